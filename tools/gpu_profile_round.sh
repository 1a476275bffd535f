# One GPU call: full bench line, kernel-trace stats of the bench, and two
# (the kernel trace runs the MSM stream one at a time, --inflight 1, so each
# launch is measured alone: its average matches the bench line's kernel_ms)
# separate PMC passes (FETCH_SIZE, WRITE_SIZE) for the HBM-traffic field.
# Usage (on the box): bash tools/gpu_profile_round.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-r01}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py --steps 20 --warmup 2 --no-cpu --proofs-per-gpu 0 --inflight 1 > $OUT/trace_log.txt 2>&1 || { echo "trace failed"; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/trace_proofs -o run --output-format csv -- python3 tools/prove_batch_once.py 128 > $OUT/trace_proofs_log.txt 2>&1 || { echo "proof trace failed"; exit 1; }
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu --proofs-per-gpu 0 > $OUT/pmc_fetch_log.txt 2>&1 || { echo "pmc fetch failed"; exit 1; }
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu --proofs-per-gpu 0 > $OUT/pmc_write_log.txt 2>&1 || { echo "pmc write failed"; exit 1; }
echo done
