# One GPU call per round for the judged evidence: -m gpu tests + smoke, the
# full bench line, kernel-trace stats (MSM stream traced one MSM at a time,
# --inflight 1, so each launch is timed alone and its average matches the
# bench line's kernel_ms; one 384-proof batch; three config-5 batch
# verifications), FETCH_SIZE / WRITE_SIZE PMC passes over the MSM bench, the
# config-5 timeline of one unprofiled pinned batch, the per-rank shard model
# (tools/shard_model.py), the k_verify_scalars phase stamps (the vst
# variant, if built), and the prover and MSM SQ counter passes
# (gpu_pmc_prover.sh, ... msm).
# Usage (on the box): bash tools/gpu_profile_round.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-r02}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.txt 2>&1 || { tail -30 $OUT/gpu_tests.txt; exit 1; }
tail -1 $OUT/gpu_tests.txt
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.txt 2>&1 || { tail $OUT/smoke.txt; exit 1; }
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench.json'));p=d['proofs'];print(d['value'],d['ms_per_step'],d['result_ok'],p['value'],p['verify_batch_proofs_per_sec'],d['verify_batch']['value'])"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py --steps 20 --warmup 2 --no-cpu --proofs-per-gpu 0 --verify-proofs 0 --no-extra --no-extra --inflight 1 > $OUT/trace_log.txt 2>&1 || { echo "trace failed"; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/trace_proofs -o run --output-format csv -- python3 tools/prove_batch_once.py ${PROOF_BATCH:-384} > $OUT/trace_proofs_log.txt 2>&1 || { echo "proof trace failed"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace_verify -o run --output-format csv -- python3 tools/verify_stages.py --reps 3 > $OUT/trace_verify_log.txt 2>&1 || { echo "verify trace failed"; exit 1; }
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu --proofs-per-gpu 0 --verify-proofs 0 --no-extra --no-extra > $OUT/pmc_fetch_log.txt 2>&1 || { echo "pmc fetch failed"; exit 1; }
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu --proofs-per-gpu 0 --verify-proofs 0 --no-extra --no-extra > $OUT/pmc_write_log.txt 2>&1 || { echo "pmc write failed"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $OUT/vtl -o run --output-format csv -- python3 tools/verify_stages.py --reps 3 --pinned > $OUT/vtl_log.txt 2>&1 || { echo "verify timeline failed"; exit 1; }
python3 tools/verify_timeline.py $OUT/vtl > $OUT/verify_timeline_pinned.txt
timeout -k 10 300 python3 tools/shard_model.py > $OUT/shard_model.json 2> $OUT/shard_model.err || { echo "shard model failed"; exit 1; }
[ -f bulletproof-perm_amd/bpperm/variants/libbpperm_vst.so ] && { BPP_LIB=bulletproof-perm_amd/bpperm/variants/libbpperm_vst.so timeout -k 10 300 python3 tools/vs_phases.py > $OUT/vs_phases.txt 2>&1 || { echo "vs phases failed"; exit 1; }; }
bash tools/gpu_pmc_prover.sh $TAG || exit 1
bash tools/gpu_pmc_prover.sh $TAG msm || exit 1
echo done
