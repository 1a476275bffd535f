set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r05sh3; mkdir -p $O
REPS=2 bash tools/ab.sh full "BENCH_ARGS=--proof-streams=16" "BENCH_ARGS=--proof-streams=24" "BENCH_ARGS=--proof-streams=32" 2>&1 | tee $O/ab.txt
