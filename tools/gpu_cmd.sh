set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r05vs2; mkdir -p $O
REPS=2 bash tools/ab.sh msmv "BENCH_ARGS=--verify-streams=4" "BENCH_ARGS=--verify-streams=6" "BENCH_ARGS=--verify-streams=8" 2>&1 | tee $O/ab.txt
