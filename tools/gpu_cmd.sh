set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r05hq; mkdir -p $O
REPS=2 bash tools/ab.sh full "GPU_MAX_HW_QUEUES=4" "GPU_MAX_HW_QUEUES=8" 2>&1 | tee $O/ab_full.txt
