set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r05hq; mkdir -p $O
B=384 T=16 REPS=2 bash tools/ab.sh prove "GPU_MAX_HW_QUEUES=4" "GPU_MAX_HW_QUEUES=8" "GPU_MAX_HW_QUEUES=12" 2>&1 | tee $O/ab.txt
REPS=2 bash tools/ab.sh msm "GPU_MAX_HW_QUEUES=4" "GPU_MAX_HW_QUEUES=8" 2>&1 | tee -a $O/ab.txt
