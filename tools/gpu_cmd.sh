set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp GPU_MAX_HW_QUEUES=8; O=gpurun_out/r05ht; mkdir -p $O
REPS=2 bash tools/ab.sh prove "B=384 T=32" "B=384 T=32 BPP_HOST_THREADS=2" "B=384 T=32 BPP_HOST_THREADS=8" "B=384 T=32 GPU_MAX_HW_QUEUES=12" 2>&1 | tee $O/ab.txt
