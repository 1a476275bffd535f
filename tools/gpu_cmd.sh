set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp GPU_MAX_HW_QUEUES=8; O=gpurun_out/r05tg; mkdir -p $O
REPS=2 bash tools/ab.sh prove "B=384 T=32" "B=384 T=32 BPP_IPA_TG=4" "B=384 T=32 BPP_DT_TG_MAX=4" "B=384 T=32 BPP_DT_PAIR=0" "B=384 T=32 BPP_IPA_LR=0" 2>&1 | tee $O/ab.txt
