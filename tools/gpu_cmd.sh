set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r05lr; mkdir -p $O
B=384 T=16 REPS=3 bash tools/ab.sh prove "BPP_IPA_LR=1" "BPP_IPA_LR=1 BPP_IPA_TG=4" "BPP_IPA_LR=0" "BPP_IPA_LR=1 BPP_IPA_TG=16" 2>&1 | tee $O/ab2.txt
