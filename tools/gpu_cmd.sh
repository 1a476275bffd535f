set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r05de; mkdir -p $O
B=384 T=16 REPS=3 bash tools/ab.sh prove "BPP_PED_DBL=0" "BPP_PED_DBL=1 BPP_DE_K=2" "BPP_PED_DBL=1 BPP_DE_K=4" "BPP_PED_DBL=1 BPP_DE_K=8" 2>&1 | tee $O/ab2.txt
B=384 REPS=2 bash tools/ab.sh one "BPP_PED_DBL=0" "BPP_PED_DBL=1 BPP_DE_K=2" "BPP_PED_DBL=1 BPP_DE_K=4" "BPP_PED_DBL=1 BPP_DE_K=8" 2>&1 | tee $O/ab2one.txt
