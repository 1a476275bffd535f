# Round-4 final call: the parallel-append replay A/B on the config-5 batch,
# then the full profile round of the final build (tools/gpu_profile_round.sh).
# Usage (on the box): bash tools/gpu_final_r04.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
V=bulletproof-perm_amd/bpperm/variants
NOTRACE=1 REPS=3 bash tools/verify_ab.sh par "BPP_X=0" "BPP_LIB=$V/libbpperm_par.so" > gpurun_out/par_ab.txt 2>&1 || { tail gpurun_out/par_ab.txt; exit 1; }
bash tools/gpu_profile_round.sh ${1:-r04f} || exit 1
echo final-done
