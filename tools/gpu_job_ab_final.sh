# round 6: the config-4 job on the last build (default) vs the build before the early completion flag (preearly), interleaved
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r06jobfin; mkdir -p $O
for rep in 1 2 3; do for v in default preearly; do
  ( [ $v = preearly ] && export BPP_LIB=bulletproof-perm_amd/bpperm/variants/libbpperm_preearly.so
    echo "$v $(timeout -k 10 200 python3 tools/job_ab.py 1024:0,128:0 2>/dev/null | tr '\n' ' ')" ) || exit 1
done; done | tee $O/job_ab.txt
