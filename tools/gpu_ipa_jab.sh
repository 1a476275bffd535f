# round 6: J rule A/B (default: J <= 32, one lane group's term per slice; jold: J <= 16, two) -- config 2 and job, interleaved
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r06s; mkdir -p $O
for rep in 1 2; do
for cfg in "LIB=default" "LIB=jold"; do
  ( [ $cfg = LIB=jold ] && export BPP_LIB=bulletproof-perm_amd/bpperm/variants/libbpperm_jold.so
    echo "$cfg c2 $(timeout -k 10 120 python3 tools/config2_once.py 20 2>/dev/null)"
    echo "$cfg $(timeout -k 10 200 python3 tools/job_ab.py 1024:0,128:0 2>/dev/null | tr '\n' ' ')" ) || exit 1
done; done | tee $O/jab.txt
