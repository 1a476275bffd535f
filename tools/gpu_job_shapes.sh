# config-4 job shapes with and without the small-batch spin (round 6)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r06n; mkdir -p $O
for cfg in "BPP_SPIN_BATCH=128" "BPP_SPIN_BATCH=1024"; do
  ( export $cfg; echo "## $cfg"; timeout -k 10 300 python3 tools/job_ab.py "1024:128,1024:256,1024:512,1024:1024,128:32,128:64,128:128" 2>/dev/null ) || exit 1
done | tee $O/job_shapes_spin.txt
