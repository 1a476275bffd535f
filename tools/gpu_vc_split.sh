# round 6: vector-commitment slices (BPP_VC_SPLIT) for config 2
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r06vc; mkdir -p $O
for rep in 1 2 3; do for j in 16 32 64; do echo "VC_SPLIT=$j c2 $(BPP_VC_SPLIT=$j timeout -k 10 120 python3 tools/config2_once.py 20 2>/dev/null)" || exit 1; done; done | tee $O/vc_split.txt
