# round 6: J sweep again after the 8-way host sums (config 2)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r06z; mkdir -p $O
for rep in 1 2 3; do for j in 32 64 16; do echo "J=$j c2 $(BPP_IPA_SPLIT=$j timeout -k 10 120 python3 tools/config2_once.py 20 2>/dev/null)" || exit 1; done; done | tee $O/c2_jsweep2.txt
