set -o pipefail
cd "$GRAFT_REPO_ROOT"
for i in 1 2 3; do
echo -n "own    "; timeout -k 10 120 python tools/prove_inflight_exp.py 128 8 16 || exit 1
echo -n "shared "; SHARED_GENS=1 timeout -k 10 120 python tools/prove_inflight_exp.py 128 8 16 || exit 1
done
