# batches in flight 8 vs 12 (8-thread host pool)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
for pass in 1 2 3; do
echo -n "T8  "; timeout -k 10 120 python tools/prove_inflight_exp.py 128 8 16 || exit 1
echo -n "T12 "; timeout -k 10 120 python tools/prove_inflight_exp.py 128 12 12 || exit 1
echo -n "T6  "; timeout -k 10 120 python tools/prove_inflight_exp.py 128 6 20 || exit 1
done
