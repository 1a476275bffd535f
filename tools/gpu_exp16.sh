# direct-table lanes per MSM after the LDS-tree change
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
for pass in 1 2 3; do
echo -n "nt256 "; timeout -k 10 120 python tools/prove_inflight_exp.py 128 8 16 || exit 1
echo -n "nt128 "; BPP_DT_NT=128 timeout -k 10 120 python tools/prove_inflight_exp.py 128 8 16 || exit 1
echo -n "nt512 "; BPP_DT_NT=512 timeout -k 10 120 python tools/prove_inflight_exp.py 128 8 16 || exit 1
done
echo -n "nt256 T1 "; timeout -k 10 120 python tools/prove_inflight_exp.py 128 1 8 || exit 1
echo -n "nt128 T1 "; BPP_DT_NT=128 timeout -k 10 120 python tools/prove_inflight_exp.py 128 1 8 || exit 1
