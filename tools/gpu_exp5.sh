# 16-bit direct tables in the 8-in-flight regime
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
for pass in 1 2; do
echo -n "c8  "; timeout -k 10 120 python tools/prove_inflight_exp.py 128 8 12 || exit 1
echo -n "c16 "; BPP_DT_C=16 timeout -k 10 120 python tools/prove_inflight_exp.py 128 8 12 || exit 1
echo -n "c16 nt128 "; BPP_DT_NT=128 BPP_DT_C=16 timeout -k 10 120 python tools/prove_inflight_exp.py 128 8 12 || exit 1
done
echo -n "c16 T=1 "; BPP_DT_C=16 timeout -k 10 120 python tools/prove_inflight_exp.py 128 1 8 || exit 1
echo -n "c8 T=1 "; timeout -k 10 120 python tools/prove_inflight_exp.py 128 1 8 || exit 1
