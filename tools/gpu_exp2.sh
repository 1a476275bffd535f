# host pool size x batches in flight for the batched prover
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
for th in 4 6 8 10; do for T in 3 4 6; do echo -n "threads=$th "; BPP_HOST_THREADS=$th timeout -k 10 120 python tools/prove_inflight_exp.py 128 $T 8 || exit 1; done; done
for sp in 50 1000; do echo -n "threads=8 spin=$sp "; BPP_POOL_SPIN_US=$sp BPP_HOST_THREADS=8 timeout -k 10 120 python tools/prove_inflight_exp.py 128 4 8 || exit 1; done
echo -n "threads=8 T=1 "; BPP_HOST_THREADS=8 timeout -k 10 120 python tools/prove_inflight_exp.py 128 1 8
echo -n "threads=16 T=1 "; BPP_HOST_THREADS=16 timeout -k 10 120 python tools/prove_inflight_exp.py 128 1 8
