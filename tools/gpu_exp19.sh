# hardware queues per process (HIP default 4) with 8 proof batches in flight
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
for pass in 1 2 3; do
for q in 4 8 16; do echo -n "hwq=$q "; GPU_MAX_HW_QUEUES=$q timeout -k 10 120 python tools/prove_inflight_exp.py 128 8 16 || exit 1; done
done
echo -n "hwq=16 T12 "; GPU_MAX_HW_QUEUES=16 timeout -k 10 120 python tools/prove_inflight_exp.py 128 12 12 || exit 1
