# 256-proof batches x T in flight under GPU_MAX_HW_QUEUES = Q (HIP's
# hardware queues per process; the box default is 4), e.g.
# bash tools/gpu_queue_sweep.sh 4:8 8:8 8:12
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export SHARED_GENS=1
for rep in 1 2; do
for cfg in "$@"; do
  Q=${cfg%%:*}; T=${cfg##*:}
  echo -n "Q=$Q T=$T: "; GPU_MAX_HW_QUEUES=$Q timeout -k 10 150 python tools/prove_inflight_exp.py 256 $T 12 || exit 1
done; done
