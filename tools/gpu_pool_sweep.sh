# In-flight prover throughput over (batches in flight T, host pool threads
# BPP_HOST_THREADS) pairs, e.g. bash tools/gpu_pool_sweep.sh 12:8 16:1 16:2
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export SHARED_GENS=1
for rep in 1 2; do
for cfg in "$@"; do
  T=${cfg%%:*}; H=${cfg##*:}
  echo -n "T=$T threads=$H: "; BPP_HOST_THREADS=$H timeout -k 10 120 python tools/prove_inflight_exp.py ${B:-256} $T ${R:-8} || exit 1
done; done
