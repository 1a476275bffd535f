# Proofs/s at batch size B x batches in flight T (shared generator set, as
# bench.py runs it) and the host CPU load.  Usage: bash tools/ab_batch_inflight.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export SHARED_GENS=1
nproc; cat /sys/fs/cgroup/cpu.max || true
for bt in "128 8 16" "256 8 8"; do
  for th in 4 8 12 16; do
    echo -n "threads=$th "; BPP_HOST_THREADS=$th timeout -k 10 120 python tools/prove_inflight_exp.py $bt || exit 1
  done
done
