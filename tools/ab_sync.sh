# 8-12-16 proof batches in flight by how a host thread waits for its stream
# (library variants: default hipStreamSynchronize; pollN = hipEventQuery with
# N-us sleeps, build.py --variant pollN -D EXP_SYNC_POLL_US=N; blk =
# hipEventBlockingSync, -D EXP_SYNC_BLOCK) and host pool size.
# Usage: bash tools/ab_sync.sh "VARIANT THREADS INFLIGHT" ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp SHARED_GENS=1
V=bulletproof-perm_amd/bpperm/variants
CFGS=("$@")
for rep in 1 2 3; do
for cfg in "${CFGS[@]}"; do
  set -- $cfg
  if [ $1 = default ]; then lib=""; else lib=$V/libbpperm_$1.so; fi
  echo -n "$1 threads=$2 T=$3 "; BPP_LIB=$lib BPP_HOST_THREADS=$2 timeout -k 10 120 python tools/prove_inflight_exp.py 128 $3 12 || exit 1
done; done
