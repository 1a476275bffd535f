# A/B of library variants at the bench's prover shape (256-proof batches x 12
# in flight, 4 pool threads), alternating, 3 rounds.
# Usage on the box: bash tools/ab_batch.sh default VARIANT ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export SHARED_GENS=1 BPP_HOST_THREADS=4
for rep in 1 2 3; do
for v in "$@"; do
  if [ "$v" = default ]; then lib=""; else lib="bulletproof-perm_amd/bpperm/variants/libbpperm_$v.so"; fi
  echo -n "$v: "; BPP_LIB=$lib timeout -k 10 150 python tools/prove_inflight_exp.py 256 ${T:-12} 12 || exit 1
done; done
