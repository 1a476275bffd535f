# A/B of library variants on 8-in-flight proofs/s (prove_inflight_exp, shared
# generators).  Usage on the box: bash tools/ab_prove.sh default VARIANT ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export SHARED_GENS=1
for rep in 1 2 3; do
for v in "$@"; do
  if [ "$v" = default ]; then lib=""; else lib="bulletproof-perm_amd/bpperm/variants/libbpperm_$v.so"; fi
  echo -n "$v: "; BPP_LIB=$lib timeout -k 10 120 python tools/prove_inflight_exp.py 128 ${T:-12} 16 || exit 1
done; done
for v in "$@"; do
  if [ "$v" = default ]; then lib=""; else lib="bulletproof-perm_amd/bpperm/variants/libbpperm_$v.so"; fi
  echo -n "$v one batch: "; BPP_LIB=$lib timeout -k 10 120 python tools/prove_inflight_exp.py 128 1 8 || exit 1
done
