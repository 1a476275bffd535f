# In-flight prover throughput per environment setting, interleaved passes
# (256-proof batches, T in flight).  Usage on the box:
#   bash tools/gpu_ab_env_prove.sh "BPP_PROVE_DEV_V=0" "BPP_PROVE_DEV_V=1" ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export SHARED_GENS=1
for rep in $(seq 1 ${REPS:-3}); do
for cfg in "$@"; do
  echo -n "$cfg: "; env $cfg timeout -k 10 120 python tools/prove_inflight_exp.py ${B:-256} ${T:-12} ${R:-8} 2>/dev/null || exit 1
done; done
