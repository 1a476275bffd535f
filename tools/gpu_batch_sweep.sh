# In-flight prover throughput over (proofs per batch B, batches in flight T,
# host pool threads H), e.g. bash tools/gpu_batch_sweep.sh 128:12:4 256:8:4
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export SHARED_GENS=1
for rep in 1 2; do
for cfg in "$@"; do
  IFS=: read -r B T H <<< "$cfg"
  R=$(( 3072 / (B * T / 128) ))
  echo -n "B=$B T=$T H=$H: "; BPP_HOST_THREADS=$H timeout -k 10 150 python tools/prove_inflight_exp.py $B $T $(( R > 4 ? R / 16 : 4 )) || exit 1
done; done
