# PMC counters of the prover's kernels under the bench's load shape (384-proof
# batches, 16 contexts in flight, PMC_SHAPE overrides; the profiler serialises dispatches, so each
# kernel's counters are its own).  One counter pass per rocprofv3 run.
# Usage (on the box): bash tools/gpu_pmc_prover.sh <tag> [msm]
#   msm: the same passes over the 2^20 MSM bench stream instead
#   verify: over config-5 batch verifications (tools/verify_stages.py)
#        (-> gpurun_out/pmc_msm_<tag>; summarise with pmc_prover_summary.py)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp SHARED_GENS=1
TAG=${1:-r02}
OUT=gpurun_out/pmc_prover_$TAG
CMD="python3 tools/prove_inflight_exp.py ${PMC_SHAPE:-384 16 2}"
if [ "$2" = "msm" ]; then
  OUT=gpurun_out/pmc_msm_$TAG
  CMD="python3 bench.py --steps 6 --warmup 1 --no-cpu --proofs-per-gpu 0 --verify-proofs 0 --no-extra --no-extra"
fi
if [ "$2" = "verify" ]; then  # one config-5 batch verification's kernels (tools/verify_stages.py)
  OUT=gpurun_out/pmc_verify_$TAG
  CMD="python3 tools/verify_stages.py --reps 2"
fi
mkdir -p $OUT
timeout -s KILL 60 rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
i=0
for PASS in "SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE" \
            "SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_BRANCH" \
            "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $PASS -d $OUT/p$i -o run --output-format csv -- $CMD > $OUT/p${i}_log.txt 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p${i}_log.txt; exit 1; }
done
echo done
