# Where does the prover's direct-table gather stall go?
# Translation (UTCL1) and L2-latency counters of k_dt_msm / k_ipa_round_dt
# under the prover's load shape, one rocprofv3 --pmc pass each, for the
# configurations given (e.g. BPP_DT_PAIR=0 / =1).  Summarise with
# tools/tlb_summary.py.
# Usage (on the box): bash tools/gpu_tlb_prover.sh TAG "CFG" ["CFG" ...]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp SHARED_GENS=1
TAG=$1; shift
CMD="python3 tools/prove_inflight_exp.py ${PMC_SHAPE:-384 16 2}"
i=0
for cfg in "$@"; do
  i=$((i+1))
  OUT=gpurun_out/tlb_$TAG/c$i
  mkdir -p $OUT
  echo "$cfg" > $OUT/cfg.txt
  j=0
  for PASS in "TCP_UTCL1_REQUEST_sum TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_PENDING_STALL_CYCLES_sum" \
              "TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_UTCL1_SERIALIZATION_STALL_sum TCP_TCP_LATENCY_sum" \
              "SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE GRBM_UTCL2_BUSY"; do
    j=$((j+1))
    ( for kv in $cfg; do export "$kv"; done
      timeout -s KILL 120 rocprofv3 --pmc $PASS -d $OUT/p$j -o run --output-format csv -- $CMD > $OUT/p${j}_log.txt 2>&1 ) \
      || { echo "cfg $i pass $j failed"; tail -5 $OUT/p${j}_log.txt; exit 1; }
  done
done
echo done
