# Kernel trace of T (8) batches of B (256) in flight + its occupancy summary.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp SHARED_GENS=1
OUT=gpurun_out/${1:-trinf}
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/tr -o run --output-format csv -- python3 tools/prove_inflight_exp.py ${B:-256} ${T:-8} 8 > $OUT/log.txt 2>&1 || { tail $OUT/log.txt; exit 1; }
tail -1 $OUT/log.txt
python3 tools/trace_inflight.py $OUT/tr $((${T:-8} * 8))
