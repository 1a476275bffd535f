# Device-side Merlin A/B (BPP_IPA_DEVICE_MERLIN): parity tests, then proofs/s
# at 12 batches (256 proofs) in flight and one batch alone, then a kernel trace of one
# batch on the device path.  Usage: bash tools/ab_dev_merlin.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp SHARED_GENS=1
OUT=gpurun_out/${1:-devm}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_merlin.py tests/test_gpu_protocol.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/tests.txt 2>&1 || { tail -30 $OUT/tests.txt; exit 1; }
tail -1 $OUT/tests.txt
for rep in 1 2 3; do for dm in 0 1; do
  echo -n "device_merlin=$dm 8 in flight: "; BPP_IPA_DEVICE_MERLIN=$dm timeout -k 10 120 python tools/prove_inflight_exp.py 256 12 8 || exit 1
done; done
for dm in 0 1; do
  echo -n "device_merlin=$dm one batch: "; BPP_IPA_DEVICE_MERLIN=$dm timeout -k 10 120 python tools/prove_inflight_exp.py 256 1 8 || exit 1
done
BPP_IPA_DEVICE_MERLIN=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 tools/prove_batch_once.py 256 > $OUT/trace.log 2>&1 || { echo "trace failed"; exit 1; }
python3 tools/kstats.py $OUT/trace/run_kernel_stats.csv > $OUT/kstats.txt && sed -n 1,16p $OUT/kstats.txt
