# A/B of the direct-table window width (BPP_DT_C) and lanes per MSM
# (BPP_DT_NT): parity first, then 8-in-flight proofs/s and one-batch kernel
# traces.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/ab_dt_c2
mkdir -p $OUT
for C in 8 11; do
  BPP_DT_C=$C timeout -k 10 300 python -u -m pytest tests/test_gpu_protocol.py tests/test_gpu_perm.py tests/test_golden_protocol.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/tests_c$C.txt 2>&1 || { echo "c=$C tests failed"; tail -30 $OUT/tests_c$C.txt; exit 1; }
  echo "c=$C $(tail -1 $OUT/tests_c$C.txt)"
done
BPP_DT_NT=512 BPP_DT_C=11 timeout -k 10 300 python -u -m pytest tests/test_gpu_perm.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/tests_nt512.txt 2>&1 || { echo "nt512 tests failed"; tail -30 $OUT/tests_nt512.txt; exit 1; }
for i in 1 2; do for C in 8 11 12; do for NT in 256 512; do
  echo -n "c=$C nt=$NT "; BPP_DT_NT=$NT BPP_DT_C=$C timeout -k 10 120 python tools/prove_inflight_exp.py 128 8 16 || exit 1
done; done; done
for C in 8 11; do for NT in 256 512; do
  BPP_DT_NT=$NT BPP_DT_C=$C timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace_c${C}_$NT -o run --output-format csv -- python3 tools/prove_batch_once.py 128 > $OUT/trace_c${C}_$NT.txt 2>&1 || { echo "trace failed"; exit 1; }
done; done
echo done
