# Prover check: -m gpu tests (protocol + perm + config 4), a kernel trace of
# one 128-proof batch, and 8-in-flight proofs/s three times.
# Usage (on the box): bash tools/gpu_r2_prover.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-r2}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_protocol.py tests/test_gpu_perm.py tests/test_gpu_config4.py tests/test_golden_protocol.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.txt 2>&1 || { tail -40 $OUT/gpu_tests.txt; exit 1; }
tail -1 $OUT/gpu_tests.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace_proofs -o run --output-format csv -- python3 tools/prove_batch_once.py 128 > $OUT/trace_proofs_log.txt 2>&1 || { echo "proof trace failed"; exit 1; }
for i in 1 2 3; do timeout -k 10 120 python tools/prove_inflight_exp.py 128 8 16 || exit 1; done
echo done
