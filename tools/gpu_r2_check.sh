# Round-2 check: -m gpu tests, bench line (result_ok), kernel trace of one
# 128-proof batch.  Usage (on the box): bash tools/gpu_r2_check.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-r2}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.txt 2>&1 || { tail -40 $OUT/gpu_tests.txt; exit 1; }
tail -1 $OUT/gpu_tests.txt
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench.json'));print(d['value'],d['ms_per_step'],d['result_ok'],d['proofs']['value'],d['proofs']['verify_batch_proofs_per_sec'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace_proofs -o run --output-format csv -- python3 tools/prove_batch_once.py 128 > $OUT/trace_proofs_log.txt 2>&1 || { echo "proof trace failed"; exit 1; }
echo done
