set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2a_gpu_tests.txt 2>&1 || { tail -30 gpurun_out/r2a_gpu_tests.txt; exit 1; }
tail -1 gpurun_out/r2a_gpu_tests.txt
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu > gpurun_out/r2a_bench.json 2> gpurun_out/r2a_bench.err || { tail gpurun_out/r2a_bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r2a_bench.json'));print(d['value'],d['ms_per_step'],d['proofs']['value'],d['proofs']['verify_batch_proofs_per_sec'])"
nproc
