set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r05n; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || { grep -E "PASS|FAIL|Error|error" $O/gpu_tests.txt | tail -30; tail -30 $O/gpu_tests.txt; exit 1; }
tail -1 $O/gpu_tests.txt
for rep in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu --proofs-per-gpu 0 --steps 10 > $O/bv.json 2> $O/bv.err || { tail $O/bv.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bv.json'));v=d['verify_batch'];print(d['value'], d['result_ok'], {k:round(x['ms_per_batch'],3) for k,x in v['splits'].items()}, round(v['stage_ms']['msm_reduce'],3), d['config2']['latency_ms'], d['msm_2e22']['latency_ms'], d['msm_2e22']['result_ok'])"
done
