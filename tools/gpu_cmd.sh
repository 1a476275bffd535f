set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r05l; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_msm.py tests/test_gpu_bench_dist.py -x -q --timeout 120 --timeout-method thread > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail $O/smoke.txt; exit 1; }
timeout -k 10 500 python bench.py > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench.json'));p=d['proofs'];v=d['verify_batch'];print(d['value'],d['ms_per_step'],d['result_ok'],d['pipelined_matches_serial'],d['config']['in_flight'],p['value'],{k:round(x['ms_per_batch'],3) for k,x in v['splits'].items()},d['host_scalars']['pipelined']['pageable']['vs_resident_pipelined'],d['config2']['latency_ms'])"
