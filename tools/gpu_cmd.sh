set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r05k; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || { tail -30 $O/gpu_tests.txt; exit 1; }
tail -1 $O/gpu_tests.txt
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail $O/smoke.txt; exit 1; }
timeout -k 10 500 python bench.py > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench.json'));p=d['proofs'];v=d['verify_batch'];print(d['value'],d['ms_per_step'],d['result_ok'],p['value'],p['batches_in_flight_per_gpu'],p['verify_batch_proofs_per_sec'],p['alu_roofline']['whole_prover_frac'],{k:round(x['ms_per_batch'],3) for k,x in v['splits'].items()},d['config2']['latency_ms'],d['msm_2e22']['latency_ms'])"
