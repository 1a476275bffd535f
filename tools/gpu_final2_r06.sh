# round 6 final check after the Q-as-doublings IPA: every -m gpu test, smoke, the default bench line, config 2 A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r06final4; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || { tail -30 $O/gpu_tests.txt; exit 1; }
tail -1 $O/gpu_tests.txt
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail $O/smoke.txt; exit 1; }
tail -2 $O/smoke.txt
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench.json'));p=d['proofs'];v=d['verify_batch']['splits'];print('msm',d['value'],'proofs',p['value'],'job',p['job']['ms_per_job'],'c5',v['single']['ms_per_batch'],v['single_pinned']['ms_per_batch'],v['streams']['value'],'c2',d['config2']['latency_ms'],d['config2']['result_ok'],'ok',d['result_ok'])"
for rep in 1 2 3; do for f in 1 0; do echo "QPOW=$f c2 $(BPP_IPA_QPOW=$f timeout -k 10 120 python3 tools/config2_once.py 20 2>/dev/null)" || exit 1; done; done | tee $O/c2_qpow_ab.txt
