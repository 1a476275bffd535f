set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r05g; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || { tail -40 $O/gpu_tests.txt; exit 1; }
tail -1 $O/gpu_tests.txt
BPP_LIB=bulletproof-perm_amd/bpperm/variants/libbpperm_vst.so timeout -k 10 300 python tools/vs_phases.py > $O/vs_phases.txt 2>&1 || { tail $O/vs_phases.txt; exit 1; }
cat $O/vs_phases.txt
for rep in 1 2; do for cfg in "X=1"; do
  env $cfg timeout -k 10 300 python bench.py --no-cpu --proofs-per-gpu 0 --no-extra --steps 10 > $O/bv.json 2> $O/bv.err || { tail $O/bv.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bv.json'));v=d['verify_batch'];print('$cfg'.ljust(60),{k:round(x['ms_per_batch'],3) for k,x in v['splits'].items()}, round(v['stage_ms']['verify_scalars'],3))"
done; done
timeout -k 10 300 python bench.py --no-cpu --proofs-per-gpu 0 --verify-proofs 0 --steps 10 > $O/b2.json 2> $O/b2.err || { tail $O/b2.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/b2.json'));print(d['value'],d['result_ok'],d['config2']['latency_ms'],d['config2']['result_ok'],d['msm_2e22']['latency_ms'],d['msm_2e22']['result_ok'])"
