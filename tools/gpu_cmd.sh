set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r05up2; mkdir -p $O
BPP_VERIFY_UP2=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_verify_dev.py tests/test_gpu_verify_split.py tests/test_gpu_perm.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for rep in 1 2 3; do for cfg in BPP_VERIFY_UP2=1 BPP_VERIFY_UP2=0; do
  env $cfg timeout -k 10 300 python bench.py --no-cpu --proofs-per-gpu 0 --no-extra --steps 10 > $O/bv.json 2> $O/bv.err || { tail $O/bv.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bv.json'));v=d['verify_batch'];print('$cfg'.ljust(20),{k:round(x['ms_per_batch'],3) for k,x in v['splits'].items()}, v['rejects_tampered'])"
done; done 2>&1 | tee $O/ab.txt
