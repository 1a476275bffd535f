set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r05r; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_verify_split.py tests/test_gpu_verify_dev.py tests/test_gpu_msm.py tests/test_gpu_msm_large.py -x -q --timeout 300 --timeout-method thread > $O/t.txt 2>&1 || { tail -30 $O/t.txt; exit 1; }
tail -1 $O/t.txt
timeout -k 10 300 python tools/shard_model.py > $O/shard_model.json 2> $O/shard_model.err || { tail $O/shard_model.err; exit 1; }
cat $O/shard_model.json
V=bulletproof-perm_amd/bpperm/variants
for rep in 1 2; do for cfg in X=1 BPP_VERIFY_SPLIT=1 "BPP_VERIFY_SPLIT=1 BPP_LIB=$V/libbpperm_vdp2.so" BPP_LIB=$V/libbpperm_vdp2.so; do
  env $cfg timeout -k 10 300 python bench.py --no-cpu --proofs-per-gpu 0 --no-extra --steps 10 > $O/bv.json 2> $O/bv.err || { tail $O/bv.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bv.json'));v=d['verify_batch'];print('$cfg'.replace('$V/','').ljust(44),{k:round(x['ms_per_batch'],3) for k,x in v['splits'].items()}, round(v['stage_ms']['verify_scalars'],3))"
done; done
