set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r05q; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_verify_split.py tests/test_gpu_bench_dist.py tests/test_gpu_verify_dev.py -x -v --timeout 300 --timeout-method thread > $O/t.txt 2>&1 || { tail -30 $O/t.txt; exit 1; }
tail -1 $O/t.txt
timeout -k 10 300 python tools/shard_model.py > $O/shard_model.json 2> $O/shard_model.err || { tail $O/shard_model.err; exit 1; }
cat $O/shard_model.json
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $O/smtr -o run --output-format csv -- python3 tools/shard_model.py --worlds 8 --reps 3 > $O/smtr_log.txt 2>&1 || { tail $O/smtr_log.txt; exit 1; }
python3 tools/verify_timeline.py $O/smtr > $O/smtr_timeline.txt 2>&1 || true
tail -40 $O/smtr_timeline.txt
for rep in 1 2; do for cfg in BPP_PIN_QUERY=1 BPP_PIN_QUERY=0; do
  env $cfg timeout -k 10 300 python bench.py --no-cpu --proofs-per-gpu 0 --no-extra --steps 10 > $O/bv.json 2> $O/bv.err || { tail $O/bv.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bv.json'));v=d['verify_batch'];print('$cfg'.ljust(24),{k:round(x['ms_per_batch'],3) for k,x in v['splits'].items()}, round(v['stage_ms']['verify_upload'],3), d['host_scalars'] if 'host_scalars' in d else '')"
done; done
