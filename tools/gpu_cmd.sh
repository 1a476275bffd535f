set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r05u; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_verify_dev.py tests/test_gpu_verify_split.py tests/test_gpu_abi_c.py -x -q --timeout 300 --timeout-method thread > $O/t.txt 2>&1 || { tail -30 $O/t.txt; exit 1; }
tail -1 $O/t.txt
for rep in 1 2 3; do for cfg in BPP_VERIFY_EARLY=0 BPP_VERIFY_EARLY=1 "BPP_VERIFY_EARLY=1 BPP_VERIFY_PIECE_KB=1024"; do
  env $cfg timeout -k 10 300 python bench.py --no-cpu --proofs-per-gpu 0 --no-extra --steps 10 > $O/bv.json 2> $O/bv.err || { tail $O/bv.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bv.json'));v=d['verify_batch'];print('$cfg'.ljust(44),{k:round(x['ms_per_batch'],3) for k,x in v['splits'].items()}, v['rejects_tampered'], all(x['all_verified'] for x in v['splits'].values()))"
done; done
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $O/vtl -o run --output-format csv -- python3 tools/verify_stages.py --reps 3 > $O/vtl_log.txt 2>&1 || { tail $O/vtl_log.txt; exit 1; }
python3 tools/verify_timeline.py $O/vtl > $O/timeline.txt 2>&1; cat $O/timeline.txt
