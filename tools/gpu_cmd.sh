set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r05f; mkdir -p $O
# 1. the verifier's kernel + copy timeline (default path), then the split replay's
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $O/vtl -o run --output-format csv -- python3 tools/verify_stages.py --reps 3 > $O/vs_log.txt 2>&1 || { tail -20 $O/vs_log.txt; exit 1; }
d=$(dirname $(find $O/vtl -name run_kernel_trace.csv | head -1)); python3 tools/verify_timeline.py $d > $O/timeline.txt
echo "--- default timeline"; cat $O/timeline.txt
export BPP_VERIFY_SPLIT=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_verify_dev.py tests/test_gpu_verify_split.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/split_tests.txt 2>&1 || { tail -30 $O/split_tests.txt; exit 1; }
tail -1 $O/split_tests.txt
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $O/vtl2 -o run --output-format csv -- python3 tools/verify_stages.py --reps 3 > $O/vs2_log.txt 2>&1 || { tail -20 $O/vs2_log.txt; exit 1; }
d=$(dirname $(find $O/vtl2 -name run_kernel_trace.csv | head -1)); python3 tools/verify_timeline.py $d > $O/timeline_split.txt
echo "--- split timeline"; cat $O/timeline_split.txt
unset BPP_VERIFY_SPLIT
# 2. verify leg A/B (pageable + pinned single batch), default vs split
for rep in 1 2; do for cfg in 0 1; do
  BPP_VERIFY_SPLIT=$cfg timeout -k 10 300 python bench.py --no-cpu --proofs-per-gpu 0 --no-extra --steps 10 > $O/bv_$cfg.json 2> $O/bv_$cfg.err || { tail $O/bv_$cfg.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bv_$cfg.json'));v=d['verify_batch'];print('split=$cfg',{k:round(x['ms_per_batch'],3) for k,x in v['splits'].items()})"
done; done
# 3. prover: merged IPA rounds, parity then A/B
BPP_IPA_MERGE=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_config4.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/merge_tests.txt 2>&1 || { tail -30 $O/merge_tests.txt; exit 1; }
tail -1 $O/merge_tests.txt
B=384 T=16 R=24 REPS=3 bash tools/ab.sh prove "BPP_IPA_MERGE=0" "BPP_IPA_MERGE=1" "BPP_IPA_MERGE=1 BPP_IPA_MERGE_US=20" > $O/merge_ab.txt 2>&1; cat $O/merge_ab.txt
