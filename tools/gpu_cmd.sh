set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r05y; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/t.txt 2>&1 || { tail -30 $O/t.txt; exit 1; }
tail -1 $O/t.txt
for rep in 1 2; do for cfg in BPP_IPA_QSLOT=0 BPP_IPA_QSLOT=1; do
  env $cfg timeout -k 10 300 python tools/config2_once.py 20 2>&1 | tail -1 | sed "s|^|$cfg |"
done; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/c2 -o run --output-format csv -- python3 tools/config2_once.py 5 > $O/c2_log.txt 2>&1 || { tail $O/c2_log.txt; exit 1; }
python3 tools/kstats.py -n 14 $O/c2/run_kernel_stats.csv
