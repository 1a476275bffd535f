set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r06k; mkdir -p $O
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace -d $O/c2tl -o run --output-format csv -- python3 tools/config2_once.py 5 > $O/c2tl_log.txt 2>&1 || { tail $O/c2tl_log.txt; exit 1; }
python3 tools/trace_tail.py $O/c2tl 1.45 > $O/c2_timeline.txt && tail -60 $O/c2_timeline.txt
for s in 100 200 400 800; do echo "spin $s: $(BPP_IPA_SPIN_US=$s timeout -k 10 120 python3 tools/config2_once.py 20 2>/dev/null)"; done
