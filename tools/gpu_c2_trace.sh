# round 6: config 2 kernel + copy timeline (the last run of 3)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r06t; mkdir -p $O
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace -d $O/tr -o run --output-format csv -- python3 tools/config2_once.py 3 > $O/log.txt 2>&1 || { tail $O/log.txt; exit 1; }
python3 tools/trace_tail.py $O/tr 1.2 > $O/timeline.txt; tail -40 $O/timeline.txt
