set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r05s; mkdir -p $O
timeout -k 10 300 python tools/shard_model.py --worlds 8,4,2 > $O/shard_model.json 2> $O/shard_model.err || { tail $O/shard_model.err; exit 1; }
cat $O/shard_model.json
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $O/smtr -o run --output-format csv -- python3 tools/shard_model.py --worlds 8 --reps 3 > $O/smtr_log.txt 2>&1 || { tail $O/smtr_log.txt; exit 1; }
python3 tools/verify_timeline.py $O/smtr > $O/smtr_timeline.txt 2>&1; cat $O/smtr_timeline.txt
