# Round-6 study 2: config-4 job with the device-side IPA transcript, the
# prover's direct-table shapes at the bench's load (term groups, table
# window c), and the sharded config-5 partial's timeline at N = 8.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r06_study2; mkdir -p $O
timeout -k 10 200 python -u -m pytest tests/test_gpu_config4.py -m gpu -x -q --timeout 150 --timeout-method thread > $O/c4_tests.txt 2>&1 || { tail -30 $O/c4_tests.txt; exit 1; }
tail -1 $O/c4_tests.txt
timeout -k 10 300 python3 tools/job_ab.py "1024:0,128:0" > $O/job_default.txt 2>&1 || { tail $O/job_default.txt; exit 1; }
cat $O/job_default.txt
BPP_IPA_DEVICE_MERLIN=1 timeout -k 10 300 python3 tools/job_ab.py "1024:0,128:0" > $O/job_devmerlin.txt 2>&1 || { tail $O/job_devmerlin.txt; exit 1; }
cat $O/job_devmerlin.txt
GPU_MAX_HW_QUEUES=8 REPS=2 timeout -k 10 700 bash tools/ab.sh prove "B=384 T=32 R=12" "B=384 T=32 R=12 BPP_DT_TG_MAX=16 BPP_IPA_TG=8" "B=384 T=32 R=12 LIB=dtc15" "B=384 T=32 R=12 LIB=dtc14" > $O/prove_shapes.txt 2>&1 || { tail $O/prove_shapes.txt; exit 1; }
cat $O/prove_shapes.txt
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $O/shard_tl -o run --output-format csv -- python3 tools/shard_model.py --worlds 8 --reps 3 --no-proof-split > $O/shard_tl_log.txt 2>&1 || { echo "shard trace failed"; tail $O/shard_tl_log.txt; exit 1; }
python3 tools/verify_timeline.py $O/shard_tl > $O/shard_rank0_timeline.txt && echo timeline ok
