set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r06f; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_rccl.py -m gpu -x -v --timeout 250 --timeout-method thread > $O/rccl_test.txt 2>&1 || { tail -40 $O/rccl_test.txt; exit 1; }
tail -1 $O/rccl_test.txt
timeout -k 10 250 python3 tools/rccl_world1.py --port 29611 > $O/rccl_world1.json 2> $O/rccl_world1.err || { tail $O/rccl_world1.err; exit 1; }
cat $O/rccl_world1.json
for K in 8 12 16 24; do
  BPP_MSM_ACC_K=$K timeout -k 10 200 python3 tools/shard_model.py --worlds 8 --reps 7 --no-proof-split > $O/shard_k$K.json 2> $O/shard_k$K.err || { tail $O/shard_k$K.err; exit 1; }
  echo "K=$K $(cat $O/shard_k$K.json)"
done
timeout -k 10 90 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29622 tools/rccl_dup_probe.py > $O/dup_probe.txt 2>&1; echo "dup probe rc=$?"; tail -15 $O/dup_probe.txt
