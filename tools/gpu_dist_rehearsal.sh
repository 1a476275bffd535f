# N=2 rehearsal of bench.py on ONE GPU (gloo collectives, 2 ranks share the
# card): window split vs point split must give the same MSM (result_prefix).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp BPP_DIST_BACKEND=gloo
for split in windows points; do
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 6 --warmup 2 --log2n 18 --no-cpu --proofs-per-gpu 32 --proof-steps 2 --msm-split $split > gpurun_out/dist_$split.json 2> gpurun_out/dist_$split.err || { tail -20 gpurun_out/dist_$split.err; exit 1; }
python -c "
import json
d=json.loads(open('gpurun_out/dist_$split.json').read().strip().splitlines()[-1]); p=d['proofs']
print('$split', d['n_gpus'], d['config']['pairs'], d['result_prefix'], d['pipelined_matches_serial'], round(d['ms_per_step'],3), p['all_verified'], round(p['value']))"
done
