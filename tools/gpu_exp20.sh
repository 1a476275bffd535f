# bench.py with GPU_MAX_HW_QUEUES 4 vs 16 (MSM stream + proofs)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
for pass in 1 2; do for q in 4 16; do
GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python bench.py --no-cpu > gpurun_out/b_q.json 2> gpurun_out/b_q.err || { tail -5 gpurun_out/b_q.err; exit 1; }
python -c "
import json
d=json.load(open('gpurun_out/b_q.json')); p=d['proofs']
print('hwq=$q', 'msm', round(d['value']/1e6,1), round(d['ms_per_step'],4), 'proofs', round(p['value']), 'verify', round(p['verify_batch_proofs_per_sec']), p['all_verified'])"
done; done
