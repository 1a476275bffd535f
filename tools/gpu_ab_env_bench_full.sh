# Full bench line (no CPU baselines) per environment setting, interleaved
# passes; prints the MSM step, proofs/s, batch-verify and config-5 rates.
#   bash tools/gpu_ab_env_bench_full.sh "GPU_MAX_HW_QUEUES=4" "GPU_MAX_HW_QUEUES=12"
set -o pipefail
cd "$GRAFT_REPO_ROOT"
for rep in $(seq 1 ${REPS:-2}); do
for cfg in "$@"; do
  env $cfg timeout -k 10 300 python bench.py --no-cpu > gpurun_out/abf.json 2> gpurun_out/abf.err || { tail gpurun_out/abf.err; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/abf.json')); p=d['proofs']; v=d['verify_batch']
print('$cfg', 'msm %.3f ms' % d['ms_per_step'], 'acc %.3f' % d['stage_ms']['msm_accumulate'], 'proofs %.0f K' % (p['value']/1e3), 'vb %.0f K' % (p['verify_batch_proofs_per_sec']/1e3), 'c5 %.2f M' % (v['splits']['single']['value']/1e6), 'c5x2 %.2f M' % (v['splits'].get('streams', {}).get('value', 0)/1e6), 'host %.2f' % d['host_scalars']['pipelined']['pageable']['vs_resident_pipelined'], 'pinned %.2f' % d['host_scalars']['pipelined']['pinned']['vs_resident_pipelined'])"
done; done
