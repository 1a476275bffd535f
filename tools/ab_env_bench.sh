# A/B of MSM env switches on the pipelined 2^20 bench: bash tools/ab_env_bench.sh "ENV=.. ENV2=.." "..." ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
for cfg in "$@"; do
  env $cfg timeout -k 10 200 python bench.py --steps 20 --no-cpu --proofs-per-gpu 0 > gpurun_out/b_ab.json 2> gpurun_out/b_ab.err || { tail -5 gpurun_out/b_ab.err; exit 1; }
  python -c "
import json
d=json.load(open('gpurun_out/b_ab.json')); s=d['stage_ms']
print('$cfg'.ljust(40), 'piped', round(d['ms_per_step'],4), 'lat', round(d['latency_ms_per_msm'],4), 'acc', round(s['msm_accumulate'],4), 'red', round(s['msm_reduce'],4), d['pipelined_matches_serial'], d['result_ok'])
v=d.get('verify_batch')
if v: print('   verify5 single', round(v['splits']['single']['ms_per_batch'],3), 'ms streams', round(v['splits']['streams']['ms_per_batch'],3), 'ms red', round(v['stage_ms']['msm_reduce'],3), 'acc', round(v['stage_ms']['msm_accumulate'],3), v['rejects_tampered'], v['splits']['single']['all_verified'])"
done
