# 3 in flight: K = 64 vs 128 entries per lane (pipelined figure only)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
run() {
  local label=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 40 --no-cpu --proofs-per-gpu 0 > gpurun_out/b_ab.json 2> gpurun_out/b_ab.err || { tail -5 gpurun_out/b_ab.err; exit 1; }
  python -c "
import json
d=json.load(open('gpurun_out/b_ab.json')); s=d['stage_ms']
print('$label'.ljust(10), 'piped', round(d['ms_per_step'],4), 'lat', round(d['latency_ms_per_msm'],4), 'acc', round(s['msm_accumulate'],4), d['pipelined_matches_serial'], d['result_prefix'])"
}
for pass in 1 2 3; do run K64 X=0; run K128 BPP_MSM_K=128; run K32 BPP_MSM_K=32; done
