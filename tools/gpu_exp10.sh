# MSM stream: in-flight depth and entries per lane
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
run() {  # label, env..., -- bench args
  local label=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 30 --no-cpu --proofs-per-gpu 0 $BARGS > gpurun_out/b_ab.json 2> gpurun_out/b_ab.err || { tail -5 gpurun_out/b_ab.err; exit 1; }
  python -c "
import json
d=json.load(open('gpurun_out/b_ab.json')); s=d['stage_ms']
print('$label'.ljust(22), 'piped', round(d['ms_per_step'],4), 'lat', round(d['latency_ms_per_msm'],4), 'acc', round(s['msm_accumulate'],4), d['pipelined_matches_serial'], d['result_prefix'])"
}
for pass in 1 2; do
BARGS="--inflight 2" run "inflight2" X=0
BARGS="--inflight 3" run "inflight3" X=0
BARGS="--inflight 2" run "K128" BPP_MSM_K=128
BARGS="--inflight 2" run "pad9000" BPP_ACC_LDS_PAD=9000
done
