# 2^20 MSM stream (bench.py's headline leg only) over (in flight, hardware
# queues), e.g. bash tools/gpu_msm_sweep.sh 3:4 4:4 3:8
set -o pipefail
cd "$GRAFT_REPO_ROOT"
for rep in 1 2; do
for cfg in "$@"; do
  I=${cfg%%:*}; Q=${cfg##*:}
  echo -n "inflight=$I queues=$Q: "
  GPU_MAX_HW_QUEUES=$Q timeout -k 10 200 python bench.py --steps 60 --warmup 3 --no-cpu --proofs-per-gpu 0 --verify-proofs 0 --inflight $I > /tmp/msm_sweep.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.loads(open('/tmp/msm_sweep.json').read().strip().splitlines()[-1]); print(round(d['ms_per_step'], 4), 'ms', d['result_ok'])"
done; done
