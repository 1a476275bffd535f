# 2^20 MSM stream: ms per MSM over K = 20 / 60 / 120 timed steps (fill and drain of the pipeline vs steady state)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
for K in 20 60 120; do
  echo "K=$K"
  BENCH_DEBUG=1 timeout -k 10 200 python bench.py --steps $K --warmup 2 --no-cpu --proofs-per-gpu 0 --verify-proofs 0 > /tmp/k.json 2> /tmp/k.err || exit 1
  grep "pipelined again" /tmp/k.err
  python3 -c "import json; d=json.loads(open('/tmp/k.json').read().strip().splitlines()[-1]); print('timed', round(d['ms_per_step'], 4), 'ms; latency', d['latency_ms_per_msm'])"
done
