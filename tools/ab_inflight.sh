set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_msm_large.py -x -q -k async --timeout 120 --timeout-method thread > gpurun_out/t_async.txt 2>&1 || { tail -30 gpurun_out/t_async.txt; exit 1; }
tail -1 gpurun_out/t_async.txt
for k in 1 2 3 4 2; do
timeout -k 10 200 python bench.py --steps 20 --no-cpu --proofs-per-gpu 0 --inflight $k > gpurun_out/b_k.json 2>/dev/null || exit 1
python -c "
import json
d=json.load(open('gpurun_out/b_k.json')); print($k, round(d['value']/1e6,1), 'Mpairs/s', 'ms/step', round(d['ms_per_step'],4), 'latency', round(d['latency_ms_per_msm'],4), d['pipelined_matches_serial'])"
done
