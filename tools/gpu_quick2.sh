# large-MSM parity tests, one bench line, rank shares at N = 1, 8
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_msm_large.py tests/test_gpu_msm.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_quick.txt 2>&1 || { tail -30 gpurun_out/t_quick.txt; exit 1; }
tail -1 gpurun_out/t_quick.txt
timeout -k 10 200 python bench.py --steps 20 --no-cpu --proofs-per-gpu 0 > gpurun_out/b_quick.json 2> gpurun_out/b_quick.err || { tail -20 gpurun_out/b_quick.err; exit 1; }
python -c "
import json
d=json.load(open('gpurun_out/b_quick.json')); print(round(d['value']/1e6,1), 'Mpairs/s', 'ms/step', round(d['ms_per_step'],4), 'latency', round(d['latency_ms_per_msm'],4), d['pipelined_matches_serial'], {k:round(v,4) for k,v in d['stage_ms'].items()}, d['result_prefix'])"
timeout -k 10 300 python tools/rank_share.py 4 8 > gpurun_out/rank_share.jsonl 2> gpurun_out/rank_share.err || { tail -5 gpurun_out/rank_share.err; exit 1; }
cat gpurun_out/rank_share.jsonl
