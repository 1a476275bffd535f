set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_msm.py tests/test_gpu_msm_large.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_msm.txt 2>&1 || { tail -30 gpurun_out/t_msm.txt; exit 1; }
tail -2 gpurun_out/t_msm.txt
for i in 1 2; do
BPP_MSM_OLD_REDUCE=1 timeout -k 10 120 python bench.py --steps 20 --no-cpu --proofs-per-gpu 0 > gpurun_out/b_old.json 2>/dev/null || exit 1
timeout -k 10 120 python bench.py --steps 20 --no-cpu --proofs-per-gpu 0 > gpurun_out/b_new.json 2>/dev/null || exit 1
python -c "
import json
for f in ['old','new']:
    d=json.load(open(f'gpurun_out/b_{f}.json')); print(f, round(d['ms_per_step'],4), {k:round(v,4) for k,v in d['stage_ms'].items()}, d['result_prefix'])"
done
