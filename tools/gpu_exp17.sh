# V commitments encoded on the host (2 (C/2), BPP_PED_DOUBLE_MAX=16384) vs on the GPU
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
BPP_PED_DOUBLE_MAX=16384 timeout -k 10 200 python -u -m pytest tests/test_gpu_perm.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_pd.txt 2>&1 || { tail -20 gpurun_out/t_pd.txt; exit 1; }
tail -1 gpurun_out/t_pd.txt
for pass in 1 2 3; do
echo -n "gpu  "; timeout -k 10 120 python tools/prove_inflight_exp.py 128 8 16 || exit 1
echo -n "host "; BPP_PED_DOUBLE_MAX=16384 timeout -k 10 120 python tools/prove_inflight_exp.py 128 8 16 || exit 1
done
echo -n "gpu  T1 "; timeout -k 10 120 python tools/prove_inflight_exp.py 128 1 8 || exit 1
echo -n "host T1 "; BPP_PED_DOUBLE_MAX=16384 timeout -k 10 120 python tools/prove_inflight_exp.py 128 1 8 || exit 1
