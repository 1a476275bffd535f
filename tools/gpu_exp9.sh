# A/B: direct-table MSM with an LDS block tree (variant lt) vs the butterfly
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
V=bulletproof-perm_amd/bpperm/variants/libbpperm_pg8.so
BPP_LIB=$V timeout -k 10 200 python -u -m pytest tests/test_gpu_perm.py tests/test_gpu_protocol.py tests/test_gpu_msm.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_pg8.txt 2>&1 || { tail -20 gpurun_out/t_pg8.txt; exit 1; }
tail -1 gpurun_out/t_pg8.txt
for pass in 1 2 3; do
echo -n "base T8 "; timeout -k 10 120 python tools/prove_inflight_exp.py 128 8 16 || exit 1
echo -n "pg8  T8 "; BPP_LIB=$V timeout -k 10 120 python tools/prove_inflight_exp.py 128 8 16 || exit 1
done
echo -n "base T1 "; timeout -k 10 120 python tools/prove_inflight_exp.py 128 1 8 || exit 1
echo -n "pg8  T1 "; BPP_LIB=$V timeout -k 10 120 python tools/prove_inflight_exp.py 128 1 8 || exit 1
