# (rejected) cross + cross-final both fused in k_ipa_terms ("cache") vs separate kernels ("upl", BPP_IPA_CROSS=1)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.txt 2>&1 || { tail -30 gpurun_out/gpu_tests.txt; exit 1; }
tail -1 gpurun_out/gpu_tests.txt
for pass in 1 2 3; do
echo -n "upl   "; BPP_IPA_CROSS=1 timeout -k 10 120 python tools/prove_inflight_exp.py 128 8 16 || exit 1
echo -n "cache "; timeout -k 10 120 python tools/prove_inflight_exp.py 128 8 16 || exit 1
done
echo -n "upl   T1 "; BPP_IPA_CROSS=1 timeout -k 10 120 python tools/prove_inflight_exp.py 128 1 8 || exit 1
echo -n "cache T1 "; timeout -k 10 120 python tools/prove_inflight_exp.py 128 1 8 || exit 1
