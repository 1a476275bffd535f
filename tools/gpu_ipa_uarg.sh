# round 6: one IPA's u words as kernel arguments (BPP_IPA_U_ARG, default on) vs read from pinned memory -- parity, config 2 A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r06uarg; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_ipa_hooks.py tests/test_gpu_protocol.py tests/test_golden_protocol.py tests/test_gpu_config4.py tests/test_gpu_perm.py tests/test_gpu_abi_c.py tests/test_gpu_compat.py tests/test_gpu_merlin.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.txt 2>&1 || { tail -40 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for rep in 1 2 3 4; do for f in 1 0; do echo "U_ARG=$f c2 $(BPP_IPA_U_ARG=$f timeout -k 10 120 python3 tools/config2_once.py 20 2>/dev/null)" || exit 1; done; done | tee $O/c2_uarg_ab.txt
