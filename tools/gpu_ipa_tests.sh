# IPA / prover parity suites (after ipa_api / host-sum changes), then config 2 A/B: 8-way partial sums (default) vs scalar (BPP_HOST_IFMA=0)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r06y; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_ipa_hooks.py tests/test_gpu_protocol.py tests/test_golden_protocol.py tests/test_gpu_config4.py tests/test_gpu_perm.py tests/test_gpu_abi_c.py tests/test_gpu_compat.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/tests.txt 2>&1 || { tail -40 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for rep in 1 2 3; do for f in 1 0; do echo "IFMA=$f c2 $(BPP_HOST_IFMA=$f timeout -k 10 120 python3 tools/config2_once.py 20 2>/dev/null)" || exit 1; done; done | tee $O/c2_sum_ab.txt
for f in 1 0; do echo "IFMA=$f $(BPP_HOST_IFMA=$f timeout -k 10 200 python3 tools/prove_phases.py 16 5 2>/dev/null | head -1)" || exit 1; done | tee $O/b16_sum_ab.txt
