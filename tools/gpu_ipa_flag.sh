# round 6: the IPA rounds' completion flag (BPP_IPA_FLAG, default on) -- parity suites, then config 2 and the job A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r06fl2; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_ipa_hooks.py tests/test_gpu_protocol.py tests/test_golden_protocol.py tests/test_gpu_config4.py tests/test_gpu_perm.py tests/test_gpu_abi_c.py tests/test_gpu_compat.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/tests.txt 2>&1 || { tail -40 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for rep in 1 2 3; do for f in 1 0; do echo "FLAG=$f c2 $(BPP_IPA_FLAG=$f timeout -k 10 120 python3 tools/config2_once.py 20 2>/dev/null)" || exit 1; done; done | tee $O/c2_flag_ab.txt
for rep in 1 2; do for f in 1 0; do echo "FLAG=$f $(BPP_IPA_FLAG=$f timeout -k 10 200 python3 tools/job_ab.py 1024:0,128:0 2>/dev/null | tr '\n' ' ')" || exit 1; done; done | tee $O/job_flag_ab.txt
