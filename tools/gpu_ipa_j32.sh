# round 6: J up to 32 -- IPA parity suites, then config 2 and the config-4 job
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r06r; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_protocol.py tests/test_golden_protocol.py tests/test_gpu_ipa_hooks.py tests/test_gpu_config4.py tests/test_gpu_perm.py tests/test_gpu_abi_c.py tests/test_gpu_compat.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for rep in 1 2 3; do echo "c2: $(timeout -k 10 120 python3 tools/config2_once.py 20 2>/dev/null)" || exit 1; done | tee $O/c2.txt
timeout -k 10 200 python3 tools/job_ab.py 1024:0,128:0 2>/dev/null | tee $O/job.txt
