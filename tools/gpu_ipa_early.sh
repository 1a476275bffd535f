# round 6: completion flag before the split round's state writes (default) vs after the whole round (prev) -- parity, config 2 A/B, job
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r06early; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_ipa_hooks.py tests/test_gpu_protocol.py tests/test_golden_protocol.py tests/test_gpu_config4.py tests/test_gpu_perm.py tests/test_gpu_abi_c.py tests/test_gpu_compat.py tests/test_gpu_merlin.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.txt 2>&1 || { tail -40 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for rep in 1 2 3; do for v in default prev; do
  ( [ $v = prev ] && export BPP_LIB=bulletproof-perm_amd/bpperm/variants/libbpperm_prev.so
    echo "$v c2 $(timeout -k 10 120 python3 tools/config2_once.py 20 2>/dev/null)" ) || exit 1
done; done | tee $O/c2_early_ab.txt
timeout -k 10 200 python3 tools/job_ab.py 1024:0 2>/dev/null | tee $O/job.txt
