# round 6: per-chunk challenge inversion on the pool + vartime y^-1 (default) vs the previous build (prev): prover parity, job and B=128 / 384 batches
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r06x; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_perm.py tests/test_gpu_config4.py tests/test_gpu_protocol.py tests/test_gpu_ipa_hooks.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for rep in 1 2; do for cfg in default prev; do
  ( [ $cfg = prev ] && export BPP_LIB=bulletproof-perm_amd/bpperm/variants/libbpperm_prev.so
    echo "$cfg $(timeout -k 10 200 python3 tools/job_ab.py 1024:0,128:0 2>/dev/null | tr '\n' ' ')"
    echo "$cfg $(timeout -k 10 200 python3 tools/prove_phases.py 128 5 2>/dev/null | head -1)" ) || exit 1
done; done | tee $O/ab.txt
