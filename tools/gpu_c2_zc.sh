# round 6: IPA inputs read in place (BPP_IPA_ZC_IN) -- parity suites, then config 2 A/B and phases
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r06v; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_protocol.py tests/test_golden_protocol.py tests/test_gpu_ipa_hooks.py tests/test_gpu_config4.py tests/test_gpu_perm.py tests/test_gpu_abi_c.py tests/test_gpu_compat.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for rep in 1 2 3; do for z in 1 0; do echo "ZC_IN=$z c2 $(BPP_IPA_ZC_IN=$z timeout -k 10 120 python3 tools/config2_once.py 20 2>/dev/null)" || exit 1; done; done | tee $O/c2_zc_ab.txt
timeout -k 10 200 python3 tools/config2_phases.py 20 > $O/phases.txt 2>&1 || { tail $O/phases.txt; exit 1; }
cat $O/phases.txt
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace -d $O/tr -o run --output-format csv -- python3 tools/config2_once.py 3 > $O/trlog.txt 2>&1 || { tail $O/trlog.txt; exit 1; }
python3 tools/trace_tail.py $O/tr 1.1 > $O/timeline.txt; head -16 $O/timeline.txt
