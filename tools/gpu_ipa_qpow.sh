# round 6: Q as its doublings in the fused IPA rounds (BPP_IPA_QPOW, default on) vs the per-call Q-slot table -- parity, config 2 A/B, a trace
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r06qp4; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_ipa_hooks.py tests/test_gpu_protocol.py tests/test_golden_protocol.py tests/test_gpu_config4.py tests/test_gpu_perm.py tests/test_gpu_abi_c.py tests/test_gpu_compat.py tests/test_gpu_merlin.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/tests.txt 2>&1 || { tail -40 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
BPP_IPA_QPOW=0 timeout -k 10 300 python -u -m pytest tests/test_gpu_ipa_hooks.py tests/test_gpu_protocol.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests_qslot.txt 2>&1 || { tail -40 $O/tests_qslot.txt; exit 1; }
tail -1 $O/tests_qslot.txt
for rep in 1 2 3; do for f in 1 0; do echo "QPOW=$f c2 $(BPP_IPA_QPOW=$f timeout -k 10 120 python3 tools/config2_once.py 20 2>/dev/null)" || exit 1; done; done | tee $O/c2_qpow_ab.txt
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace -d $O/tr -o run --output-format csv -- python3 tools/config2_once.py 3 > $O/trlog.txt 2>&1 || { tail $O/trlog.txt; exit 1; }
python3 tools/trace_tail.py $O/tr 1.0 > $O/timeline.txt; head -24 $O/timeline.txt
