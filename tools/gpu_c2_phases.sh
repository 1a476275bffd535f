# round 6: config 2 host phases (tools/config2_phases.py), device J-sum on / off (BPP_IPA_JSUM; default off since this run)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r06u; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_protocol.py tests/test_golden_protocol.py tests/test_gpu_ipa_hooks.py tests/test_gpu_config4.py tests/test_gpu_abi_c.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
BPP_IPA_JSUM=1 timeout -k 10 200 python3 tools/config2_phases.py 20 > $O/phases_jsum1.txt 2>&1 || { tail $O/phases_jsum1.txt; exit 1; }
BPP_IPA_JSUM=0 timeout -k 10 200 python3 tools/config2_phases.py 20 > $O/phases_jsum0.txt 2>&1 || { tail $O/phases_jsum0.txt; exit 1; }
for rep in 1 2; do for j in 1 0; do echo "JSUM=$j c2 $(BPP_IPA_JSUM=$j timeout -k 10 120 python3 tools/config2_once.py 20 2>/dev/null)" || exit 1; done; done | tee $O/c2_jsum_ab.txt
cat $O/phases_jsum1.txt $O/phases_jsum0.txt
