set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r05p2; mkdir -p $O
BPP_LIB=bulletproof-perm_amd/bpperm/variants/libbpperm_p2.so timeout -k 10 400 python -u -m pytest tests/test_gpu_protocol.py tests/test_gpu_config4.py tests/test_gpu_perm.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
B=384 T=16 REPS=3 bash tools/ab.sh prove "LIB=p2" "LIB=default" 2>&1 | tee $O/ab.txt
B=384 REPS=2 bash tools/ab.sh one "LIB=p2" "LIB=default" 2>&1 | tee -a $O/ab.txt
for L in bulletproof-perm_amd/bpperm/variants/libbpperm_p2.so ""; do BPP_LIB=$L timeout -k 10 120 python tools/config2_once.py 20 2>&1 | tail -1; done | tee -a $O/ab.txt
