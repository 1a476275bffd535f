set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r05lr; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_config4.py tests/test_gpu_perm.py tests/test_gpu_protocol.py tests/test_gpu_msm.py -x -q --timeout 120 --timeout-method thread > $O/tests2.log 2>&1 || { tail -30 $O/tests2.log; exit 1; }
tail -3 $O/tests2.log
B=384 T=16 REPS=3 bash tools/ab.sh prove "BPP_DT_PAIR=1" "BPP_DT_PAIR=0" 2>&1 | tee $O/ab3.txt
