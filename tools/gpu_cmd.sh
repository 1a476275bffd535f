set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r05th; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_protocol.py tests/test_gpu_config4.py tests/test_gpu_perm.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
B=384 T=16 REPS=3 bash tools/ab.sh prove "BPP_TREE_HALF=1" "BPP_TREE_HALF=0" 2>&1 | tee $O/ab.txt
for v in 1 0; do BPP_TREE_HALF=$v timeout -k 10 120 python tools/config2_once.py 20 2>&1 | tail -1; done | tee -a $O/ab.txt
