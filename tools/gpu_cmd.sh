set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r05t2; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_config4.py -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -12 $O/tests.log
