set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r06m; mkdir -p $O
for rep in 1 2 3; do
for cfg in "BPP_DT_BUILD_RPL=4" "BPP_DT_BUILD_RPL=2"; do
  ( export $cfg; echo "$cfg: $(timeout -k 10 120 python3 tools/config2_once.py 20 2>/dev/null)" ) || exit 1
done; done | tee $O/c2_build_ab2.txt
BPP_DT_BUILD_RPL=2 timeout -k 10 300 python -u -m pytest tests/test_gpu_protocol.py tests/test_golden_protocol.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
