# Round-6 GPU check: selected -m gpu tests (one process), optionally smoke + bench.
# Usage (on the box): bash tools/gpu_r06.sh TAG "pytest -k expr or file list" [bench]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-r06}
OUT=gpurun_out/$TAG
mkdir -p $OUT
SEL=${2:-tests}
timeout -k 10 900 python -u -m pytest $SEL -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.txt 2>&1 || { tail -40 $OUT/gpu_tests.txt; exit 1; }
tail -1 $OUT/gpu_tests.txt
if [ "$3" = bench ]; then
  timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.txt 2>&1 || { tail $OUT/smoke.txt; exit 1; }
  timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
  echo bench ok
fi
