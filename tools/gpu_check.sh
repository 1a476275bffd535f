# One GPU call: selected -m gpu tests, then a bench line.
# Usage (on the box): bash tools/gpu_check.sh <tag> "<pytest paths>" "<bench args>"
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-chk}
TESTS=${2:-tests}
BARGS=${3:---no-cpu}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.txt 2>&1 || { tail -40 $OUT/gpu_tests.txt; exit 1; }
tail -1 $OUT/gpu_tests.txt
timeout -k 10 400 python bench.py $BARGS > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python -c "
import json;d=json.load(open('$OUT/bench.json'))
print('msm', d['value'], d['ms_per_step'], d['result_ok'])
p=d.get('proofs') or {}
print('proofs', p.get('value'), p.get('verify_batch_proofs_per_sec'))
print('verify5', json.dumps(d.get('verify_batch')))"
echo done
