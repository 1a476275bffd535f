# host pool size x batches in flight, around 8 x 8
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
for pass in 1 2; do for cfg in "8 8" "8 12" "4 8" "4 12" "6 10" "8 16" "10 8"; do set -- $cfg; echo -n "threads=$1 "; BPP_HOST_THREADS=$1 timeout -k 10 120 python tools/prove_inflight_exp.py 128 $2 16 || exit 1; done; done
