# longer runs: host pool size x batches in flight (two passes)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
for pass in 1 2; do for cfg in "16 4" "8 4" "8 6" "6 4" "6 6" "12 4" "8 8"; do set -- $cfg; echo -n "threads=$1 "; BPP_HOST_THREADS=$1 timeout -k 10 120 python tools/prove_inflight_exp.py 128 $2 24 || exit 1; done; done
