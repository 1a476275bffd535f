# in-flight scaling of the prover + rank shares of the window-split MSM
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
for T in 1 2 4 6 8; do timeout -k 10 120 python tools/prove_inflight_exp.py 128 $T 6 || exit 1; done
for th in 8 12 24; do echo "threads=$th"; BPP_HOST_THREADS=$th timeout -k 10 120 python tools/prove_inflight_exp.py 128 4 6 || exit 1; done
for nt in 128 512; do echo "dt_nt=$nt"; BPP_DT_NT=$nt timeout -k 10 120 python tools/prove_inflight_exp.py 128 4 6 || exit 1; done
timeout -k 10 300 python tools/rank_share.py 2 4 8 > gpurun_out/rank_share.jsonl 2> gpurun_out/rank_share.err || { tail -5 gpurun_out/rank_share.err; exit 1; }
cat gpurun_out/rank_share.jsonl
