set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r05if; mkdir -p $O
REPS=3 bash tools/ab.sh msm "INFLIGHT=3" "INFLIGHT=4" "INFLIGHT=2" 2>&1 | tee $O/ab.txt
