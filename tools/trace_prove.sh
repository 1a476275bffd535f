# Kernel + memcpy timeline of warm 128-proof batches (S streams), for gap analysis.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
S=${1:-1}
OUT=gpurun_out/trace_prove_s$S
mkdir -p $OUT
BPP_PROVE_STREAMS=$S timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace -d $OUT -o run --output-format csv -- python3 tools/prove_phases.py 128 3 > $OUT/log.txt 2>&1
