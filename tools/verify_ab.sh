# Interleaved A/B of one config-5 batch verification's stages
# (tools/verify_stages.py) over environment settings, then a kernel trace of
# the default.  Usage (on the box): bash tools/verify_ab.sh TAG "CFG" "CFG" ...
# (CFG: space-separated VAR=VAL settings; REPS interleaved passes, default 2)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=$1; shift
OUT=gpurun_out/vab_$TAG
mkdir -p $OUT
for rep in $(seq 1 ${REPS:-2}); do
  for cfg in "$@"; do
    echo -n "$cfg: "
    env $cfg timeout -k 10 150 python tools/verify_stages.py --reps ${VREPS:-10} || exit 1
  done
done | tee $OUT/ab.txt
[ -n "$NOTRACE" ] || timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 tools/verify_stages.py --reps 3 > $OUT/trace_log.txt 2>&1 || { echo "trace failed"; exit 1; }
echo done
