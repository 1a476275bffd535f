# GPU busy % (sysfs gpu_busy_percent, sampled every 50 ms) while the prover
# runs 12 batches in flight for ~4 s.  Usage (on the box): bash tools/gpu_busy_probe.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp SHARED_GENS=1
F=$(ls /sys/class/drm/card*/device/gpu_busy_percent 2>/dev/null | head -1)
echo "sysfs: $F"
[ -n "$F" ] || exit 0
( for i in $(seq 1 200); do cat $F; sleep 0.05; done > gpurun_out/busy.txt ) &
BG=$!
timeout -k 10 120 python tools/prove_inflight_exp.py 128 12 40 || { kill $BG; exit 1; }
kill $BG 2>/dev/null; wait $BG 2>/dev/null
python3 -c "
v=[int(x) for x in open('gpurun_out/busy.txt').read().split()]
import statistics
print('samples', len(v), 'busy% median', statistics.median(v), 'mean', round(sum(v)/len(v),1), 'p90', sorted(v)[int(0.9*len(v))])
print(v[:80])"
