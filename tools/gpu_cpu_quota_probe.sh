# CPU quota of the box's cgroup and its throttling counters around repeated
# 12-in-flight prover runs (is the run-to-run spread CFS throttling?).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export SHARED_GENS=1
cg=/sys/fs/cgroup$(awk -F: '$1=="0"{print $3}' /proc/self/cgroup)
echo "cgroup $cg"; cat $cg/cpu.max 2>/dev/null; cat $cg/cpuset.cpus.effective 2>/dev/null
nproc; python3 -c "import os; print('affinity', len(os.sched_getaffinity(0)))"
for rep in 1 2 3 4; do
  grep -E "nr_throttled|throttled_usec|usage_usec" $cg/cpu.stat | tr '\n' ' '; echo
  timeout -k 10 120 python tools/prove_inflight_exp.py 128 ${T:-12} 16 || exit 1
done
grep -E "nr_throttled|throttled_usec|usage_usec" $cg/cpu.stat | tr '\n' ' '; echo
