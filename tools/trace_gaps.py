"""GPU busy/idle timeline of the last prove_batch in a rocprofv3 kernel +
memory-copy trace (tools/gpu_prover_study.sh gaps).  python tools/trace_gaps.py DIR"""
import csv
import sys

d = sys.argv[1]
ev = []
for r in csv.DictReader(open(f"{d}/run_kernel_trace.csv")):
    ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0][:28], r["Stream_Id"]))
try:
    for r in csv.DictReader(open(f"{d}/run_memory_copy_trace.csv")):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "copy:" + r["Direction"][:12], r.get("Stream_Id", "?")))
except FileNotFoundError:
    pass
ev.sort()
# batch starts: the first k_pedersen of each batch (3 per batch)
ped = [e for e in ev if e[2].startswith("k_pedersen")]
starts = [ped[i][0] for i in range(0, len(ped), 3)]
t0 = starts[-1] - 1
last = [e for e in ev if e[0] >= t0]
t_end = max(e[1] for e in last)
busy = 0
cur_s, cur_e = None, None
gaps = []
prev_name = None
for s, e, n, st in last:
    if cur_e is None:
        cur_s, cur_e = s, e
    elif s > cur_e:
        busy += cur_e - cur_s
        gaps.append((s - cur_e, prev_name, n, (cur_e - t0) / 1e3))
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
    prev_name = n
busy += cur_e - cur_s
span = t_end - t0
print(f"last batch span {span / 1e3:.1f} us, GPU busy {busy / 1e3:.1f} us ({100 * busy / span:.0f} %), "
      f"{len(last)} ops")
tot = {}
for s, e, n, st in last:
    tot[n] = tot.get(n, 0) + (e - s)
for n, v in sorted(tot.items(), key=lambda x: -x[1])[:14]:
    print(f"  {n:30s} {v / 1e3:8.1f} us")
print("gaps > 15 us (us, after -> before, at us):")
for g, a, b, at in gaps:
    if g > 15000:
        print(f"  {g / 1e3:7.1f}  {a} -> {b}  @{at:.0f}")
