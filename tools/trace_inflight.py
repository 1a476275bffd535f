"""Steady-state GPU occupancy of a kernel trace taken over batches in flight
(rocprofv3 --kernel-trace -- python tools/prove_inflight_exp.py B T R):
busy fraction (union of kernel intervals), mean kernels running while busy,
and per-kernel summed duration per batch.   python tools/trace_inflight.py DIR NBATCHES"""
import csv
import sys
from collections import defaultdict

d, nb = sys.argv[1], int(sys.argv[2])
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0].replace("void ", "")[:26])
            for r in csv.DictReader(open(f"{d}/run_kernel_trace.csv")))
# steady window: the middle 80 % of the prove kernels' span (skip setup/warmup tails)
ped = [e for e in ev if e[2].startswith("k_ipa_round_dt")]
lo = ped[len(ped) // 10][0]
hi = ped[len(ped) * 9 // 10][1]
win = [e for e in ev if e[0] >= lo and e[1] <= hi]
busy, cur_s, cur_e = 0, None, None
for s, e, _ in win:
    if cur_e is None or s > cur_e:
        if cur_e is not None:
            busy += cur_e - cur_s
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
busy += cur_e - cur_s
span = hi - lo
tot = sum(e - s for s, e, _ in win)
folds = sum(1 for e in win if e[2].startswith("k_ipa_round_dt"))
batches = folds / 7.0
per = defaultdict(float)
for s, e, n in win:
    per[n] += (e - s)
print(f"window {span / 1e6:.2f} ms, ~{batches:.1f} batches ({span / 1e3 / max(batches, 1):.0f} us per batch), "
      f"GPU busy {busy / span:.1%}, mean kernels running while busy {tot / busy:.2f}")
print(f"summed kernel time per batch {tot / 1e3 / batches:.0f} us")
for n, v in sorted(per.items(), key=lambda x: -x[1])[:14]:
    print(f"  {n:28s} {v / 1e3 / batches:8.1f} us/batch  {v / tot:6.1%}")
