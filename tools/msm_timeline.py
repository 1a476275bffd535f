"""Steady-state packing of the pipelined 2^20 MSM stream from a kernel trace:
rocprofv3 --kernel-trace -d DIR -o run --output-format csv -- python3 bench.py
--steps 30 --no-cpu --proofs-per-gpu 0 --verify-proofs 0.
Finds the longest run of k_msm_accumulate launches spaced < 1.05 ms apart
(the timed stream, as opposed to the one-at-a-time legs around it) and
reports, over its middle, the time per MSM, the fraction of time any kernel /
an accumulation runs, how many accumulations overlap, and every kernel's
mean and minimum duration inside the stream (alone, per bench.py stage_ms, they are shorter).
python tools/msm_timeline.py DIR"""
import csv
import statistics
import sys

d = sys.argv[1]
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0].replace("void ", ""))
            for r in csv.DictReader(open(f"{d}/run_kernel_trace.csv")))
acc = [e for e in ev if e[2].startswith("k_msm_accumulate")]
best, cur = (0, 0), 0
for i in range(1, len(acc)):
    if acc[i][0] - acc[i - 1][0] < 1_050_000:
        if i - cur > best[1] - best[0]:
            best = (cur, i)
    else:
        cur = i
a0, a1 = best
trim = (a1 - a0) // 8
a0, a1 = a0 + trim, a1 - trim
lo, hi = acc[a0][0], acc[a1][0]
n, span = a1 - a0, hi - acc[a0][0]


def union(ints):
    tot, cs, ce = 0, None, None
    for s, e in sorted((max(s, lo), min(e, hi)) for s, e in ints if min(e, hi) > max(s, lo)):
        if ce is None or s > ce:
            if ce is not None:
                tot += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    return tot + (ce - cs if ce is not None else 0)


print(f"{n} MSMs: {span / 1e3 / n:.1f} us per MSM")
print(f"any kernel running {union([(s, e) for s, e, _ in ev]) / span:.3f} of the time, "
      f"an accumulation {union([(s, e) for s, e, _ in acc]) / span:.3f}")
pts = sorted([(max(s, lo), 1) for s, e, _ in acc if e > lo and s < hi] +
             [(min(e, hi), -1) for s, e, _ in acc if e > lo and s < hi])
c, prev, hist = 0, lo, {}
for t, dv in pts:
    hist[c] = hist.get(c, 0) + t - prev
    prev, c = t, c + dv
hist[c] = hist.get(c, 0) + hi - prev
print("accumulations running at once (fraction of time):", {k: round(v / span, 3) for k, v in sorted(hist.items())})
print(f"{'kernel':28s} {'mean us':>8s} {'min us':>8s} {'us per MSM':>10s}")
for name in sorted({e[2] for e in ev}):
    dur = [(e - s) / 1e3 for s, e, nm in ev if nm == name and s >= lo and e <= hi]
    if dur:
        print(f"{name[:28]:28s} {statistics.mean(dur):8.1f} {min(dur):8.1f} {sum(dur) / n:10.1f}")
