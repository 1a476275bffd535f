"""The last `ms` milliseconds of a rocprofv3 kernel (+ memory-copy) trace as
a timeline in us from its first event (e.g. one config-2 run at the end of
tools/config2_once.py):  python tools/trace_tail.py DIR [ms]"""
import csv
import sys
from pathlib import Path


def main():
    d = Path(sys.argv[1])
    span = float(sys.argv[2]) if len(sys.argv) > 2 else 2.0
    ev = []
    for f, kind in (("run_kernel_trace.csv", "kernel"), ("run_memory_copy_trace.csv", "copy")):
        p = d / f
        if not p.exists():
            continue
        for r in csv.DictReader(open(p)):
            name = r["Kernel_Name"].split("(")[0] if kind == "kernel" else r.get("Direction", "?")
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), f"{kind} {name}"))
    ev.sort()
    end = max(e[1] for e in ev)
    t0 = None
    print("start_us  end_us  dur_us  gap_us  event")
    prev = None
    for e in ev:
        if e[1] < end - span * 1e6:
            continue
        t0 = e[0] if t0 is None else t0
        gap = (e[0] - prev) / 1e3 if prev is not None else 0.0
        print("%8.1f %8.1f %7.1f %7.1f  %s" % ((e[0] - t0) / 1e3, (e[1] - t0) / 1e3, (e[1] - e[0]) / 1e3, gap, e[2]))
        prev = max(prev or 0, e[1])


if __name__ == "__main__":
    main()
