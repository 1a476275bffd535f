"""Aggregate tools/hostprof samples: share of CPU samples per object and per
function (local symbols resolved with nm).   python tools/hostprof/report.py SAMPLES [TOP]"""
import bisect
import collections
import os
import subprocess
import sys

path = sys.argv[1]
top = int(sys.argv[2]) if len(sys.argv) > 2 else 40
rows = []
comms = []
for ln in open(path).read().splitlines():
    p = ln.split(" ", 4)
    if len(p) == 5:  # object offset caller thread-name symbol
        rows.append((p[0], p[1], p[4], p[2]))
        comms.append(p[3])
    elif len(p) == 4:
        rows.append((p[0], p[1], p[3], p[2]))
        comms.append("?")
n = len(rows)
by_obj = collections.Counter(os.path.basename(r[0]) for r in rows)
print(f"{n} samples")
for o, c in by_obj.most_common(12):
    print(f"  {c / n:6.1%}  {o}")

_tables = {}


def table(obj):
    if obj not in _tables:
        syms = []
        try:
            out = subprocess.run(["nm", "-C", "-n", "--defined-only", obj], capture_output=True, text=True).stdout
            if not out.strip():
                out = subprocess.run(["nm", "-D", "-C", "-n", "--defined-only", obj], capture_output=True, text=True).stdout
            for ln in out.splitlines():
                p = ln.split(" ", 2)
                if len(p) == 3 and p[1].lower() in ("t", "w"):
                    syms.append((int(p[0], 16), p[2]))
        except Exception:
            pass
        _tables[obj] = ([a for a, _ in syms], [s for _, s in syms])
    return _tables[obj]


by_fn = collections.Counter()
for obj, off, sname, _ in rows:
    name = sname.strip()
    if obj != "?":
        addrs, names = table(obj)
        i = bisect.bisect_right(addrs, int(off, 16)) - 1
        if i >= 0:
            name = names[i]
    by_fn[(os.path.basename(obj), name[:90])] += 1
print("top functions")
for (o, f), c in by_fn.most_common(top):
    print(f"  {c / n:6.1%}  {o:24s} {f}")

# callers (first libbpperm return address on the interrupted stack) of the
# samples outside libbpperm
bp = next((r[0] for r in rows if r[0].endswith("libbpperm.so")), None)
if bp:
    addrs, names = table(bp)
    by_caller = collections.Counter()
    for obj, off, sname, caller in rows:
        if obj.endswith("libbpperm.so") or caller == "0":
            continue
        i = bisect.bisect_right(addrs, int(caller, 16)) - 1
        by_caller[(os.path.basename(obj), names[i][:80] if i >= 0 else "?")] += 1
    print("callers in libbpperm of samples in other objects")
    for (o, f), c in by_caller.most_common(top // 2):
        print(f"  {c / n:6.1%}  {o:24s} <- {f}")

if comms:
    print("samples by thread name (object)")
    for (c, o), k in collections.Counter((c, os.path.basename(r[0])) for c, r in zip(comms, rows)).most_common(12):
        print(f"  {k / n:6.1%}  {c:16s} {o}")
