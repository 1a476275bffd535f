"""Print a rocprofv3 kernel_stats.csv compactly: name, calls, avg us, total ms.
Usage: kstats.py [-n ROWS] FILE..."""
import csv
import sys

args = sys.argv[1:]
rows = None
if args[:1] == ["-n"]:
    rows, args = int(args[1]), args[2:]
for f in args:
    print(f)
    for i, r in enumerate(csv.DictReader(open(f))):
        if rows is not None and i >= rows:
            break
        print(f"  {r['Name'].split('(')[0].replace('void ', '')[:30]:30s} {r['Calls']:>5} "
              f"{float(r['AverageNs']) / 1e3:9.1f} us  {float(r['TotalDurationNs']) / 1e6:8.3f} ms")
