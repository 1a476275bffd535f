"""Print a rocprofv3 kernel_stats.csv compactly: name, calls, avg us, total ms."""
import csv
import sys

for f in sys.argv[1:]:
    print(f)
    for r in csv.DictReader(open(f)):
        print(f"  {r['Name'].split('(')[0].replace('void ', '')[:30]:30s} {r['Calls']:>5} "
              f"{float(r['AverageNs']) / 1e3:9.1f} us  {float(r['TotalDurationNs']) / 1e6:8.3f} ms")
