"""Print a rocprofv3 kernel_stats.csv compactly: name, calls, avg/min/max us, % total."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows[: int(sys.argv[2]) if len(sys.argv) > 2 else 12]:
    print(f"{r['Name'][:64]:64s} {int(r['Calls']):6d} avg {float(r['AverageNs'])/1e3:9.2f}us "
          f"min {float(r['MinNs'])/1e3:8.2f} max {float(r['MaxNs'])/1e3:8.2f} {float(r['Percentage']):6.2f}%")
