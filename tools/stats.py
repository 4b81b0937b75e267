"""Print the top kernels of a rocprofv3 *_kernel_stats.csv (calls, average us, share, name)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
top = int(sys.argv[2]) if len(sys.argv) > 2 else 20
width = int(sys.argv[3]) if len(sys.argv) > 3 else 150
for r in rows[:top]:
    print(f"{int(r['Calls']):6d} {float(r['AverageNs']) / 1e3:9.2f}us {float(r['Percentage']):6.2f}%  {r['Name'][:width]}")
