"""Print the top kernels of a rocprofv3 kernel_stats.csv (total ms, calls, average us, name)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 25
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"total kernel time {tot / 1e6:.2f} ms over {sum(int(r['Calls']) for r in rows)} launches")
for r in rows[:n]:
    print(f"{float(r['TotalDurationNs']) / 1e6:8.2f} ms {int(r['Calls']):6d} {float(r['AverageNs']) / 1e3:8.1f}us "
          f"{r['Name'][:100]}")
