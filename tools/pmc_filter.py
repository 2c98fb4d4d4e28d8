"""Shrink a tools/pmc_r04.sh output tree in place: keep only the counter rows (and kernel-stats rows) whose kernel
name contains the given substrings, so long workloads (the meta step: thousands of dispatches per pass) fit in
gpurun's copy-back.  usage: python tools/pmc_filter.py gpurun_out/pmc_TAG SUBSTR [SUBSTR ...]"""
import csv
import pathlib
import sys

root = pathlib.Path(sys.argv[1])
keep = sys.argv[2:]
for p in list(root.rglob("*counter_collection.csv")):
    with open(p, newline="") as f:
        r = csv.reader(f)
        head = next(r)
        col = head.index("Kernel_Name")
        rows = [row for row in r if any(k in row[col] for k in keep)]
    with open(p, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(head)
        w.writerows(rows)
    print(p, len(rows), "rows kept")
