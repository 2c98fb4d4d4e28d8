"""Mean per-dispatch PMC values of the C5 step's kernels (tools/pmc_c5.sh output)."""
import collections
import csv
import glob
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc_c5"
agg = collections.defaultdict(list)
for f in glob.glob(f"{root}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")[:44]
        agg[(k, r["Counter_Name"])].append(float(r["Counter_Value"]))
for (k, c), v in sorted(agg.items()):
    if any(s in k for s in ("adam_slots", "hashgrid_", "sumsq_slots", "mlp_", "routed_", "blend_")):
        print(f"{k:46s} {c:22s} n={len(v):3d} mean={sum(v) / len(v):.5g}")
