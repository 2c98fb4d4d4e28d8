"""Summarise rocprofv3 --pmc CSVs for one kernel: mean counter value per dispatch.
python tools/pmc_summary.py gpurun_out/pmc_TAG [kernel-substring]"""
import csv, sys, glob, collections
root = sys.argv[1]
pat = sys.argv[2] if len(sys.argv) > 2 else "render_kernel"
vals = collections.defaultdict(list)
durs = []
for f in sorted(glob.glob(f"{root}/p*/run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        if pat in r["Kernel_Name"]:
            vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
            durs.append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
out = {k: sum(v) / len(v) for k, v in vals.items()}
for k, v in sorted(out.items()):
    print(f"{k:28s} {v:16.1f}  (n={len(vals[k])})")
if "GRBM_GUI_ACTIVE" in out:
    print("mean dispatch ns (profiled)", sum(durs) / len(durs))
