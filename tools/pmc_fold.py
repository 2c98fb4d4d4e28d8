"""Per-launch HBM bytes of one kernel from tools/pmc_kernel.sh passes -> profiles JSON read by bench.py.

python tools/pmc_fold.py gpurun_out/pmc_W KERNEL_SUBSTRING ALGO_BYTES_PER_LAUNCH OUT.json
FETCH_SIZE / WRITE_SIZE are kB per dispatch; on gfx950 FETCH_SIZE counts half the bytes of wide
(16 B/lane) coalesced reads (MI355X_MICROARCH.md, HBM/rocprofv3 section), so it is doubled; WRITE_SIZE
is exact for 16-B stores and float atomics.  Infinity-Cache hits are included in both."""
import csv
import glob
import json
import sys


def mean(root, sub, pat, name):
    vals = []
    for f in glob.glob(f"{root}/{sub}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if pat in r["Kernel_Name"] and r["Counter_Name"] == name:
                vals.append(float(r["Counter_Value"]))
    return sum(vals) / len(vals) if vals else None, len(vals)


def main():
    root, pat, algo, out = sys.argv[1], sys.argv[2], float(sys.argv[3]), sys.argv[4]
    fetch, nf = mean(root, "fetch", pat, "FETCH_SIZE")
    write, nw = mean(root, "write", pat, "WRITE_SIZE")
    hbm = (2.0 * fetch + write) * 1024.0
    res = {"kernel": pat, "dispatches": {"fetch": nf, "write": nw}, "fetch_size_kb": fetch, "write_size_kb": write,
           "hbm_bytes_per_launch": int(hbm), "algorithmic_bytes_per_launch": int(algo),
           "traffic_over_algorithmic": round(hbm / algo, 3) if algo else None,
           "correction": "FETCH_SIZE x2 (gfx950 half-count of 16-B/lane reads); WRITE_SIZE as reported"}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
