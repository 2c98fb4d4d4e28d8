"""Fold one gpu_round's rocprofv3 outputs into the committed profile JSON that bench.py reads.

python tools/pmc_to_json.py gpurun_out/pmc_TAG gpurun_out/prof_TAG/run_kernel_stats.csv OUT.json ROUND
Counter values are per-dispatch means of the render kernel over the --pmc passes (one counter group
per pass, tools/pmc_sets.sh); FETCH_SIZE / WRITE_SIZE are in kB as rocprofv3 reports them."""
import csv
import glob
import json
import sys
from collections import defaultdict

SAMPLES = 4096 * 256


def main():
    root, stats, out, rnd = sys.argv[1:5]
    pat = "render_kernel<1, 1, 0>"
    vals = defaultdict(list)
    for f in sorted(glob.glob(f"{root}/p*/run_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            if pat in r["Kernel_Name"]:
                vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
    c = {k: round(sum(v) / len(v), 1) for k, v in sorted(vals.items())}
    avg_ns, calls = None, None
    for r in csv.DictReader(open(stats)):
        if pat in r["Name"]:
            avg_ns, calls = float(r["AverageNs"]), int(r["Calls"])
    hit, miss = c.get("TCC_HIT_sum", 0.0), c.get("TCC_MISS_sum", 0.0)
    simd_cycles = c["GRBM_GUI_ACTIVE"] / 8 * 256 * 4 if "GRBM_GUI_ACTIVE" in c else None
    derived = {
        "tcp_accesses_per_sample": c.get("TCP_TOTAL_CACHE_ACCESSES_sum", 0) / SAMPLES,
        "l2_requests_per_sample": c.get("TCP_TCC_READ_REQ_sum", 0) / SAMPLES,
        "l2_misses_per_sample": miss / SAMPLES,
        "l2_hit_rate": hit / (hit + miss) if hit + miss else None,
        "td_busy_frac": c["TD_TD_BUSY_sum"] / (c["GRBM_GUI_ACTIVE"] / 8 * 256) if "TD_TD_BUSY_sum" in c else None,
        "td_stalled_on_tc_frac": c["TD_TC_STALL_sum"] / c["TD_TD_BUSY_sum"] if "TD_TD_BUSY_sum" in c else None,
        "mfma_busy_frac_per_simd": c["SQ_VALU_MFMA_BUSY_CYCLES"] / simd_cycles if simd_cycles else None,
        "l2_miss_bytes_per_launch_at_128B": miss * 128,
    }
    doc = {
        "kernel": "render_kernel<1,1,0> (acn_render_stratified_fwd), 4096 rays x 256 samples, 1 expert",
        "round": rnd,
        "commands": [
            "rocprofv3 --kernel-trace --stats --output-format csv -- python3 bench.py --steps 20 --warmup 3 "
            "--no-cpu-baseline",
            "tools/pmc_sets.sh: one rocprofv3 --pmc pass per counter group over python3 bench.py --steps 5 "
            "--warmup 2 --no-cpu-baseline"],
        "rocprof_avg_ns": avg_ns, "rocprof_calls": calls,
        "FETCH_SIZE_kB_per_launch": c.get("FETCH_SIZE"), "WRITE_SIZE_kB_per_launch": c.get("WRITE_SIZE"),
        "hbm_bytes_per_launch": int((c.get("FETCH_SIZE", 0) + c.get("WRITE_SIZE", 0)) * 1024),
        "counters_per_launch": c,
        "derived": derived,
        "notes": "FETCH_SIZE/WRITE_SIZE in kB (x1024), uncorrected: the gfx950 x2 read correction of "
                 "MI355X_MICROARCH.md is calibrated for 16-B/lane streaming reads, this kernel issues 8-B random "
                 "gathers. FETCH_SIZE counts requests leaving the XCD L2 with Infinity-Cache hits included (the "
                 "128 MiB table is cache-resident): an upper bound on HBM bytes. l2_miss_bytes_per_launch_at_128B "
                 "= TCC_MISS x 128 B, the line traffic the Infinity Cache serves.",
    }
    with open(out, "w") as f:
        json.dump(doc, f, indent=1)
    print(json.dumps(derived, indent=1))


if __name__ == "__main__":
    main()
