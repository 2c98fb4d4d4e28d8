"""Fold one tools/pmc_r04.sh output directory into the committed per-kernel profile JSON bench.py reads.

python tools/pmc_fold_r04.py gpurun_out/pmc_TAG KERNEL_SUBSTRING SAMPLES_PER_LAUNCH OUT.json ROUND "WHAT"

Counter values are per-dispatch means of the matching kernel over the --pmc passes.  HBM traffic follows
MI355X_MICROARCH.md 'HBM': FETCH_SIZE (kB, = TCC_EA0_RDREQ x 64 B) reports half the bytes of 128-B
requests on gfx950, so it is doubled; WRITE_SIZE is taken as reported.  TCC_MISS x 128 B (the lines the
XCD L2s fetch from the fabric) is the independent cross-check of the corrected read bytes."""
import csv
import glob
import json
import sys
from collections import defaultdict


def main():
    root, pat, samples, out, rnd, what = sys.argv[1:7]
    samples = int(samples)
    bpu = float(sys.argv[7]) if len(sys.argv) > 7 else 1024.2   # algorithmic bytes per unit (sample / record)
    vals = defaultdict(list)
    for f in sorted(glob.glob(f"{root}/p*/**/*counter_collection.csv", recursive=True)):
        for r in csv.DictReader(open(f)):
            if pat in r["Kernel_Name"]:
                vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
    c = {k: round(sum(v) / len(v), 1) for k, v in sorted(vals.items())}
    ncalls = {k: len(v) for k, v in vals.items()}
    avg_ns, calls = None, None
    for f in glob.glob(f"{root}/stats/**/*kernel_stats.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if pat in r["Name"]:
                avg_ns, calls = float(r["AverageNs"]), int(r["Calls"])
    hit, miss = c.get("TCC_HIT_sum", 0.0), c.get("TCC_MISS_sum", 0.0)
    grbm = c.get("GRBM_GUI_ACTIVE")
    # GRBM_GUI_ACTIVE is summed over the 8 XCDs (MI355X_MICROARCH.md 'DVFS give-back'): per-XCD busy cycles =
    # GRBM / 8, CU-cycles of the dispatch = GRBM / 8 x 256; SQ_WAVE_CYCLES / SQ_WAIT_* count quad-cycles
    cu_cycles = grbm / 8 * 256 if grbm else None
    fetch_raw = c.get("FETCH_SIZE", 0.0) * 1024
    write = c.get("WRITE_SIZE", 0.0) * 1024
    fetch = 2 * fetch_raw                               # gfx950 half-count correction
    traffic = int(fetch + write)
    alg = int(bpu * samples)
    derived = {
        "tcp_accesses_per_sample": c.get("TCP_TOTAL_CACHE_ACCESSES_sum", 0) / samples,
        "l2_requests_per_sample": c.get("TCP_TCC_READ_REQ_sum", 0) / samples,
        "l2_misses_per_sample": miss / samples,
        "l2_hit_rate": hit / (hit + miss) if hit + miss else None,
        "l2_miss_bytes_per_launch_at_128B": miss * 128,
        "fetch_bytes_per_launch_corrected": int(fetch),
        "fetch_corrected_over_tcc_miss_lines": fetch / (miss * 128) if miss else None,
        "traffic_over_algorithmic": traffic / alg,
        "td_busy_frac": c["TD_TD_BUSY_sum"] / cu_cycles if "TD_TD_BUSY_sum" in c and cu_cycles else None,
        "td_stalled_on_tc_frac": c["TD_TC_STALL_sum"] / c["TD_TD_BUSY_sum"] if c.get("TD_TD_BUSY_sum") else None,
        "mfma_busy_frac_per_simd": c["SQ_VALU_MFMA_BUSY_CYCLES"] / (cu_cycles * 4) if "SQ_VALU_MFMA_BUSY_CYCLES" in c and cu_cycles else None,
        "mean_waves_per_cu": 4 * c["SQ_WAVE_CYCLES"] / cu_cycles if "SQ_WAVE_CYCLES" in c and cu_cycles else None,
        "effective_clock_ghz": grbm / 8 / avg_ns if grbm and avg_ns else None,
        "wait_any_frac_of_wave_cycles": c["SQ_WAIT_ANY"] / c["SQ_WAVE_CYCLES"] if c.get("SQ_WAVE_CYCLES") else None,
        "valu_insts_per_sample": c.get("SQ_INSTS_VALU", 0) / samples,
        "vmem_rd_insts_per_sample": c.get("SQ_INSTS_VMEM_RD", 0) / samples,
        "lds_insts_per_sample": c.get("SQ_INSTS_LDS", 0) / samples,
        "mfma_insts_per_sample": c.get("SQ_INSTS_MFMA", 0) / samples,
    }
    doc = {
        "kernel": what, "kernel_match": pat, "round": rnd, "samples_per_launch": samples,
        "commands": ["tools/pmc_r04.sh (rocprofv3 --kernel-trace --stats, then one --pmc pass per counter group)"],
        "rocprof_avg_ns": avg_ns, "rocprof_calls": calls,
        "FETCH_SIZE_kB_per_launch": c.get("FETCH_SIZE"), "WRITE_SIZE_kB_per_launch": c.get("WRITE_SIZE"),
        "hbm_bytes_per_launch": traffic,
        "bytes_algorithmic_per_launch": alg,
        "counters_per_launch": c, "dispatches_per_counter": ncalls,
        "derived": derived,
        "notes": "hbm_bytes_per_launch = 2 x FETCH_SIZE + WRITE_SIZE (bytes): the gfx950 x2 read correction of "
                 "MI355X_MICROARCH.md 'HBM'; Infinity-Cache hits are counted by these fabric-side counters, so this "
                 "is the traffic beyond the XCD L2s (an upper bound on DRAM bytes). TCC_MISS x 128 B cross-checks "
                 "the corrected read bytes.",
    }
    with open(out, "w") as f:
        json.dump(doc, f, indent=1)
    print(json.dumps({"avg_ns": avg_ns, "traffic": traffic, "alg": alg, **derived}, indent=1))


if __name__ == "__main__":
    main()
