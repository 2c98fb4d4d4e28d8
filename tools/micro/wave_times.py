"""Per-wave timeline of the C2 render (developer diagnostic; needs a -DACN_DIAG_WAVETIME=1 build).

render_kernel gives every wave one ray.  The diagnostic build writes, per ray, the 100-MHz realtime stamps at the
ray's start and end and the wave's HW_ID / XCC_ID into rgb[ray] (bit patterns), so this script can tell how much of
the launch is spent with CUs partly idle: kernel span vs the mean ray (wave) time, per-CU busy fraction, and the
distribution of wave durations.
ACNERF_LIB=build_variants/libacnerf_wavetime.so python tools/micro/wave_times.py
"""
import json
import sys
from pathlib import Path

import numpy as np
import torch

REPO = Path(__file__).resolve().parent.parent.parent
sys.path.insert(0, str(REPO))

import bench  # noqa: E402
from adaptive_city_nerf_amd import render_rays  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    model, gbox, scene, sc = bench.build_model(dev, 1)
    rays = bench.make_rays(scene, gbox, dev, 4096, 1234)
    out = {}
    with torch.no_grad():
        for _ in range(5):
            render_rays(model, rays, ray_samples=256, bg_color_default="white", _want_weights=False)
        torch.cuda.synchronize()
        reps = []
        for _ in range(5):
            rgb, depth, _, acc = render_rays(model, rays, ray_samples=256, bg_color_default="white",
                                             _want_weights=False)
            torch.cuda.synchronize()
            reps.append(rgb.view(torch.int32).cpu().numpy().astype(np.int64) & 0xffffffff)
    for r, bits in enumerate(reps):
        t0, t1, hw = bits[:, 0], bits[:, 1], bits[:, 2]
        base = t0.min()
        s = (t0 - base) % (1 << 32) * 10e-3     # us (100 MHz)
        e = (t1 - base) % (1 << 32) * 10e-3
        d = e - s
        span = e.max() - s.min()
        xcc = (hw >> 16) & 0xf
        cu = (hw >> 8) & 0xf
        sh = (hw >> 12) & 0x1
        se = (hw >> 13) & 0x7
        cu_key = xcc * 1000 + se * 100 + sh * 16 + cu
        keys, inv = np.unique(cu_key, return_inverse=True)
        per_cu_busy = np.zeros(len(keys))
        per_cu_end = np.zeros(len(keys))
        per_cu_n = np.zeros(len(keys))
        np.add.at(per_cu_busy, inv, d)
        np.maximum.at(per_cu_end, inv, e)
        np.add.at(per_cu_n, inv, 1)
        rec = {"span_us": round(float(span), 2), "wave_us_mean": round(float(d.mean()), 2),
               "wave_us_p10_p50_p90_max": [round(float(np.percentile(d, q)), 2) for q in (10, 50, 90, 100)],
               "start_us_p50_p99_max": [round(float(np.percentile(s, q)), 2) for q in (50, 99, 100)],
               "end_us_p10_p50_min": [round(float(np.percentile(e, q)), 2) for q in (10, 50, 0)],
               "cus_seen": int(len(keys)), "waves_per_cu_min_max": [int(per_cu_n.min()), int(per_cu_n.max())],
               "mean_waves_resident": round(float(d.sum() / span / len(keys)), 2),
               "per_cu_end_p10_p50_min_us": [round(float(np.percentile(per_cu_end, q)), 2) for q in (10, 50, 0)]}
        out[f"rep{r}"] = rec
        print(json.dumps(rec))
    # ray duration vs ray properties for the last rep: near/far span
    Path("gpurun_out").mkdir(exist_ok=True)
    np.save("gpurun_out/wave_times_last.npy", np.stack([s, e, hw.astype(np.float64)], 1))
    json.dump(out, open("gpurun_out/wave_times.json", "w"), indent=1)


if __name__ == "__main__":
    main()
