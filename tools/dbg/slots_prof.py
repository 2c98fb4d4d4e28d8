"""Per-ray section timings of render_slots_kernel (C4 frame at S = 96 and 256, C3 batch) from its
ACN_SLOTS_PROF=1 build (tools/build_variants.sh slprof:render.hip:"-DACN_SLOTS_PROF=1"; run with
ACNERF_LIB=build_variants/libacnerf_slprof.so).  Lane 0 of each ray's wave stamps wall_clock64() (100 MHz) at:
0 round start, 1 after ray_expert_mask, 2 after the round's slot choice / restage barriers, 3 after the first
tile's field evaluation, 4 after the tile loop,
5 after the ray's background / outputs.  Prints per-section medians and totals summed over rays."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
import numpy as np
import torch

import bench
from adaptive_city_nerf_amd import _lib, parallel
from adaptive_city_nerf_amd.ray_rendering import render_rays

L = _lib.lib()
fetch = L.acn_debug_slprof_fetch
fetch.argtypes, fetch.restype = [ctypes.c_void_p, ctypes.c_int], ctypes.c_int
dev = torch.device("cuda")


def report(tag, n, ms):
    buf = np.zeros((n, 6), np.uint64)
    got = fetch(buf.ctypes.data, n)
    t = buf[:got].astype(np.float64)
    ok = (t[:, 0] > 0) & (t[:, 5] >= t[:, 0])
    t = t[ok]
    sec = {"mask": (t[:, 1] - t[:, 0]), "round barriers + restage": (t[:, 2] - t[:, 1]),
           "first tile (field only, folds included)": (t[:, 3] - t[:, 2]),
           "later tiles + compositing": (t[:, 4] - t[:, 3]), "background + outputs": (t[:, 5] - t[:, 4])}
    tot = t[:, 5] - t[:, 0]
    line = ", ".join(f"{k} {np.median(v) / 100:.2f} us ({v.sum() / tot.sum():.1%})" for k, v in sec.items())
    print(f"{tag}: {t.shape[0]} rays, kernel {ms:.2f} ms | per ray median {np.median(tot) / 100:.2f} us | {line}",
          flush=True)


for K, S, tag in ((8, 96, "C4 S=96"), (8, 256, "C4 S=256"), (4, 256, "C3")):
    torch.cuda.empty_cache()
    model, gbox, scene, sc = bench.build_model(dev, K)
    if tag.startswith("C4"):
        H, W, intr, c2w = bench.frame_camera(scene, 800, 800)
        with torch.no_grad():
            for rep in range(2):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                parallel.render_image_sharded(model, H=H, W=W, fx=intr[0], fy=intr[1], cx=intr[2], cy=intr[3],
                                              c2w=c2w, scene_box=gbox, ray_samples=S, gt_srgb=None)
                e1.record()
                torch.cuda.synchronize()
        report(tag, H * W, e0.elapsed_time(e1))
    else:
        grays = bench.make_rays(scene, gbox, dev, 4096, 1234)
        plan = parallel.expert_sorted_plan(parallel.expert_spatial_keys(grays, model), 1)
        with torch.no_grad():
            for rep in range(3):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                def fn(r):
                    o = render_rays(model, r, ray_samples=S, bg_color_default="white", _want_weights=False)
                    return o[0], o[1], o[3]
                parallel.render_rays_sharded(grays, fn, plan)
                e1.record()
                torch.cuda.synchronize()
        report(tag, 4096, e0.elapsed_time(e1))
    del model
