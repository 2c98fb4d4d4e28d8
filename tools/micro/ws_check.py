"""Self-check of render_ws_kernel (developer diagnostic; needs a -DACN_WS_CHECK=1 build): every tile's field is
evaluated twice by the same wave and a differing lane poisons its sample, so a ray with NaN rgb marks a
re-evaluation that did not reproduce (the VALU -> MFMA operand hazard class of DESIGN.md 4i).  Renders the
C2 bench batch and the K = 4 fixture rays through one expert, 10 times each, and counts poisoned rays.
ACNERF_LIB=build_variants/libacnerf_wscheck.so python tools/micro/ws_check.py"""
import sys
from pathlib import Path

import torch

REPO = Path(__file__).resolve().parent.parent.parent
sys.path.insert(0, str(REPO))
sys.path.insert(0, str(REPO / "tests"))
import bench  # noqa: E402
from adaptive_city_nerf_amd import ops, render_rays  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    model, gbox, scene, sc = bench.build_model(dev, 1)
    rays = bench.make_rays(scene, gbox, dev, 4096, 1234)
    bad = 0
    with torch.no_grad():
        for _ in range(10):
            rgb = render_rays(model, rays, ray_samples=256, bg_color_default="white", _want_weights=False)[0]
            bad += int(torch.isnan(rgb).any(dim=1).sum())
    print("C2 batch x10: poisoned rays", bad)
    import test_render_ws as T
    d, specs, routing, bgs = T._setup("k4")
    r4 = T._t(d["render:rays"])
    bad4 = 0
    with torch.no_grad():
        for S in (64, 200, 256):
            for _ in range(10):
                out = ops.render_stratified(r4, S, specs, routing, 2, bgs[0], tau=0.0)
                bad4 += int(torch.isnan(out[0]).any(dim=1).sum())
    print("K=4 fixture, active_module 2, S 64/200/256 x10: poisoned rays", bad4)


if __name__ == "__main__":
    main()
