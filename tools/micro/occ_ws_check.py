"""Bitwise check of the work-shared occupancy render (occ_ws_kernel) against occ_render_kernel (developer tool).

Run once per library build, then compare:
  ACNERF_LIB=adaptive_city_nerf_amd/libacnerf.so      python tools/micro/occ_ws_check.py gpurun_out/occ_ws.npz
  ACNERF_LIB=build_variants/libacnerf_occws0.so       python tools/micro/occ_ws_check.py gpurun_out/occ_old.npz
  python tools/micro/occ_ws_check.py --compare gpurun_out/occ_ws.npz gpurun_out/occ_old.npz
Renders the k1 / k4 occupancy fixtures' rays through one expert (active_module 0) and the bench's occ batch."""
import sys
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parent.parent.parent


def render(out):
    import torch
    sys.path.insert(0, str(REPO))
    sys.path.insert(0, str(REPO / "tests"))
    from test_occ_gpu import model_from_fixture, _t
    from adaptive_city_nerf_amd import render_rays
    res = {}
    for tag in ("k1", "k4"):
        m, d = model_from_fixture(tag)
        rays = _t(d["rays"])
        big = rays[torch.randint(0, rays.shape[0], (4096,), generator=torch.Generator().manual_seed(3)).to(rays.device)]
        for name, r in (("fixture", rays), ("4096", big.contiguous())):
            with torch.no_grad():
                o = render_rays(m, r, ray_samples=64, active_module=0, bg_color_default="white")
            for k, v in zip(("rgb", "depth", "weights", "acc"), o):
                res[f"{tag}:{name}:{k}"] = v.cpu().numpy()
    np.savez(out, **res)


def compare(a, b):
    A, B = np.load(a), np.load(b)
    bad = [k for k in A.files if not np.array_equal(A[k], B[k], equal_nan=True)]
    print("compared", len(A.files), "arrays;", "all bitwise equal" if not bad else f"DIFFER: {bad}")
    return 1 if bad else 0


if __name__ == "__main__":
    if sys.argv[1] == "--compare":
        sys.exit(compare(sys.argv[2], sys.argv[3]))
    render(sys.argv[1])
