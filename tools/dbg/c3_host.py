"""C3 step: host time per call (no sync) vs wall per call, and the same for the bare render_rays call --
is the step bound by the Python launch path?"""
import sys, time
sys.path.insert(0, ".")
import torch
import bench
from adaptive_city_nerf_amd import parallel, render_rays
dev = torch.device("cuda:0")
model, gbox, scene, sc = bench.build_model(dev, 4)
grays = bench.make_rays(scene, gbox, dev, 4096, 1234)
plan = parallel.expert_sorted_plan(parallel.expert_spatial_keys(grays, model), 1)
def rf(r):
    rgb, depth, _, acc = render_rays(model, r, ray_samples=256, bg_color_default="white", _want_weights=False)
    return rgb, depth, acc
def step():
    with torch.no_grad():
        return parallel.render_rays_sharded(grays, rf, plan)
def bare():
    with torch.no_grad():
        return rf(grays)
for name, fn in (("step", step), ("render_rays", bare)):
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(100):
        fn()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"{name}: host {1e3 * (t1 - t0) / 100:.3f} ms/call, wall {1e3 * (t2 - t0) / 100:.3f} ms/call", flush=True)
