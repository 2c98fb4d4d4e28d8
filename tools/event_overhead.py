import sys, time, torch
sys.path.insert(0, ".")
import bench
from adaptive_city_nerf_amd import render_rays, ops
dev = torch.device("cuda", 0)
model, gbox, scene, sc = bench.build_model(dev, 1)
rays = bench.make_rays(scene, gbox, dev, 4096, 1234)
def run(n, hook):
    ops.EVENT_HOOK = [] if hook else None
    torch.cuda.synchronize(); t0 = time.perf_counter()
    with torch.no_grad():
        for _ in range(n): render_rays(model, rays, ray_samples=256, bg_color_default="white")
    torch.cuda.synchronize(); dt = (time.perf_counter() - t0) / n * 1e3
    k = sum(a.elapsed_time(b) for a, b in ops.EVENT_HOOK) / n if hook else 0
    ops.EVENT_HOOK = None
    return dt, k
run(20, False)
for i in range(3):
    print("no hook %.4f ms/step" % run(200, False)[0], " hook %.4f ms/step kernel %.4f" % run(200, True))
