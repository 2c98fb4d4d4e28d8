"""cProfile of the render_rays Python launch path (C2 and C3 models): where the ~0.3 ms of host time per call goes"""
import cProfile, pstats, sys
sys.path.insert(0, ".")
import torch
import bench
from adaptive_city_nerf_amd import render_rays
dev = torch.device("cuda:0")
for K in (1, 4):
    model, gbox, scene, sc = bench.build_model(dev, K)
    rays = bench.make_rays(scene, gbox, dev, 4096, 1234)
    def fn():
        with torch.no_grad():
            return render_rays(model, rays, ray_samples=256, bg_color_default="white", _want_weights=False)
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(200):
        fn()
    pr.disable()
    torch.cuda.synchronize()
    print(f"===== K={K}")
    pstats.Stats(pr).sort_stats("tottime").print_stats(25)
