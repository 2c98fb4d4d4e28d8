"""Time the standalone hash-grid kernel (acn_hashgrid_fwd) on the bench workload's 1M sample
points: the gather floor the fused render kernel hides its MLP behind."""
import sys
from pathlib import Path
import torch
REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO))
import bench  # noqa: E402
from adaptive_city_nerf_amd import ops  # noqa: E402
dev = torch.device("cuda", 0)
model, gbox, scene, sc = bench.build_model(dev, 1)
rays = bench.make_rays(scene, gbox, dev, 4096, 1234)
sub = model.submodules[0]
S = 256
u = torch.linspace(0, 1, S, device=dev)
t = rays[:, 6:7] * (1 - u) + rays[:, 7:8] * u
pts = (rays[:, None, :3] + rays[:, None, 3:6] * t[..., None]).reshape(-1, 3)
x01 = ((pts - sub.scene_box.min) / sub.aabb_extent).clamp(1e-6, 1 - 1e-6).contiguous()
enc = sub.xyz_encoder
res = enc._res_host
for name, x in (("ray samples", x01), ("uniform random", torch.rand_like(x01))):
    for _ in range(5):
        ops.hashgrid_fwd(x, enc.hash_table, res, 20, 2, 1)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        ops.hashgrid_fwd(x, enc.hash_table, res, 20, 2, 1)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 20
    print(f"hashgrid_fwd {name}: {x.shape[0]} pts x 16 levels: {ms:.4f} ms = {x.shape[0] / ms / 1e6:.3f} Gpts/s")
