"""sys.modules stubs that let the reference be imported in THIS container (fixture generation only).

The reference imports a few packages that are absent here and are unused on the stratified
render path: nerfacc (occupancy path only; replaced by a stand-in built on the
oracle's restatement of nerfacc 0.5.3, oracle/occ_ref.py, so the reference's OWN occupancy glue can
be run to pin fixtures -- nerfacc's semantics themselves stay unpinned), jaxtyping (annotations),
viser.transforms (OrientedBox only), torchvision.utils.make_grid and
torch.utils.tensorboard.SummaryWriter (logging).  tinycudann is handled by the reference's own
try/except (models/encodings.py:8-14), so its pure-Torch fallback is what gets exercised.
"""
import sys
import types


def _nerfacc_standin():
    """nerfacc 0.5.3 stand-in (CPU, numpy/C restatement from oracle/occ_ref.py)."""
    import numpy as np
    import torch
    import torch.nn as nn
    from oracle import occ_ref as R

    m = types.ModuleType("nerfacc")

    def _enlarge(aabb, factor):
        center = (aabb[:3] + aabb[3:]) / 2
        extent = (aabb[3:] - aabb[:3]) / 2
        return torch.cat([center - extent * factor, center + extent * factor])

    class OccGridEstimator(nn.Module):
        def __init__(self, roi_aabb, resolution=128, levels=1, **kw):
            super().__init__()
            if isinstance(resolution, int):
                resolution = [resolution] * 3
            resolution = torch.tensor(resolution, dtype=torch.int32)
            self.cells_per_lvl = int(resolution.prod().item())
            self.levels = levels
            self.register_buffer("resolution", resolution)
            self.register_buffer("aabbs", torch.zeros(levels, 6))
            self.register_buffer("occs", torch.zeros(levels * self.cells_per_lvl))
            self.register_buffer("binaries", torch.zeros([levels] + resolution.tolist(), dtype=torch.bool))
            self.aabbs = torch.stack([_enlarge(roi_aabb, 2 ** i) for i in range(levels)], dim=0)
            self.last_u = None

        @torch.no_grad()
        def sampling(self, rays_o, rays_d, sigma_fn=None, alpha_fn=None, near_plane=0.0, far_plane=1e10,
                     t_min=None, t_max=None, render_step_size=1e-3, early_stop_eps=1e-4, alpha_thre=0.0,
                     stratified=False, cone_angle=0.0):
            near_planes = torch.full_like(rays_o[..., 0], fill_value=near_plane)
            far_planes = torch.full_like(rays_o[..., 0], fill_value=far_plane)
            if t_min is not None:
                near_planes = torch.clamp(near_planes, min=t_min)
            if t_max is not None:
                far_planes = torch.clamp(far_planes, max=t_max)
            if stratified:
                u = torch.rand_like(near_planes)
                self.last_u = u.clone()
                near_planes += u * render_step_size
            ri, t0, t1, _ = R.traverse(rays_o.numpy(), rays_d.numpy(), near_planes.numpy(), far_planes.numpy(),
                                       self.binaries.numpy(), self.aabbs.numpy(), render_step_size, cone_angle)
            ri, t0, t1 = torch.from_numpy(ri), torch.from_numpy(t0), torch.from_numpy(t1)
            if (alpha_thre > 0.0 or early_stop_eps > 0.0) and sigma_fn is not None:
                alpha_thre = min(alpha_thre, self.occs.mean().item())
                sig = sigma_fn(t0, t1, ri) if t0.shape[0] else torch.empty(0)
                vis = R.render_visibility_from_density(t0.numpy(), t1.numpy(), sig.detach().numpy(), ri.numpy(),
                                                       rays_o.shape[0], early_stop_eps, alpha_thre)
                mk = torch.from_numpy(vis)
                ri, t0, t1 = ri[mk], t0[mk], t1[mk]
            return ri, t0, t1

    def pack_info(ray_indices, n_rays=None):
        n = int(n_rays) if n_rays is not None else int(ray_indices.max()) + 1
        return torch.from_numpy(R.pack_info(ray_indices.numpy(), n))

    def render_weight_from_density(t_starts, t_ends, sigmas, packed_info=None, ray_indices=None, n_rays=None,
                                   prefix_trans=None):
        if ray_indices is None:
            cnt = packed_info[:, 1].numpy()
            ri = np.repeat(np.arange(len(cnt)), cnt)
            n = len(cnt)
        else:
            ri, n = ray_indices.numpy(), int(n_rays)
        w, tr, al = R.render_weight_from_density(t_starts.detach().numpy(), t_ends.detach().numpy(),
                                                 sigmas.detach().numpy(), ri, n)
        return torch.from_numpy(w), torch.from_numpy(tr), torch.from_numpy(al)

    def accumulate_along_rays(weights, values=None, ray_indices=None, n_rays=None):
        v = None if values is None else values.detach().numpy()
        return torch.from_numpy(R.accumulate_along_rays(weights.detach().numpy(), v, ray_indices.numpy(),
                                                        int(n_rays)))

    m.OccGridEstimator = OccGridEstimator
    m.pack_info = pack_info
    m.render_weight_from_density = render_weight_from_density
    m.accumulate_along_rays = accumulate_along_rays
    return m


def install() -> None:
    if "nerfacc" not in sys.modules:
        sys.modules["nerfacc"] = _nerfacc_standin()

    if "jaxtyping" not in sys.modules:
        m = types.ModuleType("jaxtyping")

        class _Ann:
            def __class_getitem__(cls, item):
                return cls

        m.Float = _Ann
        m.Int = _Ann
        m.Bool = _Ann
        sys.modules["jaxtyping"] = m

    if "viser" not in sys.modules:
        v = types.ModuleType("viser")
        vt = types.ModuleType("viser.transforms")
        v.transforms = vt
        sys.modules["viser"] = v
        sys.modules["viser.transforms"] = vt

    if "torchvision" not in sys.modules:
        tv = types.ModuleType("torchvision")
        tvu = types.ModuleType("torchvision.utils")
        tvu.make_grid = lambda *a, **k: None
        tv.utils = tvu
        sys.modules["torchvision"] = tv
        sys.modules["torchvision.utils"] = tvu

    try:
        import torch.utils.tensorboard  # noqa: F401
    except Exception:
        tb = types.ModuleType("torch.utils.tensorboard")

        class SummaryWriter:
            def __init__(self, *a, **k):
                pass

            def __getattr__(self, name):
                return lambda *a, **k: None

        tb.SummaryWriter = SummaryWriter
        sys.modules["torch.utils.tensorboard"] = tb
