"""sys.modules stubs that let the reference be imported in THIS container (fixture generation only).

The reference imports a few packages that are absent here and are unused on the stratified
render path: nerfacc (occupancy path only), jaxtyping (annotations),
viser.transforms (OrientedBox only), torchvision.utils.make_grid and
torch.utils.tensorboard.SummaryWriter (logging).  tinycudann is handled by the reference's own
try/except (models/encodings.py:8-14), so its pure-Torch fallback is what gets exercised.
"""
import sys
import types


def install() -> None:
    if "nerfacc" not in sys.modules:
        m = types.ModuleType("nerfacc")

        class OccGridEstimator:  # occupancy path is never taken (use_occ=False)
            def __init__(self, *a, **k):
                raise RuntimeError("nerfacc stub: occupancy path not available")

        def _unavailable(*a, **k):
            raise RuntimeError("nerfacc stub: occupancy path not available")

        m.OccGridEstimator = OccGridEstimator
        m.pack_info = _unavailable
        m.render_weight_from_density = _unavailable
        m.accumulate_along_rays = _unavailable
        sys.modules["nerfacc"] = m

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
