"""adaptive_city_nerf_amd -- MI355X-native volumetric ray renderer for the
psklavos1/adaptive-city-nerf stratified render hot path.

Python host code mirrors the reference's operator surface (models/encodings.py,
models/inr/meta_ngp.py, models/inr/meta_container.py, models/metamodule, nerfs/ray_sampling.py,
nerfs/ray_rendering.py, nerfs/scene_box.py) and calls hand-written gfx950 kernels through the C ABI
of libacnerf.so (include/acnerf.h).  There is no CPU fallback.
"""
import torch  # noqa: F401  (load torch's HIP runtime before libacnerf.so)

__version__ = "0.1.0"

from .encodings import FrequencyEncoder, HashGridEncoder, SHEncoder, components_from_spherical_harmonics  # noqa: E402,F401
from .meta_container import MetaContainer  # noqa: E402,F401
from .meta_ngp import MetaNGP  # noqa: E402,F401
from .metamodule import MetaBatchLinear, MetaLayerBlock, MetaLinear, MetaModule, MetaSequential  # noqa: E402,F401
from .ray_rendering import (render_expert_occ, render_image, render_rays, render_rays_occ,  # noqa: E402,F401
                            render_rays_stratified, stratified_t_vals, volume_render)
from . import nerfacc  # noqa: E402,F401
from .nerfacc import OccGridEstimator  # noqa: E402,F401
from .ray_sampling import clamp_rays_near_far, get_ray_directions, get_rays, pack_rays, unpack_rays  # noqa: E402,F401
from .scene_box import SceneBox  # noqa: E402,F401
from .trunc_exp import trunc_exp  # noqa: E402,F401
from .data import (DeviceRaysDataset, ImageMetadata, Task, TaskDataset, get_dataset,  # noqa: E402,F401
                   get_image_metadata)
from . import clusters  # noqa: E402,F401
