"""aonerf -- MI355X-native (gfx950) volumetric-render hot path of DJNing/articulated-object-nerf.

Modules mirror the reference's API surface for the path:
  aonerf.helper     <- models/vanilla_nerf/helper.py
  aonerf.model      <- models/vanilla_nerf/model.py (NeRFMLP, NeRF)
  aonerf.ray_utils  <- datasets/ray_utils.py (get_ray_directions, get_rays)
  aonerf.render     <- LitNeRF.render_rays / render_rays_test (models/vanilla_nerf/model.py)
  aonerf.interface  <- models/interface.py (PSNR definitions, image split)
  aonerf.parallel   -- row-band sharding + RCCL frame gather
All compute runs in libaonerf.so (include/aonerf.h); there is no CPU fallback.
"""
from . import _lib

__all__ = ["helper", "model", "ray_utils", "render", "interface", "parallel", "load_library"]


def load_library():
    """Load libaonerf.so now (raises ImportError if it has not been built)."""
    return _lib.lib()
