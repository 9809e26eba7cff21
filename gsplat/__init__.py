"""Import alias so reference code that does `import gsplat` (gaussian_renderer/render.py:13)
runs unchanged on the hgsr HIP rasterizer.  A Python namespace re-export only: no CUDA
API is emulated; every call lands in horizongs_amd (libhgsr.so, gfx950 kernels)."""
from horizongs_amd.gsplat_api import (  # noqa: F401
    depth_to_normal,
    rasterization,
    rasterization_2dgs,
    spherical_harmonics,
)
from horizongs_amd.gsplat_api import fully_fused_projection, fully_fused_projection_2dgs  # noqa: F401
from horizongs_amd.gsplat_api import isect_offset_encode, isect_tiles  # noqa: F401
from horizongs_amd.gsplat_api import rasterize_to_pixels, rasterize_to_pixels_2dgs  # noqa: F401

from . import cuda  # noqa: F401,E402

__version__ = "1.4.0+hgsr"
