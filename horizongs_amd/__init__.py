"""horizongs_amd — MI355X-native (gfx950) differentiable Gaussian rasterizer for Horizon-GS.

The hot path Horizon-GS reaches through gsplat (reference gaussian_renderer/render.py:13-14,
40-76, 149-186) re-built as hand-written HIP kernels behind a C ABI (include/hgsr.h,
horizongs_amd/_lib/libhgsr.so) with a gsplat-compatible Python surface.
"""
from .gsplat_api import (  # noqa: F401
    depth_to_normal,
    fully_fused_projection,
    fully_fused_projection_2dgs,
    isect_offset_encode,
    isect_tiles,
    rasterization,
    rasterization_2dgs,
    rasterize_to_pixels,
    rasterize_to_pixels_2dgs,
    spherical_harmonics,
)

__version__ = "0.1.0"
