"""`from gsplat.cuda._wrapper import fully_fused_projection, fully_fused_projection_2dgs`
(reference gaussian_renderer/render.py:14) resolves here; re-exports of horizongs_amd."""
from horizongs_amd.gsplat_api import (  # noqa: F401
    fully_fused_projection,
    fully_fused_projection_2dgs,
    isect_offset_encode,
    isect_tiles,
    rasterize_to_pixels,
    rasterize_to_pixels_2dgs,
    spherical_harmonics,
)
