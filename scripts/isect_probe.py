"""Projection + intersection only (no raster) on the c2 scene, repeated, for rocprofv3 kernel stats of
the isect kernels under probe builds (HGSR_LIB=...; e.g. an emit without key stores).  Probe builds
produce wrong intersection arrays, so nothing here reads them beyond the sort."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from horizongs_amd import gsplat_api as G  # noqa: E402
from horizongs_amd.synthetic import c2  # noqa: E402

sc = c2().to("cuda:0")
radii, means2d, depths, conics, _ = G.fully_fused_projection(sc.means, None, sc.quats, sc.scales, sc.viewmats,
                                                             sc.Ks, sc.width, sc.height)
tw, th = G._tile_grid(sc.width, sc.height, 16)
for _ in range(int(os.environ.get("ITERS", "20"))):
    st = G._isect_count(means2d, radii, 16, tw, th, depths)
    out = G._isect_finish(st)
torch.cuda.synchronize()
print("isects", int(out[1].numel()))
