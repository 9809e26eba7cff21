"""Diagnostic: per-tile bin sizes of the c2 scene (tile_sort work distribution)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from horizongs_amd import gsplat_api as G
from horizongs_amd.synthetic import c2

sc = c2().to("cuda")
r = G.fully_fused_projection(sc.means, None, sc.quats, sc.scales, sc.viewmats, sc.Ks, sc.width, sc.height)
radii, means2d, depths = r[0], r[1], r[2]
tw, th = G._tile_grid(sc.width, sc.height, 16)
tpg, ids, fl, off = G._isect_binned(means2d, radii, 16, tw, th, depths)
o = off.reshape(-1).cpu().numpy().astype(np.int64)
n = np.diff(np.append(o, ids.numel()))
print("bins", n.size, "isects", ids.numel(), "mean", n.mean(), "max", n.max(), "min", n.min())
for q in (50, 90, 99, 99.9):
    print("p%s" % q, np.percentile(n, q))
print(">256", (n > 256).sum(), ">512", (n > 512).sum(), ">1024", (n > 1024).sum(), ">2048", (n > 2048).sum())
print("tiles per gauss hist", np.bincount(tpg.reshape(-1).cpu().numpy())[:20])
