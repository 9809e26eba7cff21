"""Diagnostic: the same c2 3DGS step with the Gaussians stored in screen-tile order (as
anchor-derived scenes roughly are) instead of random order -- shows how much of
isect_emit is the scattered-write pattern.  Prints per-kernel ms for both orders."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench as B  # noqa: E402
from horizongs_amd import _native as NAT  # noqa: E402


def run(wl, steps=10):
    for _ in range(3):
        wl.step()
    torch.cuda.synchronize()
    NAT.call("hgsr_timing_reset")
    NAT.call("hgsr_timing_enable", 1)
    for _ in range(steps):
        wl.step()
    torch.cuda.synchronize()
    NAT.call("hgsr_timing_enable", 0)
    out = {}
    for k in ("isect_count", "isect_emit", "tile_sort", "raster3d_fwd", "raster3d_bwd"):
        t, c = NAT.kernel_time(k)
        if c:
            out[k] = round(t / c, 4)
    return out


def main():
    sys.argv = ["bench.py"]
    args = B.parse()
    wl = B.Workload(args, 0, torch.device("cuda", 0))
    print("random order", run(wl))
    sc = wl.sc
    fx = float(sc.Ks[0, 0, 0])
    u = sc.means[:, 0] / sc.means[:, 2] * fx + sc.Ks[0, 0, 2]
    v = sc.means[:, 1] / sc.means[:, 2] * fx + sc.Ks[0, 1, 2]
    key = (v // 128).long() * 100 + (u // 128).long()
    perm = torch.argsort(key, stable=True).to(wl.means.device)
    with torch.no_grad():
        for name in ("means", "quats", "scales", "opac", "colors"):
            t = getattr(wl, name)
            setattr(wl, name, t[perm].detach().clone().requires_grad_(True))
    wl.params = [wl.means, wl.quats, wl.scales, wl.opac, wl.colors]
    print("tile order  ", run(wl))


if __name__ == "__main__":
    main()
