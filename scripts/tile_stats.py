"""Per-tile intersection counts of the bench's c2 camera set (GPU; diagnostics only).

For each of the 16 views: the tile bins' sizes from the forward's isect_offsets, the heaviest
tile against the average share of one wave slot (tiles x 4 waves over 256 CUs x 8 slots), and
the same for the deepest tile's trimmed range (up to its latest contributor, the backward's
range).  A heaviest tile far above the per-slot share means the raster kernels' time is set by
one workgroup's sequential list, not by the chip's throughput.

usage: python scripts/tile_stats.py [--gs 3d|2d] > gpurun_out/tile_stats.json
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from horizongs_amd import gsplat_api as G  # noqa: E402
from horizongs_amd.synthetic import camera_set, make_scene  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gs", default="3d")
    ap.add_argument("--n", type=int, default=2_000_000)
    a = ap.parse_args()
    dev = "cuda:0"
    W, H = 1920, 1080
    sc = make_scene(a.n, W, H, seed=0)
    cams = camera_set(16).to(dev)
    Ks = sc.Ks.to(dev)
    means, quats, scales, opac, cols = (t.to(dev) for t in (sc.means, sc.quats, sc.scales, sc.opacities, sc.colors))
    slots = 256 * 8
    out = []
    for v in range(len(cams)):
        vm = cams[v][None]
        with torch.no_grad():
            if a.gs == "3d":
                rc, ra, meta = G.rasterization(means, quats, scales, opac, cols, vm, Ks, W, H, packed=False,
                                               render_mode="RGB+ED")
            else:
                _, meta = G.rasterization_2dgs(means, quats, scales, opac, cols, vm, Ks, W, H, render_mode="RGB+ED")
        offs = meta["isect_offsets"].reshape(-1).long().cpu().numpy()
        n = int(meta["flatten_ids"].numel())
        cnt = np.diff(np.append(offs, n))
        share = cnt.sum() * 4 / slots / 4  # a tile's list is walked by each of its 4 waves
        out.append(dict(view=v, isects=n, tiles=int(cnt.size), mean=round(float(cnt.mean()), 1),
                        p50=int(np.percentile(cnt, 50)), p99=int(np.percentile(cnt, 99)), max=int(cnt.max()),
                        per_slot_share=round(float(share), 1), max_over_share=round(float(cnt.max() / share), 2),
                        top10_sum_frac=round(float(np.sort(cnt)[-10:].sum() / cnt.sum()), 4)))
        print(json.dumps(out[-1]), flush=True)
    print(json.dumps({"summary": {"max_over_share_mean": round(float(np.mean([o["max_over_share"] for o in out])), 2),
                                  "max_over_share_max": max(o["max_over_share"] for o in out)}}))


if __name__ == "__main__":
    main()
