"""Time the densification kernels against the reference's torch formulation on the same GPU.

Reference formulations timed here (torch ops, as the reference runs them on the device):
  * training_statis: scene/basic_model.py:96-144 (mean / mean)
  * get_remove_duplicates: scene/basic_model.py:179-190 (4096-row chunked broadcast compare)
  * weed_out: scene/lod_model.py:236-249 (python loop over cameras)
Sizes: A anchors x 10 offsets (c2-decode scale, A = 500k, 70 % visible), 100k candidate
voxels against 500k occupied ones, 1000 training cameras.
Usage: python scripts/bench_densify.py  (prints one JSON line)"""
import json
import math
import os
import sys
import time
from functools import reduce
from types import SimpleNamespace

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from horizongs_amd import densify as HD  # noqa: E402

dev = "cuda"


def timeit(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps * 1e3


def ref_statis(st, sel, vis, grad, filt, opacity, W, H, k):
    temp = torch.zeros(sel.shape[0], dtype=torch.float32, device=dev)
    temp[sel] = opacity.view(-1)
    temp = temp.view(-1, k)
    cnt = sel.view(-1, k).sum(dim=1, keepdim=True).float()
    avg = temp.sum(dim=1, keepdim=True) / torch.clamp(cnt, min=1.0)
    avg[cnt == 0] = 0
    st["anchor_opacity_accum"][vis] += avg
    st["anchor_demon"][vis] += 1
    vr = vis.unsqueeze(1).repeat(1, k).view(-1)
    comb = torch.zeros_like(st["offset_gradient_accum"], dtype=torch.bool).squeeze(1)
    comb[vr] = sel
    tmp = comb.clone()
    comb[tmp] = filt
    g = grad.clone()
    g[:, 0] *= W * 0.5
    g[:, 1] *= H * 0.5
    gn = torch.norm(g[filt, :2], dim=-1, keepdim=True)
    st["offset_gradient_accum"][comb] += gn
    st["offset_denom"][comb] += 1


def ref_dedup(grid, cand):
    out = []
    for i in range(grid.shape[0] // 4096 + (1 if grid.shape[0] % 4096 else 0)):
        out.append((cand.unsqueeze(1) == grid[i * 4096:(i + 1) * 4096, :]).all(-1).any(-1).view(-1))
    return reduce(torch.logical_or, out)


def ref_weed(pos, lev, cams, sd, fork, sl, ratio):
    count = torch.zeros(pos.shape[0], dtype=torch.int, device=dev)
    for cam in cams:
        dist = torch.sqrt(torch.sum((pos - cam[:3]) ** 2, dim=1)) * cam[3]
        pred = torch.log2(sd / dist) / math.log2(fork)
        count += (lev <= torch.clamp(torch.floor(pred).int(), 0, sl - 1)).int()
    return (count / len(cams)) > ratio


def main():
    g = torch.Generator(device=dev).manual_seed(0)
    A, k = 500_000, 10
    vis = torch.rand(A, device=dev, generator=g) < 0.7
    Av = int(vis.sum())
    sel = torch.rand(Av * k, device=dev, generator=g) < 0.45
    M = int(sel.sum())
    filt = torch.rand(M, device=dev, generator=g) < 0.9
    grad = torch.randn(M, 2, device=dev, generator=g) * 1e-3
    opac = torch.rand(M, 1, device=dev, generator=g)
    mk = lambda: dict(anchor_opacity_accum=torch.zeros(A, 1, device=dev), anchor_demon=torch.zeros(A, 1, device=dev),
                      offset_gradient_accum=torch.zeros(A * k, 1, device=dev),
                      offset_denom=torch.zeros(A * k, 1, device=dev))
    st = mk()
    model = SimpleNamespace(n_offsets=k, **mk())
    pkg = dict(selection_mask=sel, visible_mask=vis, viewspace_points=SimpleNamespace(grad=grad[None]),
               visibility_filter=filt, opacity=opac, radii=torch.ones(M, dtype=torch.int32, device=dev))
    o = SimpleNamespace(pruning_type="mean", growing_type="mean")
    t_stat = timeit(lambda: HD.training_statis(model, o, pkg, 1920, 1080))
    t_stat_ref = timeit(lambda: ref_statis(st, sel, vis, grad, filt, opac, 1920, 1080, k))
    grid = torch.randint(-4000, 4000, (500_000, 3), device=dev, generator=g, dtype=torch.int32)
    cand = torch.randint(-4000, 4000, (100_000, 3), device=dev, generator=g, dtype=torch.int32)
    cand[:50_000] = grid[:50_000]
    t_dd = timeit(lambda: HD.remove_duplicates(grid, cand))
    t_dd_ref = timeit(lambda: ref_dedup(grid, cand), reps=1)
    assert torch.equal(HD.remove_duplicates(grid, cand), ref_dedup(grid, cand))
    pos = torch.rand(100_000, 3, device=dev, generator=g) * 100 - 50
    lev = torch.randint(0, 6, (100_000,), device=dev, generator=g, dtype=torch.int32)
    cams = torch.cat([torch.rand(1000, 3, device=dev, generator=g) * 80 - 40,
                      0.5 + torch.rand(1000, 1, device=dev, generator=g)], 1)
    wm = SimpleNamespace(weed_ratio=0.25, cam_infos=cams, standard_dist=20.0, fork=2, street_levels=6,
                         dist2level="floor")
    t_w = timeit(lambda: HD.weed_out(wm, pos, lev))
    t_w_ref = timeit(lambda: ref_weed(pos, lev, cams, 20.0, 2, 6, 0.25), reps=2)
    print(json.dumps({"training_statis_ms": round(t_stat, 3), "training_statis_torch_ms": round(t_stat_ref, 3),
                      "remove_duplicates_ms": round(t_dd, 3), "remove_duplicates_torch_ms": round(t_dd_ref, 1),
                      "weed_out_ms": round(t_w, 3), "weed_out_torch_ms": round(t_w_ref, 1),
                      "sizes": {"anchors": A, "visible": Av, "selected": M, "grid": 500_000, "candidates": 100_000,
                                "weed_candidates": 100_000, "cameras": 1000}}))


if __name__ == "__main__":
    main()
