"""CPU restatement of the densification kernels (TEST INFRASTRUCTURE ONLY).

Only tests/ may import this module; the product path (horizongs_amd.densify) never does.

  * training_statis  <- scene/basic_model.py:96-144 (mean / max pruning and growing types)
  * remove_duplicates <- scene/basic_model.py:179-190 get_remove_duplicates (brute force)
  * scatter_max      <- torch_scatter.scatter_max(src, index, dim=0)[0] (empty rows 0)
  * weed_out         <- scene/lod_model.py:236-249 with basic_model.py:192-210 map_to_int_level

Pinned: tests/test_oracle.py checks each against tests/golden/densify.npz, outputs of the
reference's own methods run on the CPU (scripts/make_golden.py).
"""
from __future__ import annotations

import math

import torch


def training_statis(state, sel, vis, grad, filt, opacity, radii, W, H, n_offsets, pruning_type, growing_type):
    """state: dict of the six accumulators (modified copies are returned)."""
    st = {k: v.clone() for k, v in state.items()}
    temp_opacity = torch.zeros(sel.shape[0], dtype=torch.float32)
    temp_opacity[sel] = opacity.reshape(-1)
    temp_opacity = temp_opacity.view(-1, n_offsets)
    if pruning_type == "mean":
        cnt = sel.view(-1, n_offsets).sum(dim=1, keepdim=True).float()
        avg = temp_opacity.sum(dim=1, keepdim=True) / torch.clamp(cnt, min=1.0)
        avg[cnt == 0] = 0
        st["anchor_opacity_accum"][vis] += avg
    else:
        st["anchor_opacity_accum"][vis] = torch.max(st["anchor_opacity_accum"][vis],
                                                    torch.abs(temp_opacity.sum(dim=1, keepdim=True)))
    st["anchor_demon"][vis] += 1
    vis_rep = vis.unsqueeze(1).repeat(1, n_offsets).view(-1)
    combined = torch.zeros(st["offset_gradient_accum"].shape[0], dtype=torch.bool)
    combined[vis_rep] = sel
    tmp = combined.clone()
    combined[tmp] = filt
    g = grad.reshape(-1, 2).clone()
    g[:, 0] *= W * 0.5
    g[:, 1] *= H * 0.5
    gn = torch.norm(g[filt, :2], dim=-1, keepdim=True)
    if growing_type == "mean":
        st["offset_gradient_accum"][combined] += gn
    else:
        st["offset_gradient_accum"][combined] = torch.max(st["offset_gradient_accum"][combined], torch.abs(gn))
        st["max_radii2D"][combined] = torch.max(st["max_radii2D"][combined], radii[filt].float())
        st["offset_opacity_accum"][combined] += opacity.reshape(-1, 1)[filt]
    st["offset_denom"][combined] += 1
    return st


def remove_duplicates(grid_coords, cand):
    if grid_coords.shape[0] == 0:
        return torch.zeros(cand.shape[0], dtype=torch.bool)
    return (cand.unsqueeze(1) == grid_coords.unsqueeze(0)).all(-1).any(-1)


def scatter_max(src, index, n_out):
    out = torch.full((n_out, src.shape[1]), -math.inf, dtype=src.dtype)
    out = out.scatter_reduce(0, index.view(-1, 1).expand_as(src), src, reduce="amax", include_self=True)
    out[torch.isinf(out) & (out < 0)] = 0
    return out


def int_level(pred, mode, cur):
    if mode == "floor":
        return torch.clamp(torch.floor(pred).int(), 0, cur)
    if mode == "round":
        return torch.clamp(torch.round(pred).int(), 0, cur)
    if mode == "ceil":
        return torch.clamp(torch.ceil(pred).int(), 0, cur)
    return torch.floor(torch.clamp(pred + 1.0, min=0.9999, max=cur + 0.9999)).int()


def weed_out(pos, levels, cams, standard_dist, fork, street_levels, ratio, mode="floor"):
    count = torch.zeros(pos.shape[0], dtype=torch.int32)
    for cam in cams:
        dist = torch.sqrt(torch.sum((pos - cam[:3]) ** 2, dim=1)) * cam[3]
        pred = torch.log2(standard_dist / dist) / math.log2(fork)
        count += (levels <= int_level(pred, mode, street_levels - 1)).int()
    return (count / len(cams)) > ratio
