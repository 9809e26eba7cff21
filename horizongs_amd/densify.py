"""Densification on the MI355X, host side.

Drop-ins for the periodic / per-step densification work of the reference:

* `training_statis(model, opt, render_pkg, width, height)` <- BasicModel.training_statis
  (scene/basic_model.py:96-144): one fused kernel instead of ~20 masked torch ops.
* `remove_duplicates(grid_coords, candidates)` <- BasicModel.get_remove_duplicates
  (:179-190): hash-set lookup, O(A + M) instead of the O(A*M) chunked broadcast compare.
* `scatter_max(src, index, dim_size)` <- torch_scatter.scatter_max(...)[0]
  (scene/lod_model.py:559; torch_scatter is not a dependency here).
* `weed_out(model, positions, levels)` <- GaussianLoDModel.weed_out (lod_model.py:236-249).
* `anchor_growing(model, grads, opt, offset_mask, iteration)` <- GaussianLoDModel.anchor_growing
  (lod_model.py:487-596) built from the above (same anchor order: torch.unique's sorted voxels).

There is no CPU path: tensors must be HIP device tensors.
"""
from __future__ import annotations

import torch

from .decode import visible_index

from . import _native as N
from ._native import ptr

_D2L = {"floor": 0, "round": 1, "ceil": 2, "progressive": 3}


def _check_dev(*ts):
    for t in ts:
        if t is not None and not t.is_cuda:
            raise RuntimeError("hgsr: inputs must be HIP device tensors (no CPU fallback)")


def _state(t, name):
    if t.dtype != torch.float32 or not t.is_contiguous() or not t.is_cuda:
        raise RuntimeError(f"hgsr training_statis: model.{name} must be a contiguous float32 HIP tensor")
    return t


@torch.no_grad()
def training_statis(model, opt, render_pkg, width, height):
    """BasicModel.training_statis: updates model.{anchor_opacity_accum, anchor_demon,
    offset_gradient_accum, offset_denom[, max_radii2D, offset_opacity_accum]} in place.
    Unlike the reference it leaves viewspace_points.grad unscaled."""
    sel = render_pkg["selection_mask"].reshape(-1)
    vis = render_pkg["visible_mask"].reshape(-1)
    grad = render_pkg["viewspace_points"].grad
    filt = render_pkg["visibility_filter"].reshape(-1)
    opacity = render_pkg["opacity"].reshape(-1)
    radii = render_pkg["radii"].reshape(-1)
    _check_dev(sel, vis, grad, filt, opacity, radii)
    if opt.pruning_type not in ("mean", "max"):
        raise ValueError(f"Unknown pruning_type: {opt.pruning_type}")
    if opt.growing_type not in ("mean", "max"):
        raise ValueError(f"Unknown growing_type: {opt.growing_type}")
    noff = model.n_offsets
    vm = render_pkg["visible_mask"]
    # the decode's index of the same mask object is reused (no second host sync)
    vis_idx = visible_index(vm if vm.dim() == 1 else vis) if vis.dtype == torch.bool else \
        torch.nonzero(vis, as_tuple=False).reshape(-1).to(torch.int32)
    Av = vis_idx.numel()
    if sel.numel() != Av * noff:
        raise ValueError(f"hgsr training_statis: selection_mask has {sel.numel()} slots, expected {Av * noff}")
    sel8 = sel.to(torch.uint8).contiguous()
    rank = (torch.cumsum(sel8, 0, dtype=torch.int32) - sel8).contiguous()
    gmax = opt.growing_type == "max"
    N.call("hgsr_training_statis", Av, noff, int(width), int(height), int(opt.pruning_type == "max"), int(gmax),
           ptr(vis_idx), ptr(sel8), ptr(rank), ptr(filt.to(torch.uint8).contiguous()),
           ptr(grad.reshape(-1, 2).float().contiguous()), ptr(opacity.float().contiguous()),
           ptr(radii.to(torch.int32).contiguous()) if gmax else None,
           ptr(_state(model.anchor_opacity_accum, "anchor_opacity_accum")),
           ptr(_state(model.anchor_demon, "anchor_demon")),
           ptr(_state(model.offset_gradient_accum, "offset_gradient_accum")),
           ptr(_state(model.offset_denom, "offset_denom")),
           ptr(_state(model.max_radii2D, "max_radii2D")) if gmax else None,
           ptr(_state(model.offset_opacity_accum, "offset_opacity_accum")) if gmax else None,
           N.stream(sel.device))


@torch.no_grad()
def remove_duplicates(grid_coords, candidates):
    """get_remove_duplicates: bool [U], True where the candidate voxel is already occupied."""
    _check_dev(grid_coords, candidates)
    dev = candidates.device
    g = grid_coords.to(torch.int32).reshape(-1, 3).contiguous()
    c = candidates.to(torch.int32).reshape(-1, 3).contiguous()
    found = torch.empty(c.shape[0], dtype=torch.uint8, device=dev)
    overflow = torch.empty(1, dtype=torch.int32, device=dev)
    ws_b = N.size_query("hgsr_voxel_dedup_ws_bytes", g.shape[0])
    ws = torch.empty(ws_b, dtype=torch.uint8, device=dev)
    N.call("hgsr_voxel_dedup", g.shape[0], ptr(g) if g.numel() else None, c.shape[0], ptr(c) if c.numel() else None,
           ptr(found) if c.numel() else None, ptr(overflow), ptr(ws), ws_b, N.stream(dev))
    if int(overflow.item()) != 0:
        raise RuntimeError("hgsr remove_duplicates: voxel coordinates outside +-(2^20-1)")
    return found.bool()


@torch.no_grad()
def scatter_max(src, index, dim_size=None):
    """torch_scatter.scatter_max(src, index, dim=0)[0] for 2-D src (rows no index reaches: 0)."""
    _check_dev(src, index)
    src2 = src.reshape(src.shape[0], -1).float().contiguous()
    idx = index.reshape(-1).to(torch.int64).contiguous()
    n_out = int(dim_size) if dim_size is not None else (int(idx.max().item()) + 1 if idx.numel() else 0)
    out = torch.empty(n_out, src2.shape[1], dtype=torch.float32, device=src.device)
    N.call("hgsr_scatter_max", src2.shape[0], src2.shape[1], ptr(src2) if src2.numel() else None,
           ptr(idx) if idx.numel() else None, n_out, ptr(out) if out.numel() else None, N.stream(src.device))
    return out.reshape((n_out,) + tuple(src.shape[1:]))


@torch.no_grad()
def weed_out(model, positions, levels):
    """GaussianLoDModel.weed_out: bool mask of the candidates enough cameras would render."""
    _check_dev(positions, levels)
    n = positions.shape[0]
    if getattr(model, "weed_ratio", 0) <= 0:
        return torch.ones(n, dtype=torch.bool, device=positions.device)
    cams = model.cam_infos.float().contiguous()
    mask = torch.empty(n, dtype=torch.uint8, device=positions.device)
    N.call("hgsr_weed_out", n, ptr(positions.float().contiguous()), ptr(levels.reshape(-1).to(torch.int32).contiguous()),
           cams.shape[0], ptr(cams), float(model.standard_dist), float(model.fork), int(model.street_levels),
           _D2L[model.dist2level], float(model.weed_ratio), ptr(mask), N.stream(positions.device))
    return mask.bool()


@torch.no_grad()
def anchor_growing(model, grads, opt, offset_mask, iteration):
    """GaussianLoDModel.anchor_growing (scene/lod_model.py:487-596) with the duplicate removal,
    feature scatter-max and weed-out on the HIP kernels above."""
    dev = grads.device
    noff = model.n_offsets
    init_length = model.get_anchor.shape[0]
    grads = grads.clone()
    grads[~offset_mask] = 0.0
    anchor_grads = torch.sum(grads.reshape(-1, noff), dim=-1) / (torch.sum(offset_mask.reshape(-1, noff), dim=-1) + 1e-6)
    for cur_level in range(model.street_levels):
        update_value = model.fork ** opt.update_ratio
        if model.training_stage == "coarse":
            add_level = cur_level
        elif model.training_stage == "fine":
            add_level = max(cur_level + 1, model.aerial_levels)
        else:
            raise ValueError(f"invalid training stage {model.training_stage}")
        cur_level_mask = (model.get_level == cur_level).squeeze(dim=1)
        add_level_mask = (model.get_level == add_level).squeeze(dim=1)
        if torch.sum(cur_level_mask) == 0:
            continue
        cur_threshold = opt.densify_grad_threshold * (update_value ** cur_level)
        extra_threshold = cur_threshold * opt.extra_ratio
        candidate_mask = grads >= cur_threshold
        candidate_extra_mask = anchor_grads >= extra_threshold
        length_inc = model.get_anchor.shape[0] - init_length
        if length_inc > 0:
            candidate_mask = torch.cat([candidate_mask, torch.zeros(length_inc * noff, dtype=torch.bool, device=dev)])
            candidate_extra_mask = torch.cat([candidate_extra_mask, torch.zeros(length_inc, dtype=torch.bool,
                                                                                device=dev)])
        candidate_mask = candidate_mask & cur_level_mask.repeat_interleave(noff)
        candidate_extra_mask = candidate_extra_mask & cur_level_mask
        if model.training_stage == "coarse":
            candidate_extra_mask = candidate_extra_mask & (model._level < model.aerial_levels).squeeze()
        else:
            candidate_extra_mask = candidate_extra_mask & (model._level >= model.aerial_levels).squeeze()
        model._extra_level += opt.extra_up * candidate_extra_mask.float()

        all_xyz = model.get_anchor.unsqueeze(dim=1) + model._offset * model.get_scaling[:, :3].unsqueeze(dim=1)
        voxel_size = model.voxel_size / (float(model.fork) ** (add_level - model.aerial_levels))
        grid_coords = torch.round(model.get_anchor[add_level_mask] / voxel_size - model.padding).int()
        selected_xyz = all_xyz.view([-1, 3])[candidate_mask]
        selected_grid_coords = torch.round(selected_xyz / voxel_size - model.padding).int()
        unique, inverse = torch.unique(selected_grid_coords, return_inverse=True, dim=0)
        if opt.overlap:
            keep = torch.ones(unique.shape[0], dtype=torch.bool, device=dev)
        elif unique.shape[0] > 0:
            keep = ~remove_duplicates(grid_coords, unique)
        else:
            keep = torch.zeros(0, dtype=torch.bool, device=dev)
        candidate_anchor = unique[keep] * voxel_size + model.padding * voxel_size
        new_level = torch.full((candidate_anchor.shape[0],), add_level, dtype=torch.int, device=dev)
        if candidate_anchor.shape[0] > 0:
            weed_mask = weed_out(model, candidate_anchor, new_level)
            candidate_anchor = candidate_anchor[weed_mask]
            new_level = new_level[weed_mask]
            keep_clone = keep.clone()
            keep[keep_clone] = weed_mask
        if candidate_anchor.shape[0] > 0:
            feat = model._anchor_feat.unsqueeze(dim=1).repeat([1, noff, 1]).view([-1, model.feat_dim])[candidate_mask]
            new_feat = scatter_max(feat, inverse, unique.shape[0])[keep]
            new_scaling = torch.log(torch.ones_like(candidate_anchor).repeat([1, 2]).float() * voxel_size)
            new_rotation = torch.zeros([candidate_anchor.shape[0], 4], dtype=torch.float, device=dev)
            new_rotation[:, 0] = 1.0
            new_offsets = torch.zeros_like(candidate_anchor).unsqueeze(dim=1).repeat([1, noff, 1]).float()
            d = {"anchor": candidate_anchor, "scaling": new_scaling, "rotation": new_rotation, "anchor_feat": new_feat,
                 "offset": new_offsets}
            model.anchor_demon = torch.cat([model.anchor_demon, torch.zeros([candidate_anchor.shape[0], 1],
                                                                            device=dev)], dim=0)
            model.anchor_opacity_accum = torch.cat([model.anchor_opacity_accum,
                                                    torch.zeros([candidate_anchor.shape[0], 1], device=dev)], dim=0)
            tensors = model.cat_tensors_to_optimizer(d)
            model._anchor = tensors["anchor"]
            model._scaling = tensors["scaling"]
            model._rotation = tensors["rotation"]
            model._anchor_feat = tensors["anchor_feat"]
            model._offset = tensors["offset"]
            model._level = torch.cat([model._level, new_level.unsqueeze(dim=1).float()], dim=0)
            model._extra_level = torch.cat([model._extra_level, torch.zeros(candidate_anchor.shape[0],
                                                                            dtype=torch.float, device=dev)], dim=0)
