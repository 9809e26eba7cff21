"""CPU restatement of the densification kernels (TEST INFRASTRUCTURE ONLY).

Only tests/ may import this module; the product path (horizongs_amd.densify) never does.

  * training_statis  <- scene/basic_model.py:96-144 (mean / max pruning and growing types)
  * remove_duplicates <- scene/basic_model.py:179-190 get_remove_duplicates (brute force)
  * scatter_max      <- torch_scatter.scatter_max(src, index, dim=0)[0] (empty rows 0)
  * weed_out         <- scene/lod_model.py:236-249 with basic_model.py:192-210 map_to_int_level
  * anchor_growing   <- scene/lod_model.py:487-596, control flow only; the three primitives are
                        injected (the GPU test passes the HIP ones, as densify.bind does for the
                        reference's own method)

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


@torch.no_grad()
def anchor_growing(model, grads, opt, offset_mask, prims):
    """Restatement of GaussianLoDModel.anchor_growing (reference scene/lod_model.py:487-596) with
    its three primitives injected: prims.remove_duplicates(grid, cand) (basic_model.py:179-190),
    prims.weed_out(model, pos, levels) (lod_model.py:236-249), prims.scatter_max(src, idx, n)
    (torch_scatter).  TEST INFRASTRUCTURE: tests/test_gpu_densify.py drives it with the HIP
    primitives of horizongs_amd.densify against the reference's own output (golden)."""
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
            keep = ~prims.remove_duplicates(grid_coords, unique)
        else:
            keep = torch.zeros(0, dtype=torch.bool, device=dev)
        candidate_anchor = unique[keep] * voxel_size + model.padding * voxel_size
        new_level = torch.full((candidate_anchor.shape[0],), add_level, dtype=torch.int, device=dev)
        if candidate_anchor.shape[0] > 0:
            weed_mask = prims.weed_out(model, candidate_anchor, new_level)
            candidate_anchor = candidate_anchor[weed_mask]
            new_level = new_level[weed_mask]
            keep_clone = keep.clone()
            keep[keep_clone] = weed_mask
        if candidate_anchor.shape[0] > 0:
            feat = model._anchor_feat.unsqueeze(dim=1).repeat([1, noff, 1]).view([-1, model.feat_dim])[candidate_mask]
            new_feat = prims.scatter_max(feat, inverse, unique.shape[0])[keep]
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
