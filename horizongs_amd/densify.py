"""Densification on the MI355X, host side.

Drop-ins for the periodic / per-step densification work of the reference:

* `training_statis(model, opt, render_pkg, width, height)` <- BasicModel.training_statis
  (scene/basic_model.py:96-144): one fused kernel instead of ~20 masked torch ops.
* `remove_duplicates(grid_coords, candidates)` <- BasicModel.get_remove_duplicates
  (:179-190): hash-set lookup, O(A + M) instead of the O(A*M) chunked broadcast compare.
* `scatter_max(src, index, dim_size)` <- torch_scatter.scatter_max(...)[0]
  (scene/lod_model.py:559; torch_scatter is not a dependency here).
* `weed_out(model, positions, levels)` <- GaussianLoDModel.weed_out (lod_model.py:236-249).
* `bind(scene.lod_model, scene.basic_model)` points the reference's own classes at these, so its
  GaussianLoDModel.anchor_growing (lod_model.py:487-596) runs unchanged on the HIP primitives.

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


def _as_u8(mask):
    """A bool / 0-1 mask as contiguous uint8 (a view of a contiguous bool tensor: no copy)."""
    if mask.dtype == torch.bool and mask.is_contiguous():
        return mask.view(torch.uint8)
    return mask.to(torch.uint8).contiguous()


def _state(t, name):
    if t.dtype != torch.float32 or not t.is_contiguous() or not t.is_cuda:
        raise RuntimeError(f"hgsr training_statis: model.{name} must be a contiguous float32 HIP tensor")
    return t


@torch.no_grad()
def training_statis(model, opt, render_pkg, width, height):
    """BasicModel.training_statis: updates model.{anchor_opacity_accum, anchor_demon,
    offset_gradient_accum, offset_denom[, max_radii2D, offset_opacity_accum]} in place.
    Unlike the reference it leaves viewspace_points.grad unscaled."""
    sel_t = render_pkg["selection_mask"]
    slot_row = getattr(sel_t, "_hgsr_slot_row", None)  # set by the fused decode
    sel = sel_t.reshape(-1)
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
    sel8 = _as_u8(sel)
    if slot_row is not None and slot_row.numel() == sel.numel():
        rank = slot_row  # output row of each selected slot (the decode's compaction)
    else:
        rank = (torch.cumsum(sel8, 0, dtype=torch.int32) - sel8).contiguous()
    gmax = opt.growing_type == "max"
    # converted inputs held in locals until the launch is enqueued (no aliased temporaries)
    f8, g2 = _as_u8(filt), grad.reshape(-1, 2).float().contiguous()
    op, rd = opacity.float().contiguous(), (radii.to(torch.int32).contiguous() if gmax else None)
    N.call("hgsr_training_statis", Av, noff, int(width), int(height), int(opt.pruning_type == "max"), int(gmax),
           ptr(vis_idx), ptr(sel8), ptr(rank), ptr(f8), ptr(g2), ptr(op), ptr(rd),
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
    pos, lv = positions.float().contiguous(), levels.reshape(-1).to(torch.int32).contiguous()
    N.call("hgsr_weed_out", n, ptr(pos), ptr(lv), cams.shape[0], ptr(cams), float(model.standard_dist), float(model.fork), int(model.street_levels),
           _D2L[model.dist2level], float(model.weed_ratio), ptr(mask), N.stream(positions.device))
    return mask.bool()


def scatter_max_ts(src, index, dim=0, out=None, dim_size=None):
    """torch_scatter.scatter_max signature as lod_model.py:558 calls it
    (`scatter_max(feat, inverse.unsqueeze(1).expand(-1, F), dim=0)[0]`): returns
    (values, None) -- the argmax half is never used by the reference."""
    if dim != 0 or out is not None:
        raise NotImplementedError("hgsr scatter_max: dim=0 and out=None only (the reference's call)")
    idx = index[:, 0] if index.dim() == 2 else index
    return scatter_max(src, idx, dim_size), None


def bind(lod_model_module, basic_model_module=None, base_model_module=None):
    """Point the reference's densification at the HIP primitives; its own
    GaussianLoDModel.anchor_growing (scene/lod_model.py:487-596) then runs unchanged:

        import scene.lod_model, scene.basic_model, scene.base_model
        from horizongs_amd import densify as hd
        hd.bind(scene.lod_model, scene.basic_model, scene.base_model)

    * module-level torch_scatter.scatter_max of scene/lod_model.py:20,558 -> scatter_max_ts
      (and of scene/base_model.py:439, the Scaffold-style GaussianModel's anchor_growing, when
      base_model_module is given)
    * BasicModel.get_remove_duplicates (basic_model.py:179-190) -> remove_duplicates (hash set)
    * GaussianLoDModel.weed_out (lod_model.py:236-249) -> weed_out
    * BasicModel.training_statis (basic_model.py:96-144) -> training_statis (one kernel)"""
    lod_model_module.scatter_max = scatter_max_ts
    if base_model_module is not None:
        base_model_module.scatter_max = scatter_max_ts
    lod = lod_model_module.GaussianLoDModel
    lod.weed_out = lambda self, positions, levels: weed_out(self, positions, levels)
    base = basic_model_module.BasicModel if basic_model_module is not None else lod
    base.get_remove_duplicates = (lambda self, grid_coords, selected_grid_coords_unique, use_chunk=True:
                                  remove_duplicates(grid_coords, selected_grid_coords_unique))
    base.training_statis = lambda self, opt, render_pkg, width, height: training_statis(self, opt, render_pkg,
                                                                                       width, height)
