"""Explicit (merged-scene) Gaussians on the MI355X: the c5 render path, host side.

Reference render() with pc.explicit_gs (gaussian_renderer/render.py:22-25):

* `set_gs_mask(model, cam_center, resolution_scale)` <- GaussianLoDModel.set_gs_mask
  (scene/lod_model.py:292-296): the LoD level test of set_anchor_mask on the explicit
  centres (hgsr_lod_mask, dist2level 'floor').
* `generate_explicit_gaussians(model, visible_mask)` <- BasicModel.generate_explicit_gaussians
  (scene/basic_model.py:373-383): the boolean-mask gathers of xyz, cat(features_dc,
  features_rest), opacity, scaling and rotation as ONE ordered stream compaction
  (csrc/explicit.hip: count + scan + coalesced gather; one host read of the kept count, as
  the reference's mask indexing has), differentiable (the backward scatters, overwriting).
* `bind(scene.lod_model, scene.basic_model)` points the reference's classes at these.

There is no CPU path: tensors must be HIP device tensors.
"""
from __future__ import annotations

import torch

from . import _native as N
from ._native import ptr
from .decode import lod_mask


def _check_dev(*ts):
    for t in ts:
        if t is not None and not t.is_cuda:
            raise RuntimeError("hgsr: inputs must be HIP device tensors (no CPU fallback)")


def _f32(t):
    return t.contiguous() if t.dtype == torch.float32 else t.float().contiguous()


class _ExplicitGather(torch.autograd.Function):
    @staticmethod
    def forward(ctx, mask_u8, xyz, f_dc, f_rest, opacity, scaling, rotation):
        Ng = xyz.shape[0]
        K = 1 + (0 if f_rest is None else f_rest.shape[1])
        dev = xyz.device
        ws_b = N.size_query("hgsr_explicit_ws_bytes", Ng)
        ws = torch.empty(max(ws_b, 1), dtype=torch.uint8, device=dev)
        total = torch.empty(1, dtype=torch.int64, device=dev)
        s = N.stream(dev)
        N.call("hgsr_explicit_count", Ng, None, None, None, None, 1.0, 1.0, 1.0, 0, ptr(mask_u8), None, ptr(ws),
               ws_b, ptr(total), s)
        M = int(total.item())  # the one host read (the reference's boolean indexing syncs too)
        out = [torch.empty((M, 3), dtype=torch.float32, device=dev),
               torch.empty((M, K, 3), dtype=torch.float32, device=dev),
               torch.empty((M, 1), dtype=torch.float32, device=dev),
               torch.empty((M, scaling.shape[1]), dtype=torch.float32, device=dev),
               torch.empty((M, 4), dtype=torch.float32, device=dev)]
        index = torch.empty(M, dtype=torch.int32, device=dev)
        if M > 0:
            N.call("hgsr_explicit_gather", Ng, K, ptr(mask_u8), ptr(xyz), ptr(f_dc), ptr(f_rest), ptr(opacity),
                   ptr(scaling), ptr(rotation), ptr(ws), ws_b, *[ptr(t) for t in out], ptr(index), s)
        ctx.save_for_backward(mask_u8, ws)
        ctx.cfg = (Ng, K, ws_b, f_rest is not None)
        ctx.mark_non_differentiable(index)
        return (*out, index)

    @staticmethod
    def backward(ctx, g_xyz, g_color, g_opac, g_scale, g_rot, g_index):
        mask_u8, ws = ctx.saved_tensors
        Ng, K, ws_b, has_rest = ctx.cfg
        dev = mask_u8.device
        need = ctx.needs_input_grad
        v = [torch.empty((Ng, 3), device=dev) if need[1] else None,
             torch.empty((Ng, 1, 3), device=dev) if need[2] else None,
             torch.empty((Ng, K - 1, 3), device=dev) if (has_rest and need[3]) else None,
             torch.empty((Ng, 1), device=dev) if need[4] else None,
             torch.empty((Ng, 3), device=dev) if need[5] else None,
             torch.empty((Ng, 4), device=dev) if need[6] else None]
        g = [None if x is None else _f32(x) for x in (g_xyz, g_color, g_opac, g_scale, g_rot)]
        N.call("hgsr_explicit_scatter", Ng, K, ptr(mask_u8), ptr(ws), ws_b, *[ptr(x) for x in g],
               *[ptr(x) for x in v], N.stream(dev))
        return (None, *v)


def gather(visible_mask, xyz, features_dc, features_rest, opacity, scaling, rotation):
    """The gathers of generate_explicit_gaussians: (xyz, color [M,K,3], opacity, scaling, rot, index)."""
    _check_dev(visible_mask, xyz, features_dc, features_rest, opacity, scaling, rotation)
    Ng = xyz.shape[0]
    assert visible_mask.shape[0] == Ng and features_dc.shape == (Ng, 1, 3), "bad explicit shapes"
    m = visible_mask.reshape(-1)
    m = m.view(torch.uint8) if m.dtype == torch.bool else m.to(torch.uint8)
    rest = None if features_rest is None or features_rest.shape[1] == 0 else _f32(features_rest)
    return _ExplicitGather.apply(m.contiguous(), _f32(xyz), _f32(features_dc), rest, _f32(opacity),
                                 _f32(scaling), _f32(rotation))


@torch.no_grad()
def set_gs_mask(model, cam_center, resolution_scale):
    """GaussianLoDModel.set_gs_mask: model._gs_mask = level <= LoD(dist(_xyz, camera))."""
    if getattr(model, "dist2level", "floor") != "floor":
        raise NotImplementedError("hgsr set_gs_mask: dist2level='floor' only (every reference config)")
    model._gs_mask = lod_mask(model._xyz.detach(), model._level, model._extra_level, cam_center,
                              resolution_scale, model.standard_dist, model.fork, model.street_levels)
    return model._gs_mask


def generate_explicit_gaussians(model, visible_mask=None):
    """Drop-in for BasicModel.generate_explicit_gaussians (scene/basic_model.py:373-383):
    (xyz, color [M,K,3], opacity [M,1], scaling, rot, active_sh_degree, mask [N] of ones)."""
    Ng = model._xyz.shape[0]
    if visible_mask is None:
        visible_mask = torch.ones(Ng, dtype=torch.bool, device=model._xyz.device)
    xyz, color, opacity, scaling, rot, _ = gather(visible_mask, model._xyz, model._features_dc,
                                                  model._features_rest, model._opacity, model._scaling,
                                                  model._rotation)
    mask = torch.ones(Ng, dtype=torch.bool, device=model._xyz.device)
    return xyz, color, opacity, scaling, rot, model.active_sh_degree, mask


def bind(lod_model_module, basic_model_module=None):
    """Point the reference's explicit render path at the HIP kernels:

        import scene.lod_model, scene.basic_model
        from horizongs_amd import explicit as hx
        hx.bind(scene.lod_model, scene.basic_model)
    """
    lod_model_module.GaussianLoDModel.set_gs_mask = (
        lambda self, cam_center, resolution_scale: set_gs_mask(self, cam_center, resolution_scale))
    base = basic_model_module.BasicModel if basic_model_module is not None else lod_model_module.GaussianLoDModel
    base.generate_explicit_gaussians = lambda self, visible_mask=None: generate_explicit_gaussians(self, visible_mask)

