"""Anchor -> neural-Gaussian decode on the MI355X, host side.

Mirrors the reference's per-view decode so that a Horizon-GS model can hand its
anchors to the fused HIP kernels instead of the ~10 torch launches of
`generate_neural_gaussians`:

* `lod_mask`       <- scene/lod_model.py:286-290 set_anchor_mask (dist2level 'floor')
* `prefilter`      <- set_anchor_mask + gaussian_renderer/render.py:120-197 prefilter_voxel fused:
                      one kernel (LoD test AND gsplat radius > 0) + an ordered compaction to the
                      visible-anchor index the decode consumes (`prefilter_voxel` is the drop-in)
* `decode`         <- scene/basic_model.py:297-371 generate_neural_gaussians on the
                      visible anchors, MLPs of scene/lod_model.py:67-84
* `generate_neural_gaussians(model, camera, visible_mask)` takes the reference model
  object itself and returns the same 8-tuple, so a maintainer can bind it in place of
  `BasicModel.generate_neural_gaussians`.

Supported: feat_dim 32, view_dim 0 or 3, appearance_dim 0, dist2level != 'progressive'
(smooth_complement = 1), RGB or SH colours; anything else raises NotImplementedError.
There is no CPU path: inputs must be HIP device tensors.
"""
from __future__ import annotations

import ctypes as ct
import math
import threading

import torch

from . import _native as N
from ._native import ptr

_HEADS = ("opacity", "cov", "color")


def _check_dev(*ts):
    for t in ts:
        if t is not None and not t.is_cuda:
            raise RuntimeError("hgsr: inputs must be HIP device tensors (no CPU fallback)")


def _f32(t):
    return t.contiguous() if t.dtype == torch.float32 else t.float().contiguous()


def _ptr_array(ts):
    arr = (ct.c_void_p * len(ts))(*[t.data_ptr() for t in ts])
    return arr, ct.cast(arr, ct.c_void_p)


@torch.no_grad()
def lod_mask(anchor, level, extra_level, cam_center, res_scale, standard_dist, fork, street_levels):
    """Boolean [A]: level <= clamp(floor(log2(sd/dist)/log2(fork) + extra_level), 0, street_levels-1)."""
    _check_dev(anchor, level, extra_level, cam_center)
    A = anchor.shape[0]
    mask = torch.empty(A, dtype=torch.uint8, device=anchor.device)
    # converted inputs held in locals until the launch is enqueued (no aliased temporaries)
    an, lv = _f32(anchor), level.reshape(-1).to(torch.int32).contiguous()
    el, cc = _f32(extra_level.reshape(-1)), _f32(cam_center.reshape(3))
    N.call("hgsr_lod_mask", A, ptr(an), ptr(lv), ptr(el), ptr(cc), float(res_scale), float(standard_dist),
           float(math.log2(fork)), int(street_levels) - 1, ptr(mask), N.stream(anchor.device))
    return mask.bool()


class VisibleIndex:
    """The visible-anchor index of prefilter(lazy=True) with its length still on the device:
    `buf` int32 [A] holds the ordered visible ids in its first Av entries, `counts` (device
    int64 [2]) holds Av in [1] and receives the decode's kept count in [0], so the decode reads
    both with ONE host sync instead of one each."""

    def __init__(self, buf, counts, visible):
        self.buf, self.counts, self.visible = buf, counts, visible


_pinned_dec = threading.local()


def _pinned_pair():
    buf = getattr(_pinned_dec, "buf", None)
    if buf is None:
        buf = _pinned_dec.buf = torch.empty(2, dtype=torch.int64, pin_memory=True)
    return buf


@torch.no_grad()
def prefilter(anchor, scales, quats, viewmat, K, width, height, lod=None, eps2d=0.3, near_plane=0.01,
              far_plane=1e10, lazy=False):
    """Fused set_anchor_mask + prefilter_voxel (scene/lod_model.py:286-290,
    gaussian_renderer/render.py:120-197): visible[a] = LoD test (lod = dict(level, extra_level,
    cam_center, res_scale, standard_dist, fork, street_levels), or None for all anchors) AND
    gsplat radius > 0 of the anchor projected with `scales` (activated, [A,3] or [A,6] of which
    the first three are used) and `quats`.  One kernel for the mask, then an ordered
    compaction: returns (visible bool [A], vis_idx int32 [Av]); one host read (Av).  With
    lazy=True the index is a VisibleIndex for decode() and there is no host read here."""
    _check_dev(anchor, scales, quats, viewmat, K)
    A = anchor.shape[0]
    dev = anchor.device
    vis = torch.empty(A, dtype=torch.uint8, device=dev)
    sc = scales if scales.dtype == torch.float32 and scales.stride(-1) == 1 and scales.stride(0) >= 3 else \
        scales.float().contiguous()
    stride = sc.stride(0)
    s = N.stream(dev)
    args = [None, None, None, 1.0, 1.0, 1.0, 0]
    keep = []
    if lod is not None:
        lv = lod["level"].reshape(-1).to(torch.int32).contiguous()
        el = _f32(lod["extra_level"].reshape(-1))
        cc = _f32(lod["cam_center"].reshape(3))
        keep = [lv, el, cc]
        args = [ptr(lv), ptr(el), ptr(cc), float(lod.get("res_scale", 1.0)), float(lod["standard_dist"]),
                float(math.log2(lod["fork"])), int(lod["street_levels"]) - 1]
    an, qs, vm, kk = _f32(anchor), _f32(quats), _f32(viewmat.reshape(4, 4)), _f32(K.reshape(3, 3))
    N.call("hgsr_anchor_prefilter", A, ptr(an), ptr(qs), sc.data_ptr(), stride, ptr(vm), ptr(kk), int(width),
           int(height), float(eps2d),
           float(near_plane), float(far_plane), *args, ptr(vis), s)
    ws_b = N.size_query("hgsr_explicit_ws_bytes", A)
    ws = torch.empty(max(ws_b, 1), dtype=torch.uint8, device=dev)
    counts = torch.empty(2, dtype=torch.int64, device=dev)  # [decode's kept count, Av]
    total = counts[1:]
    N.call("hgsr_explicit_count", A, None, None, None, None, 1.0, 1.0, 1.0, 0, ptr(vis), None, ptr(ws), ws_b,
           ptr(total), s)
    if lazy:
        buf = torch.empty(max(A, 1), dtype=torch.int32, device=dev)
        if A:
            N.call("hgsr_mask_index", A, ptr(vis), ptr(ws), ws_b, ptr(buf), s)
        del keep
        visible = vis.view(torch.bool)
        return visible, VisibleIndex(buf, counts, visible)
    Av = int(total.item())  # the one host read (the reference's boolean mask indexing syncs too)
    vis_idx = torch.empty(Av, dtype=torch.int32, device=dev)
    if Av:
        N.call("hgsr_mask_index", A, ptr(vis), ptr(ws), ws_b, ptr(vis_idx), s)
    del keep
    visible = vis.view(torch.bool)
    _VIS_CACHE[:] = [(visible, visible._version, vis_idx)]
    return visible, vis_idx


def prefilter_voxel(viewpoint_camera, pc):
    """Drop-in for reference prefilter_voxel (gaussian_renderer/render.py:120-197) for the 3DGS
    branch, with set_anchor_mask fused in (pc._anchor_mask is set as the reference does)."""
    if getattr(pc, "gs_attr", "3D") != "3D":
        raise NotImplementedError("hgsr prefilter: 3DGS branch only (2DGS uses fully_fused_projection_2dgs)")
    K = torch.tensor([[viewpoint_camera.fx, 0, viewpoint_camera.cx], [0, viewpoint_camera.fy, viewpoint_camera.cy],
                      [0, 0, 1]], dtype=torch.float32, device=pc.get_anchor.device)
    viewmat = viewpoint_camera.world_view_transform.transpose(0, 1)
    lod = dict(level=pc._level, extra_level=pc._extra_level, cam_center=viewpoint_camera.camera_center,
               res_scale=viewpoint_camera.resolution_scale, standard_dist=pc.standard_dist, fork=pc.fork,
               street_levels=pc.street_levels)
    pc._anchor_mask = lod_mask(pc.get_anchor, pc._level, pc._extra_level, viewpoint_camera.camera_center,
                               viewpoint_camera.resolution_scale, pc.standard_dist, pc.fork, pc.street_levels)
    visible, _ = prefilter(pc.get_anchor, pc.get_scaling, pc.get_rotation, viewmat, K,
                           int(viewpoint_camera.image_width), int(viewpoint_camera.image_height), lod=lod)
    return visible


_VIS_CACHE: list = []  # [(mask, its version counter, int32 index)]: one entry


def visible_index(visible):
    """int32 indices of a bool anchor mask (torch.nonzero: a host sync).  The last result is
    kept so that training_statis, which receives the same render_pkg["visible_mask"] after
    the backward (train.py:258-262), reuses it instead of syncing again."""
    if _VIS_CACHE and _VIS_CACHE[0][0] is visible and _VIS_CACHE[0][1] == visible._version:
        return _VIS_CACHE[0][2]
    idx = torch.nonzero(visible, as_tuple=False).reshape(-1).to(torch.int32)
    _VIS_CACHE[:] = [(visible, visible._version, idx)]
    return idx


class _Decode(torch.autograd.Function):
    @staticmethod
    def forward(ctx, anchor, feat, offset, scaling_raw, cam_center, vis_idx, cfg, *weights):
        view_dim, n_off, color_dim = cfg
        dev = anchor.device
        F = feat.shape[1]
        w = [_f32(t) for t in weights]
        arr, mlp = _ptr_array(w)
        s = N.stream(dev)
        if isinstance(vis_idx, VisibleIndex):
            # visible count still on the device: the count pass takes its upper bound A and
            # reads Av there; Av and the kept count come back with one host read
            vi = vis_idx
            cap = vi.buf.numel()
            ws_b = N.size_query("hgsr_decode_ws_bytes", cap)
            ws = torch.empty(ws_b, dtype=torch.uint8, device=dev)
            N.call("hgsr_decode_count", cap, F, view_dim, n_off, color_dim, ptr(vi.buf), ptr(anchor), ptr(feat),
                   ptr(cam_center), mlp, ptr(ws), ws_b, ptr(vi.counts), vi.counts.data_ptr() + 8, s)
            host = _pinned_pair()
            host.copy_(vi.counts, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(dev))
            ev.synchronize()
            M, Av = int(host[0]), int(host[1])
            vis_idx = vi.buf[:Av]
            _VIS_CACHE[:] = [(vi.visible, vi.visible._version, vis_idx)]
        else:
            Av = vis_idx.numel()
            ws_b = N.size_query("hgsr_decode_ws_bytes", Av)
            ws = torch.empty(ws_b, dtype=torch.uint8, device=dev)
            total = torch.empty(1, dtype=torch.int64, device=dev)
            N.call("hgsr_decode_count", Av, F, view_dim, n_off, color_dim, ptr(vis_idx), ptr(anchor), ptr(feat),
                   ptr(cam_center), mlp, ptr(ws), ws_b, ptr(total), None, s)
            M = int(total.item())  # the one host sync (the reference's boolean masking has it too)
        out = dict(xyz=(M, 3), offsets=(M, 3), color=(M, color_dim), opacity=(M, 1), scaling=(M, 3), rot=(M, 4))
        t = {k: torch.empty(v, dtype=torch.float32, device=dev) for k, v in out.items()}
        mask = torch.empty(Av * n_off, dtype=torch.uint8, device=dev)
        slot_row = torch.empty(Av * n_off, dtype=torch.int32, device=dev)
        N.call("hgsr_decode_fwd", Av, F, view_dim, n_off, color_dim, ptr(vis_idx), ptr(anchor), ptr(feat),
               ptr(offset), ptr(scaling_raw), ptr(cam_center), mlp, ptr(t["xyz"]), ptr(t["offsets"]),
               ptr(t["color"]), ptr(t["opacity"]), ptr(t["scaling"]), ptr(t["rot"]), ptr(mask), ptr(slot_row),
               ptr(ws), ws_b, s)
        del arr
        ctx.save_for_backward(anchor, feat, offset, scaling_raw, cam_center, vis_idx, slot_row, *w)
        ctx.cfg = cfg
        # the autograd inputs whose gradients are final after the backward's cov head (handed to
        # an early-gradient hook, set_early_grad_hook); weights[4:8] are the cov head's
        ctx.inputs = (offset, scaling_raw, *weights[4:8])
        sel = mask.view(torch.bool)  # 0/1 bytes: a view, no conversion kernel
        # the output row of every selected slot IS the exclusive cumsum of the selection mask:
        # training_statis takes it from here instead of recomputing it
        sel._hgsr_slot_row = slot_row
        ctx.mark_non_differentiable(sel)
        ctx.set_materialize_grads(False)  # unused outputs (mask, offsets) get no zero-filled grads
        return t["xyz"], t["offsets"], t["color"], t["opacity"], t["scaling"], t["rot"], sel

    @staticmethod
    def backward(ctx, g_xyz, g_offs, g_color, g_opac, g_scaling, g_rot, g_mask):
        anchor, feat, offset, scaling_raw, cam_center, vis_idx, slot_row, *w = ctx.saved_tensors
        view_dim, n_off, color_dim = ctx.cfg
        dev = anchor.device
        Av = vis_idx.numel()
        F = feat.shape[1]
        # every accumulated gradient carved from ONE zero-filled buffer (one fill launch, not 16)
        like = ([anchor] if ctx.needs_input_grad[0] else []) + [feat, offset, scaling_raw] + list(w)
        flat = torch.zeros(sum(t.numel() for t in like), dtype=torch.float32, device=dev)
        views, o = [], 0
        for t in like:
            views.append(flat[o:o + t.numel()].view(t.shape))
            o += t.numel()
        if not ctx.needs_input_grad[0]:
            views.insert(0, None)
        d_anchor, d_feat, d_offset, d_scaling, *d_w = views
        arr, mlp = _ptr_array(w)
        darr, dmlp = _ptr_array(d_w)
        ws_b = N.size_query("hgsr_decode_bwd_ws_bytes", Av)
        ws = torch.empty(max(ws_b, 1), dtype=torch.uint8, device=dev)
        g = [None if x is None else _f32(x) for x in (g_xyz, g_offs, g_color, g_opac, g_scaling, g_rot)]
        hook = _EARLY_GRAD[0]
        # with a data-parallel reducer attached: the cov head first (head_mask 2), whose end makes
        # d_offset, d_scaling and the cov weights final; their all-reduce is launched while the
        # opacity and colour heads run (head_mask 5).  Otherwise all heads in one call.
        for mask in ((2, 5) if hook is not None else (0,)):
            N.call("hgsr_decode_bwd", Av, F, view_dim, n_off, color_dim, ptr(vis_idx), ptr(anchor), ptr(feat),
                   ptr(offset), ptr(scaling_raw), ptr(cam_center), mlp, ptr(slot_row), *[ptr(x) for x in g],
                   ptr(d_anchor), ptr(d_feat), ptr(d_offset), ptr(d_scaling), dmlp, mask, ptr(ws), ws_b,
                   N.stream(dev))
            if mask == 2:
                src = ctx.inputs  # (offset, scaling_raw, the four cov-head tensors), the autograd inputs
                hook([(src[0], d_offset), (src[1], d_scaling)] + list(zip(src[2:], d_w[4:8])))
        del arr, darr
        return (d_anchor, d_feat, d_offset, d_scaling, None, None, None, *d_w)


_EARLY_GRAD = [None]


def set_early_grad_hook(fn):
    """fn([(input tensor, its final gradient), ...]) is called by the decode backward as soon as
    the listed gradients are final on the stream (before the rest of the backward is enqueued):
    multigpu.GradientAllReduce installs its early-reduction entry here for the duration of a
    data-parallel step.  None removes it."""
    _EARLY_GRAD[0] = fn


def decode(anchor, feat, offset, scaling_raw, cam_center, mlps, visible=None, view_dim=3, n_offsets=10,
           color_dim=3):
    """Fused generate_neural_gaussians on the visible anchors.

    mlps: (mlp_opacity, mlp_cov, mlp_color) nn.Sequentials, or a dict with
    '{opacity,cov,color}_{w1,b1,w2,b2}' tensors.  visible: bool mask [A] or int index
    tensor (None = all).  Returns (xyz, offsets, color, opacity, scaling, rot, mask)
    like the reference (colour [M, color_dim//3, 3] for SH)."""
    _check_dev(anchor, feat, offset, scaling_raw, cam_center)
    if isinstance(mlps, dict):
        weights = [mlps[f"{h}_{n}"] for h in _HEADS for n in ("w1", "b1", "w2", "b2")]
    else:
        weights = []
        for m in mlps:
            if len(m) < 3 or not isinstance(m[1], torch.nn.ReLU):
                raise NotImplementedError("hgsr decode: MLPs must be Linear -> ReLU -> Linear [-> Tanh]")
            weights += [m[0].weight, m[0].bias, m[2].weight, m[2].bias]
    A = anchor.shape[0]
    if visible is None:
        vis_idx = torch.arange(A, dtype=torch.int32, device=anchor.device)
    elif isinstance(visible, VisibleIndex):
        vis_idx = visible
    elif visible.dtype == torch.bool:
        vis_idx = visible_index(visible)
    else:
        vis_idx = visible.to(torch.int32).contiguous()
    xyz, offs, color, opac, scaling, rot, mask = _Decode.apply(
        _f32(anchor), _f32(feat), _f32(offset), _f32(scaling_raw), _f32(cam_center.reshape(3)), vis_idx,
        (int(view_dim), int(n_offsets), int(color_dim)), *weights)
    if color_dim != 3:
        color = color.reshape(color.shape[0], color_dim // 3, 3)
    return xyz, offs, color, opac, scaling, rot, mask


def generate_neural_gaussians(model, viewpoint_camera, visible_mask=None):
    """Drop-in for reference BasicModel.generate_neural_gaussians (scene/basic_model.py:297):
    returns (xyz, offsets, color, opacity, scaling, rot, active_sh_degree, mask)."""
    if getattr(model, "appearance_dim", 0) > 0:
        raise NotImplementedError("hgsr decode: appearance embeddings are not supported")
    if getattr(model, "dist2level", "floor") == "progressive":
        raise NotImplementedError("hgsr decode: dist2level='progressive' is not supported")
    if visible_mask is None:
        visible_mask = torch.ones(model.get_anchor.shape[0], dtype=torch.bool, device=model.get_anchor.device)
    xyz, offs, color, opac, scaling, rot, mask = decode(
        model.get_anchor, model.get_anchor_feat, model.get_offset, model._scaling,
        viewpoint_camera.camera_center, (model.get_opacity_mlp, model.get_cov_mlp, model.get_color_mlp),
        visible_mask, model.view_dim, model.n_offsets, model.color_dim)
    return xyz, offs, color, opac, scaling, rot, model.active_sh_degree, mask
