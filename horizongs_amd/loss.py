"""Fused training loss on the MI355X, host side.

Replaces the loss head of reference train.py:153-202 (utils/loss_utils.py:17-60):
masked L1 + D-SSIM (11x11 Gaussian window, sigma 1.5), the scale regulariser, the
sky-opacity / opacity-entropy regularisers and the per-pixel normal-consistency,
distortion and inverse-depth L1 terms -- forward and backward in two HIP passes each
instead of five depthwise conv2d plus ~25 elementwise launches.  There is no CPU path.
"""
from __future__ import annotations

import ctypes as ct

import torch

from . import _native as N
from ._native import ptr

OUTPUTS = ("loss", "l1", "ssim", "sky", "entropy", "scale_reg", "normal", "distortion", "inv_depth")


class _Terms(ct.Structure):
    """include/hgsr.h hgsr_loss_terms"""
    _fields_ = [("lambda_dssim", ct.c_float), ("lambda_sky_opa", ct.c_float), ("lambda_entropy", ct.c_float),
                ("lambda_dreg", ct.c_float), ("lambda_normal", ct.c_float), ("lambda_dist", ct.c_float),
                ("lambda_depth", ct.c_float),
                ("normals", ct.c_void_p), ("normals_strides", ct.c_int64 * 3),
                ("normals_from_depth", ct.c_void_p), ("nfd_strides", ct.c_int64 * 3),
                ("distort", ct.c_void_p), ("distort_strides", ct.c_int64 * 2),
                ("depth", ct.c_void_p), ("depth_strides", ct.c_int64 * 2),
                ("mono_invdepth", ct.c_void_p), ("depth_mask", ct.c_void_p)]


class _AuxGrads(ct.Structure):
    """include/hgsr.h hgsr_loss_aux_grads"""
    _fields_ = [("g_normals", ct.c_void_p), ("g_normals_from_depth", ct.c_void_p), ("g_distort", ct.c_void_p),
                ("g_depth", ct.c_void_p)]


def _f32(t):
    return None if t is None else (t.contiguous() if t.dtype == torch.float32 else t.float().contiguous())


def _view(t, shape=None):
    """fp32 view the kernels can address: any non-negative strides are passed through (the
    channels-last render outputs seen through permute(2,0,1) need no copy)."""
    if t is None:
        return None
    if shape is not None:
        t = t.reshape(shape)
    if t.dtype != torch.float32:
        t = t.float()
    if any(st <= 0 and sz > 1 for st, sz in zip(t.stride(), t.shape)):  # negative or broadcast
        t = t.contiguous()
    return t


def _dptr(t):
    if t is None:
        return None
    if not t.is_cuda:
        raise RuntimeError("hgsr: tensor must live on the HIP device (no CPU path)")
    return t.data_ptr()


def _strides(t, n):
    return (ct.c_int64 * n)(*(t.stride() if t is not None else (0,) * n))


def _like(t):
    """empty gradient buffer with t's strides (the kernels write through them)"""
    g = torch.empty_like(t)
    if g.stride() != t.stride():
        g = torch.empty_strided(t.shape, t.stride(), dtype=t.dtype, device=t.device)
    return g


class _FusedLoss(torch.autograd.Function):
    @staticmethod
    def forward(ctx, image, gt, mask, alpha, scaling, normals, nfd, distort, depth, mono, dmask, lams):
        C, H, W = gt.shape
        dev = image.device
        ws_b = N.size_query("hgsr_loss_ws_bytes", C, H, W)
        ws = torch.empty(ws_b, dtype=torch.uint8, device=dev)
        out = torch.empty(len(OUTPUTS), dtype=torch.float32, device=dev)
        terms = _Terms(*lams, _dptr(normals), _strides(normals, 3), _dptr(nfd), _strides(nfd, 3), _dptr(distort),
                       _strides(distort, 2), _dptr(depth), _strides(depth, 2), ptr(mono), ptr(dmask))
        n_sc, k_sc = (0, 0) if scaling is None else scaling.shape
        N.call("hgsr_loss_fwd", C, H, W, _dptr(image), _strides(image, 3), _dptr(gt), _strides(gt, 3), ptr(mask),
               ptr(alpha), ptr(scaling), n_sc, k_sc, ct.byref(terms), ptr(out), ptr(ws), ws_b, N.stream(dev))
        ctx.save_for_backward(image, gt, mask, alpha, scaling, normals, nfd, distort, depth, mono, dmask, ws)
        ctx.lams = lams
        # the rasterizer's projection of these same scales takes this loss's scale-regulariser
        # gradient into its own backward kernel (gsplat_api.GradSink): no separate sum
        ctx.sink = None if scaling is None else getattr(scaling, "_hgsr_grad_sink", None)
        # nine separate 0-dim outputs: an output the caller never uses gets no gradient
        # tensor at all (None below), so the backward builds no zeros / stack glue
        ctx.set_materialize_grads(False)
        return tuple(out.unbind(0))

    @staticmethod
    def backward(ctx, *g_outs):
        image, gt, mask, alpha, scaling, normals, nfd, distort, depth, mono, dmask, ws = ctx.saved_tensors
        C, H, W = gt.shape
        dev = image.device
        need = ctx.needs_input_grad
        g_img = _like(image)
        g_alpha = torch.empty((H, W), dtype=torch.float32, device=dev) if (alpha is not None and need[3]) else None
        g_sc = torch.empty_like(scaling) if (scaling is not None and need[4]) else None
        g_n = _like(normals) if (normals is not None and need[5]) else None
        g_f = _like(nfd) if (nfd is not None and need[6]) else None
        g_d = _like(distort) if (distort is not None and need[7]) else None
        g_z = _like(depth) if (depth is not None and need[8]) else None
        terms = _Terms(*ctx.lams, _dptr(normals), _strides(normals, 3), _dptr(nfd), _strides(nfd, 3),
                       _dptr(distort), _strides(distort, 2), _dptr(depth), _strides(depth, 2), ptr(mono), ptr(dmask))
        aux = _AuxGrads(_dptr(g_n), _dptr(g_f), _dptr(g_d), _dptr(g_z))
        n_sc, k_sc = (0, 0) if scaling is None else scaling.shape
        gs = [None if g is None else _f32(g) for g in g_outs]
        gptrs = (ct.c_void_p * len(OUTPUTS))(*[None if g is None else g.data_ptr() for g in gs])
        N.call("hgsr_loss_bwd", C, H, W, _dptr(image), _strides(image, 3), _dptr(gt), _strides(gt, 3), ptr(mask),
               ptr(alpha), ptr(scaling), n_sc, k_sc, ct.byref(terms), gptrs, _dptr(g_img),
               image.shape[0] - C, ptr(g_alpha), ptr(g_sc), ct.byref(aux), ptr(ws), ws.numel(), N.stream(dev))
        if g_alpha is not None:
            g_alpha = g_alpha.reshape(alpha.shape)
        if g_sc is not None and ctx.sink is not None and ctx.sink.put(g_sc):
            g_sc = None  # handed to the projection backward, which adds it in its kernel
        return g_img, None, None, g_alpha, g_sc, g_n, g_f, g_d, g_z, None, None, None


def fused_loss(image, gt, alpha_mask=None, lambda_dssim=0.2, alpha=None, lambda_sky_opa=0.0,
               lambda_opacity_entropy=0.0, scaling=None, lambda_dreg=0.0, normals=None, normals_from_depth=None,
               lambda_normal=0.0, distort=None, lambda_dist=0.0, depth=None, mono_invdepth=None, depth_mask=None,
               lambda_depth=0.0):
    """The reference loss head (train.py:153-202) as 0-dim tensors
    (loss, l1, ssim, sky, entropy, scale_reg, normal, distortion, inv_depth), differentiable
    w.r.t. image, alpha, scaling, normals, normals_from_depth, distort and depth.

    image, gt: [3,H,W], any layout (e.g. render_colors[0].permute(2, 0, 1) as reference
    render.py:88 builds it, read in place).  image may carry trailing channels the loss
    ignores (the permuted render of an RGB+ED render): they get a zero gradient, so no slice
    (and no slice-backward fill) is needed.  alpha_mask, alpha, distort, depth,
    mono_invdepth, depth_mask: H*W elements ([H,W], [1,H,W], [H,W,1]); normals,
    normals_from_depth: [3,H,W] views (render.py's permuted [H,W,3] renders).
    scaling: [N,k] (train.py:163-167 scaling.prod(dim=1).mean(), 0 for N = 0).  The
    normal term uses alpha detached (train.py:183)."""
    if not image.is_cuda:
        raise RuntimeError("hgsr: inputs must be HIP device tensors (no CPU fallback)")
    H, W = image.shape[-2:]
    if image.dim() != 3 or gt.dim() != 3 or gt.shape[1:] != image.shape[1:] or gt.shape[0] > image.shape[0]:
        raise ValueError(f"hgsr fused_loss: image {tuple(image.shape)} vs gt {tuple(gt.shape)}")
    if scaling is not None and scaling.dim() != 2:
        raise ValueError(f"hgsr fused_loss: scaling must be [N,k], got {tuple(scaling.shape)}")
    if (normals is None) != (normals_from_depth is None):
        raise ValueError("hgsr fused_loss: the normal term needs normals and normals_from_depth")
    if (depth is None) != (mono_invdepth is None):
        raise ValueError("hgsr fused_loss: the depth term needs depth and mono_invdepth")
    hw = lambda t: None if t is None else _f32(t.reshape(H, W))
    lams = (float(lambda_dssim), float(lambda_sky_opa), float(lambda_opacity_entropy), float(lambda_dreg),
            float(lambda_normal), float(lambda_dist), float(lambda_depth))
    out = _FusedLoss.apply(_view(image), _view(gt).detach(), hw(alpha_mask), _f32(None if alpha is None else
                                                                                  alpha.reshape(H, W)),
                           _f32(scaling), _view(normals, (3, H, W)), _view(normals_from_depth, (3, H, W)),
                           _view(distort, (H, W)), _view(depth, (H, W)), hw(mono_invdepth), hw(depth_mask), lams)
    return out
