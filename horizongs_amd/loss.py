"""Fused training loss on the MI355X, host side.

Replaces the loss head of reference train.py:153-178 (utils/loss_utils.py:17-60):
masked L1 + D-SSIM (11x11 Gaussian window, sigma 1.5) and the sky-opacity / opacity-entropy
regularisers, forward and backward in two HIP passes each instead of five depthwise conv2d
plus ~15 elementwise launches.  There is no CPU path.
"""
from __future__ import annotations

import ctypes as ct

import torch

from . import _native as N
from ._native import ptr


def _f32(t):
    return None if t is None else (t.contiguous() if t.dtype == torch.float32 else t.float().contiguous())


def _img(t):
    """fp32 [C,H,W] view the kernels can address: any non-negative strides are passed
    through (the channels-last render output seen through permute(2,0,1) needs no copy)."""
    if t.dtype != torch.float32:
        t = t.float()
    if any(st <= 0 and sz > 1 for st, sz in zip(t.stride(), t.shape)):  # negative or broadcast
        t = t.contiguous()
    return t


def _strided(t):
    """(device pointer, host int64[3] strides) of an fp32 [C,H,W] HIP tensor."""
    if not t.is_cuda:
        raise RuntimeError("hgsr: tensor must live on the HIP device (no CPU path)")
    return t.data_ptr(), (ct.c_int64 * 3)(*t.stride())


class _FusedLoss(torch.autograd.Function):
    @staticmethod
    def forward(ctx, image, gt, mask, alpha, scaling, lam_dssim, lam_sky, lam_ent, lam_dreg):
        C, H, W = gt.shape
        dev = image.device
        ws_b = N.size_query("hgsr_loss_ws_bytes", C, H, W)
        ws = torch.empty(ws_b, dtype=torch.uint8, device=dev)
        out = torch.empty(6, dtype=torch.float32, device=dev)
        ip, ist = _strided(image)
        gp, gst = _strided(gt)
        n_sc, k_sc = (0, 0) if scaling is None else scaling.shape
        N.call("hgsr_loss_fwd", C, H, W, ip, ist, gp, gst, ptr(mask), ptr(alpha), ptr(scaling), n_sc, k_sc,
               float(lam_dssim), float(lam_sky), float(lam_ent), float(lam_dreg), ptr(out), ptr(ws), ws_b,
               N.stream(dev))
        ctx.save_for_backward(image, gt, mask, alpha, scaling, ws)
        ctx.lams = (lam_dssim, lam_sky, lam_ent, lam_dreg)
        return out

    @staticmethod
    def backward(ctx, g_out):
        image, gt, mask, alpha, scaling, ws = ctx.saved_tensors
        C, H, W = gt.shape
        dev = image.device
        g_img = torch.empty_like(image)  # same strides as image (dense): written through them
        if g_img.stride() != image.stride():
            g_img = torch.empty_strided(image.shape, image.stride(), dtype=image.dtype, device=dev)
        g_alpha = torch.empty((H, W), dtype=torch.float32, device=dev) if (
            alpha is not None and ctx.needs_input_grad[3]) else None
        g_sc = torch.empty_like(scaling) if (scaling is not None and ctx.needs_input_grad[4]) else None
        n_sc, k_sc = (0, 0) if scaling is None else scaling.shape
        ip, ist = _strided(image)
        gp, gst = _strided(gt)
        N.call("hgsr_loss_bwd", C, H, W, ip, ist, gp, gst, ptr(mask), ptr(alpha), ptr(scaling), n_sc, k_sc,
               *[float(x) for x in ctx.lams], ptr(_f32(g_out)), g_img.data_ptr(), image.shape[0] - C,
               ptr(g_alpha), ptr(g_sc), ptr(ws), ws.numel(), N.stream(dev))
        if g_alpha is not None:
            g_alpha = g_alpha.reshape(alpha.shape)
        return g_img, None, None, g_alpha, g_sc, None, None, None, None


def fused_loss(image, gt, alpha_mask=None, lambda_dssim=0.2, alpha=None, lambda_sky_opa=0.0,
               lambda_opacity_entropy=0.0, scaling=None, lambda_dreg=0.0):
    """(loss, l1, ssim, sky, entropy, scale_reg) as 0-dim tensors, differentiable w.r.t.
    image, alpha and scaling.

    image, gt: [3,H,W], any layout (e.g. render_colors[0].permute(2, 0, 1) as reference
    render.py:88 builds it, read in place).  image may carry trailing channels the loss
    ignores (the permuted render of an RGB+ED render): they get a zero gradient, so no slice
    (and no slice-backward fill) is needed.  alpha_mask, alpha: [H,W] or [1,H,W].
    scaling: [N,k] (train.py:163-167 scaling.prod(dim=1).mean(), 0 for N = 0)."""
    if not image.is_cuda:
        raise RuntimeError("hgsr: inputs must be HIP device tensors (no CPU fallback)")
    H, W = image.shape[-2:]
    if image.dim() != 3 or gt.dim() != 3 or gt.shape[1:] != image.shape[1:] or gt.shape[0] > image.shape[0]:
        raise ValueError(f"hgsr fused_loss: image {tuple(image.shape)} vs gt {tuple(gt.shape)}")
    if scaling is not None and scaling.dim() != 2:
        raise ValueError(f"hgsr fused_loss: scaling must be [N,k], got {tuple(scaling.shape)}")
    mask = None if alpha_mask is None else _f32(alpha_mask.reshape(H, W).float())
    a = None if alpha is None else alpha.reshape(H, W)
    out = _FusedLoss.apply(_img(image), _img(gt).detach(), mask, _f32(a), _f32(scaling), float(lambda_dssim),
                           float(lambda_sky_opa), float(lambda_opacity_entropy), float(lambda_dreg))
    return tuple(out.unbind(0))
