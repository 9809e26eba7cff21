"""torch.autograd wrappers of the C-oracle rasterization (TEST INFRASTRUCTURE ONLY).

Only tests/ may import this module.  They let a CPU training chain differentiate through
the oracle's gsplat restatement (oracle/pipeline.py: projection, SH, tile intersection +
sort, raster forward / hand-derived backward, checked against torch autograd in
tests/test_oracle.py) exactly like the reference differentiates through
gsplat.rasterization[_2dgs] at gaussian_renderer/render.py:40-76, so that the
reference-pinned stages around it (oracle/decode_ref.decode_torch, oracle/loss_ref.loss,
torch.optim.Adam) compose into one CPU train step (train.py:150-277).

Tensors are CPU float32 or float64; the oracle precision follows the tensor dtype.
"""
from __future__ import annotations

import numpy as np
import torch

from . import pipeline as OP


def _np(t, dt):
    return None if t is None else np.ascontiguousarray(t.detach().cpu().numpy(), dtype=dt)


class Raster3DFn(torch.autograd.Function):
    """(means, quats, scales, opacities [N], colors [N,3] | [N,K,3]) ->
    (render_colors [C,H,W,D], render_alphas [C,H,W,1]) through oracle Raster3D."""

    @staticmethod
    def forward(ctx, means, quats, scales, opacities, colors, cfg):
        dt = np.float64 if means.dtype == torch.float64 else np.float32
        r = OP.Raster3D(_np(means, dt), _np(quats, dt), _np(scales, dt), _np(opacities, dt), _np(colors, dt),
                        _np(cfg["viewmats"], dt), _np(cfg["Ks"], dt), cfg["W"], cfg["H"],
                        sh_degree=cfg.get("sh_degree"), backgrounds=_np(cfg.get("bg"), dt),
                        render_mode=cfg.get("mode", "RGB+ED"), dtype=dt)
        out, ra = r.forward()
        ctx.r = r
        ctx.shapes = [t.shape for t in (means, quats, scales, opacities, colors)]
        ctx.tdt = means.dtype
        cfg["last"] = r  # the caller may read the forward's intermediates (radii, isect ids)
        return torch.from_numpy(np.array(out)), torch.from_numpy(np.array(ra))

    @staticmethod
    def backward(ctx, v_rc, v_ra):
        g = ctx.r.backward(v_rc.numpy(), v_ra.numpy())
        outs = [torch.from_numpy(np.asarray(g[k])).to(ctx.tdt).reshape(s)
                for k, s in zip(("means", "quats", "scales", "opacities", "colors"), ctx.shapes)]
        return (*outs, None)


class Raster2DFn(torch.autograd.Function):
    """2DGS: (means, quats, scales, opacities, colors [N,3]) -> (render_colors [C,H,W,4],
    render_alphas [C,H,W,1]) through oracle Raster2D (RGB+ED / RGB+D); the rendered normals
    are not returned (the normal term starts at iteration 7000, config/base/*/fine.yaml)."""

    @staticmethod
    def forward(ctx, means, quats, scales, opacities, colors, cfg):
        dt = np.float64 if means.dtype == torch.float64 else np.float32
        r = OP.Raster2D(_np(means, dt), _np(quats, dt), _np(scales, dt), _np(opacities, dt), _np(colors, dt),
                        _np(cfg["viewmats"], dt), _np(cfg["Ks"], dt), cfg["W"], cfg["H"],
                        backgrounds=_np(cfg.get("bg"), dt), render_mode=cfg.get("mode", "RGB+ED"), dtype=dt,
                        hitform=cfg.get("hitform", 0))
        out, ra, rn = r.forward()
        ctx.r = r
        ctx.rn_shape = rn.shape
        ctx.shapes = [t.shape for t in (means, quats, scales, opacities, colors)]
        ctx.tdt = means.dtype
        cfg["last"] = r
        return torch.from_numpy(np.array(out)), torch.from_numpy(np.array(ra))

    @staticmethod
    def backward(ctx, v_rc, v_ra):
        dt = ctx.r.dt
        g = ctx.r.backward(v_rc.numpy(), v_ra.numpy(), np.zeros(ctx.rn_shape, dt))
        outs = [torch.from_numpy(np.asarray(g[k])).to(ctx.tdt).reshape(s)
                for k, s in zip(("means", "quats", "scales", "opacities", "colors"), ctx.shapes)]
        return (*outs, None)


def rasterization(means, quats, scales, opacities, colors, cfg, gs="3d"):
    fn = Raster3DFn if gs == "3d" else Raster2DFn
    return fn.apply(means, quats, scales, opacities, colors, cfg)
