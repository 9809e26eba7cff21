"""Fused 3DGS parametrisation activations of a train step (csrc/activate.hip).

`activate(log_scales [N,3], logits [N]) -> (scales, opacities)`: exp and sigmoid in one HIP
pass forward and one backward, the activations the reference applies through its models'
scaling_activation (exp) and opacity_activation (sigmoid) before every render.  Matches
torch.exp / torch.sigmoid to float rounding (expf on the device).  No CPU path.
"""
from __future__ import annotations

import torch

from . import _native as N
from . import gradbuf
from ._native import ptr


class _Activate(torch.autograd.Function):
    @staticmethod
    def forward(ctx, log_scales, logits):
        n = log_scales.shape[0]
        scales = torch.empty_like(log_scales)
        opac = torch.empty_like(logits)
        N.call("hgsr_activate_fwd", n, ptr(log_scales), ptr(logits), ptr(scales), ptr(opac),
               N.stream(log_scales.device))
        ctx.save_for_backward(scales, opac)
        ctx.keys = (gradbuf.key(log_scales), gradbuf.key(logits))
        return scales, opac

    @staticmethod
    def backward(ctx, v_scales, v_opac):
        scales, opac = ctx.saved_tensors
        n = scales.shape[0]
        # in place in a DDP bucket when one is registered for the parameters (gradbuf)
        v_ls = gradbuf.alloc_key(ctx.keys[0], scales) if ctx.needs_input_grad[0] else None
        v_lg = gradbuf.alloc_key(ctx.keys[1], opac) if ctx.needs_input_grad[1] else None
        # contiguous copies held in locals until the launch is enqueued: a temporary freed
        # inside the call could hand its block to the next temporary (aliased inputs)
        vs = None if v_scales is None else v_scales.contiguous()
        vo = None if v_opac is None else v_opac.contiguous()
        N.call("hgsr_activate_bwd", n, ptr(scales), ptr(opac), ptr(vs), ptr(vo), ptr(v_ls), ptr(v_lg),
               N.stream(scales.device))
        return v_ls, v_lg


def activate(log_scales, logits):
    """(exp(log_scales), sigmoid(logits)) for log_scales [N,3], logits [N] (fp32 HIP tensors)."""
    if not (log_scales.is_cuda and logits.is_cuda):
        raise RuntimeError("hgsr: inputs must be HIP device tensors (no CPU fallback)")
    assert log_scales.dim() == 2 and log_scales.shape[1] == 3 and logits.shape == (log_scales.shape[0],)
    return _Activate.apply(log_scales.float().contiguous(), logits.float().contiguous())
