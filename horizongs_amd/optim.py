"""Drop-in for the reference optimizer: torch.optim.Adam(l, lr=0.0, eps=1e-15)
(scene/lod_model.py:320, stepped at train.py:274-277), stepped by ONE fused HIP launch
over every parameter (hgsr_adam_step, csrc/optim.hip) instead of torch's per-op
foreach kernels.

Same constructor, parameter groups, per-group "lr" (the reference rewrites it every
iteration in update_learning_rate, scene/lod_model.py:350-372) and the same per-parameter
state keys ("step" as a CPU float tensor, "exp_avg", "exp_avg_sq"), so the reference's
optimizer surgery (_prune_anchor_optimizer / cat_tensors_to_optimizer,
scene/lod_model.py:466-486,598-617, which read and replace state["exp_avg"] /
state["exp_avg_sq"] and group["params"][0]) and state_dict() / load_state_dict() work
unchanged.  amsgrad / weight_decay / maximize / capturable are not used by the reference
and raise.  No CPU path: parameters must live on the HIP device.
"""
from __future__ import annotations

import ctypes as ct

import torch

from . import _native as NAT


class _AdamTensor(ct.Structure):
    _fields_ = [("param", ct.c_void_p), ("grad", ct.c_void_p), ("exp_avg", ct.c_void_p),
                ("exp_avg_sq", ct.c_void_p), ("numel", ct.c_int64), ("lr", ct.c_double), ("step", ct.c_int64)]


class Adam(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0, amsgrad=False, *,
                 maximize=False, foreach=None, capturable=False, differentiable=False, fused=None):
        if weight_decay != 0 or amsgrad or maximize or capturable or differentiable:
            raise NotImplementedError("hgsr Adam: weight_decay / amsgrad / maximize / capturable / differentiable "
                                      "are not used by Horizon-GS and not offered")
        if not 0.0 <= lr:
            raise ValueError(f"Invalid learning rate: {lr}")
        if not 0.0 <= eps:
            raise ValueError(f"Invalid epsilon value: {eps}")
        if not 0.0 <= betas[0] < 1.0:
            raise ValueError(f"Invalid beta parameter at index 0: {betas[0]}")
        if not 0.0 <= betas[1] < 1.0:
            raise ValueError(f"Invalid beta parameter at index 1: {betas[1]}")
        defaults = dict(lr=lr, betas=betas, eps=eps, weight_decay=0, amsgrad=False, maximize=False,
                        foreach=None, capturable=False, differentiable=False, fused=None)
        super().__init__(params, defaults)

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        # one launch per distinct (betas, eps); the reference has a single setting
        batches: dict = {}
        keep = []
        for group in self.param_groups:
            b1, b2 = group["betas"]
            descs = batches.setdefault((float(b1), float(b2), float(group["eps"])), [])
            for p in group["params"]:
                if p.grad is None:
                    continue
                if p.grad.is_sparse:
                    raise RuntimeError("hgsr Adam does not support sparse gradients")
                if p.dtype != torch.float32 or p.grad.dtype != torch.float32:
                    raise RuntimeError("hgsr Adam: float32 parameters only")
                st = self.state[p]
                if len(st) == 0:
                    st["step"] = torch.tensor(0.0, dtype=torch.float32)
                    st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                    st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                g = p.grad if p.grad.is_contiguous() else p.grad.contiguous()
                for t in (p, st["exp_avg"], st["exp_avg_sq"]):
                    if not t.is_contiguous():
                        raise RuntimeError("hgsr Adam: parameters and state must be contiguous")
                st["step"] += 1
                keep.append(g)
                descs.append(_AdamTensor(NAT.ptr(p), NAT.ptr(g), NAT.ptr(st["exp_avg"]), NAT.ptr(st["exp_avg_sq"]),
                                         p.numel(), float(group["lr"]), int(st["step"].item())))
        for (b1, b2, eps), descs in batches.items():
            if not descs:
                continue
            arr = (_AdamTensor * len(descs))(*descs)
            dev = keep[0].device
            NAT.call("hgsr_adam_step", len(descs), ct.cast(arr, ct.c_void_p), b1, b2, eps, NAT.stream(dev))
        return loss
