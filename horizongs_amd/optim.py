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
    def step_params(self, params):
        """Step only `params` (a subset of the groups' parameters, e.g. one all-reduce bucket:
        multigpu.GradientAllReduce.finish(step=...)).  Adam is elementwise: stepping the
        parameters in several subsets is bit-identical to one step over all of them."""
        self.step(only={id(p) for p in params})

    @torch.no_grad()
    def step(self, closure=None, only=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        # one launch per distinct (betas, eps); the reference has a single setting.  The host
        # side is kept lean (it runs while the GPU drains the backward): the per-parameter
        # step tensors are bumped with one foreach call.
        batches: dict = {}
        keep = []
        work = []
        for group in self.param_groups:
            b1, b2 = group["betas"]
            key = (float(b1), float(b2), float(group["eps"]))
            lr = float(group["lr"])
            for p in group["params"]:
                g = p.grad
                if g is None or (only is not None and id(p) not in only):
                    continue
                if g.is_sparse:
                    raise RuntimeError("hgsr Adam does not support sparse gradients")
                if p.dtype != torch.float32 or g.dtype != torch.float32:
                    raise RuntimeError("hgsr Adam: float32 parameters only")
                if not (p.is_cuda and g.is_cuda):
                    raise RuntimeError("hgsr Adam: tensors must live on the HIP device (no CPU path)")
                st = self.state[p]
                if len(st) == 0:
                    st["step"] = torch.tensor(0.0, dtype=torch.float32)
                    st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                    st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                if not g.is_contiguous():
                    g = g.contiguous()
                m, v = st["exp_avg"], st["exp_avg_sq"]
                if not (p.is_contiguous() and m.is_contiguous() and v.is_contiguous()):
                    raise RuntimeError("hgsr Adam: parameters and state must be contiguous")
                keep.append(g)
                work.append((key, p, g, m, v, lr, st["step"]))
        if not work:
            return loss
        steps = [w[6] for w in work]
        torch._foreach_add_(steps, 1.0)
        for (key, p, g, m, v, lr, step), n in zip(work, torch.stack(steps).tolist()):
            batches.setdefault(key, []).append(
                _AdamTensor(p.data_ptr(), g.data_ptr(), m.data_ptr(), v.data_ptr(), p.numel(), lr, int(n)))
        for (b1, b2, eps), descs in batches.items():
            if not descs:
                continue
            arr = (_AdamTensor * len(descs))(*descs)
            dev = keep[0].device
            NAT.call("hgsr_adam_step", len(descs), ct.cast(arr, ct.c_void_p), b1, b2, eps, NAT.stream(dev))
        return loss
