"""Gradient destinations: the kernel that produces a leaf's gradient writes it in place.

multigpu.ShardedAdamDDP keeps each bucket's gradients in one flat buffer that it
reduce-scatters.  Without a destination, autograd hands the hook a fresh gradient tensor and
the hook copies it into the flat buffer (the c2 DDP step's means / quats / log-scales /
opacity logits: 88 MB read + written per step).  With one, the backward that
produces the gradient (the projection backward for means and quats, the activation backward
for the log-scales and opacity logits) takes its output buffer from here -- a view of the
flat buffer, shaped like the parameter -- and autograd's AccumulateGrad, which adopts a
freshly produced gradient of the parameter's layout as `.grad` without copying, leaves it
there.  The hook then finds the gradient already in place.

A destination is taken at most once (`alloc` pops it): a second use of the same parameter in
one graph gets a fresh tensor, and autograd accumulates it into the first in place.  Keys are
(data pointer, numel) of the parameter's storage, so any tensor aliasing the parameter's data
exactly (`p`, `p.detach()`, `p.contiguous()` of a contiguous p) finds it."""
from __future__ import annotations

import torch

_DEST = {}


def set_dest(p: torch.Tensor, dest: torch.Tensor) -> None:
    """The next gradient produced for `p` (by a backward that consults this table) is written
    into `dest` (same shape and dtype as p, contiguous)."""
    if dest.shape != p.shape or dest.dtype != p.dtype or not dest.is_contiguous():
        raise ValueError("hgsr gradbuf: a destination must be a contiguous tensor shaped like its parameter")
    _DEST[(p.data_ptr(), p.numel())] = dest


def clear() -> None:
    _DEST.clear()


def key(t: torch.Tensor):
    """The lookup key of `t`'s data (for a backward that keeps only its outputs: take the key
    in the forward, look it up with alloc_key in the backward)."""
    return (t.data_ptr(), t.numel())


def alloc_key(k, like: torch.Tensor) -> torch.Tensor:
    """The output buffer for a gradient shaped like `like` of the tensor whose key is `k`: its
    registered destination (taken), or a fresh torch.empty_like."""
    d = _DEST.pop(k, None)
    if d is not None and d.shape == like.shape and d.dtype == like.dtype:
        return d
    return torch.empty_like(like)


def alloc(like: torch.Tensor) -> torch.Tensor:
    """The output buffer for the gradient of `like` itself."""
    return alloc_key(key(like), like)
