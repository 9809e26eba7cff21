"""Multi-GPU mapping of the rasterizer path.

Two ways the path shards, one process per GPU (torch.distributed; backend "nccl"
is RCCL over xGMI on MI355X):

1. per-chunk (no collectives): the reference splits a large scene into m x n
   chunks (preprocess/generate_chunks_config.py:50-104) trained independently and
   joined only by merge.py (merge.py:132-217).  `chunks_for_rank` deals chunk
   configs to ranks; each rank trains its chunks alone.
2. data-parallel over views: every rank renders a different camera of one scene;
   after backward the Gaussian/anchor gradients are averaged with bucketed
   all-reduces (`GradientAllReduce`) and the densification statistics are
   reduced only at densify steps (`reduce_densify_stats`: sums, and max for the
   max-mode fields, reference scene/basic_model.py:96-144).
"""
from __future__ import annotations

from typing import Dict, Iterable, List, Sequence

import torch
import torch.distributed as dist


def chunks_for_rank(chunks: Sequence[str], rank: int, world: int) -> List[str]:
    """Round-robin deal of chunk ids (e.g. '0_0'..'3_1' for Block_A) to ranks."""
    if world < 1 or not (0 <= rank < world):
        raise ValueError(f"bad rank/world {rank}/{world}")
    return [c for i, c in enumerate(chunks) if i % world == rank]


class GradientAllReduce:
    """Bucketed gradient averaging across ranks.

    Gradients are packed into flat fp32 buckets of ~`bucket_mb` MiB (few, large
    collectives: xGMI rings are per-link bound, so fewer calls of larger
    messages amortise the latency), all-reduced asynchronously, then unpacked.
    Parameters without a gradient contribute zeros (a Gaussian may be invisible
    from a rank's view)."""

    def __init__(self, params: Iterable[torch.nn.Parameter], bucket_mb: float = 64.0, group=None):
        self.params = [p for p in params if p.requires_grad]
        self.group = group
        cap = int(bucket_mb * (1 << 20) // 4)
        self.buckets: List[List[torch.nn.Parameter]] = []
        cur, size = [], 0
        for p in self.params:
            n = p.numel()
            if cur and size + n > cap:
                self.buckets.append(cur)
                cur, size = [], 0
            cur.append(p)
            size += n
        if cur:
            self.buckets.append(cur)

    def __call__(self) -> None:
        if not dist.is_initialized() or dist.get_world_size() == 1:
            return
        world = dist.get_world_size(self.group)
        work = []
        for bucket in self.buckets:
            flat = torch.cat([(p.grad if p.grad is not None else torch.zeros_like(p)).reshape(-1)
                              for p in bucket])
            h = dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=self.group, async_op=True)
            work.append((h, flat, bucket))
        for h, flat, bucket in work:
            h.wait()
            flat.div_(world)
            off = 0
            for p in bucket:
                n = p.numel()
                g = flat[off:off + n].view_as(p)
                if p.grad is None:
                    p.grad = g.clone()
                else:
                    p.grad.copy_(g)
                off += n


MAX_FIELDS = ("max_radii2D",)


def reduce_densify_stats(stats: Dict[str, torch.Tensor], max_fields: Sequence[str] = MAX_FIELDS,
                         group=None) -> Dict[str, torch.Tensor]:
    """In-place cross-rank reduction of densification accumulators at a densify step:
    sums for the accumulators/denominators, max for the max-mode fields (and for
    offset_gradient_accum when growing_type == 'max', pass it in max_fields)."""
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return stats
    for k in sorted(stats):
        op = dist.ReduceOp.MAX if k in max_fields else dist.ReduceOp.SUM
        dist.all_reduce(stats[k], op=op, group=group)
    return stats
