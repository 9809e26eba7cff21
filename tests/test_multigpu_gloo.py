"""world_size-2 gloo tests (CPU) of the multi-GPU mapping: chunk dealing, bucketed
gradient averaging (DDP over views) and densify-statistic reduction."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from horizongs_amd.multigpu import GradientAllReduce, chunks_for_rank, reduce_densify_stats


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.manual_seed(rank)
        a = torch.nn.Parameter(torch.zeros(1000, 3))
        b = torch.nn.Parameter(torch.zeros(37))
        c = torch.nn.Parameter(torch.zeros(5))  # no grad on rank 1
        a.grad = torch.full_like(a, float(rank + 1))
        b.grad = torch.arange(37, dtype=torch.float32) * (rank + 1)
        if rank == 0:
            c.grad = torch.ones(5) * 4.0
        GradientAllReduce([a, b, c], bucket_mb=0.005)()
        stats = {"offset_gradient_accum": torch.full((4,), float(rank + 1)),
                 "max_radii2D": torch.tensor([float(rank), 10.0 - rank, 3.0, 0.0])}
        reduce_densify_stats(stats)
        q.put((rank, a.grad[0, 0].item(), b.grad[5].item(), c.grad[0].item(),
               stats["offset_gradient_accum"].tolist(), stats["max_radii2D"].tolist()))
    finally:
        dist.destroy_process_group()


def test_ddp_gradient_and_stat_reduction():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, ga, gb, gc, acc, mx in res:
        assert ga == pytest.approx(1.5)          # mean of 1 and 2
        assert gb == pytest.approx(5 * 1.5)
        assert gc == pytest.approx(2.0)          # (4 + 0) / 2: missing grads count as zeros
        assert acc == [3.0] * 4                  # sum
        assert mx == [1.0, 10.0, 3.0, 0.0]       # max


def test_chunks_dealt_once():
    chunks = [f"{m}_{n}" for m in range(4) for n in range(2)]  # Block_A 4x2
    for world in (1, 2, 3, 8):
        dealt = [c for r in range(world) for c in chunks_for_rank(chunks, r, world)]
        assert sorted(dealt) == sorted(chunks)
    assert chunks_for_rank(chunks, 3, 8) == ["1_1"]
