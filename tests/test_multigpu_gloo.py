"""world_size-2 gloo tests (CPU) of the multi-GPU mapping: chunk dealing, bucketed
gradient averaging (DDP over views) and densify-statistic reduction."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from horizongs_amd.multigpu import (GradientAllReduce, assert_replicas_agree, chunks_for_rank, reduce_densify_stats,
                                    replica_digest)


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


def _digest_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        g = torch.Generator().manual_seed(7)  # the same anchors on every rank
        anchors = [torch.randn(1001, 3, generator=g), torch.randn(1001, 32, generator=g), torch.randn(13, generator=g)]
        same = assert_replicas_agree(anchors)
        bad = [t.clone() for t in anchors]
        if rank == 1:  # one bit of one value on one rank
            bad[1].view(torch.int32)[500, 7] ^= 1
        try:
            assert_replicas_agree(bad, what="anchors")
            raised = False
        except RuntimeError as e:
            raised = "anchors" in str(e)
        q.put((rank, same, raised))
    finally:
        dist.destroy_process_group()


def test_replicas_agree_digest():
    """After a densify step every rank runs anchor_growing / prune on the same reduced
    statistics: the digest check passes for identical replicas and raises on
    every rank when one bit differs on one rank."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_digest_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res[0][1] == res[1][1]
    assert all(r[2] for r in res)
    # order- and shape-sensitive
    a, b = torch.arange(12.0), torch.arange(12.0).flip(0)
    assert int(replica_digest([a])) != int(replica_digest([b]))
    assert int(replica_digest([a.reshape(3, 4)])) != int(replica_digest([a.reshape(4, 3)]))
    assert int(replica_digest([a, b])) != int(replica_digest([b, a]))


def test_chunks_dealt_once():
    chunks = [f"{m}_{n}" for m in range(4) for n in range(2)]  # Block_A 4x2
    for world in (1, 2, 3, 8):
        dealt = [c for r in range(world) for c in chunks_for_rank(chunks, r, world)]
        assert sorted(dealt) == sorted(chunks)
    assert chunks_for_rank(chunks, 3, 8) == ["1_1"]


# ---------------------------------------------------------------------------------------
# DDP over views: 2 ranks x 1 view == 1 rank x 2 views (averaged), across densification
# ---------------------------------------------------------------------------------------
def _make_params():
    g = torch.Generator().manual_seed(0)
    a = torch.nn.Parameter(torch.randn(300, 3, generator=g))   # every view
    b = torch.nn.Parameter(torch.randn(50, generator=g))        # every view
    c = torch.nn.Parameter(torch.randn(7, 2, generator=g))      # view 0 only
    d = torch.nn.Parameter(torch.randn(5, generator=g))         # no view: grad stays None
    return [a, b, c, d]


def _view_loss(params, view):
    """CPU stand-in for render + loss of one camera view (reference train.py:150-206)."""
    a, b, c, _ = params
    w = torch.linspace(0.5, 1.5, a.numel()).reshape(a.shape) * (view + 1)
    loss = (torch.sin(a * w) ** 2).sum() + ((b * (view + 1)) ** 2).sum()
    if view == 0:
        loss = loss + (c ** 3).sum()
    return loss


def _optimizer(params):
    return torch.optim.Adam([{"params": [p], "lr": 0.01, "name": str(i)} for i, p in enumerate(params)], eps=1e-15)


def _grow(opt, params):
    """cat_tensors_to_optimizer (reference scene/basic_model.py): every group's Parameter is
    replaced by a longer one with zero-extended Adam state -- the reducer must follow."""
    new = []
    for gidx, (group, p) in enumerate(zip(opt.param_groups, params)):
        ext = torch.full((2,) + tuple(p.shape[1:]), 0.25 * (gidx + 1))
        q = torch.nn.Parameter(torch.cat([p.detach(), ext], 0))
        st = opt.state.pop(p, None)
        if st:
            st["exp_avg"] = torch.cat([st["exp_avg"], torch.zeros_like(ext)], 0)
            st["exp_avg_sq"] = torch.cat([st["exp_avg_sq"], torch.zeros_like(ext)], 0)
            opt.state[q] = st
        group["params"][0] = q
        new.append(q)
    return new


def _train(n_steps, views_per_step, reduce_fn=None, reducer=None):
    params = _make_params()
    opt = _optimizer(params)
    grads = []
    for step in range(n_steps):
        if step == 1:
            params = _grow(opt, params)
        opt.zero_grad(set_to_none=True)
        if reducer is not None:
            reducer.begin()
        loss = sum(_view_loss(params, v) for v in views_per_step) / len(views_per_step)
        loss.backward()
        if reducer is not None:
            reducer.finish()
        grads.append([None if p.grad is None else p.grad.clone() for p in params])
        opt.step()
    return grads, [p.detach().clone() for p in params]


def _step_subset(opt, subset, log):
    """Per-bucket optimizer step on the CPU (stand-in for optim.Adam.step_params, whose HIP
    kernel needs a device): torch's Adam skips parameters without a gradient."""
    ids = {id(p) for p in subset}
    log.append(sorted(ids))
    stash = []
    for g in opt.param_groups:
        for p in g["params"]:
            if id(p) not in ids and p.grad is not None:
                stash.append((p, p.grad))
                p.grad = None
    opt.step()
    for p, gr in stash:
        p.grad = gr


def _ddp_worker(rank, world, port, q, per_bucket=False):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        params = _make_params()
        opt = _optimizer(params)
        red = GradientAllReduce(opt, bucket_mb=0.0012)  # ~300 floats: several buckets
        grads, calls = [], []
        for step in range(3):
            if step == 1:
                params = _grow(opt, params)
            opt.zero_grad(set_to_none=True)
            red.begin()
            _view_loss(params, rank).backward()  # one view per rank, gradients averaged by the hooks
            if per_bucket:  # each bucket's parameters stepped right after its own collective
                log = []
                red.finish(step=lambda ps: _step_subset(opt, ps, log))
                calls.append((len(log), sorted(i for ids in log for i in ids) == sorted(id(p) for p in params)))
                grads.append([None if p.grad is None else p.grad.clone() for p in params])
            else:
                red.finish()
                grads.append([None if p.grad is None else p.grad.clone() for p in params])
                opt.step()
        # exactly one backward between begin() and finish(): a second one raises
        red.begin()
        _view_loss(params, rank).backward(retain_graph=True)
        err = None
        try:
            _view_loss(params, rank).backward()
        except RuntimeError as e:
            err = str(e)
        red.finish()
        npy = lambda t: None if t is None else t.detach().numpy().copy()  # noqa: E731
        q.put((rank, [[npy(g) for g in gs] for gs in grads], [npy(p) for p in params], len(red.buckets), calls, err))
    finally:
        dist.destroy_process_group()


def _run_ddp(per_bucket):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_ddp_worker, args=(r, world, port, q, per_bucket)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=180) for _ in range(world)], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return res


def test_ddp_per_bucket_step_equals_one_step():
    """finish(step=...) steps each bucket as its collective lands (the optimizer overlapping
    the remaining all-reduces): every parameter once per step, bit-identical parameters to
    finish() + one optimizer step; a second backward before finish() raises."""
    one, per = _run_ddp(False), _run_ddp(True)
    for (r1, g1, p1, nb, _, err1), (r2, g2, p2, _, calls, err2) in zip(one, per):
        assert nb >= 2 and all(n == nb and full for n, full in calls), calls
        for a, b in zip(p1, p2):
            assert (a == b).all(), r1  # bit for bit
        assert err1 and err2 and "exactly one backward" in err1


def test_ddp_two_ranks_match_one_rank_two_views():
    res = _run_ddp(False)
    ref_grads, ref_params = _train(3, [0, 1])
    for rank, grads, params, n_buckets, _, _ in res:
        assert n_buckets >= 2
        for step, (gs, rs) in enumerate(zip(grads, ref_grads)):
            for k, (g, r) in enumerate(zip(gs, rs)):
                if r is None:
                    assert g is None, (rank, step, k)  # no rank produced one: stays None (Adam skips it)
                else:
                    torch.testing.assert_close(torch.from_numpy(g), r, rtol=1e-6, atol=1e-7,
                                               msg=f"rank {rank} step {step} p{k}")
        for p, r in zip(params, ref_params):
            torch.testing.assert_close(torch.from_numpy(p), r, rtol=1e-6, atol=1e-7)


# ---------------------------------------------------------------------------------------
# the synchronous form red() across steps, and bucket identity across ranks after a densify
# ---------------------------------------------------------------------------------------
def _sync_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        params = _make_params()
        opt = _optimizer(params)
        red = GradientAllReduce(opt, bucket_mb=0.0012)
        grads, layouts, flats = [], [], []
        for step in range(3):
            if step == 2:
                params = _grow(opt, params)  # densification replaces every Parameter
            opt.zero_grad(set_to_none=True)
            # the hooks registered by the previous red() stay in place: this backward must
            # leave the gradients alone (they are reduced by the synchronous call below)
            _view_loss(params, rank).backward()
            red()
            grads.append([None if p.grad is None else p.grad.detach().numpy().copy() for p in params])
            layouts.append([[tuple(p.shape) for p in b["params"]] for b in red.buckets])
            flats.append([b["flat"].detach().numpy().copy() for b in red.buckets])
            opt.step()
        q.put((rank, grads, layouts, flats))
    finally:
        dist.destroy_process_group()


def test_sync_reduce_across_steps_and_bucket_identity():
    """red() (begin-less synchronous form) works step after step with its hooks left
    registered (a plain backward between steps does not raise), gives the 2-view mean every
    step, and after a densify both ranks hold the same bucket layout and reduced contents."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_sync_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=180) for _ in range(world)], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (_, g0, l0, f0), (_, g1, l1, f1) = res
    assert l0 == l1 and len(l0[-1]) >= 2  # same buckets, same order, after the growth too
    for a, b in zip(f0, f1):
        for x, y in zip(a, b):
            assert (x == y).all()  # identical reduced bucket contents on both ranks
    params = _make_params()
    opt = _optimizer(params)
    for step in range(3):  # one process, both views averaged
        if step == 2:
            params = _grow(opt, params)
        opt.zero_grad(set_to_none=True)
        (sum(_view_loss(params, v) for v in (0, 1)) / 2).backward()
        for k, p in enumerate(params):
            if p.grad is None:
                assert g0[step][k] is None and g1[step][k] is None
            else:
                torch.testing.assert_close(torch.from_numpy(g0[step][k]), p.grad, rtol=1e-6, atol=1e-7)
        opt.step()


# ---------------------------------------------------------------------------------------
# early gradients (the decode backward's cov head hands over _offset / _scaling / cov MLP
# gradients before the backward ends) and the bucket order that launches them first
# ---------------------------------------------------------------------------------------
class _EarlyStandIn(torch.autograd.Function):
    """CPU stand-in of the decode backward's hand-off: the identity on b whose backward passes
    the gradient it returns to the early hook first (decode.py _Decode.backward, head_mask 2),
    while the rest of the backward has not run yet."""

    @staticmethod
    def forward(ctx, b, red):
        ctx.b, ctx.red = b, red
        return b.view_as(b)

    @staticmethod
    def backward(ctx, g):
        from horizongs_amd import decode as HD
        gb = g.clone()
        HD._EARLY_GRAD[0]([(ctx.b, gb)])
        first = ctx.red.buckets[0]
        _EarlyStandIn.launched = first["launched"] and [id(p) for p in first["params"]] == [id(ctx.b)]
        return gb, None


def _early_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from horizongs_amd import decode as HD
        params = _make_params()
        a, b, c, d = params
        opt = _optimizer(params)
        red = GradientAllReduce(opt, bucket_mb=0.00005, order=[b])  # one parameter per bucket, b first
        out = []
        for step in range(2):
            opt.zero_grad(set_to_none=True)
            red.begin()
            assert HD._EARLY_GRAD[0] is not None  # installed for the step
            # b reaches the loss only through the stand-in, whose backward runs before a's
            _EarlyStandIn.launched = None
            loss = _view_loss([a, _EarlyStandIn.apply(b, red), c, d], rank)
            loss.backward()
            red.finish()
            assert HD._EARLY_GRAD[0] is None  # removed after the step
            out.append((_EarlyStandIn.launched,
                        [None if p.grad is None else p.grad.detach().numpy().copy() for p in params]))
            opt.step()
        # a second consumer of b besides the hand-off: autograd sums a new gradient, which the
        # early collective never saw -- refused
        opt.zero_grad(set_to_none=True)
        red.begin()
        err = None
        try:
            (_view_loss([a, _EarlyStandIn.apply(b, red), c, d], rank) + (3 * b).sum()).backward()
        except RuntimeError as e:
            err = str(e)
        red.finish()
        q.put((rank, out, err))
    finally:
        dist.destroy_process_group()


def test_early_gradients_launch_first_and_match():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_early_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=180) for _ in range(world)], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    params = _make_params()  # one process, both views averaged, no densification
    opt = _optimizer(params)
    ref_grads = []
    for _ in range(2):
        opt.zero_grad(set_to_none=True)
        (sum(_view_loss(params, v) for v in (0, 1)) / 2).backward()
        ref_grads.append([None if p.grad is None else p.grad.clone() for p in params])
        opt.step()
    for rank, out, err in res:
        assert err and "handed over early" in err, err
        for step, (launched_early, grads) in enumerate(out):
            assert launched_early, (rank, step)  # the early bucket's collective was in flight before backward
            for g, r in zip(grads, ref_grads[step]):
                if r is None:
                    assert g is None
                else:
                    torch.testing.assert_close(torch.from_numpy(g), r, rtol=1e-6, atol=1e-7)


# ---------------------------------------------------------------------------------------
# the sharded optimizer (ZeRO-1): reduce-scatter -> Adam on each rank's shard -> all-gather
# ---------------------------------------------------------------------------------------
def _cpu_adam(descs, betas, eps, device):
    """CPU restatement of the fused HIP Adam on segments: torch's single-tensor Adam order
    (lerp, mul + addcmul, sqrt / sqrt(bc2) + eps, addcdiv; torch/optim/adam.py)."""
    import math
    b1, b2 = betas
    for p, g, m, v, lr, step in descs:
        m.lerp_(g, 1 - b1)
        v.mul_(b2).addcmul_(g, g, value=1 - b2)
        bc1, bc2 = 1 - b1 ** step, 1 - b2 ** step
        denom = (v.sqrt() / math.sqrt(bc2)).add_(eps)
        p.addcdiv_(m, denom, value=-lr / bc1)


def _sharded_params():
    g = torch.Generator().manual_seed(0)
    return [torch.nn.Parameter(torch.randn(301, 3, generator=g)), torch.nn.Parameter(torch.randn(53, generator=g)),
            torch.nn.Parameter(torch.randn(7, 2, generator=g))]


def _sharded_loss(params, view):
    a, b, c = params
    w = torch.linspace(0.5, 1.5, a.numel()).reshape(a.shape) * (view + 1)
    return (torch.sin(a * w) ** 2).sum() + ((b * (view + 1)) ** 2).sum() + (c ** 3).sum() * (view + 1)


def _sharded_worker(rank, world, port, q, defer=False):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from horizongs_amd.multigpu import ShardedAdamDDP
        params = _sharded_params()
        opt = torch.optim.Adam([{"params": [p], "lr": 0.01 * (i + 1)} for i, p in enumerate(params)], eps=1e-15)
        if defer == "first":  # the deferred bucket first in order (its reduce-scatter launches first):
            # finish() still steps and gathers it last
            red = ShardedAdamDDP(opt, adam_fn=_cpu_adam, order=[[params[2]], [params[0]], [params[1]]],
                                 defer=[params[2]])
        elif defer:  # explicit buckets, the last one's all-gather left in flight until the next use
            red = ShardedAdamDDP(opt, adam_fn=_cpu_adam, order=[[params[0]], [params[1]], [params[2]]],
                                 defer=[params[2]])
        else:
            red = ShardedAdamDDP(opt, bucket_mb=0.0012, adam_fn=_cpu_adam)  # ~300 floats: several buckets
        for _ in range(3):
            red.begin()
            red.wait_deferred()  # what rasterization's parameter-ready hook does before reading them
            _sharded_loss(params, rank).backward()
            red.finish()
        red.wait_deferred()
        errs = []
        red.begin()  # a parameter without a gradient on this rank: refused, not a desynchronised collective
        try:
            (params[0].sum() + params[1].sum()).backward()
            red.finish()
        except RuntimeError as e:
            errs.append(str(e))
        q.put((rank, [p.detach().numpy().copy() for p in params], len(red.buckets), errs,
               sum(int(s[2].numel()) for s in red.state_shard())))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,defer", [(2, False), (3, False), (2, True), (2, "first")])
def test_sharded_adam_matches_one_rank_two_views(world, defer):
    """N ranks x 1 view with the sharded optimizer == 1 process x N views averaged with
    torch.optim.Adam (reference train.py:274-277 over the batch), parameters identical on
    every rank, each rank holding 1/N of the Adam state (world 3: buckets padded to a multiple
    of the world size); a parameter missing its gradient on a rank raises."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_sharded_worker, args=(r, world, port, q, defer)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=180) for _ in range(world)], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    params = _sharded_params()
    opt = torch.optim.Adam([{"params": [p], "lr": 0.01 * (i + 1)} for i, p in enumerate(params)], eps=1e-15,
                           foreach=False)
    for _ in range(3):
        opt.zero_grad(set_to_none=True)
        (sum(_sharded_loss(params, v) for v in range(world)) / world).backward()
        opt.step()
    nb = res[0][2]
    assert nb >= 2 and (nb == 3 if defer else True)
    total = sum(p.numel() for p in params)
    shards = [r[4] for r in res]
    assert sum(shards) >= total and max(shards) <= total // world + nb  # each rank holds ~1/N of the state
    for k, ref in enumerate(params):
        for r in res[1:]:
            assert (r[1][k] == res[0][1][k]).all()  # the all-gather leaves every rank with the same parameters
        torch.testing.assert_close(torch.from_numpy(res[0][1][k]), ref.detach(), rtol=1e-6, atol=1e-7)
    for r in res:
        assert r[3] and "no gradient this step" in r[3][0]
