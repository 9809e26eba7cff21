"""The explicit-Gaussian DDP step with two ranks on ONE GPU (gloo carries the collectives on
device tensors; the driver's N > 1 runs use RCCL across GPUs): each rank renders its own view
through gsplat_api.rasterization + the fused loss, multigpu.ShardedAdamDDP reduce-scatters the
gradients from the autograd hooks, steps the HIP Adam on its shard (offsets != 0, the colours'
bucket reduced in place) and all-gathers, the colours' gather left in flight until the next
rasterization's parameter-ready hook.  Against one process rendering both views per step and
stepping hgsr's Adam on the averaged gradient (reference train.py:206,274-277 over a batch of two
views).

Every gradient of the last step lands in its bucket without a copy (gradbuf: the projection and
activation backwards write into the flat buffers; the colours' bucket reduces autograd's tensor).

Equality: every backward is deterministic (round 6), and the one process's halving at the top
of its backward (the loss averaged) commutes exactly with the fp32 arithmetic below it, as does
the ranks' halving of each view's gradient before the sum: the parameters are bit-identical to
the one-process batch (profiles/r06_ddp_two_ranks.json).  (Before round 6 the float-atomic raster
backward made them differ in the last bits, and Adam with eps = 1e-15 turned a sign flip of a
near-zero gradient into a 2 lr step; those bounds are kept below as the failure report's
context: the parameters must
agree within 1e-3 lr except for at most 0.2 % of the elements, and within 2 lr x steps everywhere.
The ranks' parameters must be bit-identical."""
import json
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

N, W, H, V, STEPS = 20_000, 160, 96, 4, 3
LRS = [1.6e-4, 1e-3, 5e-3, 5e-2, 2.5e-3]  # means, quats, log-scales, opacity logits, colours (bench.py)


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")


def _setup(dev):
    from horizongs_amd.synthetic import camera_set, make_scene
    sc = make_scene(N, W, H, seed=0)
    cams = camera_set(V).to(dev)
    ps = [sc.means, sc.quats, torch.log(sc.scales), torch.logit(sc.opacities), sc.colors]
    ps = [p.to(dev).clone().requires_grad_(True) for p in ps]
    targets = [torch.rand(3, H, W, generator=torch.Generator().manual_seed(100 + v)).to(dev) for v in range(V)]
    return sc.Ks.to(dev), cams, ps, targets


def _view_loss(ps, Ks, cams, targets, view):
    from horizongs_amd import gsplat_api as G
    from horizongs_amd.activations import activate
    from horizongs_amd.loss import fused_loss
    means, quats, log_scales, opac_logit, colors = ps
    scales, opac = activate(log_scales, opac_logit)
    out, alpha, _ = G.rasterization(means, quats, scales, opac, colors, cams[view][None], Ks, W, H, packed=False,
                                    backgrounds=torch.zeros(1, 3, device=means.device), render_mode="RGB+ED")
    img = out.reshape(H, W, -1).permute(2, 0, 1)
    return fused_loss(img, targets[view], None, 0.2, alpha.reshape(H, W), 0.05, 0.05, scales, 0.01)[0]


def _optimizer(ps):
    from horizongs_amd.optim import Adam
    return Adam([{"params": [p], "lr": lr} for p, lr in zip(ps, LRS)], lr=0.0, eps=1e-15)


def _rank(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from horizongs_amd import gsplat_api as G
        from horizongs_amd.multigpu import ShardedAdamDDP
        dev = "cuda"
        Ks, cams, ps, targets = _setup(dev)
        means, quats, log_scales, opac_logit, colors = ps
        red = ShardedAdamDDP(_optimizer(ps), order=[[colors], [means, quats], [log_scales, opac_logit]],
                             defer=[colors])
        remove = G.register_param_ready_hook(red.wait_deferred)
        try:
            for s in range(STEPS):
                loss = _view_loss(ps, Ks, cams, targets, (s * world + rank) % V)
                red.begin()
                loss.backward()
                red.finish()
            red.wait_deferred()
            torch.cuda.synchronize()
            # the last step's gradients all landed in place: the colours' bucket reduces autograd's
            # tensor, the projection / activation backwards wrote the rest into the flat buffers
            direct = ([b["direct"] for b in red.buckets], red.copies)
            q.put((rank, [p.detach().cpu().numpy() for p in ps], direct, None))
        finally:
            remove()
    except Exception as e:  # noqa: BLE001  (reported to the parent, which fails the test)
        q.put((rank, None, None, f"{type(e).__name__}: {e}"))
    finally:
        dist.destroy_process_group()


def test_sharded_ddp_two_ranks_one_gpu_matches_two_view_batch():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = [ctx.Process(target=_rank, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=240) for _ in range(world)], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
    assert all(r[3] is None for r in res), [r[3] for r in res]
    assert all(p.exitcode == 0 for p in procs)
    assert res[0][2] == ([True, False, False], 0)  # no gradient copied into a bucket (gradbuf)
    # the reference: one process, both views of each step, averaged, one Adam step
    Ks, cams, ps, targets = _setup("cuda")
    init = [p.detach().cpu().numpy().copy() for p in ps]
    opt = _optimizer(ps)
    for s in range(STEPS):
        opt.zero_grad(set_to_none=True)
        loss = sum(_view_loss(ps, Ks, cams, targets, (s * world + r) % V) for r in range(world)) / world
        loss.backward()
        opt.step()
    torch.cuda.synchronize()
    stats = {}
    for k, (p, lr) in enumerate(zip(ps, LRS)):
        d = np.abs(res[0][1][k] - p.detach().cpu().numpy())
        stats[k] = {"lr": lr, "max_abs_diff": float(d.max()), "frac_above_1e-3_lr": float((d > 1e-3 * lr).mean()),
                    "frac_moved": float((np.abs(p.detach().cpu().numpy() - init[k]) > 0).mean())}
    os.makedirs("gpurun_out", exist_ok=True)
    with open(os.path.join("gpurun_out", "ddp_two_ranks.json"), "w") as f:
        json.dump(stats, f)
    for k, (p, lr) in enumerate(zip(ps, LRS)):
        ref = p.detach().cpu().numpy()
        a, b = res[0][1][k], res[1][1][k]
        assert np.array_equal(a, b), f"param {k}: the ranks' all-gathered parameters differ"
        d = np.abs(a - ref)
        assert d.max() <= 2 * lr * STEPS + 1e-6, (k, float(d.max()))
        assert (d > 1e-3 * lr).mean() <= 2e-3, (k, float((d > 1e-3 * lr).mean()))
        assert np.array_equal(a, ref), (k, float(d.max()), float((d > 0).mean()))
        assert (np.abs(ref - init[k]) > 0).mean() > 0.05  # the steps moved the parameters


# ---------------------------------------------------------------------------------------
# the anchor model (reference train.py:206,257-277): GradientAllReduce across a densify step
# ---------------------------------------------------------------------------------------
A_ANCHORS, A_STEPS, A_GROW_AT, A_K = 3000, 4, 1, 10


def _anchor_workload(rank, world):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    args = bench.resolve(bench.parse(["--config", "c5", "--anchors", str(A_ANCHORS), "--width", "320", "--height",
                                      "192", "--cameras", "4", "--mode", "ddp", "--no-cpu-baseline", "--no-secondary",
                                      "--no-quality", "--no-timing"]), world)
    return bench.Workload(args, rank, torch.device("cuda", 0), world)


def _grow_anchors(wl):
    """A densify step of the anchor model on statistics every rank holds identically (reduced
    over the ranks when distributed): the most often visible anchors (offset_denom counts are
    integers, so their sums are exact in any order -- the one-process reference accumulates the
    views in another order than the ranks' reduction) grow a neighbour, and every anchor
    Parameter is replaced by a longer one with zero-extended Adam state
    (cat_tensors_to_optimizer, reference scene/lod_model.py:487-541) -- the reducer must rebuild
    its buckets around the new objects."""
    st = wl.stats
    A = wl.anchor.shape[0]
    cnt = st["offset_denom"].view(A, A_K).sum(1)
    sel = torch.nonzero(cnt >= 0.5 * cnt.max()).squeeze(1)[:256]
    add = {"anchor": wl.anchor.detach()[sel] + 0.01, "feat": wl.feat.detach()[sel],
           "offset": torch.zeros(sel.numel(), A_K, 3, device=sel.device), "scaling_raw": wl.scaling_raw.detach()[sel]}
    opt = wl.optimizer
    for name, ext in add.items():
        old = getattr(wl, name)
        q = torch.nn.Parameter(torch.cat([old.detach(), ext], 0))
        for g in opt.param_groups:
            if g["params"][0] is old:
                s = opt.state.pop(old, None)
                if s:
                    s["exp_avg"] = torch.cat([s["exp_avg"], torch.zeros_like(ext)], 0)
                    s["exp_avg_sq"] = torch.cat([s["exp_avg_sq"], torch.zeros_like(ext)], 0)
                    opt.state[q] = s
                g["params"][0] = q
        setattr(wl, name, q)
    n = sel.numel()
    mlp_ps = [p for m in wl.mlps for p in m.parameters()]
    wl.params = [wl.anchor, wl.feat, wl.offset, wl.scaling_raw] + mlp_ps
    wl.ddp_order = [wl.offset, wl.scaling_raw, *wl.mlps[1].parameters(), wl.feat, wl.anchor]
    wl.allreduce.order = wl.ddp_order
    for k, v in list(st.items()):  # the statistics restart after a densify (train.py:263-273)
        per = v.shape[0] // A
        st[k] = torch.zeros((A + n) * per, 1, device=v.device)
    wl.stats_model = type("Stats", (), dict(n_offsets=A_K, **st))
    wl.lod["level"] = torch.cat([wl.lod["level"], wl.lod["level"][sel]])
    wl.lod["extra_level"] = torch.cat([wl.lod["extra_level"], wl.lod["extra_level"][sel]])
    wl.anchor_quats = torch.cat([wl.anchor_quats, wl.anchor_quats[sel]])
    return n


def _anchor_rank(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from horizongs_amd.multigpu import assert_replicas_agree, reduce_densify_stats
        wl = _anchor_workload(rank, world)
        grown, buckets = 0, []
        for s in range(A_STEPS):
            wl.step()  # GradientAllReduce: early cov-head buckets, per-bucket HIP Adam
            buckets.append(sum(b["n"] for b in wl.allreduce.buckets))
            if s == A_GROW_AT:
                reduce_densify_stats(wl.stats)
                assert_replicas_agree(list(wl.stats.values()), what="densify statistics")
                grown = _grow_anchors(wl)
        torch.cuda.synchronize()
        digest = assert_replicas_agree(wl.params, what="anchor parameters")
        q.put((rank, [p.detach().cpu().numpy() for p in wl.params], grown, buckets, digest, None))
    except Exception as e:  # noqa: BLE001  (reported to the parent, which fails the test)
        q.put((rank, None, None, None, None, f"{type(e).__name__}: {e}"))
    finally:
        dist.destroy_process_group()


def _anchor_reference(world):
    """One process, the ranks' views of each step (rank r's view and target), gradients summed
    and halved -- what the all-reduce of the 1/world-scaled gradients computes -- one Adam step."""
    wl = _anchor_workload(0, 1)
    targets = [wl.target]
    g = torch.Generator().manual_seed(1000 + 1)
    targets.append(torch.rand(3, wl.args.height, wl.args.width, generator=g).to(wl.dev))
    wl.args.freeze = True  # step() leaves the gradients, the optimizer is stepped here
    wl.world = world
    grown = 0
    for s in range(A_STEPS):
        acc = None
        for r in range(world):
            wl.rank, wl.n_steps, wl.target = r, s, targets[r]
            wl.step()
            gs = [p.grad.clone() if p.grad is not None else None for p in wl.params]
            acc = gs if acc is None else [a if b is None else (b if a is None else a + b) for a, b in zip(acc, gs)]
        for p, a in zip(wl.params, acc):
            p.grad = None if a is None else a * (1.0 / world)
        wl.optimizer.step()
        if s == A_GROW_AT:
            grown = _grow_anchors(wl)
    torch.cuda.synchronize()
    return [p.detach().cpu().numpy() for p in wl.params], grown


def test_anchor_ddp_two_ranks_across_densify():
    """The anchor model's DDP step (multigpu.GradientAllReduce: buckets in gradient order, the
    fused decode backward's early cov-head buckets, per-bucket HIP Adam) with two ranks on one GPU,
    across a densify step: the statistics reduced over the ranks, every rank growing the same
    anchors (replica digest), the buckets rebuilt around the new Parameters; after the steps the
    ranks' parameters are bit-identical, and bit-identical to one process stepping the two views'
    averaged gradient: every backward is deterministic, and halving before the sum (the hooks'
    1/world) equals halving after it in fp32 (profiles/r06_ddp_anchor_two_ranks.json)."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = [ctx.Process(target=_anchor_rank, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=240) for _ in range(world)], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
    assert all(r[5] is None for r in res), [r[5] for r in res]
    assert all(p.exitcode == 0 for p in procs)
    (_, p0, grown0, b0, d0, _), (_, p1, grown1, b1, d1, _) = res
    assert grown0 == grown1 > 0 and d0 == d1
    assert b0[A_GROW_AT + 1] > b0[A_GROW_AT], b0  # the buckets were rebuilt around the grown anchors
    ref, grown_ref = _anchor_reference(world)
    assert grown_ref == grown0
    stats = {}
    for k, (a, b, r) in enumerate(zip(p0, p1, ref)):
        assert np.array_equal(a, b), f"param {k}: the ranks differ"
        assert a.shape == r.shape, (k, a.shape, r.shape)
        d = np.abs(a - r)
        stats[k] = {"shape": list(a.shape), "max_abs_diff": float(d.max()), "frac_differing": float((d > 0).mean())}
    os.makedirs("gpurun_out", exist_ok=True)
    with open(os.path.join("gpurun_out", "ddp_anchor_two_ranks.json"), "w") as f:
        json.dump({"grown": grown0, "bucket_floats": b0, "params": stats}, f)
    for k, st in stats.items():
        assert st["max_abs_diff"] == 0.0, (k, st)
