"""GPU parity of the fused HIP Adam step (K17, horizongs_amd.optim.Adam) against the
reference's optimizer, torch.optim.Adam(..., eps=1e-15) (scene/lod_model.py:320), run on
the CPU with the same parameters and gradients, over several steps.  Covers: many
tensors (> 16 per launch -> several launches), ragged sizes (chunk tails), a
misaligned parameter (scalar path), parameters without a gradient on some steps
(per-parameter step counts), lr = 0 groups, and the reference's optimizer surgery
(prune rows of a parameter and its exp_avg / exp_avg_sq, scene/lod_model.py:466-486).
Tolerance: 2e-6 relative + 2e-6 of each array's max magnitude (torch's own CPU vs GPU
Adam differ by contraction/rounding at that level)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")


def _close(a, b, what):
    a = a.detach().float().cpu().numpy()
    b = b.detach().float().cpu().numpy()
    np.testing.assert_allclose(a, b, rtol=2e-6, atol=2e-6 * max(float(np.abs(b).max()), 1e-30), err_msg=what)


def _pair(shapes, lrs, seed=0, misalign=()):
    g = torch.Generator().manual_seed(seed)
    ref, mine = [], []
    for i, s in enumerate(shapes):
        x = torch.randn(s, generator=g)
        ref.append(torch.nn.Parameter(x.clone()))
        if i in misalign:  # a parameter whose storage starts 4 B into an allocation
            base = torch.empty(x.numel() + 1, device=DEV)
            base[1:] = x.reshape(-1).to(DEV)
            mine.append(torch.nn.Parameter(base[1:].view(s)))
        else:
            mine.append(torch.nn.Parameter(x.to(DEV)))
    groups = lambda ps: [{"params": [p], "lr": lr} for p, lr in zip(ps, lrs)]
    from horizongs_amd.optim import Adam
    return ref, mine, torch.optim.Adam(groups(ref), lr=0.0, eps=1e-15), Adam(groups(mine), lr=0.0, eps=1e-15)


def test_adam_matches_torch_over_steps():
    shapes = [(2_000_003, 3), (4096,), (4097,), (1, 10, 3), (70, 32), (70,), (35, 32), (32,), (10, 32), (10,),
              (30, 32), (30,), (5,), (123457,), (16, 16), (3,), (99, 7), (12, 4), (8192, 2), (1,)]
    lrs = [1e-3 * (i % 4) for i in range(len(shapes))]
    ref, mine, oref, omine = _pair(shapes, lrs, misalign=(2, 13))
    assert mine[2].data_ptr() % 16 != 0
    g = torch.Generator().manual_seed(1)
    for t in range(4):
        for i, (a, b) in enumerate(zip(ref, mine)):
            if (i + t) % 5 == 0:  # no gradient this step: skipped, its step count lags
                a.grad = None
                b.grad = None
                continue
            gr = torch.randn(a.shape, generator=g) * (0.1 ** t)
            a.grad = gr.clone()
            b.grad = gr.to(DEV)
        oref.step()
        omine.step()
        torch.cuda.synchronize()
        for i, (a, b) in enumerate(zip(ref, mine)):
            _close(b, a, f"param {i} step {t}")
            if oref.state[a]:
                assert float(omine.state[b]["step"]) == float(oref.state[a]["step"])
                _close(omine.state[b]["exp_avg"], oref.state[a]["exp_avg"], f"exp_avg {i} step {t}")
                _close(omine.state[b]["exp_avg_sq"], oref.state[a]["exp_avg_sq"], f"exp_avg_sq {i} step {t}")


def test_adam_after_reference_prune_surgery():
    """_prune_anchor_optimizer (scene/lod_model.py:466-486): rows of a parameter and its
    moment buffers are masked, the group's param and state are replaced; later steps
    continue from the kept rows."""
    ref, mine, oref, omine = _pair([(5000, 32), (5000, 3)], [1e-2, 1e-3], seed=3)
    keep = torch.rand(5000, generator=torch.Generator().manual_seed(4)) > 0.3

    def prune(opt, mask):
        for group in opt.param_groups:
            p = group["params"][0]
            st = opt.state.get(p, None)
            st["exp_avg"] = st["exp_avg"][mask]
            st["exp_avg_sq"] = st["exp_avg_sq"][mask]
            del opt.state[p]
            group["params"][0] = torch.nn.Parameter(p[mask].requires_grad_(True))
            opt.state[group["params"][0]] = st

    g = torch.Generator().manual_seed(5)
    for t in range(3):
        if t == 1:
            prune(oref, keep)
            prune(omine, keep.to(DEV))
        for ga, gb in zip(oref.param_groups, omine.param_groups):
            gr = torch.randn(ga["params"][0].shape, generator=g)
            ga["params"][0].grad = gr.clone()
            gb["params"][0].grad = gr.to(DEV)
        oref.step()
        omine.step()
    for ga, gb in zip(oref.param_groups, omine.param_groups):
        _close(gb["params"][0], ga["params"][0], "pruned param")
        _close(omine.state[gb["params"][0]]["exp_avg_sq"], oref.state[ga["params"][0]]["exp_avg_sq"], "pruned v")


def test_adam_state_dict_round_trip():
    _, mine, _, omine = _pair([(100, 3)], [1e-3])
    mine[0].grad = torch.ones_like(mine[0])
    omine.step()
    sd = omine.state_dict()
    assert set(sd["state"][0]) == {"step", "exp_avg", "exp_avg_sq"}
    from horizongs_amd.optim import Adam
    o2 = Adam([{"params": [mine[0]], "lr": 1e-3}], lr=0.0, eps=1e-15)
    o2.load_state_dict(sd)
    assert float(o2.state[mine[0]]["step"]) == 1.0


def test_adam_step_params_subsets_bit_identical():
    """Adam.step_params (one fused launch per all-reduce bucket, multigpu.GradientAllReduce
    .finish(step=...)) stepping the parameters in subsets gives bit-identical parameters and
    state to one step over all of them."""
    from horizongs_amd.optim import Adam
    shapes = [(300_001, 3), (4096,), (70, 32), (5,), (123, 7), (1,)]
    g = torch.Generator().manual_seed(9)
    base = [torch.randn(s, generator=g) for s in shapes]
    pa = [b.to(DEV).clone().requires_grad_(True) for b in base]
    pb = [b.to(DEV).clone().requires_grad_(True) for b in base]
    oa = Adam([{"params": [p], "lr": 1e-3 * (i + 1)} for i, p in enumerate(pa)], lr=0.0, eps=1e-15)
    ob = Adam([{"params": [p], "lr": 1e-3 * (i + 1)} for i, p in enumerate(pb)], lr=0.0, eps=1e-15)
    for t in range(3):
        for a, b in zip(pa, pb):
            gr = torch.randn(a.shape, generator=g).to(DEV)
            a.grad, b.grad = gr.clone(), gr.clone()
        oa.step()
        for sub in ([pb[5], pb[0]], [pb[2]], [pb[1], pb[3], pb[4]]):  # buckets in reverse-ish order
            ob.step_params(sub)
        torch.cuda.synchronize()
        for a, b in zip(pa, pb):
            assert torch.equal(a, b)
            assert torch.equal(oa.state[a]["exp_avg_sq"], ob.state[b]["exp_avg_sq"])
            assert float(oa.state[a]["step"]) == float(ob.state[b]["step"]) == t + 1


def test_adam_alignment_bit_identical():
    """A parameter whose storage is not 16-B aligned (the scalar path of csrc/optim.hip, e.g. a
    shard segment at an odd offset of a flat bucket) steps bit-identically to an aligned copy
    (the float4 path)."""
    from horizongs_amd.optim import Adam
    n = 3 * 4096 + 7
    g = torch.Generator().manual_seed(4)
    base = torch.randn(n, generator=g)
    pa = base.to(DEV).clone().requires_grad_(True)
    buf = torch.zeros(n + 1, device=DEV)
    pb = buf[1:]
    pb.copy_(base.to(DEV))
    pb.requires_grad_(True)
    assert pa.data_ptr() % 16 == 0 and pb.data_ptr() % 16 != 0
    oa, ob = Adam([pa], lr=1e-2, eps=1e-15), Adam([pb], lr=1e-2, eps=1e-15)
    for _ in range(4):
        gr = torch.randn(n, generator=g).to(DEV)
        pa.grad, pb.grad = gr.clone(), gr.clone()
        oa.step()
        ob.step()
    torch.cuda.synchronize()
    assert torch.equal(pa.detach(), pb.detach()), float((pa - pb).abs().max())
    assert torch.equal(oa.state[pa]["exp_avg_sq"], ob.state[pb]["exp_avg_sq"])


def test_sharded_adam_one_rank_rccl_matches_adam(monkeypatch):
    """multigpu.ShardedAdamDDP through a one-rank RCCL group (the HGSR_DDP_FORCE rehearsal path:
    hooks, explicit buckets, reduce-scatter, the HIP Adam over shard segments, all-gather, the
    last bucket's all-gather deferred to the next use) gives the parameters of hgsr's Adam stepping
    the same gradients, bit for bit."""
    import socket
    import torch.distributed as dist
    from horizongs_amd import multigpu as MG
    from horizongs_amd.optim import Adam
    monkeypatch.setattr(MG, "_FORCE", True)
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", world_size=1, rank=0)
    try:
        g = torch.Generator().manual_seed(3)
        shapes = [(100_003, 3), (77_001, 4), (5, 3)]
        base = [torch.randn(sh, generator=g) for sh in shapes]
        pa = [b.to(DEV).clone().requires_grad_(True) for b in base]
        pb = [b.to(DEV).clone().requires_grad_(True) for b in base]
        oa = Adam([{"params": [p], "lr": 1e-3 * (i + 1)} for i, p in enumerate(pa)], lr=0.0, eps=1e-15)
        ob = Adam([{"params": [p], "lr": 1e-3 * (i + 1)} for i, p in enumerate(pb)], lr=0.0, eps=1e-15)
        red = MG.ShardedAdamDDP(ob, order=[[pb[2]], [pb[0], pb[1]]], defer=[pb[2]])  # deferred first: stepped last
        for _ in range(3):
            w = [torch.randn(sh, generator=g).to(DEV) for sh in shapes]
            oa.zero_grad(set_to_none=True)
            sum((a * c).sin().sum() for a, c in zip(pa, w)).backward()
            oa.step()
            red.begin()
            red.wait_deferred()
            sum((b * c).sin().sum() for b, c in zip(pb, w)).backward()
            red.finish()
        red.wait_deferred()
        torch.cuda.synchronize()
        for i, (a, b) in enumerate(zip(pa, pb)):
            assert torch.equal(a.detach(), b.detach()), (i, float((a - b).abs().max()))
    finally:
        dist.destroy_process_group()


def test_replica_digest_device_independent():
    """multigpu.replica_digest (the post-densification replica check) gives the same value for
    the same bytes on the device and on the host, and changes with one flipped bit."""
    from horizongs_amd.multigpu import replica_digest
    g = torch.Generator().manual_seed(11)
    host = [torch.randn(50_001, 32, generator=g), torch.randn(7, generator=g), torch.randint(0, 9, (333,), generator=g)]
    dev = [t.to(DEV) for t in host]
    assert int(replica_digest(host)) == int(replica_digest(dev))
    dev[0].view(torch.int32)[25_000, 3] ^= 1
    assert int(replica_digest(host)) != int(replica_digest(dev))
