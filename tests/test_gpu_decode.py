"""GPU parity of the fused anchor decode (horizongs_amd.decode) -- SURVEY 8(f) rank 1.

Forward and LoD mask against tests/golden/decode_{rgb,sh2}.npz (outputs of the
reference module itself, scripts/make_golden.py); backward against torch autograd of
the oracle restatement oracle/decode_ref.py in fp64 (and fp32 for the conditioning-aware
check).  Tolerance: fp32, 1e-5 abs / 1e-4 rel (exact-f32 MFMA with a different
summation order than the reference GEMM)."""
import os

import numpy as np
import pytest
import torch

from oracle import decode_ref as D
from oracle.checks import close, cond_close

pytestmark = pytest.mark.gpu
DEV = "cuda"
GOLD = os.path.join(os.path.dirname(__file__), "golden")


def _gold(tag):
    return np.load(os.path.join(GOLD, f"decode_{tag}.npz"))


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")


@pytest.mark.parametrize("tag", ["rgb", "sh2"])
def test_lod_mask_matches_reference(tag):
    from horizongs_amd import decode as HD
    g = _gold(tag)
    t = lambda a: torch.from_numpy(np.asarray(a)).to(DEV)
    m = HD.lod_mask(t(g["anchor"]), t(g["level"]), t(g["extra_level"]), t(g["cam_center"]), float(g["res_scale"]),
                    float(g["standard_dist"]), int(g["fork"]), int(g["street_levels"]))
    np.testing.assert_array_equal(m.cpu().numpy(), g["anchor_mask"])


@pytest.mark.parametrize("tag", ["rgb", "sh2"])
def test_decode_forward_matches_reference(tag):
    from horizongs_amd import decode as HD
    g = _gold(tag)
    a = D.golden_inputs(g, torch.float32)
    t = lambda x: x.to(DEV)
    mlps = {k: t(v) for k, v in a["mlps"].items()}
    vis = torch.from_numpy(g["anchor_mask"]).to(DEV)
    xyz, offs, col, op, sc, rot, mask = HD.decode(t(torch.from_numpy(g["anchor"])),
                                                  t(torch.from_numpy(g["anchor_feat"])),
                                                  t(torch.from_numpy(g["offset"])),
                                                  t(torch.from_numpy(g["scaling"])), t(a["cam_center"]), mlps, vis,
                                                  a["view_dim"], a["n_offsets"], a["color_dim"])
    np.testing.assert_array_equal(mask.cpu().numpy(), g["out_mask"])
    close(xyz.cpu().numpy(), g["out_xyz"], name="xyz")
    close(col.cpu().numpy(), g["out_color"], name="color")
    close(op.cpu().numpy(), g["out_opacity"], name="opacity")
    close(sc.cpu().numpy(), g["out_scaling"], name="scaling")
    close(rot.cpu().numpy(), g["out_rot"], name="rot")


def _random_model(n_anchor, view_dim, color_dim, seed, n_off=10):
    gen = torch.Generator().manual_seed(seed)
    F = 32
    r = lambda *s, sd=1.0: torch.randn(*s, generator=gen) * sd
    anchor = r(n_anchor, 3, sd=2.0)
    inputs = dict(anchor=anchor, feat=r(n_anchor, F, sd=0.3), offset=r(n_anchor, n_off, 3, sd=0.1),
                  scaling_raw=np.log(0.01) + r(n_anchor, 6, sd=0.1), cam_center=torch.tensor([0.3, -0.5, 6.0]))
    K1 = F + view_dim
    mlps = {}
    for h, O in (("opacity", n_off), ("cov", 7 * n_off), ("color", color_dim * n_off)):
        mlps[f"{h}_w1"] = r(F, K1, sd=1 / np.sqrt(K1))
        mlps[f"{h}_b1"] = r(F, sd=0.1)
        mlps[f"{h}_w2"] = r(O, F, sd=1 / np.sqrt(F))
        mlps[f"{h}_b2"] = r(O, sd=0.1)
    return inputs, mlps


@pytest.mark.parametrize("view_dim,color_dim,n_anchor,n_off,col_one", [
    (3, 3, 1000, 10, 1), (0, 27, 700, 10, 1), (3, 3, 20011, 10, 1), (3, 3, 1500, 5, 1), (3, 3, 333, 11, 1),
    # SH colour heads: the one-launch colour backward (17 / 9 / 15 tiles, view_dim 0 / 3) and
    # the chunked launches it replaces
    (0, 27, 5003, 10, 1), (3, 27, 1500, 10, 1), (0, 27, 900, 5, 1), (3, 48, 777, 5, 1), (0, 27, 700, 10, 0)])
def test_decode_backward(view_dim, color_dim, n_anchor, n_off, col_one, request):
    """All input and weight gradients vs fp64 / fp32 autograd of the oracle restatement.
    n_offsets 5 is the Block_A chunk setting (config/ours/large_scene/block_A/config.yaml:11),
    11 the largest the kernels take."""
    from horizongs_amd import decode as HD
    from horizongs_amd import _native as NAT
    old = NAT.lib().hgsr_decode_set_color_bwd(col_one)
    request.addfinalizer(lambda: NAT.lib().hgsr_decode_set_color_bwd(old))
    inputs, mlps = _random_model(n_anchor, view_dim, color_dim, seed=5 + n_anchor, n_off=n_off)
    gen = torch.Generator().manual_seed(77)
    vis = torch.rand(n_anchor, generator=gen) < 0.8

    def run_ref(dtype):
        ins = {k: v.to(dtype).clone().requires_grad_(k != "cam_center") for k, v in inputs.items()}
        ws = {k: v.to(dtype).clone().requires_grad_(True) for k, v in mlps.items()}
        sub = {k: (v[vis] if k != "cam_center" else v) for k, v in ins.items()}
        outs = D.decode_torch(sub["anchor"], sub["feat"], sub["offset"], sub["scaling_raw"], sub["cam_center"], ws,
                              view_dim, n_off, color_dim)
        return ins, ws, outs

    ins32, ws32, outs32 = run_ref(torch.float32)
    mask_ref = outs32[6]
    gg = torch.Generator().manual_seed(78)
    ups = [torch.randn(o.shape, generator=gg) for o in outs32[:6]]
    sum(((o * u.to(o.dtype)).sum() for o, u in zip(outs32[:6], ups))).backward()
    ins64, ws64, outs64 = run_ref(torch.float64)
    assert torch.equal(outs64[6], mask_ref)
    sum(((o * u.to(o.dtype)).sum() for o, u in zip(outs64[:6], ups))).backward()

    dev_in = {k: v.to(DEV).clone().requires_grad_(k != "cam_center") for k, v in inputs.items()}
    dev_w = {k: v.to(DEV).clone().requires_grad_(True) for k, v in mlps.items()}
    outs = HD.decode(dev_in["anchor"], dev_in["feat"], dev_in["offset"], dev_in["scaling_raw"], dev_in["cam_center"],
                     dev_w, vis.to(DEV), view_dim, n_off, color_dim)
    np.testing.assert_array_equal(outs[6].cpu().numpy(), mask_ref.numpy())
    for o, r32, r64, name in zip(outs[:6], outs32[:6], outs64[:6], ("xyz", "offsets", "color", "opacity", "scaling",
                                                                   "rot")):
        cond_close(o.detach().cpu().numpy(), r32.detach().numpy(), r64.detach().numpy(), name)
    sum(((o * u.to(DEV)).sum() for o, u in zip(outs[:6], ups))).backward()
    for k in ("anchor", "feat", "offset", "scaling_raw"):
        cond_close(dev_in[k].grad.cpu().numpy(), ins32[k].grad.numpy(), ins64[k].grad.numpy(), "d_" + k)
    for k in mlps:
        cond_close(dev_w[k].grad.cpu().numpy(), ws32[k].grad.numpy(), ws64[k].grad.numpy(), "d_" + k)


@pytest.mark.parametrize("with_lod", [False, True])
def test_anchor_prefilter_matches_projection_and_lod(with_lod):
    """decode.prefilter (fused set_anchor_mask + prefilter_voxel, render.py:120-197) vs the oracle
    projection's radii > 0 and the LoD restatement: the visible mask and its ordered index
    bit-exact (the same projection bits as hgsr_project3d_fwd)."""
    from horizongs_amd import decode as HD
    from horizongs_amd.synthetic import make_scene
    from oracle import explicit_ref as XR
    from oracle import oracle as O
    A = 20000
    sc = make_scene(A, 320, 240, seed=11, scale_range=(0.002, 0.4), depth_range=(0.005, 30.0))
    g = torch.Generator().manual_seed(3)
    scal6 = torch.exp(torch.randn(A, 6, generator=g) * 0.5 - 4.0)
    quats = sc.quats / sc.quats.norm(dim=-1, keepdim=True)
    r, _, _, _ = O.proj3d_fwd(sc.means.numpy(), quats.numpy(), scal6[:, :3].contiguous().numpy(),
                              sc.viewmats.numpy(), sc.Ks.numpy(), 320, 240)
    ref = torch.from_numpy(r[0] > 0)
    lod = None
    if with_lod:
        level = torch.randint(0, 4, (A,), generator=g, dtype=torch.int32)
        extra = torch.rand(A, generator=g) - 0.5
        cam = torch.tensor([0.0, 0.0, 0.5])
        ref &= XR.gs_mask(sc.means, level, extra, cam, 1.0, 8.0, 2, 4)
        lod = dict(level=level.to(DEV), extra_level=extra.to(DEV), cam_center=cam.to(DEV), res_scale=1.0,
                   standard_dist=8.0, fork=2, street_levels=4)
    assert 0 < int(ref.sum()) < A
    vis, idx = HD.prefilter(sc.means.to(DEV), scal6.to(DEV), quats.to(DEV), sc.viewmats[0].to(DEV),
                            sc.Ks[0].to(DEV), 320, 240, lod=lod)
    np.testing.assert_array_equal(vis.cpu().numpy(), ref.numpy())
    np.testing.assert_array_equal(idx.cpu().numpy(), torch.nonzero(ref).reshape(-1).numpy())


def test_lazy_prefilter_decode_equals_eager():
    """prefilter(lazy=True) keeps the visible count on the device (one host read less per
    view): decode through it gives bit-identical outputs, selection mask, gradients and the
    slot rows training_statis reuses, as through the eager index."""
    from horizongs_amd import decode as HD
    from horizongs_amd.synthetic import make_scene
    A = 30000
    sc = make_scene(A, 640, 480, seed=5)
    g = torch.Generator().manual_seed(4)
    anchor = sc.means.to(DEV)
    feat = (torch.randn(A, 32, generator=g) * 0.3).to(DEV)
    offset = (torch.randn(A, 10, 3, generator=g) * 0.1).to(DEV)
    scaling = (np.log(0.02) + torch.randn(A, 6, generator=g) * 0.2).float().to(DEV)
    quats = torch.zeros(A, 4, device=DEV)
    quats[:, 0] = 1.0
    torch.manual_seed(7)
    mlps = [torch.nn.Sequential(torch.nn.Linear(35, 32), torch.nn.ReLU(True), torch.nn.Linear(32, o)).to(DEV)
            for o in (10, 70, 30)]
    cam = torch.zeros(3, device=DEV)
    outs = []
    for lazy in (False, True):
        vis, idx = HD.prefilter(anchor, torch.exp(scaling), quats, sc.viewmats[0].to(DEV), sc.Ks[0].to(DEV), 640, 480,
                                lazy=lazy)
        ps = [t.clone().requires_grad_(True) for t in (feat, offset, scaling)]
        xyz, offs, col, op, scl, rot, sel = HD.decode(anchor, ps[0], ps[1], ps[2], cam, mlps, idx, 3, 10, 3)
        assert 1000 < xyz.shape[0]
        loss = xyz.square().sum() + col.sum() + op.sum() + scl.sum() + rot.sum()
        loss.backward()
        vis_idx = HD.visible_index(vis)  # cached by the decode in both modes
        outs.append([vis.cpu(), vis_idx.cpu(), xyz.detach().cpu(), col.detach().cpu(), op.detach().cpu(),
                     sel.cpu(), sel._hgsr_slot_row.cpu()] + [p.grad.cpu() for p in ps])
    assert torch.equal(outs[0][1], torch.nonzero(outs[0][0]).reshape(-1).to(torch.int32))
    for a, b in zip(*outs):
        assert torch.equal(a, b)


@pytest.mark.parametrize("view_dim,color_dim", [(3, 3), (0, 27)])
def test_decode_backward_split_heads_equal_one_call(view_dim, color_dim):
    """With a data-parallel reducer attached the decode backward runs as two launches (the cov
    head first, head_mask 2, then the opacity + colour heads, head_mask 5, the second one
    read-modify-writing d_scaling) instead of one all-heads call (head_mask 0): every input
    and weight gradient must come out the same, and the hook must receive exactly the cov
    head's final gradients."""
    from horizongs_amd import decode as HD
    inputs, mlps = _random_model(3001, view_dim, color_dim, seed=41)
    vis = (torch.rand(3001, generator=torch.Generator().manual_seed(42)) < 0.8).to(DEV)
    gg = torch.Generator().manual_seed(43)
    res = {}
    for split in (False, True):
        dev_in = {k: v.to(DEV).clone().requires_grad_(k != "cam_center") for k, v in inputs.items()}
        dev_w = {k: v.to(DEV).clone().requires_grad_(True) for k, v in mlps.items()}
        handed = []
        HD.set_early_grad_hook((lambda pairs: handed.extend((id(p), g.clone()) for p, g in pairs)) if split else None)
        try:
            outs = HD.decode(dev_in["anchor"], dev_in["feat"], dev_in["offset"], dev_in["scaling_raw"],
                             dev_in["cam_center"], dev_w, vis, view_dim, 10, color_dim)
            if not res:
                ups = [torch.randn(o.shape, generator=gg).to(DEV) for o in outs[:6]]
            sum((o * u).sum() for o, u in zip(outs[:6], ups)).backward()
        finally:
            HD.set_early_grad_hook(None)
        torch.cuda.synchronize()
        grads = {k: dev_in[k].grad.cpu().numpy() for k in ("anchor", "feat", "offset", "scaling_raw")}
        grads.update({k: dev_w[k].grad.cpu().numpy() for k in mlps})
        res[split] = grads
        if split:
            early = dict(handed)
            want = [dev_in["offset"], dev_in["scaling_raw"]] + [dev_w[f"cov_{n}"] for n in ("w1", "b1", "w2", "b2")]
            assert sorted(early) == sorted(id(t) for t in want)
            for t in want:  # what the hook saw is the final gradient
                np.testing.assert_array_equal(early[id(t)].cpu().numpy(), t.grad.cpu().numpy())
    for k in res[False]:
        # the same kernels and per-head reduction order: identical up to float-atomic order of the
        # input gradients summed across heads (d_scaling, d_feat, d_anchor)
        np.testing.assert_allclose(res[True][k], res[False][k], rtol=1e-5, atol=1e-6 * float(np.abs(res[False][k]).max()),
                                   err_msg=k)
