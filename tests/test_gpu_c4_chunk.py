"""Config c4 (MatrixCity Block_A per-chunk fine: color_attr SH2, view_dim 0, 10 offsets, colour
head [32, 270]; reference config/ours/large_scene/block_A/chunk_fine/0_0.yaml,
scene/lod_model.py:67-84) through the decode-inclusive train step on the GPU:

  prefilter_voxel (render.py:120-197) -> generate_neural_gaussians (basic_model.py:297-371)
  -> gsplat.rasterization(sh_degree=2, RGB+ED) (render.py:40-54) -> loss head (train.py:153-178)
  -> backward

* test_c4_golden_chain: the reference's own decode inputs (tests/golden/decode_sh2.npz, written
  by the reference module) -> the whole step vs the CPU chain (decode restatement pinned to the
  same golden -> C-oracle rasterization with SH2 -> loss restatement pinned to losses.npz),
  every decoded output, the image, the loss and every gradient (anchor features, offsets,
  scalings and all twelve MLP tensors), f32 checker + f64 truth per element;
* test_c4_fullsize_chunk_step: a 500k-anchor SH2 chunk at 1920x1080: decoded outputs vs the
  restatement (f32 / f64), the rasterization fwd + bwd vs the oracle on a band of rows, and the
  decode backward fed with the GPU raster's own gradients vs the restatement's autograd."""
from types import SimpleNamespace

import numpy as np
import pytest
import torch

from horizongs_amd import decode as HD
from horizongs_amd import gsplat_api as G
from horizongs_amd.loss import fused_loss
from oracle import autograd as OA
from oracle import decode_ref as D
from oracle import loss_ref as LR
from oracle.checks import close, cond_close
from tests import raster_parity as RP

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
HEADS = ("opacity", "cov", "color")


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")


def _camera(cam_center, W, H, fov_deg=90.0):
    """world -> camera = translation by -cam_center (camera at the decode's cam_center, +z forward)."""
    vm = torch.eye(4)
    vm[:3, 3] = -torch.as_tensor(cam_center, dtype=torch.float32)
    f = 0.5 * W / np.tan(np.radians(fov_deg) / 2)
    K = torch.tensor([[f, 0, W / 2], [0, f, H / 2], [0, 0, 1.0]])
    return vm[None], K[None]


def test_c4_golden_chain():
    import os
    g = np.load(os.path.join(os.path.dirname(__file__), "golden", "decode_sh2.npz"))
    assert int(g["view_dim"]) == 0 and g["color_w2"].shape == (270, 32)  # the c4 colour head
    W, H = 160, 128
    vm, K = _camera(g["cam_center"], W, H)
    target = torch.rand(3, H, W, generator=torch.Generator().manual_seed(3))
    bg = torch.tensor([[0.1, 0.2, 0.3]])

    def cpu_chain(dtype):
        a = D.golden_inputs(g, dtype)
        ins = {k: a[k].clone().requires_grad_(True) for k in ("feat", "offset", "scaling_raw")}
        ws = {k: v.clone().requires_grad_(True) for k, v in a["mlps"].items()}
        xyz, _, col, op, sc, rot, mask = D.decode_torch(a["anchor"], ins["feat"], ins["offset"], ins["scaling_raw"],
                                                        a["cam_center"], ws, 0, 10, 27)
        cfg = dict(viewmats=vm, Ks=K, W=W, H=H, sh_degree=2, bg=bg, mode="RGB+ED")
        out, ra = OA.rasterization(xyz, rot, sc, op.reshape(-1), col, cfg)
        img = out[0, ..., :3].permute(2, 0, 1)
        loss = LR.loss(img, target.to(dtype), None, 0.2, ra[0, ..., 0], 0.05, 0.05, sc, 0.01)[0]
        loss.backward()
        return dict(xyz=xyz, color=col, opacity=op, scaling=sc, rot=rot, mask=mask, out=out, alpha=ra, loss=loss,
                    ref=cfg["last"], **{"d_" + k: v.grad for k, v in {**ins, **ws}.items()})

    c32, c64 = cpu_chain(torch.float32), cpu_chain(torch.float64)
    assert c32["ref"].isect_ids.size > 50  # the visible golden Gaussians do reach the image

    t = lambda x: torch.from_numpy(np.asarray(x)).to(DEV)
    ins = {"feat": t(g["anchor_feat"]), "offset": t(g["offset"]), "scaling_raw": t(g["scaling"])}
    ins = {k: v.clone().requires_grad_(True) for k, v in ins.items()}
    ws = {k: t(v).clone().requires_grad_(True) for k, v in D.golden_inputs(g, torch.float32)["mlps"].items()}
    vis = t(g["anchor_mask"])
    xyz, _, col, op, sc, rot, mask = HD.decode(t(g["anchor"]), ins["feat"], ins["offset"], ins["scaling_raw"],
                                               t(g["cam_center"]), ws, vis, 0, 10, 27)
    # stage 1: the decode against the reference's own outputs
    np.testing.assert_array_equal(mask.cpu().numpy(), g["out_mask"])
    for name, x in (("xyz", xyz), ("color", col), ("opacity", op), ("scaling", sc), ("rot", rot)):
        close(x.detach().cpu().numpy(), g["out_" + name], name=name)
    out, alpha, meta = G.rasterization(xyz, rot, sc, op.reshape(-1), col, vm.to(DEV), K.to(DEV), W, H, packed=False,
                                       backgrounds=bg.to(DEV), render_mode="RGB+ED", sh_degree=2)
    np.testing.assert_array_equal(meta["isect_ids"].cpu().numpy(), c32["ref"].isect_ids)
    np.testing.assert_array_equal(meta["flatten_ids"].cpu().numpy(), c32["ref"].flatten_ids)
    cond_close(out.detach().cpu().numpy(), c32["out"].detach().numpy(), c64["out"].detach().numpy(), "render")
    cond_close(alpha.detach().cpu().numpy(), c32["alpha"].detach().numpy(), c64["alpha"].detach().numpy(), "alpha")
    img = out[0].permute(2, 0, 1)
    loss = fused_loss(img, target.to(DEV), None, 0.2, alpha[0, ..., 0], 0.05, 0.05, sc, 0.01)[0]
    cond_close(np.array([float(loss)]), np.array([float(c32["loss"])]), np.array([float(c64["loss"])]), "loss")
    loss.backward()
    m = g["anchor_mask"]  # the restatement takes the visible anchors only
    for k, v in {**ins, **ws}.items():
        got = v.grad.cpu().numpy()
        if k in ins:
            assert not got[~m].any()  # invisible anchors get no gradient
            got = got[m]
        cond_close(got, c32["d_" + k].numpy(), c64["d_" + k].numpy(), "d_" + k)


@pytest.mark.slow
def test_c4_fullsize_chunk_step():
    """500k anchors, SH2 colour head, view_dim 0, 1920x1080 (bench.py --config c4 inputs)."""
    from horizongs_amd.synthetic import make_scene
    A, W, H = 500_000, 1920, 1080
    sc0 = make_scene(A, W, H, seed=0)
    gen = torch.Generator().manual_seed(2)
    anchor = sc0.means
    feat = torch.randn(A, 32, generator=gen) * 0.1
    offset = torch.randn(A, 10, 3, generator=gen) * 0.1
    scaling = (np.log(0.01) + torch.randn(A, 6, generator=gen) * 0.1).float()
    torch.manual_seed(2)
    ws = {}
    for h, o in zip(HEADS, (10, 70, 270)):
        l1, l2 = torch.nn.Linear(32, 32), torch.nn.Linear(32, o)
        ws.update({f"{h}_w1": l1.weight.detach(), f"{h}_b1": l1.bias.detach(), f"{h}_w2": l2.weight.detach(),
                   f"{h}_b2": l2.bias.detach()})
    cam = torch.zeros(3)
    quats = torch.zeros(A, 4)
    quats[:, 0] = 1
    vis, idx = HD.prefilter(anchor.to(DEV), torch.exp(scaling).to(DEV), quats.to(DEV), sc0.viewmats[0].to(DEV),
                            sc0.Ks[0].to(DEV), W, H)
    v = vis.cpu()
    assert int(v.sum()) > 0.9 * A
    dins = {k: x.to(DEV).clone().requires_grad_(True) for k, x in (("feat", feat), ("offset", offset),
                                                                   ("scaling", scaling))}
    dws = {k: x.to(DEV).clone().requires_grad_(True) for k, x in ws.items()}
    outs = HD.decode(anchor.to(DEV), dins["feat"], dins["offset"], dins["scaling"], cam.to(DEV), dws, idx, 0, 10, 27)

    def ref(dtype):
        ins = {k: x.to(dtype)[v].clone().requires_grad_(True) for k, x in (("feat", feat), ("offset", offset),
                                                                          ("scaling", scaling))}
        w = {k: x.to(dtype).clone().requires_grad_(True) for k, x in ws.items()}
        o = D.decode_torch(anchor.to(dtype)[v], ins["feat"], ins["offset"], ins["scaling"], cam.to(dtype), w, 0, 10,
                           27)
        return ins, w, o

    i32, w32, o32 = ref(torch.float32)
    i64, w64, o64 = ref(torch.float64)
    np.testing.assert_array_equal(outs[6].cpu().numpy(), o32[6].numpy())
    names = ("xyz", "offsets", "color", "opacity", "scaling", "rot")
    for k in (0, 2, 3, 4, 5):
        cond_close(outs[k].detach().cpu().numpy(), o32[k].detach().numpy(), o64[k].detach().numpy(), names[k])
    M = outs[0].shape[0]
    assert 2_000_000 < M < 4_000_000, M
    # the rasterization of the decoded chunk vs the oracle on a band (every output and gradient)
    xyz, _, col, op, scl, rot, _ = outs
    sub = SimpleNamespace(means=xyz.detach().cpu(), quats=rot.detach().cpu(), scales=scl.detach().cpu(),
                          opacities=op.detach().reshape(-1).cpu(), colors=col.detach().cpu(), viewmats=sc0.viewmats,
                          Ks=sc0.Ks, width=W, height=H)
    (max_tile, _, _), _, x = RP.run_3dgs(sub, "RGB+ED", torch.tensor([[0.1, 0.2, 0.3]]), rows=96, seed=9, sh=2)
    assert max_tile >= 256, max_tile
    # decode backward fed with the GPU raster's own gradients (the chain's upstream), vs autograd
    gr = x["grads"]
    ups = [gr["means"], gr["colors"], gr["opacities"].reshape(-1, 1), gr["scales"], gr["quats"]]
    torch.autograd.backward([xyz, col, op, scl, rot], [u.to(DEV) for u in ups])
    for o, ins, w in ((o32, i32, w32), (o64, i64, w64)):
        outs_r = [o[0], o[2], o[3], o[4], o[5]]
        torch.autograd.backward(outs_r, [u.cpu().to(o[0].dtype) for u in ups])
    for k in ("feat", "offset", "scaling"):
        cond_close(dins[k].grad[idx.long()].cpu().numpy(), i32[k].grad.numpy(), i64[k].grad.numpy(), "d_" + k)
    for k in ws:
        cond_close(dws[k].grad.cpu().numpy(), w32[k].grad.numpy(), w64[k].grad.numpy(), "d_" + k)
