"""GPU parity of the fused loss (horizongs_amd.loss) -- SURVEY 8(f) rank 2.

Values against tests/golden/losses.npz (the reference's own l1 / ssim) and the oracle
restatement oracle/loss_ref.py; gradients of every output against torch autograd of the
oracle in fp64 (fp32 for the conditioning-aware check).  Tolerance 1e-5 abs / 1e-4 rel."""
import os

import numpy as np
import pytest
import torch

from oracle import loss_ref as L
from oracle.checks import cond_close

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")


def test_loss_matches_reference_golden():
    from horizongs_amd.loss import fused_loss
    g = np.load(os.path.join(os.path.dirname(__file__), "golden", "losses.npz"))
    img, gt = torch.from_numpy(g["img"]).to(DEV), torch.from_numpy(g["gt"]).to(DEV)
    loss, l1, s = fused_loss(img, gt, lambda_dssim=0.2)[:3]
    assert abs(float(l1) - float(g["l1"])) <= 1e-6
    assert abs(float(s) - float(g["ssim"])) <= 1e-5
    assert abs(float(loss) - (0.8 * float(g["l1"]) + 0.2 * (1 - float(g["ssim"])))) <= 1e-5


@pytest.mark.parametrize("H,W,masked,alpha_terms,n_sc", [(64, 80, False, False, 0), (67, 93, True, True, 1000),
                                                         (1080 // 4, 1920 // 4, True, True, 300007),
                                                         (40, 50, False, True, 0)])
def test_loss_gradients(H, W, masked, alpha_terms, n_sc):
    """n_sc = 0 with a scaling tensor is the reference's empty-model branch (train.py:163-166)."""
    from horizongs_amd.loss import fused_loss
    gen = torch.Generator().manual_seed(H * 7 + W)
    img = torch.rand(3, H, W, generator=gen)
    gt = (img + 0.1 * torch.randn(3, H, W, generator=gen)).clamp(0, 1)
    mask = (torch.rand(H, W, generator=gen) > 0.2).float() if masked else None
    alpha = torch.rand(H, W, generator=gen) if alpha_terms else None
    scaling = (0.02 * torch.rand(n_sc, 3, generator=gen)) if (n_sc or alpha_terms) else None
    lam = dict(lambda_dssim=0.2, lambda_sky=0.05 if alpha_terms else 0.0, lambda_ent=0.01 if alpha_terms else 0.0,
               lambda_dreg=0.01 if scaling is not None else 0.0)
    ups = torch.randn(9, generator=gen)

    def ref(dtype):
        i = img.to(dtype).clone().requires_grad_(True)
        a = alpha.to(dtype).clone().requires_grad_(True) if alpha is not None else None
        sc = scaling.to(dtype).clone().requires_grad_(True) if scaling is not None else None
        outs = L.loss(i, gt.to(dtype), None if mask is None else mask.to(dtype), alpha=a, scaling=sc, **lam)
        sum(o * u for o, u in zip(outs, ups.to(dtype))).backward()
        g_sc = sc.grad.numpy() if (sc is not None and sc.grad is not None) else None
        return [o.detach().numpy() for o in outs], i.grad.numpy(), (a.grad.numpy() if a is not None else None), g_sc

    o32, gi32, ga32, gs32 = ref(torch.float32)
    o64, gi64, ga64, gs64 = ref(torch.float64)
    i = img.to(DEV).clone().requires_grad_(True)
    a = alpha.to(DEV).clone().requires_grad_(True) if alpha is not None else None
    sc = scaling.to(DEV).clone().requires_grad_(True) if scaling is not None else None
    outs = fused_loss(i, gt.to(DEV), None if mask is None else mask.to(DEV), lam["lambda_dssim"], a,
                      lam["lambda_sky"], lam["lambda_ent"], sc, lam["lambda_dreg"])
    assert len(outs) == 9
    for o, r32, r64, name in zip(outs, o32, o64, ("loss", "l1", "ssim", "sky", "entropy", "scale_reg")):
        cond_close(o.detach().cpu().numpy(), r32, r64, name)
    sum(o * u for o, u in zip(outs, ups.to(DEV))).backward()
    cond_close(i.grad.cpu().numpy(), gi32, gi64, "d_image")
    if a is not None:
        cond_close(a.grad.cpu().numpy(), ga32, ga64, "d_alpha")
    if gs32 is not None:
        cond_close(sc.grad.cpu().numpy(), gs32, gs64, "d_scaling")


@pytest.mark.parametrize("extra", [0, 1])
def test_loss_channels_last_view(extra):
    """render_colors[0].permute(2, 0, 1) of a channels-last [H,W,3+extra] render (render.py:81-95)
    is read in place: outputs and the RGB gradient are bit-identical to the contiguous CHW
    call, and trailing channels (RGB+ED depth) get an exact zero gradient."""
    from horizongs_amd.loss import fused_loss
    H, W = 75, 131
    gen = torch.Generator().manual_seed(31 + extra)
    hwc = torch.rand(H, W, 3 + extra, generator=gen).to(DEV)
    gt = torch.rand(3, H, W, generator=gen).to(DEV)
    mask = (torch.rand(H, W, generator=gen) > 0.3).float().to(DEV)
    alpha = torch.rand(H, W, generator=gen).to(DEV)
    ups = torch.randn(9, generator=gen).to(DEV)

    a = hwc.clone().requires_grad_(True)
    outs = fused_loss(a.permute(2, 0, 1), gt, mask, 0.2, alpha, 0.05, 0.01)
    sum(o * u for o, u in zip(outs, ups)).backward()
    b = hwc[..., :3].permute(2, 0, 1).contiguous().requires_grad_(True)
    ref = fused_loss(b, gt, mask, 0.2, alpha, 0.05, 0.01)
    sum(o * u for o, u in zip(ref, ups)).backward()
    for o, r in zip(outs, ref):
        assert torch.equal(o, r)
    assert a.grad.is_contiguous()
    assert torch.equal(a.grad[..., :3].permute(2, 0, 1), b.grad)
    if extra:
        assert torch.equal(a.grad[..., 3:], torch.zeros_like(a.grad[..., 3:]))


@pytest.mark.parametrize("H,W,masked", [(48, 70, True), (1080 // 4, 1920 // 4, False)])
def test_loss_aux_terms(H, W, masked):
    """Normal consistency, distortion and inverse-depth L1 (train.py:180-199) on channels-last
    render views, every gradient vs fp64 / fp32 autograd of the oracle."""
    from horizongs_amd.loss import fused_loss
    gen = torch.Generator().manual_seed(H + 3 * W)
    img = torch.rand(3, H, W, generator=gen)
    gt = torch.rand(3, H, W, generator=gen)
    mask = (torch.rand(H, W, generator=gen) > 0.25).float() if masked else None
    alpha = torch.rand(H, W, generator=gen)
    nrm = torch.nn.functional.normalize(torch.randn(H, W, 3, generator=gen), dim=-1)
    nfd = torch.nn.functional.normalize(torch.randn(H, W, 3, generator=gen), dim=-1)
    dist = torch.rand(H, W, 1, generator=gen) * 0.1
    depth = torch.where(torch.rand(H, W, generator=gen) > 0.1, 1.0 + 9.0 * torch.rand(H, W, generator=gen),
                        torch.zeros(H, W))
    mono = 1.0 / (1.0 + 9.0 * torch.rand(H, W, generator=gen))
    dmask = (torch.rand(H, W, generator=gen) > 0.2).float()
    lam = dict(lambda_normal=0.05, lambda_dist=100.0, lambda_depth=0.3)
    ups = torch.randn(9, generator=gen)

    def ref(dtype):
        t = {k: v.to(dtype).clone().requires_grad_(True) for k, v in
             dict(img=img, alpha=alpha, nrm=nrm, nfd=nfd, dist=dist, depth=depth).items()}
        outs = L.loss(t["img"], gt.to(dtype), None if mask is None else mask.to(dtype), 0.2, t["alpha"], 0.0, 0.0,
                      None, 0.0, t["nrm"].permute(2, 0, 1), t["nfd"].permute(2, 0, 1), lam["lambda_normal"],
                      t["dist"][..., 0], lam["lambda_dist"], t["depth"], mono.to(dtype), dmask.to(dtype),
                      lam["lambda_depth"])
        sum(o * u for o, u in zip(outs, ups.to(dtype))).backward()
        return [o.detach().numpy() for o in outs], {k: (v.grad.numpy() if v.grad is not None else None)
                                                    for k, v in t.items()}

    o32, g32 = ref(torch.float32)
    o64, g64 = ref(torch.float64)
    d = {k: v.to(DEV).clone().requires_grad_(True) for k, v in
         dict(img=img, alpha=alpha, nrm=nrm, nfd=nfd, dist=dist, depth=depth).items()}
    outs = fused_loss(d["img"], gt.to(DEV), None if mask is None else mask.to(DEV), 0.2, d["alpha"],
                      normals=d["nrm"].permute(2, 0, 1), normals_from_depth=d["nfd"].permute(2, 0, 1),
                      distort=d["dist"], depth=d["depth"], mono_invdepth=mono.to(DEV), depth_mask=dmask.to(DEV),
                      **lam)
    names = ("loss", "l1", "ssim", "sky", "entropy", "scale_reg", "normal", "distortion", "inv_depth")
    for o, r32, r64, name in zip(outs, o32, o64, names):
        cond_close(o.detach().cpu().numpy(), r32, r64, name)
    sum(o * u for o, u in zip(outs, ups.to(DEV))).backward()
    for k in ("img", "alpha", "nrm", "nfd", "dist", "depth"):
        assert d[k].grad is not None, k
        if g32[k] is None:  # alpha only reaches the normal term, detached: zero gradient
            assert torch.count_nonzero(d[k].grad) == 0, k
            continue
        cond_close(d[k].grad.cpu().numpy(), g32[k], g64[k], "d_" + k)
