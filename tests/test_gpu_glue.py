"""The torch glue folded into the kernels (DESIGN.md §3 "glue"), checked against the unfolded
composition it replaces:

* the loss head's scale-regulariser gradient handed to the projection backward
  (gsplat_api.GradSink; reference train.py:163-167 regularises the same scales the rasterizer
  projects) instead of autograd's separate sum -- bit-identical gradients (the kernel performs
  the same single f32 addition);
* rasterization_2dgs' world-frame normals and K13 (render_normals_from_depth) inside the fused
  raster Function, their gradients entering its backward kernel, instead of separate rotate /
  depth_to_normal launches and the slice-backward fill + copy + sum of the depth channel
  (reference gaussian_renderer/render.py:62-76, train.py:180-188);
* rasterization()'s SH colour step: its means gradient (dirs = means - campos) handed to the
  projection backward's kernel in the same way (v_means_in)."""
import numpy as np
import pytest
import torch

from horizongs_amd import gsplat_api as G
from horizongs_amd.activations import activate
from horizongs_amd.loss import fused_loss
from horizongs_amd.synthetic import make_scene

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _train_step(sc, gs, twice=False):
    means, quats, cols = (t.to(DEV).clone().requires_grad_(True) for t in (sc.means, sc.quats, sc.colors))
    log_s = torch.log(sc.scales).to(DEV).requires_grad_(True)
    logit = torch.logit(sc.opacities).to(DEV).requires_grad_(True)
    scales, opac = activate(log_s, logit)
    W, H = sc.width, sc.height
    vm, K = sc.viewmats.to(DEV), sc.Ks.to(DEV)
    bg = torch.zeros(1, 3, device=DEV)
    gt = torch.rand(3, H, W, generator=torch.Generator().manual_seed(3)).to(DEV)
    if gs == "3d":
        out, alpha, meta = G.rasterization(means, quats, scales, opac, cols, vm, K, W, H, packed=False,
                                           backgrounds=bg, render_mode="RGB+ED")
        aux = {}
    else:
        (out, alpha, nrm, nfd, _, _), meta = G.rasterization_2dgs(means, quats, scales, opac, cols, vm, K, W, H,
                                                                   packed=False, backgrounds=bg, render_mode="RGB+ED")
        aux = dict(normals=nrm.reshape(H, W, 3).permute(2, 0, 1), normals_from_depth=nfd.reshape(H, W, 3).permute(2, 0, 1),
                   lambda_normal=0.05)
    img = out.reshape(H, W, -1).permute(2, 0, 1)
    loss = fused_loss(img, gt, None, 0.2, alpha.reshape(H, W), 0.05, 0.05, scales, 0.01, **aux)[0]
    loss.backward(retain_graph=twice)
    grads = [t.grad.clone() for t in (means, quats, log_s, logit, cols)]
    if twice:  # a second backward through the same graph: the sink is closed, autograd sums again
        for t in (means, quats, log_s, logit, cols):
            t.grad = None
        loss.backward()
        grads += [t.grad.clone() for t in (means, quats, log_s, logit, cols)]
    torch.cuda.synchronize()
    return [g.cpu().numpy() for g in grads]


@pytest.mark.parametrize("gs", ["3d", "2d"])
def test_scale_reg_grad_sink_matches_autograd_sum(gs, monkeypatch):
    sc = make_scene(6000, 160, 120, seed=21, scale_range=(0.01, 0.05), depth_range=(2.0, 6.0))
    monkeypatch.setattr(G, "_GRAD_SINK", False)
    ref = _train_step(sc, gs)
    monkeypatch.setattr(G, "_GRAD_SINK", True)
    got = _train_step(sc, gs, twice=True)
    # the log-scale gradient is the only one the hand-off touches: the same one f32 addition
    # (in the kernel instead of by autograd's add)
    for i, (a, b) in enumerate(zip(got[:5], ref)):
        np.testing.assert_allclose(a, b, rtol=1e-4, atol=1e-5 * float(np.abs(b).max()), err_msg=f"grad {i}")
    for i, (a, b) in enumerate(zip(got[5:], ref)):  # second backward: the same gradients again
        np.testing.assert_allclose(a, b, rtol=1e-4, atol=1e-5 * float(np.abs(b).max()), err_msg=f"2nd grad {i}")
    # the raster backward is deterministic: a second backward through the same graph (a fresh
    # workspace, the gradient slots' piece count cleared again) repeats every gradient the sink
    # does not touch bit for bit
    for i in (0, 1, 3, 4):
        assert np.array_equal(got[i], got[5 + i]), f"grad {i}: the second backward differs"
    assert np.abs(got[2]).max() > 0


def _sh_step(sc, twice=False):
    means, quats, scales, opac, coeffs = (t.to(DEV).clone().requires_grad_(True) for t in (
        sc.means, sc.quats, sc.scales, sc.opacities, sc.colors))
    out, alpha, _ = G.rasterization(means, quats, scales, opac, coeffs, sc.viewmats.to(DEV), sc.Ks.to(DEV),
                                    sc.width, sc.height, packed=False, sh_degree=2, render_mode="RGB+ED")
    g = torch.Generator().manual_seed(9)
    ups = [torch.randn(t.shape, generator=g).to(DEV) for t in (out, alpha)]
    loss = (out * ups[0]).sum() + (alpha * ups[1]).sum()
    loss.backward(retain_graph=twice)
    ts = (means, quats, scales, opac, coeffs)
    grads = [t.grad.clone() for t in ts]
    if twice:  # the sink is closed: the SH means gradient returns through autograd's sum
        for t in ts:
            t.grad = None
        loss.backward()
        grads += [t.grad.clone() for t in ts]
    torch.cuda.synchronize()
    return [x.cpu().numpy() for x in grads]


def test_sh_means_grad_sink_matches_autograd_sum(monkeypatch):
    """The SH colour step's means gradient (view directions) handed to the projection backward
    (v_means_in) instead of autograd's add: the same single f32 addition of the same two terms,
    so every gradient -- the means' included -- is bit-identical, in both backwards."""
    sc = make_scene(6000, 160, 120, seed=31, scale_range=(0.01, 0.05), depth_range=(2.0, 6.0), sh_degree=2)
    monkeypatch.setattr(G, "_GRAD_SINK", False)
    ref = _sh_step(sc)
    monkeypatch.setattr(G, "_GRAD_SINK", True)
    got = _sh_step(sc, twice=True)
    for i in range(5):
        assert np.array_equal(got[i], ref[i]), f"grad {i}"
        assert np.array_equal(got[5 + i], ref[i]), f"2nd grad {i}"
    assert np.abs(got[0]).max() > 0


def _render_2dgs(sc, seed):
    means, quats, scales, opac, cols = (t.to(DEV).clone().requires_grad_(True) for t in (
        sc.means, sc.quats, sc.scales, sc.opacities, sc.colors))
    th = 0.3
    vm = torch.eye(4)
    vm[:3, :3] = torch.tensor([[np.cos(th), 0, np.sin(th)], [0, 1, 0], [-np.sin(th), 0, np.cos(th)]],
                              dtype=torch.float32)
    vm[:3, 3] = torch.tensor([0.3, -0.1, 0.5])  # a rotated camera: world frame != camera frame
    vm = vm[None].to(DEV)
    (out, alpha, nrm, nfd, _, _), meta = G.rasterization_2dgs(means, quats, scales, opac, cols, vm, sc.Ks.to(DEV),
                                                               sc.width, sc.height, packed=False,
                                                               render_mode="RGB+ED")
    g = torch.Generator().manual_seed(seed)
    ups = [torch.randn(t.shape, generator=g).to(DEV) for t in (out, alpha, nrm, nfd)]
    sum((t * u).sum() for t, u in zip((out, alpha, nrm, nfd), ups)).backward()
    torch.cuda.synchronize()
    return ([t.detach().cpu().numpy() for t in (out, alpha, nrm, nfd)],
            [t.grad.cpu().numpy() for t in (means, quats, scales, opac, cols)])


def test_2dgs_fused_frame_matches_separate_kernels(monkeypatch):
    sc = make_scene(8000, 192, 144, seed=23, scale_range=(0.01, 0.06), depth_range=(2.0, 6.0))
    sc.means[:, 2] += 1.0
    monkeypatch.setattr(G, "_FUSE_FRAME", False)
    ref_out, ref_g = _render_2dgs(sc, 5)
    monkeypatch.setattr(G, "_FUSE_FRAME", True)
    out, gr = _render_2dgs(sc, 5)
    np.testing.assert_array_equal(out[0], ref_out[0])  # colours + depth: the same kernels
    np.testing.assert_array_equal(out[1], ref_out[1])
    np.testing.assert_allclose(out[2], ref_out[2], rtol=1e-5, atol=1e-6)  # R^T n in the raster kernel
    np.testing.assert_array_equal(out[3], ref_out[3])  # K13 on the same depth channel
    assert np.abs(out[2]).max() > 0.1 and np.abs(out[3]).max() > 0.1
    for i, (a, b) in enumerate(zip(gr, ref_g)):
        np.testing.assert_allclose(a, b, rtol=1e-4, atol=1e-5 * float(np.abs(b).max()), err_msg=f"grad {i}")


def test_grad_sink_second_projection_falls_back_to_autograd():
    """A second projection of the same scales before the first one's backward (a render whose
    graph is never backpropagated) closes the open sink: the loss then returns its scale
    gradient through autograd, so no gradient lands in an orphaned sink."""
    sc = make_scene(6000, 160, 120, seed=21, scale_range=(0.01, 0.05), depth_range=(2.0, 6.0))
    ref = _train_step(sc, "3d")
    means, quats, cols = (t.to(DEV).clone().requires_grad_(True) for t in (sc.means, sc.quats, sc.colors))
    log_s = torch.log(sc.scales).to(DEV).requires_grad_(True)
    logit = torch.logit(sc.opacities).to(DEV).requires_grad_(True)
    scales, opac = activate(log_s, logit)
    W, H = sc.width, sc.height
    vm, K = sc.viewmats.to(DEV), sc.Ks.to(DEV)
    bg = torch.zeros(1, 3, device=DEV)
    gt = torch.rand(3, H, W, generator=torch.Generator().manual_seed(3)).to(DEV)
    out, alpha, _ = G.rasterization(means, quats, scales, opac, cols, vm, K, W, H, packed=False, backgrounds=bg,
                                    render_mode="RGB+ED")
    G.rasterization(means, quats, scales, opac, cols, vm, K, W, H, packed=False, backgrounds=bg,
                    render_mode="RGB+ED")  # an orphaned render of the same scales, never backpropagated
    img = out.reshape(H, W, -1).permute(2, 0, 1)
    fused_loss(img, gt, None, 0.2, alpha.reshape(H, W), 0.05, 0.05, scales, 0.01)[0].backward()
    got = [t.grad.cpu().numpy() for t in (means, quats, log_s, logit, cols)]
    for i, (a, b) in enumerate(zip(got, ref)):
        np.testing.assert_allclose(a, b, rtol=1e-4, atol=1e-5 * float(np.abs(b).max()), err_msg=f"grad {i}")
