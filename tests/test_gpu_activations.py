"""GPU check of the fused 3DGS activations (horizongs_amd.activations): exp / sigmoid and their
vjps vs torch on the CPU (float rounding of expf), including a gradient arriving on only one
output."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def test_activate_fwd_bwd_vs_torch():
    from horizongs_amd.activations import activate
    g = torch.Generator().manual_seed(0)
    ls = torch.randn(10007, 3, generator=g) * 2 - 4
    lg = torch.randn(10007, generator=g) * 3
    a, b = ls.to(DEV).requires_grad_(True), lg.to(DEV).requires_grad_(True)
    s, o = activate(a, b)
    rs, ro = torch.exp(ls.double()), torch.sigmoid(lg.double())
    np.testing.assert_allclose(s.detach().cpu().numpy(), rs.numpy(), rtol=2e-7, atol=0)
    np.testing.assert_allclose(o.detach().cpu().numpy(), ro.numpy(), rtol=3e-7, atol=1e-30)
    vs, vo = torch.randn(10007, 3, generator=g), torch.randn(10007, generator=g)
    ((s * vs.to(DEV)).sum() + (o * vo.to(DEV)).sum()).backward()
    np.testing.assert_allclose(a.grad.cpu().numpy(), (vs.double() * rs).numpy(), rtol=1e-6, atol=1e-30)
    # torch's own fp32 sigmoid backward (the reference's) is v * (1 - y) * y on the fp32 output, whose
    # (1 - y) cancels near y = 1: compare with that formula on our fp32 output
    o32 = o.detach().cpu()
    np.testing.assert_allclose(b.grad.cpu().numpy(), (vo * (1 - o32) * o32).numpy(), rtol=2e-7, atol=1e-30)
    lb = lg.clone().requires_grad_(True)
    (torch.sigmoid(lb) * vo).sum().backward()
    np.testing.assert_allclose(b.grad.cpu().numpy(), lb.grad.numpy(), rtol=1e-5, atol=2e-7)
    # gradient on the scales only: the logits' vjp is exactly zero
    a.grad = b.grad = None
    s, o = activate(a, b)
    s.sum().backward()
    assert float(b.grad.abs().max()) == 0.0


def test_activate_unaligned_views():
    """Views starting off a 16-B boundary take the scalar path: same values as aligned ones."""
    from horizongs_amd.activations import activate
    g = torch.Generator().manual_seed(1)
    ls = (torch.randn(1001, 3, generator=g) - 3).to(DEV)
    lg = torch.randn(1001, generator=g).to(DEV)
    s0, o0 = activate(ls[1:].clone(), lg[1:].clone())
    s1, o1 = activate(ls[1:], lg[1:])  # 12-B / 4-B offset bases
    assert torch.equal(s0, s1) and torch.equal(o0, o1)
