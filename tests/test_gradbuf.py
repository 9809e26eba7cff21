"""Gradient destinations (horizongs_amd/gradbuf.py): a backward that takes its output buffer
from the table writes the gradient where multigpu.ShardedAdamDDP reduce-scatters it, and
autograd adopts that buffer as `.grad` (no copy)."""
import torch

from horizongs_amd import gradbuf


class _Twice(torch.autograd.Function):
    """y = 2 x with the gradient buffer taken the way the projection backward takes it."""

    @staticmethod
    def forward(ctx, x):
        ctx.save_for_backward(x)
        return 2 * x

    @staticmethod
    def backward(ctx, g):
        (x,) = ctx.saved_tensors
        out = gradbuf.alloc(x)
        torch.mul(g, 2.0, out=out)
        return out


def test_destination_is_adopted_as_grad():
    flat = torch.zeros(16)
    p = torch.randn(3, 4, requires_grad=True)
    gradbuf.set_dest(p, flat[2:14].view(3, 4))  # no other reference: autograd may adopt it
    _Twice.apply(p).sum().backward()
    assert p.grad.data_ptr() == flat[2:].data_ptr()  # adopted, not copied
    assert torch.equal(flat[2:14], torch.full((12,), 2.0))
    assert flat[:2].abs().sum() == 0 and flat[14:].abs().sum() == 0
    gradbuf.clear()


def test_destination_taken_once_second_use_accumulates():
    flat = torch.zeros(12)
    p = torch.randn(3, 4, requires_grad=True)
    gradbuf.set_dest(p, flat.view(3, 4))
    (_Twice.apply(p).sum() + 3 * _Twice.apply(p).sum()).backward()
    assert torch.equal(p.grad, torch.full((3, 4), 8.0))
    # autograd sums the two uses (in place in the destination or not); either way the DDP hook
    # sees a .grad that is not the destination whenever it must copy
    assert p.grad.data_ptr() == flat.data_ptr() or not torch.equal(flat, p.grad.reshape(-1))
    gradbuf.clear()


def test_no_destination_or_mismatch_gives_fresh_buffer():
    p = torch.randn(5, 3, requires_grad=True)
    _Twice.apply(p).sum().backward()
    assert torch.equal(p.grad, torch.full((5, 3), 2.0))
    q = torch.randn(5, 3)
    gradbuf._DEST[gradbuf.key(q)] = torch.zeros(15)  # wrong shape: ignored
    out = gradbuf.alloc(q)
    assert out.shape == q.shape and not gradbuf._DEST
    try:
        gradbuf.set_dest(q, torch.zeros(3, 5))
        raise AssertionError("a mis-shaped destination must be refused")
    except ValueError:
        pass
