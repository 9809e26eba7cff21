"""Optimizer step (K17): the oracle restatement vs torch.optim.Adam on CPU (the
reference's optimizer, scene/lod_model.py:320), and the C-ABI argument checks.
GPU parity of the fused HIP Adam is in tests/test_gpu_optim.py."""
import ctypes as ct

import numpy as np
import torch

from oracle import optim_ref as OR


def test_oracle_matches_torch_adam():
    rng = np.random.default_rng(0)
    shapes = [(1000, 3), (257,), (64, 10, 3)]
    ps = [torch.tensor(rng.standard_normal(s), dtype=torch.float32, requires_grad=True) for s in shapes]
    lrs = [1e-3, 0.0, 5e-2]
    opt = torch.optim.Adam([{"params": [p], "lr": lr} for p, lr in zip(ps, lrs)], lr=0.0, eps=1e-15)
    mine = [(p.detach().numpy().copy(), np.zeros(s, np.float32), np.zeros(s, np.float32)) for p, s in zip(ps, shapes)]
    for t in range(1, 6):
        gs = [rng.standard_normal(s).astype(np.float32) * (10.0 ** -t) for s in shapes]
        for p, g in zip(ps, gs):
            p.grad = torch.from_numpy(g.copy())
        opt.step()
        for (q, m, v), g, lr in zip(mine, gs, lrs):
            OR.adam_step(q, g, m, v, lr, t, eps=1e-15)
        for p, (q, m, v) in zip(ps, mine):
            # lerp / subtraction cancel: absolute part scaled to each array's magnitude
            st = opt.state[p]
            for a, b in ((q, p.detach().numpy()), (m, st["exp_avg"].numpy()), (v, st["exp_avg_sq"].numpy())):
                np.testing.assert_allclose(a, b, rtol=1e-6, atol=1e-6 * float(np.abs(b).max()))


def test_abi_rejects_bad_descriptors():
    from horizongs_amd import _native
    from horizongs_amd.optim import _AdamTensor
    lib = _native.lib()
    d = (_AdamTensor * 1)(_AdamTensor(None, 8, None, None, 10, 1e-3, 1))
    assert lib.hgsr_adam_step(1, ct.cast(d, ct.c_void_p), 0.9, 0.999, 1e-15, None) == -1
    assert b"null pointer" in lib.hgsr_last_error()
    d = (_AdamTensor * 1)(_AdamTensor(8, 8, 8, 8, 10, 1e-3, 0))
    assert lib.hgsr_adam_step(1, ct.cast(d, ct.c_void_p), 0.9, 0.999, 1e-15, None) == -1
    assert b"step" in lib.hgsr_last_error()
    assert lib.hgsr_adam_step(1, ct.cast(d, ct.c_void_p), 1.0, 0.999, 1e-15, None) == -1
    # no tensors / no gradients: nothing to launch
    assert lib.hgsr_adam_step(0, None, 0.9, 0.999, 1e-15, None) == 0


def test_optimizer_rejects_unsupported_options():
    import pytest
    from horizongs_amd.optim import Adam
    p = torch.zeros(3, requires_grad=True)
    for kw in (dict(amsgrad=True), dict(weight_decay=0.1), dict(maximize=True)):
        with pytest.raises(NotImplementedError):
            Adam([p], **kw)
