"""TEST INFRASTRUCTURE ONLY (checker, never the product path).

numpy restatement of the reference optimizer step: torch.optim.Adam(l, lr=0.0, eps=1e-15)
(scene/lod_model.py:320) stepped at train.py:274-277, amsgrad / weight_decay / maximize
off.  torch's single-tensor / foreach Adam (torch/optim/adam.py) computes, per
parameter with its own step count t:
    exp_avg.lerp_(grad, 1 - beta1)                   # m + (1 - beta1) (g - m)
    exp_avg_sq.mul_(beta2).addcmul_(grad, grad, value=1 - beta2)
    step_size = lr / (1 - beta1 ** t); bc2_sqrt = (1 - beta2 ** t) ** 0.5
    denom = exp_avg_sq.sqrt() / bc2_sqrt + eps
    param.addcdiv_(exp_avg, denom, value=-step_size)
Pinned against torch.optim.Adam itself (the reference's optimizer, importable here) by
tests/test_optim.py."""
import numpy as np


def adam_step(p, g, m, v, lr, t, beta1=0.9, beta2=0.999, eps=1e-8):
    """One in-place step on float32 arrays; t is the 1-based step count."""
    f = np.float32
    w1 = f(1.0 - beta1)
    m += w1 * (g - m)
    v *= f(beta2)
    v += f(1.0 - beta2) * g * g
    step_size = f(lr / (1.0 - beta1 ** t))
    bc2 = f((1.0 - beta2 ** t) ** 0.5)
    denom = np.sqrt(v) / bc2 + f(eps)
    p += (-step_size) * (m / denom)
    return p, m, v
