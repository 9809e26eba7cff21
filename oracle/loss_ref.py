"""CPU restatement of the reference loss head (TEST INFRASTRUCTURE ONLY).

Only tests/ may import this module.  Follows reference utils/loss_utils.py:17-60 (l1_loss,
gaussian/create_window, _ssim with conv2d, zero padding, C1 = 0.01^2, C2 = 0.03^2) and the
scale / alpha regularisers and per-pixel normal / distortion / inverse-depth terms of
train.py:162-202, in torch ops so autograd gives the reference
gradients.  Pinned by tests/golden/losses.npz (l1 and ssim of the reference module itself).
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F


def _window(dtype):
    g = torch.tensor([math.exp(-(x - 5) ** 2 / float(2 * 1.5 ** 2)) for x in range(11)], dtype=dtype)
    g = g / g.sum()
    return (g[:, None] @ g[None, :])


def ssim(img1, img2):
    C = img1.shape[-3]
    w = _window(img1.dtype).expand(C, 1, 11, 11).contiguous()
    x, y = img1[None], img2[None]
    mu1 = F.conv2d(x, w, padding=5, groups=C)
    mu2 = F.conv2d(y, w, padding=5, groups=C)
    mu1_sq, mu2_sq, mu1_mu2 = mu1.pow(2), mu2.pow(2), mu1 * mu2
    s1 = F.conv2d(x * x, w, padding=5, groups=C) - mu1_sq
    s2 = F.conv2d(y * y, w, padding=5, groups=C) - mu2_sq
    s12 = F.conv2d(x * y, w, padding=5, groups=C) - mu1_mu2
    C1, C2 = 0.01 ** 2, 0.03 ** 2
    m = ((2 * mu1_mu2 + C1) * (2 * s12 + C2)) / ((mu1_sq + mu2_sq + C1) * (s1 + s2 + C2))
    return m.mean()


def loss(image, gt, mask=None, lambda_dssim=0.2, alpha=None, lambda_sky=0.0, lambda_ent=0.0, scaling=None,
         lambda_dreg=0.0, normals=None, nfd=None, lambda_normal=0.0, distort=None, lambda_dist=0.0, depth=None,
         mono=None, dmask=None, lambda_depth=0.0):
    """train.py:153-202: returns (loss, l1, ssim, sky, entropy, scale_reg, normal, distortion, inv_depth).
    normals / nfd [3,H,W], distort / depth / mono / dmask [H,W]; mask [H,W] or None."""
    mask_hw = mask
    if mask is not None:
        image = image * mask
        gt = gt * mask
    l1 = (image - gt).abs().mean()
    s = ssim(image, gt)
    total = (1 - lambda_dssim) * l1 + lambda_dssim * (1 - s)
    dreg = torch.zeros((), dtype=image.dtype)
    if scaling is not None and scaling.shape[0] > 0:  # train.py:163-167
        dreg = scaling.prod(dim=1).mean()
        total = total + lambda_dreg * dreg
    sky = ent = torch.zeros((), dtype=image.dtype)
    if alpha is not None:
        o = alpha.clamp(1e-6, 1 - 1e-6)
        skym = mask if mask is not None else torch.ones_like(alpha)
        sky = (-(1 - skym) * torch.log(1 - o)).mean()
        ent = -(o * torch.log(o)).mean()
        total = total + lambda_sky * sky + lambda_ent * ent
    z = torch.zeros((), dtype=image.dtype)
    mk = mask_hw if mask_hw is not None else torch.ones(image.shape[-2:], dtype=image.dtype)
    nrm = dist = dep = z
    if normals is not None:  # train.py:180-188 (alpha detached)
        a = alpha.detach() if alpha is not None else torch.ones_like(mk)
        err = 1 - (normals * (nfd * a[None])).sum(0)
        nrm = (err * mk).mean()
        total = total + lambda_normal * nrm
    if distort is not None:  # train.py:190-191
        dist = (distort * mk).mean()
        total = total + lambda_dist * dist
    if depth is not None:  # train.py:193-199
        # train.py:195 uses where(depth > 0, 1/depth, 0), whose backward is NaN at depth == 0
        # (0 * -inf); the inner where keeps that gradient 0, as the HIP kernel defines it
        pos = depth > 0.0
        inv = torch.where(pos, 1.0 / torch.where(pos, depth, torch.ones_like(depth)), torch.zeros_like(depth))
        dm = dmask if dmask is not None else torch.ones_like(depth)
        dep = torch.abs((inv - mono) * dm).mean()
        total = total + lambda_depth * dep
    return total, l1, s, sky, ent, dreg, nrm, dist, dep
