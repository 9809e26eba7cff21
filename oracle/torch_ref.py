"""Dense, autograd-differentiated torch restatement of the rasterizer path.

TEST INFRASTRUCTURE ONLY.  It exists to check the hand-derived backward passes
of the C oracle (oracle/hgsr_oracle.c) and of the HIP kernels with an
*independent* implementation: every gradient here comes from torch autograd,
not from a hand-written VJP.  It evaluates every (pixel, Gaussian) pair densely,
so it is only usable on small problems (a few thousand pairs per pixel row).

Semantics restated (gsplat, as called at reference gaussian_renderer/render.py
:40-76): EWA projection with eps2d blur and the 0.3*tan_fov clamp; 2DGS ray-splat
with the 2.0 low-pass filter; per-tile culling by the 16x16 tile rectangle of each
Gaussian's 3-sigma (3.33 for 2DGS) radius; front-to-back compositing with the
alpha<1/255 skip, the 0.999 clamp and the T<=1e-4 exclusive stop.
"""
from __future__ import annotations

import math

import torch

SH_C0 = 0.28209479177387814
SH_C1 = 0.4886025119029199
SH_C2 = [1.0925484305920792, -1.0925484305920792, 0.31539156525252005, -1.0925484305920792,
         0.5462742152960396]
SH_C3 = [-0.5900435899266435, 2.890611442640554, -0.4570457994644658, 0.3731763325901154,
         -0.4570457994644658, 1.445305721320277, -0.5900435899266435]


def quat_to_rotmat(q):
    q = q / q.norm(dim=-1, keepdim=True)
    w, x, y, z = q.unbind(-1)
    return torch.stack([
        1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y),
        2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x),
        2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)], -1).reshape(q.shape[:-1] + (3, 3))


def project3d(means, quats, scales, viewmat, K, W, H, eps2d=0.3):
    """One camera. Returns means2d [N,2], conics [N,3], depths [N], radius [N] (float, no grad)."""
    R, t = viewmat[:3, :3], viewmat[:3, 3]
    mc = means @ R.T + t
    Rq = quat_to_rotmat(quats)
    M = Rq * scales[:, None, :]
    cov = M @ M.transpose(1, 2)
    covc = R @ cov @ R.T
    fx, fy, cx, cy = K[0, 0], K[1, 1], K[0, 2], K[1, 2]
    x, y, z = mc.unbind(-1)
    tanx, tany = 0.5 * W / fx, 0.5 * H / fy
    lxp, lxn = (W - cx) / fx + 0.3 * tanx, cx / fx + 0.3 * tanx
    lyp, lyn = (H - cy) / fy + 0.3 * tany, cy / fy + 0.3 * tany
    tx = z * torch.minimum(torch.maximum(x / z, -lxn), lxp)
    ty = z * torch.minimum(torch.maximum(y / z, -lyn), lyp)
    zero = torch.zeros_like(z)
    J = torch.stack([fx / z, zero, -fx * tx / z ** 2, zero, fy / z, -fy * ty / z ** 2], -1).reshape(-1, 2, 3)
    c2 = J @ covc @ J.transpose(1, 2)
    c2 = c2 + eps2d * torch.eye(2, dtype=c2.dtype)
    det = c2[:, 0, 0] * c2[:, 1, 1] - c2[:, 0, 1] * c2[:, 1, 0]
    conics = torch.stack([c2[:, 1, 1] / det, -c2[:, 0, 1] / det, c2[:, 0, 0] / det], -1)
    means2d = torch.stack([fx * x / z + cx, fy * y / z + cy], -1)
    with torch.no_grad():
        b = 0.5 * (c2[:, 0, 0] + c2[:, 1, 1])
        v1 = b + torch.sqrt(torch.clamp(b * b - det, min=0.01))
        radius = torch.ceil(3.0 * torch.sqrt(v1))
    return means2d, conics, z, radius


def project2d(means, quats, scales, viewmat, K):
    """One camera. Returns means2d [N,2], ray_transforms [N,3,3], depths [N], normals [N,3], radius."""
    R, t = viewmat[:3, :3], viewmat[:3, 3]
    mc = means @ R.T + t
    RRq = R @ quat_to_rotmat(quats)
    RS0 = RRq[:, :, 0] * scales[:, 0:1]
    RS1 = RRq[:, :, 1] * scales[:, 1:2]
    WH = torch.stack([RS0, RS1, mc], -1)  # columns
    M = K @ WH
    e = torch.tensor([1.0, 1.0, -1.0], dtype=means.dtype)
    dist = (e * M[:, 2] * M[:, 2]).sum(-1)
    mx = (e * M[:, 0] * M[:, 2]).sum(-1) / dist
    my = (e * M[:, 1] * M[:, 2]).sum(-1) / dist
    n = RRq[:, :, 2]
    with torch.no_grad():
        sgn = torch.where((-n * mc).sum(-1) > 0, 1.0, -1.0).to(means.dtype)
        tpx = (e * M[:, 0] * M[:, 0]).sum(-1) / dist
        tpy = (e * M[:, 1] * M[:, 1]).sum(-1) / dist
        he = torch.maximum(mx * mx - tpx, my * my - tpy)
        radius = torch.ceil(3.33 * torch.sqrt(torch.clamp(he, min=1e-4)))
    return torch.stack([mx, my], -1), M, mc[:, 2], n * sgn[:, None], radius


def sh_eval(deg, coeffs, dirs):
    """coeffs [N,K,3], dirs [N,3] (unnormalised) -> [N,3]; polynomials of utils/sh_utils.py."""
    d = dirs / dirs.norm(dim=-1, keepdim=True)
    x, y, z = d[:, 0:1], d[:, 1:2], d[:, 2:3]
    res = SH_C0 * coeffs[:, 0]
    if deg > 0:
        res = res - SH_C1 * y * coeffs[:, 1] + SH_C1 * z * coeffs[:, 2] - SH_C1 * x * coeffs[:, 3]
    if deg > 1:
        xx, yy, zz, xy, yz, xz = x * x, y * y, z * z, x * y, y * z, x * z
        res = (res + SH_C2[0] * xy * coeffs[:, 4] + SH_C2[1] * yz * coeffs[:, 5]
               + SH_C2[2] * (2 * zz - xx - yy) * coeffs[:, 6] + SH_C2[3] * xz * coeffs[:, 7]
               + SH_C2[4] * (xx - yy) * coeffs[:, 8])
    if deg > 2:
        res = (res + SH_C3[0] * y * (3 * xx - yy) * coeffs[:, 9] + SH_C3[1] * xy * z * coeffs[:, 10]
               + SH_C3[2] * y * (4 * zz - xx - yy) * coeffs[:, 11]
               + SH_C3[3] * z * (2 * zz - 3 * xx - 3 * yy) * coeffs[:, 12]
               + SH_C3[4] * x * (4 * zz - xx - yy) * coeffs[:, 13] + SH_C3[5] * z * (xx - yy) * coeffs[:, 14]
               + SH_C3[6] * x * (xx - 3 * yy) * coeffs[:, 15])
    return res


def _cover(means2d, radius, W, H, tile=16):
    """[P, N] bool: Gaussian's tile rectangle covers the pixel's tile (gsplat isect_tiles)."""
    tw, th = (W + tile - 1) // tile, (H + tile - 1) // tile
    m = means2d.detach().float()  # rect math in f32 like the kernels
    r = radius.detach().float()
    tr = r / tile
    txc, tyc = m[:, 0] / tile, m[:, 1] / tile
    x0 = torch.clamp(torch.floor(txc - tr), 0, tw)
    y0 = torch.clamp(torch.floor(tyc - tr), 0, th)
    x1 = torch.clamp(torch.ceil(txc + tr), 0, tw)
    y1 = torch.clamp(torch.ceil(tyc + tr), 0, th)
    jj, ii = torch.meshgrid(torch.arange(W), torch.arange(H), indexing="xy")
    ptx = (jj // tile).reshape(-1, 1).float()
    pty = (ii // tile).reshape(-1, 1).float()
    return (ptx >= x0) & (ptx < x1) & (pty >= y0) & (pty < y1)


def _composite(alpha, valid, feats, bgs, order):
    """alpha [P,N] (grad), valid [P,N] bool; feats list of [N,Dk]; returns outs, T_final."""
    alpha = alpha[:, order]
    valid = valid[:, order]
    with torch.no_grad():
        a0 = torch.where(valid, alpha, torch.zeros_like(alpha))
        t_after = torch.cumprod(1 - a0, dim=1)
        contrib = valid & (t_after > 1e-4)
    ac = torch.where(contrib, alpha, torch.zeros_like(alpha))
    one_m = 1 - ac
    t_before = torch.cat([torch.ones_like(one_m[:, :1]), torch.cumprod(one_m, 1)[:, :-1]], 1)
    w = ac * t_before
    T_final = torch.prod(one_m, 1)
    outs = []
    for f, bg in zip(feats, bgs):
        o = w @ f[order]
        if bg is not None:
            o = o + T_final[:, None] * bg[None]
        outs.append(o)
    return outs, T_final


def raster3d(means2d, conics, colors, opacities, depths, radius, W, H, bg=None):
    """Dense front-to-back compositing. Returns image [H,W,D], alpha [H,W,1]."""
    jj, ii = torch.meshgrid(torch.arange(W), torch.arange(H), indexing="xy")
    px = (jj.reshape(-1) + 0.5).to(means2d.dtype)
    py = (ii.reshape(-1) + 0.5).to(means2d.dtype)
    dx = means2d[None, :, 0] - px[:, None]
    dy = means2d[None, :, 1] - py[:, None]
    a, b, c = conics[:, 0], conics[:, 1], conics[:, 2]
    sigma = 0.5 * (a * dx * dx + c * dy * dy) + b * dx * dy
    alpha = torch.clamp(opacities[None] * torch.exp(-sigma), max=0.999)
    vis_g = (radius > 0)[None]
    valid = _cover(means2d, radius, W, H) & vis_g & (sigma >= 0) & (alpha >= 1.0 / 255.0)
    order = torch.argsort(depths.detach().float(), stable=True)
    (img,), T = _composite(alpha, valid, [colors], [bg], order)
    return img.reshape(H, W, -1), (1 - T).reshape(H, W, 1)


def raster2d(means2d, rt, colors, opacities, normals, depths, radius, W, H, bg=None):
    jj, ii = torch.meshgrid(torch.arange(W), torch.arange(H), indexing="xy")
    px = (jj.reshape(-1) + 0.5).to(means2d.dtype)[:, None, None]
    py = (ii.reshape(-1) + 0.5).to(means2d.dtype)[:, None, None]
    u, v, w = rt[None, :, 0], rt[None, :, 1], rt[None, :, 2]
    hu = px * w - u
    hv = py * w - v
    cr = torch.cross(hu, hv, dim=-1)
    sx = cr[..., 0] / cr[..., 2]
    sy = cr[..., 1] / cr[..., 2]
    g3 = sx * sx + sy * sy
    dx = means2d[None, :, 0] - px[..., 0]
    dy = means2d[None, :, 1] - py[..., 0]
    g2 = 2.0 * (dx * dx + dy * dy)
    sigma = 0.5 * torch.minimum(g3, g2)
    alpha = torch.clamp(opacities[None] * torch.exp(-sigma), max=0.999)
    valid = _cover(means2d, radius, W, H) & (radius > 0)[None] & (sigma >= 0) & (alpha >= 1.0 / 255.0)
    order = torch.argsort(depths.detach().float(), stable=True)
    (img, nrm), T = _composite(alpha, valid, [colors, normals], [bg, None], order)
    return img.reshape(H, W, -1), (1 - T).reshape(H, W, 1), nrm.reshape(H, W, 3)


def depth_to_normal(depths, camtoworlds, Ks, z_depth=True, origin=True, jitter=None):
    """The gsplat fork's depth_to_normal restated in torch (any device / dtype; autograd):
    unproject the depth map [C,H,W,1] through the pinhole rays, central differences along
    y (dx) and x (dy), normalize(cross(dx, dy)), zero one-pixel border -> [C,H,W,3].
    origin=False: the points without the camera origin, which cancels from every difference in
    exact arithmetic -- a second correct f32 evaluation order (the HIP kernel's), used by the
    parity tests as the element's other f32 error sample (checks.cond_close alt32).
    jitter ([C,H,W,3], f64 runs): relative perturbation of every unprojected point coordinate,
    e.g. uniform +-u -- the two roundings (ray direction, depth product) of an f32 unprojection -- so that f64 runs with
    several jitters sample the spread of correct f32 evaluations (k13_error_samples)."""
    import torch.nn.functional as F
    height, width = depths.shape[-3:-1]
    dev, dt = depths.device, depths.dtype
    x, y = torch.meshgrid(torch.arange(width, device=dev, dtype=dt), torch.arange(height, device=dev, dtype=dt),
                          indexing="xy")
    fx, fy, cx, cy = Ks[..., 0, 0], Ks[..., 1, 1], Ks[..., 0, 2], Ks[..., 1, 2]
    camera_dirs = F.pad(torch.stack([(x - cx[..., None, None] + 0.5) / fx[..., None, None],
                                     (y - cy[..., None, None] + 0.5) / fy[..., None, None]], dim=-1),
                        (0, 1), value=1.0)
    directions = torch.einsum("...ij,...hwj->...hwi", camtoworlds[..., :3, :3], camera_dirs)
    origins = camtoworlds[..., :3, -1]
    if not z_depth:
        directions = F.normalize(directions, dim=-1)
    points = origins[..., None, None, :] + depths * directions if origin else depths * directions
    if jitter is not None:
        points = points * (1 + jitter)
    dx = points[..., 2:, 1:-1, :] - points[..., :-2, 1:-1, :]
    dy = points[..., 1:-1, 2:, :] - points[..., 1:-1, :-2, :]
    normals = F.normalize(torch.cross(dx, dy, dim=-1), dim=-1)
    return F.pad(normals, (0, 0, 1, 1, 1, 1), value=0.0)


def k13_error_samples(depth, c2w, Ks, gup, z_depth=True, n_jitter=4, seed=0):
    """K13 (depth_to_normal) forward / backward error samples for the conditioning-aware checks.
    Returns (n64, g64, [(n, g), ...]): the f64 normals and depth gradient (loss sum(n * gup)),
    then correct f32-level evaluations of the same quantities -- the fork's f32 order, the f32
    order without the camera origin (the HIP kernel's), and n_jitter f64 runs whose unprojected
    points carry a random relative perturbation of +-u (u = 2^-24).  The per-element spread of
    these samples around f64 is what any correct f32 evaluation may show at that element."""
    import torch

    def run(dt, origin=True, jitter=None):
        d = depth.detach().cpu().to(dt).requires_grad_(True)
        n = depth_to_normal(d, c2w.cpu().to(dt), Ks.cpu().to(dt), z_depth=z_depth, origin=origin, jitter=jitter)
        (n * gup.cpu().to(dt)).sum().backward()
        return n.detach().double().numpy(), d.grad.double().numpy()

    n64, g64 = run(torch.float64)
    samples = [run(torch.float32), run(torch.float32, origin=False)]
    g = torch.Generator().manual_seed(seed)
    shape = tuple(depth.shape[:-1]) + (3,)
    for _ in range(n_jitter):
        j = (torch.rand(shape, generator=g, dtype=torch.float64) * 2 - 1) * 2.0 ** -24
        samples.append(run(torch.float64, jitter=j))
    return n64, g64, samples
