"""Seeded synthetic Gaussian scenes.

There is no dataset or checkpoint in this environment, so every benchmark and
parity test runs on these scenes.  Inputs are generated on the host with a
torch.Generator so CPU and GPU see identical bits.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import torch


@dataclass
class Scene:
    means: torch.Tensor      # [N,3]
    quats: torch.Tensor      # [N,4] (w,x,y,z), unnormalised
    scales: torch.Tensor     # [N,3]
    opacities: torch.Tensor  # [N]
    colors: torch.Tensor     # [N,3] or SH [N,K,3]
    viewmats: torch.Tensor   # [1,4,4] world->camera
    Ks: torch.Tensor         # [1,3,3]
    width: int
    height: int
    backgrounds: torch.Tensor  # [1,3]
    sh_degree: int | None = None

    def to(self, device):
        kw = {k: (v.to(device) if isinstance(v, torch.Tensor) else v) for k, v in self.__dict__.items()}
        return Scene(**kw)


def make_scene(n: int, width: int, height: int, seed: int = 0,
               scale_range=(0.002, 0.012), depth_range=(2.0, 10.0), fov_deg: float = 60.0,
               sh_degree: int | None = None, sh_std: float = 0.3, opacity_range=(0.05, 0.95),
               viewmat: torch.Tensor | None = None) -> Scene:
    """c1/c2 spec: pixel-uniform centres, depth ~ U[2,10], log-uniform scales.

    fx = fy = (W/2)/tan(fov/2) (fov 60 deg: 221.70 at 256 px, 1662.77 at 1920 px),
    cx = W/2, cy = H/2, viewmat = I unless given.
    """
    g = torch.Generator().manual_seed(seed)
    fx = 0.5 * width / math.tan(math.radians(fov_deg) * 0.5)
    fy = fx
    cx, cy = 0.5 * width, 0.5 * height
    u = torch.rand(n, generator=g) * width
    v = torch.rand(n, generator=g) * height
    z = depth_range[0] + torch.rand(n, generator=g) * (depth_range[1] - depth_range[0])
    x = (u - cx) * z / fx
    y = (v - cy) * z / fy
    means = torch.stack([x, y, z], -1)
    quats = torch.randn(n, 4, generator=g)
    quats = quats / quats.norm(dim=-1, keepdim=True)
    lo, hi = math.log(scale_range[0]), math.log(scale_range[1])
    scales = torch.exp(lo + torch.rand(n, 3, generator=g) * (hi - lo))
    opacities = opacity_range[0] + torch.rand(n, generator=g) * (opacity_range[1] - opacity_range[0])
    if sh_degree is None:
        colors = torch.rand(n, 3, generator=g)
    else:
        K = (sh_degree + 1) ** 2
        colors = torch.randn(n, K, 3, generator=g) * sh_std
    if viewmat is None:
        viewmat = torch.eye(4)
    Ks = torch.tensor([[fx, 0.0, cx], [0.0, fy, cy], [0.0, 0.0, 1.0]])
    return Scene(means.float(), quats.float(), scales.float(), opacities.float(), colors.float(),
                 viewmat[None].float(), Ks[None].float(), width, height, torch.zeros(1, 3),
                 sh_degree)


def c1(seed: int = 0) -> Scene:
    """c1 plumbing: 1k Gaussians, 256x256."""
    return make_scene(1000, 256, 256, seed)


def c2(seed: int = 0, n: int = 2_000_000) -> Scene:
    """c2 north-star: 2M Gaussians at 1920x1080."""
    return make_scene(n, 1920, 1080, seed)


def look_at(eye, target, up=(0.0, -1.0, 0.0)) -> torch.Tensor:
    """world -> camera viewmat [4,4] (OpenCV axes as the synthetic scenes: x right, y down, z forward)
    of a camera at `eye` looking at `target`."""
    eye, target, up = (torch.tensor(v, dtype=torch.float64) for v in (eye, target, up))
    z = target - eye
    z = z / z.norm()
    x = torch.linalg.cross(-up, z)
    x = x / x.norm()
    y = torch.linalg.cross(z, x)
    R = torch.stack([x, y, z])  # rows: camera axes in world coordinates
    vm = torch.eye(4, dtype=torch.float64)
    vm[:3, :3] = R
    vm[:3, 3] = -R @ eye
    return vm.float()


def camera_set(n_views: int = 16, seed: int = 0, centre=(0.0, 0.0, 6.0), radius: float = 6.0) -> torch.Tensor:
    """A seeded training-camera set around a synthetic scene: [n_views, 4, 4] viewmats.

    Horizon-GS trains one camera per iteration, picked at random from aerial and street views
    (reference train.py:133-148), whose intersection counts differ widely.  View 0 is the scene's
    own identity camera; the others sit on a ring around the scene centre (yaw within +-25 deg),
    at elevations within +-15 deg, at 0.5-1.5x the identity camera's distance -- close "street"
    views (fewer Gaussians in view, larger footprints) to far "aerial" ones (everything in view,
    small footprints)."""
    g = torch.Generator().manual_seed(1000 + seed)
    c = torch.tensor(centre, dtype=torch.float64)
    views = [torch.eye(4)]
    for i in range(1, n_views):
        yaw = math.radians(float(torch.rand(1, generator=g)) * 50.0 - 25.0)
        pitch = math.radians(float(torch.rand(1, generator=g)) * 30.0 - 15.0)
        dist = radius * (0.5 + 1.0 * (i - 1) / max(n_views - 2, 1))  # spread over the range, shuffled below
        d = torch.tensor([math.sin(yaw) * math.cos(pitch), math.sin(pitch), -math.cos(yaw) * math.cos(pitch)],
                         dtype=torch.float64)
        views.append(look_at((c + dist * d).tolist(), c.tolist()))
    perm = [0] + (1 + torch.randperm(n_views - 1, generator=g)).tolist()
    return torch.stack([views[i] for i in perm])
