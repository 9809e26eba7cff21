"""Generate golden vectors by importing the reference's own Python on CPU.

Run in the build container only (the reference does not exist on the GPU box):
    python scripts/make_golden.py
Writes small seeded .npz fixtures into tests/golden/.  The fixtures are data
(inputs and the reference's outputs); no reference source is copied.

Pinned here:
  * utils/sh_utils.py:57-112 eval_sh (SH basis constants + sign conventions), deg 0-3
  * scene/lod_model.py:286-290 set_anchor_mask + scene/basic_model.py:192-210 map_to_int_level
  * scene/basic_model.py:297-371 generate_neural_gaussians (anchor -> Gaussian decode),
    RGB (view_dim=3) and SH2 (view_dim=0) variants, MLP shapes of scene/lod_model.py:67-84
  * utils/loss_utils.py:17-60 l1_loss / ssim and utils/image_utils.py:18-20 psnr
  * scene/basic_model.py:96-144 training_statis, :179-190 get_remove_duplicates and
    scene/lod_model.py:236-249 weed_out (their device="cuda" allocations mapped to the CPU)
  * scene/lod_model.py:487-596 anchor_growing (fine stage), with torch_scatter.scatter_max
    (absent third-party dependency, torch_scatter 2.x) restated in _scatter_max_restated
"""
from __future__ import annotations

import contextlib
import os
import sys
import types

import numpy as np
import torch

REF = "/root/reference"
OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden")


class _Subscriptable:
    def __class_getitem__(cls, item):
        return cls


def _stub_modules():
    """Stub third-party imports the reference pulls in but the decode never touches."""
    for name in ["torch_scatter", "plyfile", "jaxtyping", "cv2", "kornia", "laspy", "colorama",
                 "simple_knn", "simple_knn._C"]:
        if name not in sys.modules:
            m = types.ModuleType(name)
            m.scatter_max = None
            m.PlyData = m.PlyElement = object
            m.Float = m.Int = m.Shaped = _Subscriptable
            m.Fore = m.Style = types.SimpleNamespace(RED="", GREEN="", RESET_ALL="", RESET="")
            m.init = lambda *a, **k: None
            sys.modules[name] = m


def golden_sh():
    from utils.sh_utils import eval_sh
    g = torch.Generator().manual_seed(11)
    out = {}
    for deg in range(4):
        n = 257
        K = (deg + 1) ** 2
        sh = torch.randn(n, 3, K, generator=g)       # reference layout [..., C, K]
        dirs = torch.randn(n, 3, generator=g)
        dirs = dirs / dirs.norm(dim=-1, keepdim=True)
        res = eval_sh(deg, sh, dirs)                   # [n, 3]
        out[f"deg{deg}_coeffs_nk3"] = sh.permute(0, 2, 1).contiguous().numpy()  # gsplat layout
        out[f"deg{deg}_dirs"] = dirs.numpy()
        out[f"deg{deg}_colors"] = res.numpy()
    np.savez(os.path.join(OUT, "sh_eval.npz"), **out)


def _make_lod_model(n_anchor, view_dim, color_attr, seed):
    import torch.nn as nn
    from scene.lod_model import GaussianLoDModel
    feat_dim, n_offsets = 32, 10
    model = GaussianLoDModel.__new__(GaussianLoDModel)
    model.feat_dim, model.view_dim, model.n_offsets = feat_dim, view_dim, n_offsets
    model.appearance_dim = 0
    model.color_attr = color_attr
    model.dist2level = "floor"
    model.standard_dist, model.fork, model.street_levels = 26.686, 2, 8
    if color_attr == "RGB":
        model.active_sh_degree, model.color_dim = None, 3
    else:
        model.active_sh_degree, model.color_dim = 2, 27
    model.setup_functions()
    g = torch.Generator().manual_seed(seed)
    torch.manual_seed(seed)
    model.mlp_opacity = nn.Sequential(nn.Linear(feat_dim + view_dim, feat_dim), nn.ReLU(True),
                                      nn.Linear(feat_dim, n_offsets), nn.Tanh())
    model.mlp_cov = nn.Sequential(nn.Linear(feat_dim + view_dim, feat_dim), nn.ReLU(True),
                                  nn.Linear(feat_dim, 7 * n_offsets))
    model.mlp_color = nn.Sequential(nn.Linear(feat_dim + view_dim, feat_dim), nn.ReLU(True),
                                    nn.Linear(feat_dim, model.color_dim * n_offsets))
    model._anchor = torch.rand(n_anchor, 3, generator=g) * 40 - 20
    model._anchor_feat = torch.randn(n_anchor, feat_dim, generator=g) * 0.5
    model._offset = torch.randn(n_anchor, n_offsets, 3, generator=g) * 0.1
    model._scaling = torch.log(torch.full((n_anchor, 6), 0.01)) + torch.randn(n_anchor, 6, generator=g) * 0.1
    model._rotation = torch.zeros(n_anchor, 4)
    model._rotation[:, 0] = 1
    model._level = torch.randint(0, 8, (n_anchor, 1), generator=g, dtype=torch.int32)
    model._extra_level = torch.randn(n_anchor, generator=g) * 0.2
    model.smooth_complement = lambda visible_mask: torch.ones((int(visible_mask.sum()), 1))
    return model


def golden_decode():
    from types import SimpleNamespace
    for tag, view_dim, color_attr in [("rgb", 3, "RGB"), ("sh2", 0, "SH2")]:
        model = _make_lod_model(1000, view_dim, color_attr, seed=21 if tag == "rgb" else 22)
        cam_center = torch.tensor([0.5, -1.0, 2.0])
        res_scale = 1.0
        model.set_anchor_mask(cam_center, res_scale)
        anchor_mask = model._anchor_mask.clone()
        cam = SimpleNamespace(camera_center=cam_center)
        with torch.no_grad():
            xyz, offsets, color, opacity, scaling, rot, sh_degree, mask = model.generate_neural_gaussians(
                cam, anchor_mask)
        sd = {}
        for name, mlp in [("opacity", model.mlp_opacity), ("cov", model.mlp_cov), ("color", model.mlp_color)]:
            sd[f"{name}_w1"] = mlp[0].weight.detach().numpy()
            sd[f"{name}_b1"] = mlp[0].bias.detach().numpy()
            sd[f"{name}_w2"] = mlp[2].weight.detach().numpy()
            sd[f"{name}_b2"] = mlp[2].bias.detach().numpy()
        np.savez(os.path.join(OUT, f"decode_{tag}.npz"),
                 anchor=model._anchor.numpy(), anchor_feat=model._anchor_feat.numpy(),
                 offset=model._offset.numpy(), scaling=model._scaling.numpy(),
                 level=model._level.numpy(), extra_level=model._extra_level.numpy(),
                 cam_center=cam_center.numpy(), res_scale=np.float32(res_scale),
                 standard_dist=np.float32(model.standard_dist), fork=np.int32(model.fork),
                 street_levels=np.int32(model.street_levels), view_dim=np.int32(view_dim),
                 anchor_mask=anchor_mask.numpy(),
                 out_xyz=xyz.numpy(), out_color=color.numpy(), out_opacity=opacity.numpy(),
                 out_scaling=scaling.numpy(), out_rot=rot.numpy(), out_mask=mask.numpy(),
                 **sd)


def golden_losses():
    from utils.image_utils import psnr
    from utils.loss_utils import l1_loss, ssim
    g = torch.Generator().manual_seed(31)
    a = torch.rand(3, 64, 80, generator=g)
    b = (a + 0.1 * torch.randn(3, 64, 80, generator=g)).clamp(0, 1)
    np.savez(os.path.join(OUT, "losses.npz"), img=a.numpy(), gt=b.numpy(),
             l1=np.float32(l1_loss(a, b).item()), ssim=np.float32(ssim(a, b).item()),
             psnr=psnr(a[None], b[None]).numpy())


@contextlib.contextmanager
def _cuda_as_cpu():
    """Run reference code that allocates with device="cuda" / calls .cuda() on the CPU."""
    names = ["zeros", "ones", "empty", "full", "tensor", "arange", "zeros_like", "ones_like"]
    saved = {n: getattr(torch, n) for n in names}

    def wrap(orig):
        def f(*a, **k):
            if "device" in k and str(k["device"]).startswith("cuda"):
                k["device"] = "cpu"
            return orig(*a, **k)
        return f

    for n in names:
        setattr(torch, n, wrap(saved[n]))
    saved_cuda = torch.Tensor.cuda
    torch.Tensor.cuda = lambda self, *a, **k: self
    try:
        yield
    finally:
        for n in names:
            setattr(torch, n, saved[n])
        torch.Tensor.cuda = saved_cuda


def golden_densify():
    """scene/basic_model.py:96-144 training_statis (mean/mean and max/max), :179-190
    get_remove_duplicates, scene/lod_model.py:236-249 weed_out."""
    from types import SimpleNamespace
    out = {}
    g = torch.Generator().manual_seed(41)
    A, k = 300, 10
    model = _make_lod_model(A, 3, "RGB", seed=41)
    vis = torch.rand(A, generator=g) < 0.7
    Av = int(vis.sum())
    sel = torch.rand(Av * k, generator=g) < 0.6
    M = int(sel.sum())
    radii = torch.randint(0, 12, (M,), generator=g, dtype=torch.int32)
    filt = radii > 0
    grad = torch.randn(1, M, 2, generator=g) * 1e-3
    opac = torch.rand(M, 1, generator=g)
    W, H = 640, 360
    out.update(vis=vis.numpy(), sel=sel.numpy(), radii=radii.numpy(), filt=filt.numpy(), grad=grad.numpy(),
               opacity=opac.numpy(), W=np.int32(W), H=np.int32(H), n_offsets=np.int32(k))
    for tag, ptype, gtype in [("mean", "mean", "mean"), ("max", "max", "max")]:
        st = dict(anchor_opacity_accum=torch.rand(A, 1, generator=g), anchor_demon=torch.randint(0, 5, (A, 1), generator=g).float(),
                  offset_gradient_accum=torch.rand(A * k, 1, generator=g) * 1e-2,
                  offset_denom=torch.randint(0, 5, (A * k, 1), generator=g).float(),
                  max_radii2D=torch.randint(0, 8, (A * k,), generator=g).float(),
                  offset_opacity_accum=torch.rand(A * k, 1, generator=g))
        for n, v in st.items():
            out[f"{tag}_in_{n}"] = v.numpy().copy()
            setattr(model, n, v.clone())
        vsp = grad.clone().requires_grad_(True)
        vsp.grad = grad.clone()
        pkg = dict(selection_mask=sel, visible_mask=vis, viewspace_points=vsp, visibility_filter=filt,
                   opacity=opac, radii=radii)
        with _cuda_as_cpu():
            model.training_statis(SimpleNamespace(pruning_type=ptype, growing_type=gtype), pkg, W, H)
        for n in st:
            out[f"{tag}_out_{n}"] = getattr(model, n).numpy()
    # get_remove_duplicates: existing voxels and candidates with a known overlap
    grid = torch.unique(torch.randint(-300, 300, (5000, 3), generator=g, dtype=torch.int32), dim=0)
    cand = torch.cat([grid[torch.randperm(grid.shape[0], generator=g)[:700]],
                      torch.randint(-300, 300, (900, 3), generator=g, dtype=torch.int32)])
    cand = torch.unique(cand, dim=0)
    with _cuda_as_cpu():
        dup = model.get_remove_duplicates(grid, cand)
    out.update(grid_coords=grid.numpy(), cand_coords=cand.numpy(), duplicates=dup.numpy())
    # weed_out over 137 cameras
    model.weed_ratio = 0.3
    model.cam_infos = torch.cat([torch.rand(137, 3, generator=g) * 40 - 20, 0.5 + torch.rand(137, 1, generator=g)], 1)
    pos = torch.rand(2000, 3, generator=g) * 60 - 30
    lev = torch.randint(0, 8, (2000,), generator=g, dtype=torch.int32)
    with _cuda_as_cpu():
        wm = model.weed_out(pos, lev)
    out.update(weed_pos=pos.numpy(), weed_levels=lev.numpy(), weed_cams=model.cam_infos.numpy(),
               weed_ratio=np.float32(model.weed_ratio), weed_mask=wm.numpy(),
               standard_dist=np.float32(model.standard_dist), fork=np.int32(model.fork),
               street_levels=np.int32(model.street_levels))
    np.savez(os.path.join(OUT, "densify.npz"), **out)


def _scatter_max_restated(src, index, dim=0, out=None, dim_size=None):
    """torch_scatter 2.x scatter_max (the reference's dependency, absent here), restated:
    out[i] = elementwise max of the src rows with index i, 0 for rows no index reaches;
    the argmax output is not used by the reference (lod_model.py:559 takes [0])."""
    n = int(index.max()) + 1 if dim_size is None else dim_size
    res = torch.full((n,) + tuple(src.shape[1:]), float("-inf"), dtype=src.dtype)
    res = res.scatter_reduce(0, index, src, reduce="amax", include_self=True)
    res[torch.isinf(res) & (res < 0)] = 0
    return res, None


def golden_anchor_growing():
    """scene/lod_model.py:487-596 anchor_growing (fine stage, weed_out active) on the CPU."""
    import torch.nn as nn
    from types import SimpleNamespace
    import scene.lod_model as LM
    LM.scatter_max = _scatter_max_restated
    g = torch.Generator().manual_seed(51)
    A, k = 400, 10
    model = _make_lod_model(A, 3, "RGB", seed=51)
    model._level = torch.randint(0, 4, (A, 1), generator=g).float()
    model.training_stage, model.aerial_levels, model.street_levels = "fine", 1, 4
    model.voxel_size, model.padding = 0.5, 0.0
    model.weed_ratio = 0.05
    model.cam_infos = torch.cat([torch.rand(64, 3, generator=g) * 40 - 20, 0.5 + torch.rand(64, 1, generator=g)], 1)
    model.anchor_demon = torch.rand(A, 1, generator=g)
    model.anchor_opacity_accum = torch.rand(A, 1, generator=g)
    for n in ("_anchor", "_offset", "_anchor_feat", "_scaling", "_rotation"):
        setattr(model, n, nn.Parameter(getattr(model, n).clone()))
    model.optimizer = torch.optim.Adam([
        {"params": [model._anchor], "name": "anchor"}, {"params": [model._offset], "name": "offset"},
        {"params": [model._anchor_feat], "name": "anchor_feat"}, {"params": [model._scaling], "name": "scaling"},
        {"params": [model._rotation], "name": "rotation"}], lr=0.0)
    before = {n: getattr(model, n).detach().numpy().copy() for n in
              ("_anchor", "_offset", "_anchor_feat", "_scaling", "_rotation", "_level", "_extra_level",
               "anchor_demon", "anchor_opacity_accum")}
    grads = torch.rand(A * k, generator=g) * 0.0004
    offset_mask = torch.rand(A * k, generator=g) < 0.7
    opt = SimpleNamespace(update_ratio=0.5, densify_grad_threshold=0.0002, extra_ratio=0.25, extra_up=0.01,
                          overlap=False)
    with _cuda_as_cpu():
        model.anchor_growing(grads.clone(), opt, offset_mask, 1000)
    after = {n: getattr(model, n).detach().numpy() for n in before}
    np.savez(os.path.join(OUT, "anchor_growing.npz"), grads=grads.numpy(), offset_mask=offset_mask.numpy(),
             cam_infos=model.cam_infos.numpy(), standard_dist=np.float32(model.standard_dist),
             **{"in" + n: v for n, v in before.items()}, **{"out" + n: v for n, v in after.items()})


def main():
    os.makedirs(OUT, exist_ok=True)
    sys.path.insert(0, REF)
    _stub_modules()
    golden_sh()
    golden_decode()
    golden_losses()
    golden_densify()
    golden_anchor_growing()
    print("wrote", sorted(os.listdir(OUT)))


if __name__ == "__main__":
    main()
