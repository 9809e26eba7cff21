"""Run-to-run reproducibility of the raster kernels ("two launches of the
same 2DGS backward are bit-identical").

The forwards are atomic-free.  The backwards write every (tile, Gaussian, wave) partial sum to
its own gradient slot and each Gaussian's slots are summed in one fixed order (DESIGN.md,
"Deterministic gradient slots"), so the same inputs must give bit-identical images AND
gradients on every launch.  Three launches are compared element by element; the per-tensor
report (fraction of bit-identical elements, which must be 1.0) goes to
gpurun_out/run_to_run_*.json."""
import json
import os

import pytest
import torch

from horizongs_amd import gsplat_api as G
from horizongs_amd.synthetic import make_scene

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _inputs(seed=7, n=20000, W=640, H=480):
    sc = make_scene(n, W, H, seed=seed, scale_range=(0.01, 0.06), depth_range=(2.0, 6.0),
                    opacity_range=(0.2, 0.95))
    ts = [torch.as_tensor(t).to(DEV).contiguous() for t in (sc.means, sc.quats, sc.scales, sc.opacities,
                                                              sc.colors, sc.viewmats, sc.Ks)]
    return ts, W, H


def _launch(gs, ts, W, H, wts):
    means, quats, scales, opac, cols, vm, K = ts
    ps = [t.clone().requires_grad_(True) for t in (means, quats, scales, opac, cols)]
    if gs == "3d":
        rc, ra, _ = G.rasterization(*ps, vm, K, W, H, packed=False, render_mode="RGB+ED")
        outs = [rc, ra]
    else:
        (rc, ra, rn, _nfd, _rd, _rm), _ = G.rasterization_2dgs(*ps, vm, K, W, H, render_mode="RGB+ED")
        outs = [rc, ra, rn]
    loss = sum((o * w).sum() for o, w in zip(outs, wts))
    loss.backward()
    torch.cuda.synchronize()
    return [o.detach().clone() for o in outs], {k: p.grad.detach().clone() for k, p in
                                                 zip(("means", "quats", "scales", "opacities", "colors"), ps)}


@pytest.mark.parametrize("gs", ["3d", "2d"])
def test_backward_run_to_run_spread(gs):
    ts, W, H = _inputs()
    g = torch.Generator(device="cpu").manual_seed(11)
    shapes = [(1, H, W, 4), (1, H, W, 1)] + ([(1, H, W, 3)] if gs == "2d" else [])
    wts = [torch.randn(s, generator=g).to(DEV) for s in shapes]
    runs = [_launch(gs, ts, W, H, wts) for _ in range(3)]
    outs0, grads0 = runs[0]
    for outs, _ in runs[1:]:
        for a, b in zip(outs, outs0):
            assert torch.equal(a, b), "the forward must be bit-reproducible"
    report = {}
    for k, g0 in grads0.items():
        scale = float(g0.abs().max())
        assert scale > 0, k
        same = min(float((r[1][k] == g0).float().mean()) for r in runs[1:])
        spread = max(float((r[1][k] - g0).abs().max()) for r in runs[1:]) / scale
        report[k] = {"bit_identical_fraction": round(same, 6), "max_diff_over_max_abs": spread}
    os.makedirs("gpurun_out", exist_ok=True)
    with open(os.path.join("gpurun_out", f"run_to_run_{gs}.json"), "w") as f:
        json.dump({"gs": gs, "gaussians": int(ts[0].shape[0]), "width": W, "height": H, "launches": 3,
                   "grads": report}, f, indent=1)
    print(gs, report)
    for k, r in report.items():
        assert r["bit_identical_fraction"] == 1.0 and r["max_diff_over_max_abs"] == 0.0, (k, r)
