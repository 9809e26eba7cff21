"""Diagnostic: GPU vs oracle f32 vs oracle f64 gradient errors for rasterization()."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from horizongs_amd import gsplat_api as G
from horizongs_amd.synthetic import make_scene
from oracle import pipeline as OP
DEV = "cuda:0"
for mode, sh in [("RGB+ED", None), ("RGB", None), ("RGB+ED", 2)]:
    sc = make_scene(600, 96, 80, seed=11, scale_range=(0.01, 0.06), depth_range=(2.0, 6.0), sh_degree=sh, opacity_range=(0.2, 0.95))
    bg = torch.tensor([[0.1, 0.3, 0.2]])
    refs = {}
    for dt in (np.float32, np.float64):
        r = OP.Raster3D(sc.means, sc.quats, sc.scales, sc.opacities, sc.colors, sc.viewmats, sc.Ks, sc.width, sc.height,
                        sh_degree=sh, backgrounds=bg, render_mode=mode, dtype=dt)
        rc, ra = r.forward()
        refs[dt] = r
    g = torch.Generator().manual_seed(12)
    vrc = torch.randn(rc.shape, generator=g); vra = torch.randn(ra.shape, generator=g)
    gr32 = refs[np.float32].backward(vrc.numpy(), vra.numpy())
    gr64 = refs[np.float64].backward(vrc.numpy(), vra.numpy())
    t = [x.to(DEV) for x in (sc.means, sc.quats, sc.scales, sc.opacities, sc.colors, sc.viewmats, sc.Ks, bg)]
    means, quats, scales, opac, cols, vm, K, gbg = t
    for x in (means, quats, scales, opac, cols): x.requires_grad_(True)
    out, alpha, meta = G.rasterization(means, quats, scales, opac, cols, vm, K, sc.width, sc.height, packed=False, sh_degree=sh, backgrounds=gbg, render_mode=mode)
    meta["means2d"].retain_grad()
    ((out * vrc.to(DEV)).sum() + (alpha * vra.to(DEV)).sum()).backward()
    gpu = {"means2d": meta["means2d"].grad, "opacities": opac.grad, "colors": cols.grad, "means": means.grad, "quats": quats.grad, "scales": scales.grad}
    print("mode", mode, "sh", sh, "fwd err gpu-64", np.abs(out.detach().cpu().numpy() - refs[np.float64].render_colors).max(),
          "o32-64", np.abs(refs[np.float32].render_colors - refs[np.float64].render_colors).max())
    for k, v in gpu.items():
        a = v.detach().cpu().numpy().astype(np.float64); b = gr64[k]; c = gr32[k].astype(np.float64)
        eg = np.abs(a - b); eo = np.abs(c - b)
        print(f"  {k:10s} max|g| {np.abs(b).max():9.3g}  gpu-64 max {eg.max():9.3g}  o32-64 max {eo.max():9.3g}  gpu-o32 max {np.abs(a-c).max():9.3g}  ratio(gpu/o32 err) {eg.max()/max(eo.max(),1e-30):6.2f}")
