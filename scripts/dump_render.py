"""Save GPU forward renders (last-contributor ids, images) of the parity scenes for CPU-side
debugging of the near-threshold branch resolution (tests/raster_parity.py) against the oracle.
Developer tool, GPU box: python scripts/dump_render.py -> gpurun_out/dump_<name>.npz"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from horizongs_amd import gsplat_api as G  # noqa: E402
from horizongs_amd.synthetic import c2  # noqa: E402
from tests.raster_parity import gpu_last, to_dev  # noqa: E402
from tests.test_gpu_parity_dense import _dense_scene  # noqa: E402


def dump(name, sc, gs, bg, rows):
    means, quats, scales, opac, cols, vm, K = to_dev(sc.means, sc.quats, sc.scales, sc.opacities, sc.colors,
                                                     sc.viewmats, sc.Ks)
    gbg = bg.to("cuda:0")
    out = {}
    means.requires_grad_(True)  # keep the autograd node (gpu_last reads its saved tensors)
    if gs == "3d":
        o, a, meta = G.rasterization(means, quats, scales, opac, cols, vm, K, sc.width, sc.height, packed=False,
                                     backgrounds=gbg, render_mode="RGB+ED")
    else:
        (o, a, n, nfd, dist, med), meta = G.rasterization_2dgs(means, quats, scales, opac, cols, vm, K, sc.width,
                                                               sc.height, packed=False, backgrounds=gbg,
                                                               render_mode="RGB+ED")
        out["normals"] = n[:, :rows].detach().cpu().numpy()
    out["render_colors"] = o[:, :rows].detach().cpu().numpy()
    out["ra"] = a[:, :rows].detach().cpu().numpy()
    out["last"] = gpu_last(o)[:, :rows].cpu().numpy()
    np.savez_compressed(os.path.join(ROOT, "gpurun_out", f"dump_{name}.npz"), **out)
    print(name, {k: v.shape for k, v in out.items()})


def main():
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    torch.set_grad_enabled(True)
    sc = c2()
    dump("c2_3dgs", sc, "3d", torch.tensor([[0.2, 0.1, 0.3]]), 320)
    dump("c3_2dgs", sc, "2d", torch.tensor([[0.2, 0.1, 0.3]]), 320)
    sd = _dense_scene(n=24000, seed=7, opacity_range=(0.05, 0.6))
    dump("dense_2dgs", sd, "2d", torch.tensor([[0.2, 0.1, 0.4]]), sd.height)


if __name__ == "__main__":
    main()
