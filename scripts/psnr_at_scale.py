"""PSNR parity at scale, reference side (TEST INFRASTRUCTURE; run on the CPU, here).

Runs the CPU chain of tests/pipeline_fit.py -- prefilter_voxel -> the reference-pinned decode
(oracle/decode_ref.py) -> the C-oracle rasterization(_2dgs) -> the reference-pinned loss head
(oracle/loss_ref.py) -> torch.optim.Adam(eps=1e-15) -- for ITERS iterations on an anchor model
of A anchors at W x H, at the fine-stage learning rates x LR_SCALE (reference train.py:150-277,
config/base/small_scene/fine.yaml), twice: from the initialisation and from the same
initialisation perturbed by 1e-6 (relative), which measures the chain's own noise floor.
Writes tests/golden/psnr_scale_{3d,2d}.json: the window / final PSNRs of both runs and the
loss curve; tests/test_gpu_training_parity.py::test_psnr_parity_at_scale_* runs the HIP chain
on the GPU with the same seeds and compares.

The CPU chain takes ~1 s per iteration at 50k anchors / 480x270 on 8 host threads, far beyond
a GPU-suite test, so its result is committed as a fixture together with this script.

usage: python scripts/psnr_at_scale.py --gs 3d [--anchors 50000 --width 480 --height 270
       --iters 500 --lr-scale 1.0]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from tests import pipeline_fit as PF  # noqa: E402

# the at-scale problem (tests/test_gpu_training_parity.py reads these from the fixture)
SEEDS = dict(target=41, anchors=42, params=300, perturb=5)


def problem(A, W, H, gs):
    # ~2 target Gaussians per pixel (the small test's density: 40k at 160x120)
    n_target = int(round(40000 * W * H / (160 * 120)))
    gt = PF.target(n_target, W, H, seed=SEEDS["target"], gs=gs)
    p0, cfg = PF.anchor_model(A, W, H, seed=SEEDS["anchors"], param_seed=SEEDS["params"])
    return gt, p0, cfg, n_target


TARGET = os.path.join(ROOT, "tests", "golden", "psnr_target_{gs}.npz")


def problem_from_fixture(A, W, H, gs):
    """problem() with the target render read from tests/golden/psnr_target_{gs}.npz (the
    C-oracle render of the seeded target scene, written by --write-target): what bench.py uses
    to measure the HIP chain's PSNR live without running the oracle."""
    import numpy as np
    gt = torch.from_numpy(np.load(TARGET.format(gs=gs))["target"])
    assert gt.shape == (3, H, W), gt.shape
    p0, cfg = PF.anchor_model(A, W, H, seed=SEEDS["anchors"], param_seed=SEEDS["params"])
    return gt, p0, cfg


def perturbed(p0, seed=None):
    g = torch.Generator().manual_seed(SEEDS["perturb"] if seed is None else seed)
    return {k: (v * (1 + 1e-6 * torch.randn(v.shape, generator=g)) if k != "anchor" else v) for k, v in p0.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gs", choices=["3d", "2d"], required=True)
    ap.add_argument("--anchors", type=int, default=50000)
    ap.add_argument("--width", type=int, default=480)
    ap.add_argument("--height", type=int, default=270)
    ap.add_argument("--iters", type=int, default=500)
    ap.add_argument("--lr-scale", type=float, default=1.0)
    ap.add_argument("--window", type=int, default=50)
    ap.add_argument("--out", default=None)
    ap.add_argument("--write-target", action="store_true",
                    help="only write the target render to tests/golden/psnr_target_{gs}.npz")
    ap.add_argument("--perturb-seed", type=int, default=None,
                    help="ensemble member: run ONLY the chain from the initialisation perturbed with this seed "
                         "and write it to --out (merged into the fixture by scripts/psnr_ensemble.py)")
    a = ap.parse_args()
    gt, p0, cfg, n_target = problem(a.anchors, a.width, a.height, a.gs)
    if a.write_target:
        import numpy as np
        np.savez_compressed(TARGET.format(gs=a.gs), target=gt.numpy())
        return
    with torch.no_grad():
        psnr_init = PF.psnr(PF.cpu_render(p0, cfg, a.gs)[0], gt)
    res = dict(gs=a.gs, anchors=a.anchors, width=a.width, height=a.height, iterations=a.iters, lr_scale=a.lr_scale,
               window=a.window, target_gaussians=n_target, seeds=SEEDS, psnr_init_db=round(psnr_init, 4),
               threads=torch.get_num_threads(), omp_num_threads=os.environ.get("OMP_NUM_THREADS"))
    runs = ((("ref", p0), ("ref_perturbed_1e-6", perturbed(p0))) if a.perturb_seed is None
            else ((f"ref_perturbed_1e-6_seed{a.perturb_seed}", perturbed(p0, a.perturb_seed)),))
    for name, p in runs:
        t0 = time.time()
        fin, win, losses = PF.fit(p, cfg, gt, a.iters, gs=a.gs, window=a.window, lr_scale=a.lr_scale)
        res[name] = dict(final_db=round(fin, 4), window_db=round(win, 4), seconds=round(time.time() - t0, 1),
                         loss_first=losses[0], loss_last=losses[-1], losses_every_10=[round(x, 6) for x in losses[::10]])
        print(name, res[name]["final_db"], res[name]["window_db"], res[name]["seconds"], "s", flush=True)
    if a.perturb_seed is None:
        res["noise_floor_window_db"] = round(res["ref_perturbed_1e-6"]["window_db"] - res["ref"]["window_db"], 4)
        res["noise_floor_final_db"] = round(res["ref_perturbed_1e-6"]["final_db"] - res["ref"]["final_db"], 4)
    out = a.out or os.path.join(ROOT, "tests", "golden", f"psnr_scale_{a.gs}.json")
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps({k: v for k, v in res.items() if not isinstance(v, dict)}))


if __name__ == "__main__":
    main()
