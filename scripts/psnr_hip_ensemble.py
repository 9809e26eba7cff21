"""HIP-chain ensemble of the at-scale PSNR problem (diagnostic, GPU).

The HIP chain of tests/pipeline_fit.py at the scripts/psnr_at_scale.py problem (50k anchors,
480x270, 500 iterations), from the unperturbed initialisation R times (run-to-run spread of
the product path alone) and from the 1e-6-perturbed initialisations of the reference ensemble
(seeds 5..12, scripts/psnr_ensemble_run.sh), so its spread can be set against the reference
chain's.  Also counts the gradient elements that differ between two launches of the same step.

usage: python scripts/psnr_hip_ensemble.py --gs 2d --lr-scale 0.3 [--repeat 3] [--seeds 5-12]
       -> gpurun_out/psnr_hip_ensemble_{gs}.json
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

from scripts import psnr_at_scale as PS  # noqa: E402
from tests import pipeline_fit as PF  # noqa: E402


def step_grads(p0, cfg, gt, gs):
    p = {k: v.cuda().clone().requires_grad_(k != "anchor") for k, v in p0.items()}
    loss = PF.gpu_loss(p, cfg, gt.cuda(), gs)[0]
    loss.backward()
    return {k: v.grad.detach().clone() for k, v in p.items() if k != "anchor"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gs", choices=["3d", "2d"], required=True)
    ap.add_argument("--lr-scale", type=float, required=True)
    ap.add_argument("--repeat", type=int, default=3)
    ap.add_argument("--seeds", default="5-12")
    ap.add_argument("--iters", type=int, default=500)
    a = ap.parse_args()
    lo, hi = (int(x) for x in a.seeds.split("-"))
    gt, p0, cfg, _ = PS.problem(50000, 480, 270, a.gs)
    res = dict(gs=a.gs, lr_scale=a.lr_scale, iterations=a.iters, anchors=50000, width=480, height=270, runs={})
    g1, g2 = step_grads(p0, cfg, gt, a.gs), step_grads(p0, cfg, gt, a.gs)
    res["step_grad_elements_differing"] = {k: int((g1[k] != g2[k]).sum()) for k in g1}
    res["step_grad_elements"] = {k: int(g1[k].numel()) for k in g1}
    runs = [(f"unperturbed_{r}", p0) for r in range(a.repeat)]
    runs += [(f"seed{s}", PS.perturbed(p0, s)) for s in range(lo, hi + 1)]
    for name, p in runs:
        t0 = time.time()
        fin, win, losses = PF.fit(p, cfg, gt, a.iters, gs=a.gs, device="cuda", lr_scale=a.lr_scale)
        res["runs"][name] = dict(final_db=round(fin, 4), window_db=round(win, 4), seconds=round(time.time() - t0, 1),
                                 loss_last=losses[-1])
        print(name, res["runs"][name], flush=True)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", f"psnr_hip_ensemble_{a.gs}.json"), "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res["step_grad_elements_differing"]))


if __name__ == "__main__":
    main()
