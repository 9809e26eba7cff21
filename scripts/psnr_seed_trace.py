"""Diagnostic (round 6): per-iteration render MSE of the HIP at-scale chain for one seed over the
whole run (the window PSNR averages the last 50): a transient spike shows as a few iterations."""
import json
import math
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from scripts import psnr_at_scale as PS  # noqa: E402
from tests import pipeline_fit as PF  # noqa: E402


def main():
    gs, seed = sys.argv[1], int(sys.argv[2])
    gold = json.load(open(os.path.join(ROOT, "tests", "golden", f"psnr_scale_{gs}.json")))
    gt, p0, cfg, _ = PS.problem(gold["anchors"], gold["width"], gold["height"], gs)
    p0 = p0 if seed < 0 else PS.perturbed(p0, seed)
    from horizongs_amd.optim import Adam
    p = {k: v.to("cuda").clone().requires_grad_(k != "anchor") for k, v in p0.items()}
    opt = Adam([{"params": [p[k]], "lr": gold["lr_scale"] * PF._lr(k)} for k in p if k != "anchor"], lr=0.0, eps=1e-15)
    gtd = gt.to("cuda")
    mses = []
    for it in range(gold["iterations"]):
        opt.zero_grad(set_to_none=True)
        loss, img = PF.gpu_loss(p, cfg, gtd, gs)
        loss.backward()
        opt.step()
        mses.append(float(((img[:3].detach().double() - gtd.double()) ** 2).mean()))
    w = mses[-gold["window"]:]
    print(json.dumps({"seed": seed, "window_db": round(10 * math.log10(len(w) / sum(w)), 4),
                      "window_mse": [round(x, 8) for x in w], "max_mse_it": int(max(range(len(mses)), key=lambda i: mses[i] if i > 100 else 0)),
                      "mse_every_10": [round(x, 7) for x in mses[::10]]}))


if __name__ == "__main__":
    main()
