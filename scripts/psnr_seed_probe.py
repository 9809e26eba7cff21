"""Diagnostic (round 6): the HIP 2DGS at-scale chain for given perturbation seeds -- window PSNR
and the loss every 10 iterations -- to tell a chaotic draw from a gradient event."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from scripts import psnr_at_scale as PS  # noqa: E402
from tests import pipeline_fit as PF  # noqa: E402


def main():
    gs = sys.argv[1]
    seeds = [int(x) for x in sys.argv[2].split(",")]
    gold = json.load(open(os.path.join(ROOT, "tests", "golden", f"psnr_scale_{gs}.json")))
    gt, p0, cfg, _ = PS.problem(gold["anchors"], gold["width"], gold["height"], gs)
    for s in seeds:
        p = p0 if s < 0 else PS.perturbed(p0, s)
        fin, win, losses = PF.fit(p, cfg, gt, gold["iterations"], gs=gs, device="cuda", window=gold["window"],
                                  lr_scale=gold["lr_scale"])
        print(json.dumps({"seed": s, "final_db": round(fin, 4), "window_db": round(win, 4),
                          "losses_every_10": [round(x, 6) for x in losses[::10]]}), flush=True)


if __name__ == "__main__":
    main()
