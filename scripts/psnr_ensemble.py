"""Merge the reference-chain ensemble into the at-scale PSNR fixtures (TEST INFRASTRUCTURE).

scripts/psnr_ensemble_run.sh runs the CPU chain of scripts/psnr_at_scale.py from initialisations
perturbed by 1e-6 with seeds 6..12 (tests/golden/psnr_ensemble/{gs}_seed<N>.json); the fixture
already holds the unperturbed run ("ref") and seed 5 ("ref_perturbed_1e-6").  This adds
"ensemble": {seed: {window_db, final_db, loss_last}} for seeds 5..12 and the spread statistics
of the reference chain (its window PSNR over the unperturbed run and the perturbed ones) that
tests/test_gpu_training_parity.py takes its bar from.

usage: python scripts/psnr_ensemble.py --gs 2d [--fixture psnr_scale_2d]
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import statistics

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gs", choices=["2d", "3d"], required=True)
    ap.add_argument("--fixture", default=None)
    ap.add_argument("--prefix", default=None, help="ensemble file prefix (default: the --gs value)")
    a = ap.parse_args()
    path = os.path.join(ROOT, "tests", "golden", f"{a.fixture or 'psnr_scale_' + a.gs}.json")
    fx = json.load(open(path))
    ens = {5: fx["ref_perturbed_1e-6"]}
    for f in sorted(glob.glob(os.path.join(ROOT, "tests", "golden", "psnr_ensemble", f"{a.prefix or a.gs}_seed*.json"))):
        d = json.load(open(f))
        if d["lr_scale"] != fx["lr_scale"] or d["iterations"] != fx["iterations"] or d["anchors"] != fx["anchors"]:
            continue
        seed = int(os.path.basename(f).split("seed")[1].split(".")[0])
        ens[seed] = d[f"ref_perturbed_1e-6_seed{seed}"]
    fx["ensemble"] = {str(s): {k: r[k] for k in ("window_db", "final_db", "loss_last", "seconds")}
                      for s, r in sorted(ens.items())}
    w = [fx["ref"]["window_db"]] + [r["window_db"] for r in ens.values()]
    fin = [fx["ref"]["final_db"]] + [r["final_db"] for r in ens.values()]
    fx["ensemble_stats"] = {
        "members": len(w), "window_mean_db": round(statistics.mean(w), 4), "window_sd_db": round(statistics.stdev(w), 4),
        "window_range_db": round(max(w) - min(w), 4), "final_mean_db": round(statistics.mean(fin), 4),
        "final_sd_db": round(statistics.stdev(fin), 4),
        "note": ("the reference chain from its unperturbed initialisation and from initialisations perturbed by 1e-6 "
                 "(seeds " + ", ".join(str(s) for s in sorted(ens)) + "): draws of the chain's own spread")}
    with open(path, "w") as f:
        json.dump(fx, f, indent=1)
    print(json.dumps(fx["ensemble_stats"]))


if __name__ == "__main__":
    main()
