"""Diagnostic (round 6): how the c2 / c3 bench views' gradient slots are spread over the
reducer's 64-Gaussian waves -- slots per wave (max, percentiles) and the largest tile counts."""
import json
import sys

import numpy as np
import torch

sys.argv = [sys.argv[0]] + sys.argv[1:] + ["--no-cpu-baseline", "--no-secondary", "--no-quality", "--no-timing"]
sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
import bench  # noqa: E402


def main():
    args = bench.resolve(bench.parse(), 1)
    wl = bench.Workload(args, 0, torch.device("cuda", 0), 1)
    out = []
    for v in range(16):
        wl.step()
        torch.cuda.synchronize()
        tpg = wl.meta["tiles_per_gauss"].reshape(-1).to(torch.int64).cpu().numpy()
        n = tpg.size
        pad = (-n) % 64
        per_wave = np.concatenate([tpg, np.zeros(pad, np.int64)]).reshape(-1, 64).sum(1)
        out.append({"view": v, "slots": int(tpg.sum()), "max_tpg": int(tpg.max()),
                    "tpg_p99": float(np.percentile(tpg, 99)), "n_tpg_gt16": int((tpg > 16).sum()),
                    "n_tpg_gt64": int((tpg > 64).sum()), "n_tpg_gt1024": int((tpg > 1024).sum()),
                    "wave_slots_max": int(per_wave.max()), "wave_slots_p99": float(np.percentile(per_wave, 99)),
                    "wave_slots_mean": float(per_wave.mean())})
        print(json.dumps(out[-1]), flush=True)


if __name__ == "__main__":
    main()
