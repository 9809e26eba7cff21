"""Host-side cost of the bench train step: wall time per step vs the time the host spends
blocked in the intersection-count sync (the only sync of a step).  wall - wait = host work
per step; if it approaches the device time the step is host-bound.
Usage: python scripts/host_timing.py [--gs 3d|2d] [--anchors A] [--steps K]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402

_wait = [0.0]
_orig = torch.cuda.Event.synchronize


def _sync(self):
    t = time.perf_counter()
    _orig(self)
    _wait[0] += time.perf_counter() - t


torch.cuda.Event.synchronize = _sync
sys.argv = [sys.argv[0]] + sys.argv[1:]
args = bench.parse()
dev = torch.device("cuda", 0)
wl = bench.Workload(args, 0, dev)
for _ in range(5):
    wl.step()
torch.cuda.synchronize()
for rep in range(3):
    _wait[0] = 0.0
    t0 = time.perf_counter()
    for _ in range(args.steps):
        wl.step()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    n = args.steps
    print(f"rep {rep}: wall/step {(t2 - t0) / n * 1e3:.3f} ms, enqueue-loop/step {(t1 - t0) / n * 1e3:.3f} ms, "
          f"sync wait/step {_wait[0] / n * 1e3:.3f} ms, host work/step {((t1 - t0) - _wait[0]) / n * 1e3:.3f} ms")
