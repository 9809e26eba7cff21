"""cProfile of the bench train step's host side (where the Python / launch time goes).
Usage: python scripts/host_profile.py [bench args] -- prints the top functions by own time."""
import cProfile
import os
import pstats
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402

args = bench.parse()
dev = torch.device("cuda", 0)
wl = bench.Workload(args, 0, dev)
for _ in range(5):
    wl.step()
torch.cuda.synchronize()
pr = cProfile.Profile()
pr.enable()
for _ in range(args.steps):
    wl.step()
torch.cuda.synchronize()
pr.disable()
st = pstats.Stats(pr)
st.sort_stats("tottime").print_stats(28)
