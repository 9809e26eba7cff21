"""Per-phase shader-clock breakdown of the decode backward (variant build with
-DHGSR_DECODE_PROF; run with HGSR_LIB=build/dprof/libhgsr.so).  Phases: 0 stage X,
1 hidden layer, 2 Y recompute, 3 dY (slot work), 4 per-anchor sums, 5 dW2/db2, 6 dH,
7 dW1/db1, 8 dX + d feat / d anchor, 9 after the tile loop."""
import ctypes as ct
import sys
import types

import torch

sys.path.insert(0, ".")
import bench  # noqa: E402
from horizongs_amd import _native as NAT  # noqa: E402

args = types.SimpleNamespace(gpus=1, steps=3, warmup=2, n=2_000_000, width=1920, height=1080, gs="3d", mode="chunk",
                             no_cpu_baseline=True, no_timing=True, anchors=int(sys.argv[1]) if len(sys.argv) > 1 else 500000)
wl = bench.Workload(args, 0, torch.device("cuda", 0))
for _ in range(args.warmup):
    wl.step()
torch.cuda.synchronize()
lib = NAT.lib()
buf = (ct.c_ulonglong * 48)()
lib.hgsr_debug_decode_prof(buf, 1)
for _ in range(args.steps):
    wl.step()
torch.cuda.synchronize()
lib.hgsr_debug_decode_prof(buf, 0)
names = ["stageX", "hidden", "Yrecomp", "dY/slots", "anchor sums", "dW2", "dH", "dW1", "dX+RMW", "tail"]
for h, hn in enumerate(("opacity", "cov", "colour")):
    row = [buf[h * 16 + k] / args.steps for k in range(10)]
    tot = sum(row)
    print(hn, " ".join(f"{n}={v / tot * 100:.1f}%" for n, v in zip(names, row)), f"total={tot:.3g} clk/step")
