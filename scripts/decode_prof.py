"""Per-phase shader-clock breakdown of the anchor decode backward (developer tool).

Needs the instrumented library: make -C horizongs_amd/csrc OUT=../_lib_prof EXTRA=-DHGSR_DECODE_PROF
Run:  HGSR_LIB=horizongs_amd/_lib_prof/libhgsr.so python scripts/decode_prof.py --config c4
Phases (decode.hip DPROF_T): 0 stage X / slot rows, 1 hidden layer + gathers, 2 recompute Y,
3 dY, 4 per-anchor sums, 5 dW2, 6 dH, 7 dW1, 8 dX + stores, 9 tail."""
import ctypes as ct
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402
from horizongs_amd import _native as NAT  # noqa: E402

args = bench.resolve(bench.parse(sys.argv[1:] + ["--no-secondary", "--no-timing"]), 1)
wl = bench.Workload(args, 0, torch.device("cuda", 0))
for _ in range(3):
    wl.step()
torch.cuda.synchronize()
lib = NAT.lib()
fn = lib.hgsr_debug_decode_prof
fn.argtypes = [ct.c_void_p, ct.c_int]
buf = (ct.c_ulonglong * 48)()
fn(buf, 1)
steps = 5
for _ in range(steps):
    wl.step()
torch.cuda.synchronize()
fn(buf, 1)
names = ["stage", "hidden+gathers", "recompute Y", "dY", "anchor sums", "dW2", "dH", "dW1", "dX+stores", "tail"]
for h, head in enumerate(("opacity", "cov", "color")):
    row = [buf[h * 16 + k] for k in range(10)]
    tot = sum(row)
    if not tot:
        continue
    print(f"{head:8s} total {tot / steps:.3e} wave-clocks/step: " +
          ", ".join(f"{n} {v / tot:.1%}" for n, v in zip(names, row)))
