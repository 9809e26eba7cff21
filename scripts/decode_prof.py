"""Per-phase shader-clock split of the decode backward (developer instrumentation).
Build:  make -C horizongs_amd/csrc OUT=../_lib_dprof EXTRA=-DHGSR_DECODE_PROF
Run:    HGSR_LIB=horizongs_amd/_lib_dprof/libhgsr.so python scripts/decode_prof.py
Phases (decode.hip DPROF_T): 0 setup + slot gathers issued, 1 hidden layer, 2 Y recompute,
3 dY (activation derivatives), 4 per-anchor sums, 5 dW2, 6 dH, 7 dW1, 8 dX + stores, 9 tail."""
import ctypes as ct
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from horizongs_amd import _native as NAT  # noqa: E402

sys.argv = [sys.argv[0], "--anchors", "500000", "--steps", "5"]
args = bench.parse()
wl = bench.Workload(args, 0, torch.device("cuda", 0))
for _ in range(3):
    wl.step()
torch.cuda.synchronize()
lib = NAT.lib()
fn = lib.hgsr_debug_decode_prof
fn.argtypes = [ct.c_void_p, ct.c_int]
buf = (ct.c_ulonglong * 48)()
fn(buf, 1)
for _ in range(args.steps):
    wl.step()
torch.cuda.synchronize()
fn(buf, 0)
names = ["setup", "hidden", "Y", "dY", "sums", "dW2", "dH", "dW1", "dX", "tail"]
for h in range(3):
    row = [buf[h * 16 + k] for k in range(10)]
    tot = sum(row) or 1
    print(f"head {h}: " + "  ".join(f"{n} {v / tot:.2f}" for n, v in zip(names, row)) + f"  total {tot:.3e}")
