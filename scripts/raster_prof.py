"""Per-phase shader-clock breakdown of raster3d_bwd (developer tool).

Needs the instrumented library: make -C horizongs_amd/csrc OUT=../_lib_rprof EXTRA=-DHGSR_RASTER_PROF
Run:  HGSR_LIB=horizongs_amd/_lib_rprof/libhgsr.so python scripts/raster_prof.py [bench args]
Phases (raster3d.hip RPROF_T): setup, batch head (DMA wait + staging + barrier), list build,
group loop, end-of-batch barrier, tail; plus batches and 4-step groups per wave."""
import ctypes as ct
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402
from horizongs_amd import _native as NAT  # noqa: E402

args = bench.resolve(bench.parse(sys.argv[1:] + ["--no-secondary", "--no-timing"]), 1)
print("setup", flush=True)
wl = bench.Workload(args, 0, torch.device("cuda", 0))
print("warmup", flush=True)
for _ in range(3):
    wl.step()
torch.cuda.synchronize()
fn = NAT.lib().hgsr_debug_raster_prof
fn.argtypes = [ct.c_void_p, ct.c_int]
buf = (ct.c_ulonglong * 8)()
fn(buf, 1)
print("profiling", flush=True)
steps = 5
for _ in range(steps):
    wl.step()
torch.cuda.synchronize()
fn(buf, 1)
names = ["setup", "batch head", "list build", "group loop", "end barrier", "tail"]
tot = sum(buf[k] for k in range(6))
print(f"raster3d_bwd: {tot / steps:.3e} wave-clocks/step; " +
      ", ".join(f"{n} {buf[k] / tot:.1%}" for k, n in enumerate(names)))
print(f"batches/step {buf[6] / steps:.0f}, groups/step {buf[7] / steps:.0f}, "
      f"clocks/group (loop) {buf[3] / max(buf[7], 1):.0f}, clocks/batch (head+list+barrier) "
      f"{(buf[1] + buf[2] + buf[4]) / max(buf[6], 1):.0f}")
