"""Wait-site attribution of raster3d_bwd (developer probe).

Runs the c2 bench workload on the library built with the wait-site hooks live
(`make -C horizongs_amd/csrc probe-wait` -> horizongs_amd/_lib_probe_wait/libhgsr.so, loaded
through HGSR_LIB) and reads the kernel's per-site shader-clock sums (csrc/common.h HGSR_WP_*):
  0 setup (pixel terms, last ids, first DMA)    4 compaction (quadrant bits -> wave list)
  1 batch-top vmcnt(0) wait (DMA, slot loads,   5 the steps + pass 2 (VALU, LDS transposes,
    previous batch's row stores)                  the row stores issue)
  2 DMA / slot-load issue                        6 second barrier (waves waiting for the slowest)
  3 first barrier                                7 tail
Each s_memtime read waits for the wave's outstanding LDS operations, so the probe perturbs
the kernel (it runs slower); the split is an attribution, not a timing.
usage: python scripts/micro/wait_probe.py [--steps K] > gpurun_out/<tag>/wait_probe.json
"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["HGSR_LIB"] = os.path.join(ROOT, "horizongs_amd", "_lib_probe_wait", "libhgsr.so")
steps = int(sys.argv[sys.argv.index("--steps") + 1]) if "--steps" in sys.argv else 16
sys.argv = [sys.argv[0], "--no-cpu-baseline", "--no-secondary", "--no-quality", "--no-timing"]
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402
from horizongs_amd import _native  # noqa: E402

SITES = ["setup", "vmcnt_wait", "dma_issue", "barrier1", "compaction", "steps_pass2", "barrier2", "tail"]


def main():
    lib = _native.lib()
    rd = lib.hgsr_probe_wait_read
    rd.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
    rd.restype = ctypes.c_int
    buf = (ctypes.c_ulonglong * 16)()
    args = bench.resolve(bench.parse(), 1)
    wl = bench.Workload(args, 0, torch.device("cuda", 0), 1)
    for _ in range(3):
        wl.step()
    torch.cuda.synchronize()
    assert rd(buf, 1) == 0
    for _ in range(steps):
        wl.step()
    torch.cuda.synchronize()
    assert rd(buf, 1) == 0
    wl.close()
    v = list(buf)
    tot = sum(v[:8])
    out = {"steps": steps, "waves": v[8], "cycles_total": tot,
           "fraction": {s: round(v[k] / tot, 4) for k, s in enumerate(SITES)},
           "cycles_per_wave": {s: round(v[k] / max(v[8], 1), 1) for k, s in enumerate(SITES)},
           "library": os.environ["HGSR_LIB"]}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
