"""Per-workgroup timing of the 3DGS raster kernels over the bench's camera set (GPU; diagnostics).

Needs the probe build: make -C horizongs_amd/csrc OUT=../_lib_wgt EXTRA=-DHGSR_PROBE_WGTIME=1.
For each view the forward and backward's workgroups (one per tile) record start / end on the
100-MHz real-time counter.  Reported per kernel: the launch span, the longest workgroup and
when it started, the mean workgroup time, the occupancy the durations imply (sum of workgroup
times over span x resident-workgroup capacity) and how the time of a tile relates to its bin
size and to its trimmed range (latest contributor).

usage: HGSR_LIB=horizongs_amd/_lib_wgt/libhgsr.so python scripts/wg_time.py > gpurun_out/wg_time.jsonl
"""
import ctypes as ct
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from horizongs_amd import _native  # noqa: E402
from horizongs_amd import gsplat_api as G  # noqa: E402
from horizongs_amd.synthetic import camera_set, make_scene  # noqa: E402

SLOTS = 16384


def main():
    dev = "cuda:0"
    W, H = 1920, 1080
    sc = make_scene(2_000_000, W, H, seed=0)
    cams = camera_set(16).to(dev)
    Ks = sc.Ks.to(dev)
    lib = _native.lib()
    fn = lib.hgsr_debug_wgtime
    fn.argtypes = [ct.c_void_p]
    buf = np.zeros((2, SLOTS, 3), np.uint64)
    g = torch.Generator().manual_seed(5)
    for v in list(range(0, 16, 3)):
        ps = [t.to(dev).clone().requires_grad_(True) for t in (sc.means, sc.quats, sc.scales, sc.opacities, sc.colors)]
        rc, ra, meta = G.rasterization(*ps, cams[v][None], Ks, W, H, packed=False, render_mode="RGB+ED")
        w = torch.randn(rc.shape, generator=g).to(dev)
        (rc * w).sum().backward()
        torch.cuda.synchronize()
        assert fn(buf.ctypes.data) == 0
        offs = meta["isect_offsets"].reshape(-1).long().cpu().numpy()
        n = int(meta["flatten_ids"].numel())
        cnt = np.diff(np.append(offs, n))
        nb = cnt.size
        rec = {"view": v, "isects": n, "bins": nb}
        for k, name in ((0, "fwd"), (1, "bwd")):
            t0, t1, b = (buf[k, :nb, i].astype(np.int64) for i in range(3))
            d = (t1 - t0) * 10e-3  # us
            span = (t1.max() - t0.min()) * 10e-3
            i = int(np.argmax(d))
            # 256 CUs x 8 workgroups (fwd: 4 waves each, one per SIMD, 8 waves/SIMD); bwd: 7
            cap = 256 * (8 if k == 0 else 7)
            c = cnt[b]
            rec[name] = {"span_us": round(float(span), 1), "wg_mean_us": round(float(d.mean()), 2),
                         "wg_p99_us": round(float(np.percentile(d, 99)), 1), "wg_max_us": round(float(d.max()), 1),
                         "max_wg_start_us": round(float((t0[i] - t0.min()) * 10e-3), 1), "max_wg_bin_count": int(c[i]),
                         "implied_resident_wgs_per_cu": round(float(d.sum() / span / 256), 2), "capacity_wgs_per_cu": cap // 256,
                         "last_start_us": round(float((t0.max() - t0.min()) * 10e-3), 1),
                         "corr_time_count": round(float(np.corrcoef(d, c)[0, 1]), 3)}
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
