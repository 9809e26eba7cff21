"""Measurement-only: price the raster3d backward's float atomics (plain-store build)."""
import ctypes as ct, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from horizongs_amd import _native as NAT, gsplat_api as G
from horizongs_amd.synthetic import c2
sc = c2(); dev = "cuda:0"
t = [x.to(dev) for x in (sc.means, sc.quats, sc.scales, sc.opacities, sc.colors, sc.viewmats, sc.Ks)]
means, quats, scales, opac, cols, vm, K = t
out, alpha, meta = G.rasterization(means, quats, scales, opac, cols, vm, K, 1920, 1080, packed=False, render_mode="RGB+ED")
C, N, H, W = 1, means.shape[0], 1080, 1920
c4 = torch.cat([cols[None], meta["depths"][..., None]], -1).contiguous()
ws_b = NAT.size_query("hgsr_raster3d_fwd_ws_bytes", C, N, 4)
ws = torch.empty(ws_b, dtype=torch.uint8, device=dev)
rc = torch.empty(C, H, W, 4, device=dev); ra = torch.empty(C, H, W, 1, device=dev); last = torch.empty(C, H, W, dtype=torch.int32, device=dev)
NAT.call("hgsr_raster3d_fwd", C, N, 4, NAT.ptr(meta["means2d"].detach().contiguous()), NAT.ptr(meta["conics"].detach().contiguous()), NAT.ptr(c4), NAT.ptr(meta["opacities"].contiguous()), None, W, H, 16, 120, 68, NAT.ptr(meta["isect_offsets"]), meta["flatten_ids"].numel(), NAT.ptr(meta["flatten_ids"]), NAT.ptr(rc), NAT.ptr(ra), NAT.ptr(last), NAT.ptr(ws), ws_b, NAT.stream())
rows = torch.zeros(C * N * 16, device=dev)
vrc = torch.randn(C, H, W, 4, device=dev); vra = torch.randn(C, H, W, 1, device=dev)
f = NAT.lib().hgsr_diag_raster3d_bwd_noatomic_ms
f.restype = ct.c_double
f.argtypes = [ct.c_int, ct.c_int, ct.c_void_p, ct.c_void_p, ct.c_int, ct.c_int, ct.c_int, ct.c_int, ct.c_void_p, ct.c_int64, ct.c_void_p, ct.c_void_p, ct.c_void_p, ct.c_void_p, ct.c_void_p, ct.c_int, ct.c_void_p]
res = {0: [], 1: []}
for rep in range(6):
    for na in (0, 1):
        res[na].append(f(C, N, rows.data_ptr(), ws.data_ptr(), W, H, 120, 68, meta["isect_offsets"].data_ptr(), meta["flatten_ids"].numel(), meta["flatten_ids"].data_ptr(), ra.data_ptr(), last.data_ptr(), vrc.data_ptr(), vra.data_ptr(), na, NAT.stream()))
print("bwd with atomics ms", sorted(res[0]))
print("bwd plain stores ms", sorted(res[1]))
