"""ctypes binding of libhgsr.so (the C ABI declared in include/hgsr.h).

The product path has no CPU fallback: if the library is missing, or a tensor is
not on the HIP device, the call raises.  Device pointers and the current torch
stream are passed straight through; the library never allocates.
"""
from __future__ import annotations

import ctypes as ct
import os
import threading

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
# HGSR_LIB: developer override (benchmarking alternative builds of the same sources)
LIB_PATH = os.environ.get("HGSR_LIB") or os.path.join(_HERE, "_lib", "libhgsr.so")

_lock = threading.Lock()
_lib = None

P = ct.c_void_p
I = ct.c_int
I64 = ct.c_int64
F = ct.c_float
SZ = ct.c_size_t

# name -> (restype, argtypes)
_SIGS = {
    "hgsr_version": (I, []),
    "hgsr_last_error": (ct.c_char_p, []),
    "hgsr_project3d_fwd": (I, [I, I, P, P, P, P, P, I, I, F, F, F, F, P, P, P, P, P]),
    "hgsr_project3d_bwd": (I, [I, I, P, P, P, P, P, I, I, F, P, P, P, P, P, P, P, P, P, P, P]),
    "hgsr_project2d_fwd": (I, [I, I, P, P, P, P, P, I, I, F, F, F, P, P, P, P, P, P]),
    "hgsr_project2d_bwd": (I, [I, I, P, P, P, P, P, I, I, P, P, P, P, P, P, P, P, P, P, P]),
    "hgsr_sh_fwd": (I, [I, I, I64, P, P, P, P, P]),
    "hgsr_sh_bwd": (I, [I, I, I64, P, P, P, P, P, P, P]),
    "hgsr_sh_rgb_fwd": (I, [I, I, I, I, P, P, P, P, I, P, P, P]),
    "hgsr_sh_rgb_bwd": (I, [I, I, I, I, P, P, P, P, I, P, P, P, P, P]),
    "hgsr_isect_ws1_bytes": (SZ, [I, I, I, I]),
    "hgsr_isect_ws2_bytes": (SZ, [I64, I64]),
    "hgsr_isect_count": (I, [I, I, P, P, I, I, I, P, P, P, P, SZ, P]),
    "hgsr_isect_emit_sorted": (I, [I, I, P, P, P, I, I, I, P, I64, I64, P, P, P, SZ, P, SZ, P, P]),
    "hgsr_isect_emit_unsorted": (I, [I, I, P, P, P, I, I, I, P, P, P, P]),
    "hgsr_isect_offset_encode": (I, [I64, P, I, I, I, P, P]),
    "hgsr_raster3d_fwd_ws_bytes": (SZ, [I, I, I]),
    "hgsr_raster3d_fwd": (I, [I, I, I, P, P, P, P, P, I, I, I, I, I, P, I64, P, P, P, P, P, SZ, P]),
    "hgsr_raster3d_bwd_ws_bytes": (SZ, [I, I, I, I64, I]),
    "hgsr_raster3d_bwd": (I, [I, I, I, P, P, P, P, P, I, I, I, I, I, P, I64, P, P, P, P, P, P, P, P, P, P, P,
                              P, SZ, P]),
    "hgsr_raster3d_fwd_fused": (I, [I, I, I, P, P, P, I, P, I, P, I, P, I, I, I, I, I, P, I64, P, P, P, P, P, SZ,
                                    P]),
    "hgsr_raster3d_bwd_fused": (I, [I, I, I, P, P, P, I, P, I, P, I, P, I, I, I, I, I, P, I64, P, P, P, P, P, P,
                                    P, P, P, P, P, P, P, P, SZ, P, SZ, I, P, I, P]),
    "hgsr_raster3d_qmask_bytes": (SZ, [I, I, I, I64]),
    "hgsr_raster3d_pack_fused": (I, [I, I, I, P, P, P, I, P, P, I, P, P, I, I, I, P, SZ, P]),
    "hgsr_raster3d_fwd_packed": (I, [I, I, I, I, I, P, I, I, I, I, I, P, I64, P, P, P, P, P, SZ, P, SZ, P, SZ,
                                     P, P]),
    "hgsr_raster2d_fwd_ws_bytes": (SZ, [I, I, I]),
    "hgsr_raster2d_fwd": (I, [I, I, I, P, P, P, P, P, P, I, I, I, I, I, P, I64, P, P, P, P, P, P, P, P, P, SZ, P]),
    "hgsr_raster2d_pack_fused": (I, [I, I, I, P, P, P, I, P, P, I, P, P, P, I, I, I, P, SZ, P]),
    "hgsr_raster2d_fwd_packed": (I, [I, I, I, I, I, P, I, I, I, I, I, P, I64, P, P, P, P, P, P, P, P, P, SZ, P, SZ,
                                     P, SZ, P, P, P]),
    "hgsr_raster2d_bwd_ws_bytes": (SZ, [I, I, I, I64, I]),
    "hgsr_raster2d_bwd": (I, [I, I, I, P, P, P, P, P, P, I, I, I, I, I, P, I64, P, P, P, P, P, P, P, P, P, P,
                              P, P, P, P, SZ, P]),
    "hgsr_raster2d_fwd_fused": (I, [I, I, I, P, P, P, I, P, I, P, I, P, P, I, I, I, I, I, P, I64, P, P, P, P, P, P,
                                    P, P, P, SZ, P]),
    "hgsr_raster2d_bwd_fused": (I, [I, I, I, P, P, P, I, P, I, P, I, P, P, I, I, I, I, I, P, I64, P, P, P, P, P,
                                    P, P, P, P, P, P, P, P, P, P, P, SZ, P, SZ, I, P, P, P, I, P]),
    "hgsr_lod_mask": (I, [I, P, P, P, P, F, F, F, I, P, P]),
    "hgsr_decode_ws_bytes": (SZ, [I]),
    "hgsr_decode_count": (I, [I, I, I, I, I, P, P, P, P, P, P, SZ, P, P, P]),
    "hgsr_decode_fwd": (I, [I, I, I, I, I, P, P, P, P, P, P, P, P, P, P, P, P, P, P, P, P, SZ, P]),
    "hgsr_decode_bwd_ws_bytes": (SZ, [I]),
    "hgsr_decode_set_color_bwd": (I, [I]),
    "hgsr_decode_bwd": (I, [I, I, I, I, I, P, P, P, P, P, P, P, P, P, P, P, P, P, P, P, P, P, P, P, I, P, SZ, P]),
    "hgsr_loss_ws_bytes": (SZ, [I, I, I]),
    "hgsr_training_statis": (I, [I, I, I, I, I, I, P, P, P, P, P, P, P, P, P, P, P, P, P, P]),
    "hgsr_voxel_dedup_ws_bytes": (SZ, [I64]),
    "hgsr_voxel_dedup": (I, [I64, P, I64, P, P, P, P, SZ, P]),
    "hgsr_scatter_max": (I, [I64, I, P, P, I64, P, P]),
    "hgsr_weed_out": (I, [I64, P, P, I, P, F, F, I, I, F, P, P]),
    "hgsr_loss_fwd": (I, [I, I, I, P, P, P, P, P, P, P, I64, I, P, P, P, SZ, P]),
    "hgsr_loss_bwd": (I, [I, I, I, P, P, P, P, P, P, P, I64, I, P, P, P, I, P, P, P, P, SZ, P]),
    "hgsr_depth_normal_fwd": (I, [I, I, I, P, P, P, P, I, I, P, P]),
    "hgsr_depth_normal_bwd": (I, [I, I, I, P, P, P, P, I, I, P, P, P]),
    "hgsr_rotate3": (I, [I, I64, P, I, I, I, P, P, P]),
    "hgsr_adam_step": (I, [I, P, ct.c_double, ct.c_double, ct.c_double, P]),
    "hgsr_explicit_ws_bytes": (SZ, [I64]),
    "hgsr_explicit_count": (I, [I64, P, P, P, P, F, F, F, I, P, P, P, SZ, P, P]),
    "hgsr_explicit_gather": (I, [I64, I, P, P, P, P, P, P, P, P, SZ, P, P, P, P, P, P, P]),
    "hgsr_explicit_scatter": (I, [I64, I, P, P, SZ, P, P, P, P, P, P, P, P, P, P, P, P]),
    "hgsr_mask_index": (I, [I64, P, P, SZ, P, P]),
    "hgsr_anchor_prefilter": (I, [I, P, P, P, I, P, P, I, I, F, F, F, P, P, P, F, F, F, I, P, P]),
    "hgsr_activate_fwd": (I, [I64, P, P, P, P, P]),
    "hgsr_activate_bwd": (I, [I64, P, P, P, P, P, P, P]),
    "hgsr_timing_enable": (I, [I]),
    "hgsr_timing_reset": (I, []),
    "hgsr_timing_only": (I, [ct.c_char_p]),
    "hgsr_timing_pairs": (I, [ct.POINTER(ct.c_ulonglong), I]),
    "hgsr_timing_exec_pairs": (I, [ct.POINTER(ct.c_ulonglong)]),
    "hgsr_timing_query": (I, [ct.c_char_p, ct.POINTER(ct.c_double), ct.POINTER(I64)]),
}

EXPORTED = tuple(n for n in _SIGS)


def lib():
    """Load libhgsr.so once (raises if it was not built)."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise RuntimeError(
                    f"hgsr native library not found at {LIB_PATH}; build it with "
                    "`python -c 'import __graft_entry__ as g; g.build()'` (no CPU fallback exists)")
            h = ct.CDLL(LIB_PATH)
            for name, (res, args) in _SIGS.items():
                fn = getattr(h, name)
                fn.restype = res
                fn.argtypes = args
            _lib = h
    return _lib


def call(name, *args):
    st = getattr(lib(), name)(*args)
    if st != 0:
        msg = lib().hgsr_last_error().decode(errors="replace")
        raise RuntimeError(f"{name} failed ({st}): {msg}")


def kernel_time(kernel: str):
    """(total_ms, launches) recorded for `kernel` since the last hgsr_timing_reset()."""
    tot = ct.c_double(0.0)
    cnt = ct.c_int64(0)
    call("hgsr_timing_query", kernel.encode(), ct.byref(tot), ct.byref(cnt))
    return tot.value, cnt.value


def size_query(name, *args) -> int:
    return int(getattr(lib(), name)(*args))


def stream(dev=None) -> int:
    return torch.cuda.current_stream(dev).cuda_stream


def ptr(t):
    """Device pointer of a contiguous HIP tensor (None -> NULL)."""
    if t is None:
        return None
    if not t.is_cuda:
        raise RuntimeError("hgsr: tensor must live on the HIP device (no CPU path)")
    if not t.is_contiguous():
        raise RuntimeError("hgsr: tensor must be contiguous")
    return t.data_ptr()
