"""ctypes front-end of the C oracle (oracle/hgsr_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py as the checker.  The product package
(horizongs_amd / gsplat alias) never imports this module.

All arrays are numpy, C-contiguous; dtype float32 for the f32 build ("checker",
same operation order as the HIP kernels) or float64 for the f64 build (used for
finite-difference checks).  Every function follows the gsplat semantics that the
reference calls at gaussian_renderer/render.py:40-76 and :149-186.
"""
from __future__ import annotations

import ctypes as ct
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIBS: dict = {}

P = ct.c_void_p
I32 = ct.c_int
I64 = ct.c_int64


def build() -> None:
    """Compile the oracle shared objects (gcc, no GPU needed)."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def _lib(dtype):
    key = np.dtype(dtype).name
    if key in _LIBS:
        return _LIBS[key]
    name = "liboracle_f32.so" if key == "float32" else "liboracle_f64.so"
    path = os.path.join(_HERE, "_build", name)
    if not os.path.exists(path):
        build()
    lib = ct.CDLL(path)
    _LIBS[key] = lib
    return lib


def _fn(dtype, name):
    pfx = "oracle32_" if np.dtype(dtype) == np.float32 else "oracle64_"
    return getattr(_lib(dtype), pfx + name)


def _p(a):
    if a is None:
        return None
    assert a.flags["C_CONTIGUOUS"], "oracle arrays must be C-contiguous"
    return a.ctypes.data_as(P)


def _c(a, dtype):
    return np.ascontiguousarray(a, dtype=dtype)


def _real(dtype):
    return ct.c_float if np.dtype(dtype) == np.float32 else ct.c_double


# --------------------------------------------------------------------------
# projection
# --------------------------------------------------------------------------
def proj3d_fwd(means, quats, scales, viewmats, Ks, W, H, eps2d=0.3, near=0.01, far=1e10,
               radius_clip=0.0, dtype=np.float32):
    means, quats, scales = _c(means, dtype), _c(quats, dtype), _c(scales, dtype)
    viewmats, Ks = _c(viewmats, dtype), _c(Ks, dtype)
    C, N = viewmats.shape[0], means.shape[0]
    radii = np.zeros((C, N), np.int32)
    means2d = np.zeros((C, N, 2), dtype)
    depths = np.zeros((C, N), dtype)
    conics = np.zeros((C, N, 3), dtype)
    R = _real(dtype)
    _fn(dtype, "proj3d_fwd")(I32(C), I32(N), _p(means), _p(quats), _p(scales), _p(viewmats), _p(Ks),
                             I32(W), I32(H), R(eps2d), R(near), R(far), R(radius_clip), _p(radii),
                             _p(means2d), _p(depths), _p(conics))
    return radii, means2d, depths, conics


def proj3d_bwd(means, quats, scales, viewmats, Ks, W, H, radii, conics, v_means2d, v_depths,
               v_conics, eps2d=0.3, dtype=np.float32):
    means, quats, scales = _c(means, dtype), _c(quats, dtype), _c(scales, dtype)
    viewmats, Ks = _c(viewmats, dtype), _c(Ks, dtype)
    C, N = viewmats.shape[0], means.shape[0]
    v_means = np.zeros((N, 3), dtype)
    v_quats = np.zeros((N, 4), dtype)
    v_scales = np.zeros((N, 3), dtype)
    _fn(dtype, "proj3d_bwd")(I32(C), I32(N), _p(means), _p(quats), _p(scales), _p(viewmats), _p(Ks),
                             I32(W), I32(H), _real(dtype)(eps2d), _p(_c(radii, np.int32)),
                             _p(_c(conics, dtype)), _p(_c(v_means2d, dtype)), _p(_c(v_depths, dtype)),
                             _p(_c(v_conics, dtype)), _p(v_means), _p(v_quats), _p(v_scales))
    return v_means, v_quats, v_scales


def proj2d_fwd(means, quats, scales, viewmats, Ks, W, H, near=0.01, far=1e10, radius_clip=0.0,
               dtype=np.float32):
    means, quats, scales = _c(means, dtype), _c(quats, dtype), _c(scales, dtype)
    viewmats, Ks = _c(viewmats, dtype), _c(Ks, dtype)
    C, N = viewmats.shape[0], means.shape[0]
    radii = np.zeros((C, N), np.int32)
    means2d = np.zeros((C, N, 2), dtype)
    depths = np.zeros((C, N), dtype)
    rt = np.zeros((C, N, 3, 3), dtype)
    normals = np.zeros((C, N, 3), dtype)
    R = _real(dtype)
    _fn(dtype, "proj2d_fwd")(I32(C), I32(N), _p(means), _p(quats), _p(scales), _p(viewmats), _p(Ks),
                             I32(W), I32(H), R(near), R(far), R(radius_clip), _p(radii), _p(means2d),
                             _p(depths), _p(rt), _p(normals))
    return radii, means2d, depths, rt, normals


def proj2d_bwd(means, quats, scales, viewmats, Ks, W, H, radii, ray_transforms, v_means2d,
               v_depths, v_ray_transforms, v_normals, dtype=np.float32):
    means, quats, scales = _c(means, dtype), _c(quats, dtype), _c(scales, dtype)
    viewmats, Ks = _c(viewmats, dtype), _c(Ks, dtype)
    C, N = viewmats.shape[0], means.shape[0]
    v_means = np.zeros((N, 3), dtype)
    v_quats = np.zeros((N, 4), dtype)
    v_scales = np.zeros((N, 3), dtype)
    _fn(dtype, "proj2d_bwd")(I32(C), I32(N), _p(means), _p(quats), _p(scales), _p(viewmats), _p(Ks),
                             I32(W), I32(H), _p(_c(radii, np.int32)), _p(_c(ray_transforms, dtype)),
                             _p(_c(v_means2d, dtype)), _p(_c(v_depths, dtype)),
                             _p(_c(v_ray_transforms, dtype)), _p(_c(v_normals, dtype)), _p(v_means),
                             _p(v_quats), _p(v_scales))
    return v_means, v_quats, v_scales


# --------------------------------------------------------------------------
# spherical harmonics
# --------------------------------------------------------------------------
def sh_fwd(degree, dirs, coeffs, masks=None, dtype=np.float32):
    dirs = _c(dirs, dtype).reshape(-1, 3)
    K = coeffs.shape[-2]
    coeffs = _c(coeffs, dtype).reshape(-1, K, 3)
    n = dirs.shape[0]
    m = None if masks is None else _c(masks, np.uint8).reshape(-1)
    out = np.zeros((n, 3), dtype)
    _fn(dtype, "sh_fwd")(I32(degree), I32(K), I64(n), _p(dirs), _p(coeffs), _p(m), _p(out))
    return out


def sh_bwd(degree, dirs, coeffs, v_colors, masks=None, dtype=np.float32):
    dirs = _c(dirs, dtype).reshape(-1, 3)
    K = coeffs.shape[-2]
    coeffs = _c(coeffs, dtype).reshape(-1, K, 3)
    n = dirs.shape[0]
    m = None if masks is None else _c(masks, np.uint8).reshape(-1)
    v_coeffs = np.zeros_like(coeffs)
    v_dirs = np.zeros_like(dirs)
    _fn(dtype, "sh_bwd")(I32(degree), I32(K), I64(n), _p(dirs), _p(coeffs), _p(m),
                         _p(_c(v_colors, dtype).reshape(-1, 3)), _p(v_coeffs), _p(v_dirs))
    return v_coeffs, v_dirs


# --------------------------------------------------------------------------
# tile intersection / sort / offsets
# --------------------------------------------------------------------------
def tile_grid(W, H, tile_size=16):
    return (W + tile_size - 1) // tile_size, (H + tile_size - 1) // tile_size


def isect_tiles(means2d, radii, depths, tile_size, tw, th, sort=True, dtype=np.float32):
    means2d, depths = _c(means2d, dtype), _c(depths, dtype)
    radii = _c(radii, np.int32)
    C, N = radii.shape
    tpg = np.zeros((C, N), np.int32)
    f = _fn(dtype, "isect_tiles")
    f.restype = I64
    n = f(I32(C), I32(N), _p(means2d), _p(radii), _p(depths), I32(tile_size), I32(tw), I32(th),
          _p(tpg), None, None, I32(0))
    ids = np.zeros((max(n, 1),), np.int64)
    fl = np.zeros((max(n, 1),), np.int32)
    f(I32(C), I32(N), _p(means2d), _p(radii), _p(depths), I32(tile_size), I32(tw), I32(th), _p(tpg),
      _p(ids), _p(fl), I32(1 if sort else 0))
    return tpg, ids[:n], fl[:n]


def isect_offsets(isect_ids, C, tw, th):
    isect_ids = _c(isect_ids, np.int64)
    out = np.zeros((C, th, tw), np.int32)
    _lib(np.float32).oracle_isect_offsets(I64(isect_ids.shape[0]), _p(isect_ids), I32(C), I32(tw),
                                          I32(th), _p(out))
    return out


# --------------------------------------------------------------------------
# rasterization
# --------------------------------------------------------------------------
def raster3d_fwd(means2d, conics, colors, opacities, backgrounds, W, H, tile_size, offsets,
                 flatten_ids, dtype=np.float32, return_stopped=False):
    C, N = means2d.shape[:2]
    D = colors.shape[-1]
    th, tw = offsets.shape[1:]
    rc = np.zeros((C, H, W, D), dtype)
    ra = np.zeros((C, H, W, 1), dtype)
    last = np.zeros((C, H, W), np.int32)
    stopped = np.zeros((C, H, W), np.uint8)  # 1 where the list ended at the T <= 1e-4 stop
    margin = np.zeros((C, H, W), dtype)       # smallest relative distance of a value decision to its threshold
    gmargin = np.zeros((C, H, W), dtype)      # ... of any decision, incl. gradient-path switches
    bg = None if backgrounds is None else _c(backgrounds, dtype)
    _fn(dtype, "raster3d_fwd")(I32(C), I32(N), I32(D), _p(_c(means2d, dtype)), _p(_c(conics, dtype)),
                               _p(_c(colors, dtype)), _p(_c(opacities, dtype)), _p(bg), I32(W), I32(H),
                               I32(tile_size), I32(tw), I32(th), _p(_c(offsets, np.int32)),
                               I64(flatten_ids.shape[0]), _p(_c(flatten_ids, np.int32)), _p(rc),
                               _p(ra), _p(last), _p(stopped), _p(margin), _p(gmargin))
    return (rc, ra, last, stopped, margin, gmargin) if return_stopped else (rc, ra, last)


def raster3d_bwd(means2d, conics, colors, opacities, backgrounds, W, H, tile_size, offsets,
                 flatten_ids, render_alphas, last_ids, v_render_colors, v_render_alphas,
                 dtype=np.float32):
    C, N = means2d.shape[:2]
    D = colors.shape[-1]
    th, tw = offsets.shape[1:]
    v_means2d = np.zeros((C, N, 2), dtype)
    v_conics = np.zeros((C, N, 3), dtype)
    v_colors = np.zeros((C, N, D), dtype)
    v_opac = np.zeros((C, N), dtype)
    bg = None if backgrounds is None else _c(backgrounds, dtype)
    _fn(dtype, "raster3d_bwd")(I32(C), I32(N), I32(D), _p(_c(means2d, dtype)), _p(_c(conics, dtype)),
                               _p(_c(colors, dtype)), _p(_c(opacities, dtype)), _p(bg), I32(W), I32(H),
                               I32(tile_size), I32(tw), I32(th), _p(_c(offsets, np.int32)),
                               I64(flatten_ids.shape[0]), _p(_c(flatten_ids, np.int32)),
                               _p(_c(render_alphas, dtype)), _p(_c(last_ids, np.int32)),
                               _p(_c(v_render_colors, dtype)), _p(_c(v_render_alphas, dtype)),
                               _p(v_means2d), _p(v_conics), _p(v_colors), _p(v_opac))
    return v_means2d, v_conics, v_colors, v_opac


def raster2d_fwd(means2d, ray_transforms, colors, opacities, normals, backgrounds, W, H,
                 tile_size, offsets, flatten_ids, dtype=np.float32, return_stopped=False):
    C, N = means2d.shape[:2]
    D = colors.shape[-1]
    th, tw = offsets.shape[1:]
    rc = np.zeros((C, H, W, D), dtype)
    ra = np.zeros((C, H, W, 1), dtype)
    rn = np.zeros((C, H, W, 3), dtype)
    rd = np.zeros((C, H, W, 1), dtype)
    rm = np.zeros((C, H, W, 1), dtype)
    last = np.zeros((C, H, W), np.int32)
    med = np.zeros((C, H, W), np.int32)
    stopped = np.zeros((C, H, W), np.uint8)
    margin = np.zeros((C, H, W), dtype)
    gmargin = np.zeros((C, H, W), dtype)
    bg = None if backgrounds is None else _c(backgrounds, dtype)
    _fn(dtype, "raster2d_fwd")(I32(C), I32(N), I32(D), _p(_c(means2d, dtype)),
                               _p(_c(ray_transforms, dtype)), _p(_c(colors, dtype)),
                               _p(_c(opacities, dtype)), _p(_c(normals, dtype)), _p(bg), I32(W), I32(H),
                               I32(tile_size), I32(tw), I32(th), _p(_c(offsets, np.int32)),
                               I64(flatten_ids.shape[0]), _p(_c(flatten_ids, np.int32)), _p(rc),
                               _p(ra), _p(rn), _p(rd), _p(rm), _p(last), _p(med), _p(stopped),
                               _p(margin), _p(gmargin))
    out = (rc, ra, rn, rd, rm, last, med)
    return out + (stopped, margin, gmargin) if return_stopped else out


def raster2d_bwd(means2d, ray_transforms, colors, opacities, normals, backgrounds, W, H,
                 tile_size, offsets, flatten_ids, render_alphas, last_ids, v_render_colors,
                 v_render_alphas, v_render_normals, dtype=np.float32):
    C, N = means2d.shape[:2]
    D = colors.shape[-1]
    th, tw = offsets.shape[1:]
    v_means2d = np.zeros((C, N, 2), dtype)
    v_rt = np.zeros((C, N, 3, 3), dtype)
    v_colors = np.zeros((C, N, D), dtype)
    v_opac = np.zeros((C, N), dtype)
    v_normals = np.zeros((C, N, 3), dtype)
    v_dens = np.zeros((C, N, 2), dtype)
    bg = None if backgrounds is None else _c(backgrounds, dtype)
    _fn(dtype, "raster2d_bwd")(I32(C), I32(N), I32(D), _p(_c(means2d, dtype)),
                               _p(_c(ray_transforms, dtype)), _p(_c(colors, dtype)),
                               _p(_c(opacities, dtype)), _p(_c(normals, dtype)), _p(bg), I32(W), I32(H),
                               I32(tile_size), I32(tw), I32(th), _p(_c(offsets, np.int32)),
                               I64(flatten_ids.shape[0]), _p(_c(flatten_ids, np.int32)),
                               _p(_c(render_alphas, dtype)), _p(_c(last_ids, np.int32)),
                               _p(_c(v_render_colors, dtype)), _p(_c(v_render_alphas, dtype)),
                               _p(_c(v_render_normals, dtype)), _p(v_means2d), _p(v_rt),
                               _p(v_colors), _p(v_opac), _p(v_normals), _p(v_dens))
    return v_means2d, v_rt, v_colors, v_opac, v_normals, v_dens


def set_envelope(on, dtype=np.float64):
    """Switch the raster backwards of one build into envelope mode (see hgsr_oracle.c)."""
    _fn(dtype, "set_envelope")(I32(int(bool(on))))


def set_hitform(form, dtype=np.float32):
    """2DGS hit evaluation of one build: 0 gsplat's per-pixel cross product, 1 the plane form."""
    _fn(dtype, "set_hitform")(I32(int(form)))


def set_pixmask(mask, dtype=np.float32):
    """Raster forwards composite only pixels whose mask byte is set (hgsr_oracle.c set_pixmask;
    None clears).  The caller keeps `mask` (uint8, C-contiguous [C*rows*W]) alive while set."""
    _fn(dtype, "set_pixmask")(None if mask is None else _p(mask))


def set_alphaform(form, dtype=np.float32):
    """3DGS alpha evaluation of one build: 0 gsplat's exp(-sigma), 1 the kernels' log2(e)-scaled
    conic with explicit FMAs and exp2 (hgsr_oracle.c vis3)."""
    _fn(dtype, "set_alphaform")(I32(int(form)))


NEAR_K = 8  # hgsr_oracle.c NEAR_K
_NEAR_KEEP = {}


def set_near(near, dtype=np.float32):
    """Near-threshold decision lists of one build (hgsr_oracle.c set_near): None, or a dict with
    "thr" (> 0: record mode, 0: force mode) and arrays "n" [P] int32, "idx" [P,K] int64, "kind" /
    "out" [P,K] int32, "m" [P,K] float64 (P = C x rows x W).  Held until the next call."""
    key = np.dtype(dtype).name
    if near is None:
        _NEAR_KEEP.pop(key, None)
        _fn(dtype, "set_near")(ct.c_double(0.0), None, None, None, None, None)
        return
    for k, t in (("n", np.int32), ("idx", np.int64), ("kind", np.int32), ("out", np.int32), ("m", np.float64)):
        assert near[k].dtype == t and near[k].flags["C_CONTIGUOUS"], k
    _NEAR_KEEP[key] = near
    _fn(dtype, "set_near")(ct.c_double(float(near["thr"])), _p(near["n"]), _p(near["idx"]), _p(near["kind"]),
                           _p(near["out"]), _p(near["m"]))
