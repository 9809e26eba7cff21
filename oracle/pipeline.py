"""Oracle composition of gsplat.rasterization / rasterization_2dgs (numpy + C oracle).

TEST INFRASTRUCTURE ONLY (checker for tests/, smoke() and the bench CPU
baseline).  Restates the glue gsplat performs around its kernels, as the
reference calls it (gaussian_renderer/render.py:40-76): SH colour (+0.5,
clamp_min 0) when sh_degree is given, RGB+ED depth channel with a zero
background channel, tile intersection + sort, rasterization, expected-depth
normalisation by clamp_min(alpha, 1e-10).  backward() propagates upstream
gradients through the same chain to means / quats / scales / opacities / colors.
"""
from __future__ import annotations

import numpy as np

from . import oracle as O


def _campos(viewmats):
    R = viewmats[:, :3, :3]
    t = viewmats[:, :3, 3]
    return -np.einsum("cji,cj->ci", R, t)


class Raster3D:
    """3DGS forward + backward through the C oracle (float32 by default)."""

    def __init__(self, means, quats, scales, opacities, colors, viewmats, Ks, W, H, sh_degree=None,
                 backgrounds=None, render_mode="RGB+ED", eps2d=0.3, near=0.01, far=1e10, tile_size=16,
                 dtype=np.float32):
        self.dt = dtype
        c = lambda a: None if a is None else np.ascontiguousarray(a, dtype=dtype)  # noqa: E731
        self.means, self.quats, self.scales = c(means), c(quats), c(scales)
        self.opacities, self.colors = c(opacities), c(colors)
        self.viewmats, self.Ks = c(viewmats), c(Ks)
        self.W, self.H, self.sh_degree = W, H, sh_degree
        self.bg = c(backgrounds)
        self.mode = render_mode
        self.eps2d, self.near, self.far, self.ts = eps2d, near, far, tile_size

    def forward(self):
        dt = self.dt
        C, Nn = self.viewmats.shape[0], self.means.shape[0]
        self.radii, self.means2d, self.depths, self.conics = O.proj3d_fwd(
            self.means, self.quats, self.scales, self.viewmats, self.Ks, self.W, self.H, self.eps2d, self.near,
            self.far, dtype=dt)
        if self.sh_degree is None:
            cols = np.broadcast_to(self.colors, (C,) + self.colors.shape).astype(dt)
            self.sh_pre = None
        else:
            self.dirs = (self.means[None] - _campos(self.viewmats)[:, None]).astype(dt)
            K = self.colors.shape[-2]
            shs = np.broadcast_to(self.colors, (C, Nn, K, 3))
            raw = O.sh_fwd(self.sh_degree, self.dirs.reshape(-1, 3), shs.reshape(-1, K, 3),
                           (self.radii > 0).reshape(-1), dtype=dt).reshape(C, Nn, 3)
            self.sh_pre = raw + dt(0.5)
            cols = np.maximum(self.sh_pre, 0).astype(dt)
        bg = self.bg
        if self.mode in ("RGB+D", "RGB+ED"):
            cols = np.concatenate([cols, self.depths[..., None]], -1)
            if bg is not None:
                bg = np.concatenate([bg, np.zeros((C, 1), dt)], -1)
        elif self.mode in ("D", "ED"):
            cols = self.depths[..., None].copy()
            bg = None if bg is None else np.zeros((C, 1), dt)
        self.cols, self.bg_r = np.ascontiguousarray(cols, dt), bg
        self.tw, self.th = O.tile_grid(self.W, self.H, self.ts)
        self.tpg, self.isect_ids, self.flatten_ids = O.isect_tiles(self.means2d, self.radii, self.depths, self.ts,
                                                                   self.tw, self.th, dtype=dt)
        self.offsets = O.isect_offsets(self.isect_ids, C, self.tw, self.th)
        self.opac_c = np.ascontiguousarray(np.broadcast_to(self.opacities, (C, Nn)), dt)
        self.rc_raw, self.ra, self.last = O.raster3d_fwd(self.means2d, self.conics, self.cols, self.opac_c,
                                                         self.bg_r, self.W, self.H, self.ts, self.offsets,
                                                         self.flatten_ids, dtype=dt)
        out = self.rc_raw.copy()
        if self.mode in ("ED", "RGB+ED"):
            out[..., -1:] = self.rc_raw[..., -1:] / np.maximum(self.ra, dt(1e-10))
        self.render_colors = out
        return out, self.ra

    def backward(self, v_render_colors, v_render_alphas):
        """Returns dict of grads: means, quats, scales, opacities, colors, means2d."""
        dt = self.dt
        C, Nn = self.viewmats.shape[0], self.means.shape[0]
        v_rc = np.array(v_render_colors, dt)
        v_ra = np.array(v_render_alphas, dt)
        if self.mode in ("ED", "RGB+ED"):
            den = np.maximum(self.ra, dt(1e-10))
            g = v_rc[..., -1:]
            v_ra = v_ra + np.where(self.ra >= dt(1e-10), -g * self.rc_raw[..., -1:] / (den * den), 0).astype(dt)
            v_rc = v_rc.copy()
            v_rc[..., -1:] = g / den
        vm2, vcon, vcol, vop = O.raster3d_bwd(self.means2d, self.conics, self.cols, self.opac_c, self.bg_r, self.W,
                                              self.H, self.ts, self.offsets, self.flatten_ids, self.ra, self.last,
                                              v_rc, v_ra, dtype=dt)
        v_depths = np.zeros((C, Nn), dt)
        if self.mode in ("RGB+D", "RGB+ED", "D", "ED"):
            v_depths += vcol[..., -1]
            vcol_rgb = vcol[..., :-1]
        else:
            vcol_rgb = vcol
        grads = {"means2d": vm2, "conics": vcon, "opacities": vop.sum(0)}
        v_means_extra = np.zeros((Nn, 3), dt)
        if self.mode not in ("D", "ED"):
            if self.sh_degree is None:
                grads["colors"] = vcol_rgb.sum(0)
            else:
                v_sh = np.where(self.sh_pre >= 0, vcol_rgb, 0).astype(dt)
                K = self.colors.shape[-2]
                shs = np.broadcast_to(self.colors, (C, Nn, K, 3))
                v_coeffs, v_dirs = O.sh_bwd(self.sh_degree, self.dirs.reshape(-1, 3), shs.reshape(-1, K, 3),
                                            v_sh.reshape(-1, 3), (self.radii > 0).reshape(-1), dtype=dt)
                grads["colors"] = v_coeffs.reshape(C, Nn, K, 3).sum(0)
                v_means_extra += v_dirs.reshape(C, Nn, 3).sum(0)
        vm, vq, vs = O.proj3d_bwd(self.means, self.quats, self.scales, self.viewmats, self.Ks, self.W, self.H,
                                  self.radii, self.conics, vm2, v_depths, vcon, self.eps2d, dtype=dt)
        grads["means"] = vm + v_means_extra
        grads["quats"] = vq
        grads["scales"] = vs
        return grads


class Raster2D:
    """2DGS forward (+ backward of colors/alphas/normals outputs) through the C oracle."""

    def __init__(self, means, quats, scales, opacities, colors, viewmats, Ks, W, H, backgrounds=None,
                 render_mode="RGB+ED", near=0.01, far=1e10, tile_size=16, dtype=np.float32):
        self.dt = dtype
        c = lambda a: None if a is None else np.ascontiguousarray(a, dtype=dtype)  # noqa: E731
        self.means, self.quats, self.scales = c(means), c(quats), c(scales)
        self.opacities, self.colors = c(opacities), c(colors)
        self.viewmats, self.Ks = c(viewmats), c(Ks)
        self.W, self.H, self.bg = W, H, c(backgrounds)
        self.mode, self.near, self.far, self.ts = render_mode, near, far, tile_size

    def forward(self):
        dt = self.dt
        C, Nn = self.viewmats.shape[0], self.means.shape[0]
        (self.radii, self.means2d, self.depths, self.rt,
         self.normals) = O.proj2d_fwd(self.means, self.quats, self.scales, self.viewmats, self.Ks, self.W, self.H,
                                      self.near, self.far, dtype=dt)
        cols = np.broadcast_to(self.colors, (C,) + self.colors.shape).astype(dt)
        bg = self.bg
        assert self.mode in ("RGB+ED", "RGB+D")
        cols = np.concatenate([cols, self.depths[..., None]], -1)
        if bg is not None:
            bg = np.concatenate([bg, np.zeros((C, 1), dt)], -1)
        self.cols, self.bg_r = np.ascontiguousarray(cols, dt), bg
        self.tw, self.th = O.tile_grid(self.W, self.H, self.ts)
        self.tpg, self.isect_ids, self.flatten_ids = O.isect_tiles(self.means2d, self.radii, self.depths, self.ts,
                                                                   self.tw, self.th, dtype=dt)
        self.offsets = O.isect_offsets(self.isect_ids, C, self.tw, self.th)
        self.opac_c = np.ascontiguousarray(np.broadcast_to(self.opacities, (C, Nn)), dt)
        (self.rc_raw, self.ra, self.rn, self.rd, self.rm, self.last,
         self.med) = O.raster2d_fwd(self.means2d, self.rt, self.cols, self.opac_c, self.normals, self.bg_r, self.W,
                                    self.H, self.ts, self.offsets, self.flatten_ids, dtype=dt)
        out = self.rc_raw.copy()
        if self.mode == "RGB+ED":
            out[..., -1:] = self.rc_raw[..., -1:] / np.maximum(self.ra, dt(1e-10))
        self.render_colors = out
        return out, self.ra, self.rn

    def backward(self, v_render_colors, v_render_alphas, v_render_normals_cam):
        """Upstream grads w.r.t. render colors / alphas / CAMERA-frame normals -> Gaussian grads."""
        dt = self.dt
        C, Nn = self.viewmats.shape[0], self.means.shape[0]
        v_rc = np.array(v_render_colors, dt)
        v_ra = np.array(v_render_alphas, dt)
        if self.mode == "RGB+ED":
            den = np.maximum(self.ra, dt(1e-10))
            g = v_rc[..., -1:]
            v_ra = v_ra + np.where(self.ra >= dt(1e-10), -g * self.rc_raw[..., -1:] / (den * den), 0).astype(dt)
            v_rc = v_rc.copy()
            v_rc[..., -1:] = g / den
        vm2, vrt, vcol, vop, vn, vdens = O.raster2d_bwd(
            self.means2d, self.rt, self.cols, self.opac_c, self.normals, self.bg_r, self.W, self.H, self.ts,
            self.offsets, self.flatten_ids, self.ra, self.last, v_rc, v_ra, np.asarray(v_render_normals_cam, dt),
            dtype=dt)
        v_depths = vcol[..., -1].copy()
        vm, vq, vs = O.proj2d_bwd(self.means, self.quats, self.scales, self.viewmats, self.Ks, self.W, self.H,
                                  self.radii, self.rt, vm2, v_depths, vrt, vn, dtype=dt)
        return {"means": vm, "quats": vq, "scales": vs, "opacities": vop.sum(0), "colors": vcol[..., :-1].sum(0),
                "means2d": vm2, "densify": vdens}
