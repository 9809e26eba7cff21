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


class _Band:
    # near-threshold decision lists of the raster calls (hgsr_oracle.c set_near): None, or the
    # dict of oracle.set_near (record mode: thr > 0, filled by forward(); force mode: thr = 0)
    decisions = None
    # uint8 [C*rows*W] or None: the raster calls composite only these pixels (hgsr_oracle.c
    # set_pixmask) -- for branch candidates whose other pixels are never read
    pixmask = None

    @property
    def Hr(self):
        return self.H if self.rows is None else min(self.rows, self.H)

    def _thresholds(self):
        """Context: the raster calls inside use this instance's decision lists."""
        band = self

        class _Ctx:
            def __enter__(self):
                if band.decisions is not None:
                    O.set_near(band.decisions, band.dt)
                if band.pixmask is not None:
                    O.set_pixmask(band.pixmask, band.dt)

            def __exit__(self, *exc):
                if band.decisions is not None:
                    O.set_near(None, band.dt)
                if band.pixmask is not None:
                    O.set_pixmask(None, band.dt)
        return _Ctx()

    def _shape(self):
        return (self.viewmats.shape[0], self.Hr, self.W)

    def record_near(self, thr):
        """Record mode: forward() lists every decision with margin < thr per pixel."""
        P = int(np.prod(self._shape()))
        K = O.NEAR_K
        self.decisions = {"thr": float(thr), "n": np.zeros(P, np.int32), "idx": np.full((P, K), -1, np.int64),
                     "kind": np.zeros((P, K), np.int32), "out": np.zeros((P, K), np.int32),
                     "m": np.zeros((P, K), np.float64)}

    def force_near(self, near):
        """Force mode: the listed decisions take the listed outcomes (forward and backward)."""
        self.decisions = {"thr": 0.0, "n": np.ascontiguousarray(near["n"], np.int32),
                     "idx": np.ascontiguousarray(near["idx"], np.int64),
                     "kind": np.ascontiguousarray(near["kind"], np.int32),
                     "out": np.ascontiguousarray(near["out"], np.int32),
                     "m": np.ascontiguousarray(near.get("m", np.zeros(near["idx"].shape)), np.float64)}


class Raster3D(_Band):
    """3DGS forward + backward through the C oracle (float32 by default)."""

    def __init__(self, means, quats, scales, opacities, colors, viewmats, Ks, W, H, sh_degree=None,
                 backgrounds=None, render_mode="RGB+ED", eps2d=0.3, near=0.01, far=1e10, tile_size=16,
                 dtype=np.float32, rows=None, alphaform=0):
        self.dt = dtype
        self.rows = rows  # rasterise only image rows [0, rows) (banded checks); None = all
        self.alphaform = alphaform  # 3DGS alpha evaluation form (hgsr_oracle.c vis3)
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
        O.set_alphaform(self.alphaform, dt)
        try:
            with self._thresholds():
                self.rc_raw, self.ra, self.last, self.stopped, self.margin, self.gmargin = O.raster3d_fwd(
                    self.means2d, self.conics, self.cols, self.opac_c, self.bg_r, self.W, self.Hr, self.ts,
                    self.offsets, self.flatten_ids, dtype=dt, return_stopped=True)
        finally:
            O.set_alphaform(0, dt)
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
        O.set_alphaform(self.alphaform, dt)
        try:
            with self._thresholds():
                vm2, vcon, vcol, vop = O.raster3d_bwd(self.means2d, self.conics, self.cols, self.opac_c, self.bg_r,
                                                      self.W, self.Hr, self.ts, self.offsets, self.flatten_ids,
                                                      self.ra, self.last, v_rc, v_ra, dtype=dt)
        finally:
            O.set_alphaform(0, dt)
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

    def envelope(self, v_render_colors, v_render_alphas):
        """Per-element magnitude envelopes E of every gradient of backward() (same keys):
        the raster backward in envelope mode (sum of |term| per output, hgsr_oracle.c) on
        |upstream|, then propagated through the projection / SH backward as |J|^T E, one
        input component at a time.  Any f32 evaluation of gradient i is within a small
        multiple of u * E_i of the exact value.  Use on the float64 instance after forward()."""
        dt = self.dt
        C, Nn = self.viewmats.shape[0], self.means.shape[0]
        v_rc = np.abs(np.array(v_render_colors, dt))
        v_ra = np.abs(np.array(v_render_alphas, dt))
        if self.mode in ("ED", "RGB+ED"):
            den = np.maximum(self.ra, dt(1e-10))
            g = v_rc[..., -1:]
            # alpha = 1 - T carries an absolute rounding error ~u, so the ED divide amplifies the
            # relative error of every term it feeds by ~(1 + 1 / alpha)
            k = 1 + 1 / den
            v_ra = v_ra + np.where(self.ra >= dt(1e-10), k * g * np.abs(self.rc_raw[..., -1:]) / (den * den),
                                   0).astype(dt)
            v_rc = v_rc.copy()
            v_rc[..., -1:] = k * g / den
        O.set_envelope(True, dt)
        try:
            with self._thresholds():
                vm2, vcon, vcol, vop = O.raster3d_bwd(self.means2d, self.conics, self.cols, self.opac_c, self.bg_r,
                                                      self.W, self.Hr, self.ts, self.offsets, self.flatten_ids,
                                                      self.ra, self.last, v_rc, v_ra, dtype=dt)
        finally:
            O.set_envelope(False, dt)
        v_depths = np.zeros((C, Nn), dt)
        if self.mode in ("RGB+D", "RGB+ED", "D", "ED"):
            v_depths += vcol[..., -1]
            vcol_rgb = vcol[..., :-1]
        else:
            vcol_rgb = vcol
        env = {"means2d": vm2, "conics": vcon, "opacities": vop.sum(0)}
        v_means_extra = np.zeros((Nn, 3), dt)
        if self.mode not in ("D", "ED"):
            if self.sh_degree is None:
                env["colors"] = vcol_rgb.sum(0)
            else:
                K = self.colors.shape[-2]
                shs = np.broadcast_to(self.colors, (C, Nn, K, 3))
                ec = np.zeros((C * Nn, K, 3), dt)
                for ch in range(3):  # |J|^T E one colour channel at a time
                    e1 = np.zeros((C * Nn, 3), dt)
                    e1[:, ch] = np.where(self.sh_pre >= 0, vcol_rgb, 0).reshape(-1, 3)[:, ch]
                    vc, vd = O.sh_bwd(self.sh_degree, self.dirs.reshape(-1, 3), shs.reshape(-1, K, 3), e1,
                                      (self.radii > 0).reshape(-1), dtype=dt)
                    ec += np.abs(vc)
                    v_means_extra += np.abs(vd).reshape(C, Nn, 3).sum(0)
                env["colors"] = ec.reshape(C, Nn, K, 3).sum(0)
        ups = {"m2x": None, "m2y": None, "d": None, "c0": None, "c1": None, "c2": None}
        acc = [np.zeros((Nn, 3), dt), np.zeros((Nn, 4), dt), np.zeros((Nn, 3), dt)]
        for key in ups:
            a2, ad, ac = np.zeros_like(vm2), np.zeros_like(v_depths), np.zeros_like(vcon)
            if key == "m2x":
                a2[..., 0] = vm2[..., 0]
            elif key == "m2y":
                a2[..., 1] = vm2[..., 1]
            elif key == "d":
                ad[...] = v_depths
            else:
                ac[..., int(key[1])] = vcon[..., int(key[1])]
            out = O.proj3d_bwd(self.means, self.quats, self.scales, self.viewmats, self.Ks, self.W, self.H,
                               self.radii, self.conics, a2, ad, ac, self.eps2d, dtype=dt)
            for t, o in zip(acc, out):
                t += np.abs(o)
        env["means"] = acc[0] + v_means_extra
        env["quats"] = acc[1]
        env["scales"] = acc[2]
        return env


class Raster2D(_Band):
    """2DGS forward (+ backward of colors/alphas/normals outputs) through the C oracle."""

    def __init__(self, means, quats, scales, opacities, colors, viewmats, Ks, W, H, backgrounds=None,
                 render_mode="RGB+ED", near=0.01, far=1e10, tile_size=16, dtype=np.float32, rows=None,
                 hitform=0):
        self.dt = dtype
        self.hitform = hitform  # 2DGS hit evaluation form (hgsr_oracle.c eval_splat2d)
        self.rows = rows  # rasterise only image rows [0, rows) (banded checks); None = all
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
        O.set_hitform(self.hitform, dt)
        with self._thresholds():
            (self.rc_raw, self.ra, self.rn, self.rd, self.rm, self.last, self.med, self.stopped, self.margin,
             self.gmargin) = O.raster2d_fwd(self.means2d, self.rt, self.cols, self.opac_c, self.normals, self.bg_r,
                                            self.W, self.Hr, self.ts, self.offsets, self.flatten_ids, dtype=dt,
                                            return_stopped=True)
        O.set_hitform(0, dt)
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
        O.set_hitform(self.hitform, dt)
        try:
            with self._thresholds():
                vm2, vrt, vcol, vop, vn, vdens = O.raster2d_bwd(
                    self.means2d, self.rt, self.cols, self.opac_c, self.normals, self.bg_r, self.W, self.Hr, self.ts,
                    self.offsets, self.flatten_ids, self.ra, self.last, v_rc, v_ra,
                    np.asarray(v_render_normals_cam, dt), dtype=dt)
        finally:
            O.set_hitform(0, dt)
        v_depths = vcol[..., -1].copy()
        vm, vq, vs = O.proj2d_bwd(self.means, self.quats, self.scales, self.viewmats, self.Ks, self.W, self.H,
                                  self.radii, self.rt, vm2, v_depths, vrt, vn, dtype=dt)
        return {"means": vm, "quats": vq, "scales": vs, "opacities": vop.sum(0), "colors": vcol[..., :-1].sum(0),
                "means2d": vm2, "densify": vdens}

    def envelope(self, v_render_colors, v_render_alphas, v_render_normals_cam):
        """Per-element magnitude envelopes of every gradient of backward(); see
        Raster3D.envelope.  Use on the float64 instance after forward()."""
        dt = self.dt
        C, Nn = self.viewmats.shape[0], self.means.shape[0]
        v_rc = np.abs(np.array(v_render_colors, dt))
        v_ra = np.abs(np.array(v_render_alphas, dt))
        if self.mode == "RGB+ED":
            den = np.maximum(self.ra, dt(1e-10))
            g = v_rc[..., -1:]
            # alpha = 1 - T carries an absolute rounding error ~u, so the ED divide amplifies the
            # relative error of every term it feeds by ~(1 + 1 / alpha)
            k = 1 + 1 / den
            v_ra = v_ra + np.where(self.ra >= dt(1e-10), k * g * np.abs(self.rc_raw[..., -1:]) / (den * den),
                                   0).astype(dt)
            v_rc = v_rc.copy()
            v_rc[..., -1:] = k * g / den
        O.set_envelope(True, dt)
        try:
            with self._thresholds():
                vm2, vrt, vcol, vop, vn, vdens = O.raster2d_bwd(
                    self.means2d, self.rt, self.cols, self.opac_c, self.normals, self.bg_r, self.W, self.Hr, self.ts,
                    self.offsets, self.flatten_ids, self.ra, self.last, v_rc, v_ra,
                    np.abs(np.asarray(v_render_normals_cam, dt)), dtype=dt)
        finally:
            O.set_envelope(False, dt)
        v_depths = vcol[..., -1].copy()
        acc = [np.zeros((Nn, 3), dt), np.zeros((Nn, 4), dt), np.zeros((Nn, 3), dt)]
        comps = [("m2", k) for k in range(2)] + [("d", 0)] + [("rt", k) for k in range(9)] + [("n", k) for k in range(3)]
        for kind, k in comps:
            a2, ad = np.zeros_like(vm2), np.zeros_like(v_depths)
            art, an = np.zeros(vrt.shape[:2] + (9,), dt), np.zeros_like(vn)
            if kind == "m2":
                a2[..., k] = vm2[..., k]
            elif kind == "d":
                ad[...] = v_depths
            elif kind == "rt":
                art[..., k] = vrt.reshape(art.shape)[..., k]
            else:
                an[..., k] = vn[..., k]
            out = O.proj2d_bwd(self.means, self.quats, self.scales, self.viewmats, self.Ks, self.W, self.H,
                               self.radii, self.rt, a2, ad, art.reshape(vrt.shape), an, dtype=dt)
            for t, o in zip(acc, out):
                t += np.abs(o)
        return {"means": acc[0], "quats": acc[1], "scales": acc[2], "opacities": vop.sum(0),
                "colors": vcol[..., :-1].sum(0), "means2d": vm2, "densify": vdens}
