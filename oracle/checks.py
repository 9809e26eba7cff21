"""Comparison helpers shared by the GPU parity tests and __graft_entry__.smoke().

TEST INFRASTRUCTURE ONLY.  Tolerance bar of BASELINE.json: 1e-5 abs / 1e-4 rel (fp32).
"""
from __future__ import annotations

import numpy as np

ATOL, RTOL = 1e-5, 1e-4
U32 = 2.0 ** -24  # fp32 unit roundoff


def close(a, b, atol=ATOL, rtol=RTOL, frac_ok=0.0, name=""):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    assert a.shape == b.shape, (name, a.shape, b.shape)
    bad = np.abs(a - b) > atol + rtol * np.abs(b)
    frac = bad.mean() if bad.size else 0.0
    worst = np.abs(a - b).max() if bad.size else 0.0
    assert frac <= frac_ok, f"{name}: {bad.sum()}/{bad.size} outside tol, max abs err {worst:.3g}"


def grad_close(a, b, name, rel_floor=1e-4):
    """Within 1e-5 abs / 1e-4 rel, the relative part against max(|b|, rel_floor*max|b|):
    gradients sum thousands of per-pixel terms in a different order (atomics), so
    near-cancelled entries are judged against the tensor's scale."""
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    scale = np.maximum(np.abs(b), rel_floor * (np.abs(b).max() if b.size else 0.0))
    bad = np.abs(a - b) > ATOL + RTOL * scale
    assert not bad.any(), f"{name}: {bad.sum()}/{bad.size} bad, max err {np.abs(a - b).max():.3g}"


def strict_rate(a, b, atol=ATOL, rtol=RTOL):
    """Fraction of elements within the bare north-star bar |a - b| <= atol + rtol |b|."""
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float((np.abs(a - b) <= atol + rtol * np.abs(b)).mean()) if b.size else 1.0


def cond_close(a, b32, b64, name, rel_floor=1e-4, factor=3.0, min_strict=None, dilate_axes=None, env=None,
               alt32=None, env_k=1.0, dilate=3):
    """fp32-conditioning-aware check (expected-depth normalisation, x depth channel, 2DGS,
    deep tiles).  Per element: the GPU value must be within 1e-5 abs / 1e-4 rel (relative
    part against max(|b32|, rel_floor * max|b32|)) of the f32 oracle PLUS twice that
    element's own f32-oracle error |b32 - b64|, and no further from the f64 answer than
    `factor` x that error + the same bar.  The slack is per element: an ill-conditioned
    low-alpha pixel loosens only itself.  Returns the fraction of elements that meet the
    bare 1e-5 / 1e-4 bar against the f32 oracle (asserted >= min_strict when given).

    dilate_axes (image-shaped tensors only, e.g. the (H, W) axes of a depth-derived normal
    map): the per-element error is max-filtered over the 3-neighbourhood along those axes,
    since a pixel's conditioning is shared with the neighbours it is differenced against and
    one particular f32 operation order can be accidentally exact at a single pixel.  dilate:
    the neighbourhood width (3; 5 for a quantity whose stencil reaches two pixels, e.g. the
    depth gradient of K13, which sums the vjps of the normals at +-1, each differencing +-1).

    env (raster gradients): the element's rounding envelope E (oracle Raster*.envelope: sum
    of |terms| weighted by compositing depth); u * E (u = 2^-24) is added to its slack, so a
    single f32 sample that happens to be exact at one element does not set a bar no other
    f32 evaluation order could meet.  Used with rel_floor=0: nothing tensor-wide remains.

    alt32: a second correct f32 evaluation of the same quantity (e.g. the 2DGS plane-form
    hit, oracle set_hitform), or a list of them; the element's f32 error is the largest.

    env_k: multiple of u * E allowed (E is a first-order bound; the resolved-branch re-check
    of tests/raster_parity.py, which keeps the near-threshold pixels' gradients, uses 2)."""
    a = np.asarray(a, np.float64)
    b = np.asarray(b32, np.float64)
    c = np.asarray(b64, np.float64)
    assert a.shape == b.shape == c.shape, (name, a.shape, b.shape, c.shape)
    if not b.size:
        return 1.0
    e32 = np.abs(b - c)
    if alt32 is not None:
        for alt in (alt32 if isinstance(alt32, (list, tuple)) else [alt32]):
            e32 = np.maximum(e32, np.abs(np.asarray(alt, np.float64) - c))
    if dilate_axes:
        from scipy.ndimage import maximum_filter
        size = [dilate if ax in [d % e32.ndim for d in dilate_axes] else 1 for ax in range(e32.ndim)]
        e32 = maximum_filter(e32, size=size, mode="nearest")
    scale = np.maximum(np.abs(b), rel_floor * np.abs(b).max()) if rel_floor else np.abs(b)
    bar = ATOL + RTOL * scale
    if env is not None:
        env = np.asarray(env, np.float64)
        assert env.shape == b.shape, (name, env.shape, b.shape)
        bar = bar + env_k * U32 * env
    err = np.abs(a - b)
    bad = err > bar + 2.0 * e32
    if env is not None and bad.any():  # how many envelopes the worst elements miss by
        need = (err - (bar - env_k * U32 * env) - 2.0 * e32) / (U32 * env + 1e-300)
        print(f"{name}: failing elements need {np.sort(need[bad])[-10:]} x u*E (|g| {np.abs(c[bad])[:5]}, "
              f"E {env[bad][:5]})")
    assert not bad.any(), (f"{name}: {bad.sum()}/{bad.size} bad, worst excess {(err - bar - 2 * e32).max():.3g} "
                           f"(max err {err.max():.3g}, max e32 {e32.max():.3g})")
    e64 = np.abs(a - c)
    far = e64 > factor * e32 + bar
    assert not far.any(), (f"{name}: {far.sum()}/{far.size} further from f64 than {factor}x the f32 oracle, "
                           f"worst {e64[far].max():.3g}")
    rate = strict_rate(a, b)
    if min_strict is not None:
        assert rate >= min_strict, f"{name}: strict 1e-5/1e-4 pass rate {rate:.6f} < {min_strict}"
    return rate


# relative decision margins (oracle forward `margin`) below which another correct f32
# evaluation order may take the other branch: 3DGS alpha / stop decisions (the kernels'
# exp2 of the log2(e)-prescaled conic vs expf: a few ulps of a sigma <= ~6) and 2DGS (taken
# over both correct hit forms, the per-pixel cross product and the plane form, see
# tests/raster_parity.run_2dgs)
DELTA_3D, DELTA_2D = 2e-5, 5e-5
MAX_AMBIGUOUS = 0.01       # value decisions: at most this fraction of pixels within the margin
MAX_GRAD_AMBIGUOUS = 0.03  # + gradient-path switches (0.999 clamp, 2DGS surface / low-pass branch)


def ambiguous(ref, delta, gradient=False):
    """bool [C, rows, W]: pixels with a discrete decision within `delta` of its threshold
    (gradient=True: also the decisions that switch only a gradient path)."""
    return np.asarray(ref.gmargin if gradient else ref.margin) < delta


def image_close(a, b32, b64, amb, name, min_strict=None, margin=None, alt32=None, **kw):
    """cond_close on the pixels of an image [C,H,W,K] whose decisions are unambiguous.
    Ambiguous pixels (a threshold decision within a few ulps) are excluded from the
    bar and only counted; their upstream gradients are zeroed by the callers, so no
    gradient check depends on the branch they took.  Returns (strict pass rate, n_amb)."""
    a, b, c = (np.asarray(x, np.float64) for x in (a, b32, b64))
    amb = np.asarray(amb, bool)
    assert amb.shape == a.shape[:amb.ndim], (amb.shape, a.shape)
    n_amb = int(amb.sum())
    assert n_amb <= MAX_AMBIGUOUS * amb.size, f"{name}: {n_amb}/{amb.size} ambiguous pixels"
    keep = ~amb
    if margin is not None:  # diagnostics: decision margins of the pixels that fail the bar
        m = np.asarray(margin)
        e32 = np.abs(b - c) if alt32 is None else np.maximum(np.abs(b - c), np.abs(np.asarray(alt32) - c))
        bar = ATOL + RTOL * np.abs(b) + 2.0 * e32
        badpix = (np.abs(a - b) > bar).reshape(amb.shape + (-1,)).any(-1) & keep
        if badpix.any():
            print(f"{name}: {int(badpix.sum())} failing pixels, margins {np.sort(m[badpix])[:20]}")
    alt = None if alt32 is None else np.asarray(alt32, np.float64)[keep]
    # images: no further from f64 than the (larger) f32 oracle error + the bar -- factor 1
    # (round-4 element-wise report: the GPU is never measurably worse than f32 on images)
    kw.setdefault("factor", 1.0)
    return cond_close(a[keep], b[keep], c[keep], name, min_strict=min_strict, alt32=alt, **kw), n_amb
