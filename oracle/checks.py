"""Comparison helpers shared by the GPU parity tests and __graft_entry__.smoke().

TEST INFRASTRUCTURE ONLY.  Tolerance bar of BASELINE.json: 1e-5 abs / 1e-4 rel (fp32).
"""
from __future__ import annotations

import numpy as np

ATOL, RTOL = 1e-5, 1e-4


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


def cond_close(a, b32, b64, name, rel_floor=1e-4, factor=3.0):
    """fp32-conditioning-aware check (expected-depth normalisation, x depth channel, 2DGS):
    the GPU result must be within 1e-5 abs / 1e-4 rel of the f32 oracle PLUS twice the f32
    oracle's own measured distance to the f64 oracle on that tensor, and no further from the
    f64 answer than `factor` x the f32 oracle (the kernels use the hardware exp / reciprocal
    and FMA contraction, the oracle correctly rounded ops)."""
    a = np.asarray(a, np.float64)
    b = np.asarray(b32, np.float64)
    c = np.asarray(b64, np.float64)
    e32 = np.abs(b - c).max() if b.size else 0.0
    scale = np.maximum(np.abs(b), rel_floor * (np.abs(b).max() if b.size else 0.0))
    bad = np.abs(a - b) > ATOL + RTOL * scale + 2.0 * e32
    assert not bad.any(), f"{name}: {bad.sum()}/{bad.size} bad, max err {np.abs(a - b).max():.3g} (e32 {e32:.3g})"
    assert np.abs(a - c).max() <= factor * e32 + ATOL, (
        f"{name}: GPU err {np.abs(a - c).max():.3g} vs f32 oracle err {e32:.3g} (max|g| {np.abs(c).max():.3g})")
