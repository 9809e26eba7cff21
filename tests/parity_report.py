"""Element-wise strict-rate report of the raster parity tests.  TEST INFRASTRUCTURE.

For every image and gradient tensor a raster parity run checks (tests/raster_parity.py), one
row with, against the bare north-star bar |x - ref| <= 1e-5 + 1e-4 |ref|:

  gpu~g32 / gpu~k32 / gpu~f64   pass rate of the GPU against the gsplat-form f32 oracle, the
                                kernel-form f32 oracle (3DGS: log2(e)-prescaled conic + exp2,
                                hgsr_oracle.c vis3; 2DGS: the plane-form hit) and the f64 oracle;
  g32~f64 / k32~f64             the same rate of the two f32 oracles against f64 (what any
                                correct f32 evaluation achieves on this tensor);
  worse_g32 / worse_k32         fraction of elements where the GPU is further from f64 than the
                                gsplat-form (kernel-form) f32 oracle is, by more than the bar:
                                |gpu - f64| > |o32 - f64| + 1e-5 + 1e-4 |f64|;
  worse_best                    ... further than the closer of the two f32 oracles;
  better_g32 / better_k32       the mirror image: fraction where that f32 oracle is further from
                                f64 than the GPU is, by more than the bar.  worse ~ better means
                                the GPU and that oracle are two equally accurate f32 evaluations
                                whose errors fall on different elements (gradient sums in another
                                order); worse >> better would mean a systematically worse GPU.

Rows are kept in RECORDS (printed by tests/conftest.py's terminal summary, so the suite's own
log carries them) and appended as JSON lines to $HGSR_PARITY_REPORT (default
gpurun_out/parity_strict.jsonl).
"""
from __future__ import annotations

import json
import os

import numpy as np

from oracle.checks import ATOL, RTOL

RECORDS = []
_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _rate(a, ref):
    return float((np.abs(a - ref) <= ATOL + RTOL * np.abs(ref)).mean()) if ref.size else 1.0


def _test_name():
    t = os.environ.get("PYTEST_CURRENT_TEST", "")
    return t.split(" ")[0].split("::")[-1] if t else "?"


def tensor(name, gpu, g32, k32, f64, mask=None):
    """Record one tensor (mask: elements included, e.g. the unambiguous pixels of an image)."""
    a, b, k, c = (np.asarray(x, np.float64) for x in (gpu, g32, k32, f64))
    if mask is not None:
        m = np.asarray(mask, bool)
        a, b, k, c = a[m], b[m], k[m], c[m]
    a, b, k, c = (x.reshape(-1) for x in (a, b, k, c))
    bar = ATOL + RTOL * np.abs(c)
    e = np.abs(a - c)
    eg, ek = np.abs(b - c), np.abs(k - c)
    row = {"test": _test_name(), "tensor": name, "n": int(a.size),
           "gpu~g32": _rate(a, b), "gpu~k32": _rate(a, k), "gpu~f64": _rate(a, c),
           "g32~f64": _rate(b, c), "k32~f64": _rate(k, c),
           "worse_g32": float((e > eg + bar).mean()) if a.size else 0.0,
           "worse_k32": float((e > ek + bar).mean()) if a.size else 0.0,
           "worse_best": float((e > np.minimum(eg, ek) + bar).mean()) if a.size else 0.0,
           "better_g32": float((eg > e + bar).mean()) if a.size else 0.0,
           "better_k32": float((ek > e + bar).mean()) if a.size else 0.0}
    RECORDS.append(row)
    path = os.environ.get("HGSR_PARITY_REPORT") or os.path.join(_ROOT, "gpurun_out", "parity_strict.jsonl")
    try:
        os.makedirs(os.path.dirname(path), exist_ok=True)
        with open(path, "a") as f:
            f.write(json.dumps(row) + "\n")
    except OSError:
        pass
    return row


COLS = ("gpu~g32", "gpu~k32", "gpu~f64", "g32~f64", "k32~f64", "worse_g32", "worse_k32", "worse_best", "better_g32",
        "better_k32")


def table(rows=None):
    rows = RECORDS if rows is None else rows
    out = ["strict 1e-5 abs / 1e-4 rel pass rates and GPU-worse-than-f32 fractions (tests/parity_report.py)",
           f"{'test':40s} {'tensor':16s} {'n':>9s} " + " ".join(f"{c:>10s}" for c in COLS)]
    for r in rows:
        out.append(f"{r['test'][:40]:40s} {r['tensor'][:16]:16s} {r['n']:9d} "
                   + " ".join(f"{r[c]:10.6f}" if c in r else f"{'-':>10s}" for c in COLS))
    return "\n".join(out)
