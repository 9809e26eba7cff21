"""Per-chunk training on the device through the launcher: two chunks
trained by two concurrent child processes sharing the box's GPU (HIP_VISIBLE_DEVICES=0 for both
slots) against the same chunks run one after the other.  Each chunk is an independent unit and
the whole training step is deterministic (the raster backwards sum fixed-order gradient slots,
the decode backward reduces its weight gradients in a fixed f64 order), so every merge input --
each chunk's coarse and fine PLYs and the merged explicit PLY (merge.py:132-217) -- must be
byte-identical between the concurrent and the sequential run."""
import os
import sys

import numpy as np
import pytest

from horizongs_amd import chunk_train as CT
from horizongs_amd.chunks import consolidate_explicit, run_chunks
from horizongs_amd.ply import read_ply

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _cmd(out):
    return lambda c, st: [sys.executable, "-m", "horizongs_amd.chunk_train", "--chunk", c, "--stage", st, "--out", out,
                          "--anchors", "4000", "--iters", "10", "--width", "256", "--height", "144", "--views", "4",
                          "--lr-scale", "0.3"]


def test_two_chunk_processes_equal_sequential(tmp_path):
    env = dict(os.environ, PYTHONPATH=ROOT + os.pathsep + os.environ.get("PYTHONPATH", ""))
    chunks = ["0_0", "1_0"]
    par, seq = str(tmp_path / "par"), str(tmp_path / "seq")
    run_chunks(chunks, ["0", "0"], _cmd(par), env=env, log_dir=str(tmp_path / "lp"), timeout=240)
    run_chunks(chunks, ["0"], _cmd(seq), env=env, log_dir=str(tmp_path / "ls"), timeout=240)
    for c in chunks:
        for st, names in (("coarse", ("point_cloud.ply",)), ("fine", ("point_cloud.ply", "point_cloud_explicit.ply"))):
            for n in names:
                pa, pb = os.path.join(par, c, st, n), os.path.join(seq, c, st, n)
                with open(pa, "rb") as fa, open(pb, "rb") as fb:
                    ba, bb = fa.read(), fb.read()
                if ba != bb:  # name the first differing property for the record
                    a, _, _ = read_ply(pa)
                    b, _, _ = read_ply(pb)
                    diff = [k for k in b if k not in a or not np.array_equal(a[k], b[k])]
                    raise AssertionError(f"{c}/{st}/{n}: concurrent != sequential, properties {diff[:8]}")
        init, _ = CT.init_model(c, 4000)
        trained, _, _ = read_ply(os.path.join(seq, c, "fine", "point_cloud.ply"))
        assert np.abs(trained["f_anchor_feat_0"] - init["feat"][:, 0].numpy()).max() > 1e-3  # it trained
    merged = {}
    for name, root in (("par", par), ("seq", seq)):
        parts = [(c, os.path.join(root, c, "fine", "point_cloud_explicit.ply"), CT.true_bounds(c)) for c in chunks]
        kept = consolidate_explicit(parts, [0, 2], str(tmp_path / f"{name}.ply"))
        assert all(v > 1000 for v in kept.values()), kept
        with open(tmp_path / f"{name}.ply", "rb") as f:
            merged[name] = f.read()
    assert merged["par"] == merged["seq"], "merged explicit PLYs differ"
