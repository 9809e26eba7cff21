"""The per-chunk launcher and merge (horizongs_amd/chunks.py; SURVEY.md §4 item 5, §8(e) mapping 1).

The reference trains every chunk config with its own train.py process (coarse, then fine on
the coarse output: preprocess/generate_chunks_config.py:77-104) and joins them only in
merge.py (merge.py:132-217).  On the CPU the children run the plumbing mode of
horizongs_amd.chunk_train (--dry: the same files, no device work): chunks spread over two
device slots must produce exactly the outputs of one slot running them in sequence, each
stage in a fresh process with its slot's HIP_VISIBLE_DEVICES, fine after its own coarse; the
merge crops and concatenates like consolidate_lod."""
import os
import sys

import numpy as np
import pytest

from horizongs_amd import chunk_train as CT
from horizongs_amd.chunks import chunk_ids, consolidate_explicit, crop_mask, run_chunks
from horizongs_amd.ply import read_ply

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _cmd(out, extra=()):
    return lambda c, st: [sys.executable, "-m", "horizongs_amd.chunk_train", "--chunk", c, "--stage", st, "--out", out,
                          "--anchors", "500", *extra]


def _files(out):
    got = {}
    for d, _, fs in os.walk(out):
        for f in fs:
            if f != "device.txt":
                p = os.path.join(d, f)
                got[os.path.relpath(p, out)] = open(p, "rb").read()
    return got


def test_chunk_ids_follow_generate_chunks_config():
    assert chunk_ids(4, 2) == ["0_0", "0_1", "1_0", "1_1", "2_0", "2_1", "3_0", "3_1"]  # Block_A: 4 x 2


def test_parallel_chunks_equal_sequential(tmp_path):
    chunks = chunk_ids(2, 2)
    env = dict(os.environ, PYTHONPATH=ROOT + os.pathsep + os.environ.get("PYTHONPATH", ""))
    par, seq = str(tmp_path / "par"), str(tmp_path / "seq")
    res = run_chunks(chunks, ["0", "1"], _cmd(par, ["--dry"]), env=env, log_dir=str(tmp_path / "logs"), timeout=300)
    assert sorted(res) == chunks and {r["device"] for r in res.values()} == {"0", "1"}
    for c, r in res.items():
        assert r["returncodes"] == {"coarse": 0, "fine": 0}
        for st in ("coarse", "fine"):  # each stage ran in a process that saw its slot's device
            assert open(os.path.join(par, c, st, "device.txt")).read() == r["device"]
    run_chunks(chunks, ["0"], _cmd(seq, ["--dry"]), env=env, timeout=300)
    a, b = _files(par), _files(seq)
    assert sorted(a) == sorted(b) and len(a) == 4 * 3
    for k in a:
        assert a[k] == b[k], k  # byte-identical merge inputs
    # merge.py: crop every chunk to its true bounds on the ground plane (x, z) and concatenate
    parts = [(c, os.path.join(par, c, "fine", "point_cloud_explicit.ply"), CT.true_bounds(c)) for c in chunks]
    merged = str(tmp_path / "merged.ply")
    kept = consolidate_explicit(parts, [0, 2], merged)
    cols, info, _ = read_ply(merged)
    ref = []
    for c, path, bnd in parts:
        cc, _, _ = read_ply(path)
        xyz = np.stack([cc["x"], cc["y"], cc["z"]], 1)
        m = crop_mask(xyz, bnd, [0, 2])
        assert 0 < m.sum() < len(m)  # the overlap padding is cropped away, the cell kept
        assert kept[c] == int(m.sum())
        ref.append({k: v[m] for k, v in cc.items()})
    for k in cols:
        np.testing.assert_array_equal(cols[k], np.concatenate([r[k] for r in ref]))
    assert info[0].startswith("standard_dist")
    # every merged Gaussian lies in exactly one chunk's cell
    xyz = np.stack([cols["x"], cols["y"], cols["z"]], 1)
    owners = sum(crop_mask(xyz, CT.true_bounds(c), [0, 2]).astype(int) for c in chunks)
    assert np.all(owners >= 1)


def test_failed_stage_stops_its_chunk(tmp_path):
    """A coarse stage that fails: its fine stage never starts, the other chunks finish, and the
    launcher raises naming the failed chunk."""
    env = dict(os.environ, PYTHONPATH=ROOT + os.pathsep + os.environ.get("PYTHONPATH", ""))
    out = str(tmp_path / "o")

    def cmd(c, st):
        if c == "0_1" and st == "coarse":
            return [sys.executable, "-c", "import sys; sys.exit(3)"]
        return _cmd(out, ["--dry"])(c, st)

    with pytest.raises(RuntimeError, match="0_1"):
        run_chunks(chunk_ids(1, 2), ["0", "0"], cmd, env=env, timeout=300)
    assert os.path.exists(os.path.join(out, "0_0", "fine", "point_cloud_explicit.ply"))
    assert not os.path.exists(os.path.join(out, "0_1", "fine"))


def test_launch_errors_fail_their_chunk(tmp_path):
    """A stage whose executable does not exist, or whose command() raises, is a failed stage
    (ADVICE r05): the launcher still runs the other chunks and raises naming the chunks, instead
    of losing them with the slot thread."""
    env = dict(os.environ, PYTHONPATH=ROOT + os.pathsep + os.environ.get("PYTHONPATH", ""))
    out = str(tmp_path / "o")

    def cmd(c, st):
        if c == "0_0":
            return [str(tmp_path / "no_such_binary")]
        if c == "0_1":
            raise ValueError("bad chunk config")
        return _cmd(out, ["--dry"])(c, st)

    with pytest.raises(RuntimeError) as ei:
        run_chunks(chunk_ids(1, 3), ["0"], cmd, env=env, timeout=300)
    msg = str(ei.value)
    assert "0_0" in msg and "0_1" in msg and "bad chunk config" in msg and "0_2" not in msg.split("never run")[0]
    assert os.path.exists(os.path.join(out, "0_2", "fine", "point_cloud_explicit.ply"))
