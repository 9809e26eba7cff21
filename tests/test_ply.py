"""On-disk formats, CPU: PLY codec, anchor / explicit PLY round trips with
the reference's property layout (scene/lod_model.py:374-464, 681-832), TorchScript MLPs
(:598-617).  The reference ships no PLY fixture and plyfile is absent, so the byte layout
is checked against the PLY header plyfile writes for these files (format line, obj_info
lines, one float vertex element) -- parity unpinned beyond that."""
import numpy as np
import torch

from horizongs_amd import ply as P


def test_header_layout_and_roundtrip(tmp_path):
    f = tmp_path / "a.ply"
    cols = {"x": np.arange(3, dtype=np.float32), "level": np.array([0, 1, 2], np.float32)}
    P.write_ply(f, cols, obj_info=["standard_dist 26.686000", "street_levels 8.000000"])
    raw = f.read_bytes()
    want = (b"ply\nformat binary_little_endian 1.0\nobj_info standard_dist 26.686000\n"
            b"obj_info street_levels 8.000000\nelement vertex 3\nproperty float x\nproperty float level\n"
            b"end_header\n")
    assert raw.startswith(want)
    assert raw[len(want):] == np.stack([cols["x"], cols["level"]], 1).astype("<f4").tobytes()
    back, info, _ = P.read_ply(f)
    assert info == ["standard_dist 26.686000", "street_levels 8.000000"]
    for k in cols:
        np.testing.assert_array_equal(back[k], cols[k])


def test_ascii_and_big_endian(tmp_path):
    f = tmp_path / "t.ply"
    f.write_bytes(b"ply\nformat ascii 1.0\nelement vertex 2\nproperty float x\nproperty uchar c\nend_header\n"
                  b"1.5 7\n-2 255\n")
    cols, _, _ = P.read_ply(f)
    np.testing.assert_array_equal(cols["x"], np.array([1.5, -2], np.float32))
    np.testing.assert_array_equal(cols["c"], np.array([7, 255], np.uint8))
    g = tmp_path / "b.ply"
    body = np.array([(1.25, 3), (4.0, -1)], dtype=[("x", ">f4"), ("i", ">i4")]).tobytes()
    g.write_bytes(b"ply\nformat binary_big_endian 1.0\nelement vertex 2\nproperty float x\nproperty int i\n"
                  b"end_header\n" + body)
    cols, _, _ = P.read_ply(g)
    np.testing.assert_array_equal(cols["x"], [1.25, 4.0])
    np.testing.assert_array_equal(cols["i"], [3, -1])


def test_anchor_ply_roundtrip(tmp_path):
    g = torch.Generator().manual_seed(3)
    A, k, F = 257, 10, 32
    anchor = torch.randn(A, 3, generator=g)
    level = torch.randint(0, 8, (A, 1), generator=g).float()
    extra = torch.randn(A, generator=g)
    offset = torch.randn(A, k, 3, generator=g)
    feat = torch.randn(A, F, generator=g)
    scaling = torch.randn(A, 6, generator=g)
    rot = torch.randn(A, 4, generator=g)
    f = tmp_path / "point_cloud.ply"
    P.save_anchor_ply(f, anchor, level, extra, offset, feat, scaling, rot, 26.686, 1, 8)
    cols, info, _ = P.read_ply(f)
    names = list(cols)
    assert names[:5] == ["x", "y", "z", "level", "extra_level"]
    assert names[5:5 + 3 * k] == [f"f_offset_{i}" for i in range(3 * k)]
    # the reference stores offsets transposed: f_offset_{c*k + j} = offset[:, j, c]
    np.testing.assert_array_equal(cols["f_offset_1"], offset[:, 1, 0].numpy())
    np.testing.assert_array_equal(cols[f"f_offset_{k}"], offset[:, 0, 1].numpy())
    assert info == ["standard_dist 26.686000", "aerial_levels 1.000000", "street_levels 8.000000"]
    d = P.load_anchor_ply(f, device="cpu")
    for key, ref in (("anchor", anchor), ("extra_level", extra), ("offset", offset), ("anchor_feat", feat),
                     ("scaling", scaling), ("rotation", rot)):
        assert torch.equal(d[key], ref), key
    assert torch.equal(d["level"], level.int())
    assert d["aerial_levels"] == 1 and d["street_levels"] == 8 and abs(d["standard_dist"] - 26.686) < 1e-6


def test_explicit_ply_roundtrip(tmp_path):
    g = torch.Generator().manual_seed(4)
    N, K = 301, 9
    xyz = torch.randn(N, 3, generator=g)
    dc = torch.randn(N, 1, 3, generator=g)
    rest = torch.randn(N, K - 1, 3, generator=g)
    f = tmp_path / "point_cloud_explicit.ply"
    P.save_explicit_ply(f, xyz, torch.zeros(N, 1), torch.ones(N), dc, rest, torch.rand(N, 1, generator=g),
                        torch.rand(N, 3, generator=g), torch.randn(N, 4, generator=g), 26.686, 1, 8)
    cols, _, _ = P.read_ply(f)
    # channel-major SH: f_dc_c = dc[:, 0, c]; f_rest_{c*(K-1) + j} = rest[:, j, c]
    np.testing.assert_array_equal(cols["f_dc_2"], dc[:, 0, 2].numpy())
    np.testing.assert_array_equal(cols[f"f_rest_{K - 1}"], rest[:, 0, 1].numpy())
    d = P.load_explicit_ply(f, device="cpu")
    assert torch.equal(d["xyz"], xyz) and torch.equal(d["features_dc"], dc) and torch.equal(d["features_rest"], rest)


def test_torchscript_mlps_roundtrip(tmp_path):
    nn = torch.nn
    torch.manual_seed(5)
    heads = [nn.Sequential(nn.Linear(35, 32), nn.ReLU(True), nn.Linear(32, o)) for o in (10, 70, 30)]
    heads[0].append(nn.Tanh())
    P.save_mlp_checkpoints(tmp_path, *heads, in_dim=35)
    w = P.load_mlp_checkpoints(tmp_path, device="cpu")
    for (name, _), m in zip(P._HEADS, heads):
        assert torch.equal(w[f"{name}_w1"], m[0].weight.detach())
        assert torch.equal(w[f"{name}_b2"], m[2].bias.detach())
