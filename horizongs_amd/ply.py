"""On-disk formats of the reference: anchor PLY, explicit PLY,
TorchScript MLP checkpoints.

* `save_anchor_ply` / `load_anchor_ply`   <- GaussianLoDModel.save_ply / load_ply
  (scene/lod_model.py:374-464): vertex properties x, y, z, level, extra_level,
  f_offset_* (offsets transposed to [A, 3, k] then flattened), f_anchor_feat_*, scale_*,
  rot_*, all float32, plus obj_info lines standard_dist / aerial_levels / street_levels.
* `save_explicit_ply` / `load_explicit_ply` <- save_explicit / load_explicit
  (scene/lod_model.py:681-832, merge.py:42-53,132-217): x, y, z, level, extra_level,
  f_dc_0..2, f_rest_*, opacity, scale_0..2, rot_0..3.
* `export_explicit` decodes a view-independent anchor model with the fused HIP decode and
  writes the explicit PLY (the reference's save_explicit; device work on the MI355X).
* `load_mlp_checkpoints` / `save_mlp_checkpoints` <- lod_model.py:598-617 (TorchScript
  opacity_mlp.pt / cov_mlp.pt / color_mlp.pt), giving the decode's weight dict.

The PLY codec is self-contained (plyfile is not a dependency): it writes what plyfile
writes for these files -- binary little-endian, `obj_info` header lines after the format
line, one `vertex` element of float properties -- and reads binary (either byte order) or
ASCII PLY with scalar properties.
"""
from __future__ import annotations

import os

import numpy as np
import torch

_PLY_TYPES = {
    "char": "i1", "int8": "i1", "uchar": "u1", "uint8": "u1", "short": "i2", "int16": "i2", "ushort": "u2",
    "uint16": "u2", "int": "i4", "int32": "i4", "uint": "u4", "uint32": "u4", "float": "f4", "float32": "f4",
    "double": "f8", "float64": "f8",
}
_NP_TO_PLY = {"i1": "char", "u1": "uchar", "i2": "short", "u2": "ushort", "i4": "int", "u4": "uint", "f4": "float",
              "f8": "double"}


# --------------------------------------------------------------------- codec
def write_ply(path, columns, obj_info=(), comments=()):
    """columns: ordered {name: 1-D array}; one `vertex` element, binary little-endian."""
    names = list(columns)
    n = len(columns[names[0]]) if names else 0
    dtype = [(nm, "<" + np.asarray(columns[nm]).dtype.str[1:]) for nm in names]
    arr = np.empty(n, dtype=dtype)
    for nm in names:
        col = np.asarray(columns[nm]).reshape(-1)
        if col.shape[0] != n:
            raise ValueError(f"ply column {nm}: {col.shape[0]} rows, expected {n}")
        arr[nm] = col
    lines = ["ply", "format binary_little_endian 1.0"]
    lines += [f"comment {c}" for c in comments]
    lines += [f"obj_info {c}" for c in obj_info]
    lines.append(f"element vertex {n}")
    for nm, dt in dtype:
        lines.append(f"property {_NP_TO_PLY[dt[1:]]} {nm}")
    lines.append("end_header")
    d = os.path.dirname(os.path.abspath(path))
    os.makedirs(d, exist_ok=True)
    with open(path, "wb") as f:
        f.write(("\n".join(lines) + "\n").encode("ascii"))
        f.write(arr.tobytes())


def read_ply(path):
    """-> (columns {name: np.ndarray} of the `vertex` element, obj_info [str], comments [str])."""
    with open(path, "rb") as f:
        data = f.read()
    end = data.find(b"end_header")
    if not data.startswith(b"ply") or end < 0:
        raise ValueError(f"{path}: not a PLY file")
    nl = data.find(b"\n", end)
    header = data[:end].decode("ascii").splitlines()
    body = data[nl + 1:]
    fmt, obj_info, comments, elements = None, [], [], []
    for ln in header[1:]:
        tok = ln.strip().split()
        if not tok:
            continue
        if tok[0] == "format":
            fmt = tok[1]
        elif tok[0] == "comment":
            comments.append(ln.strip()[len("comment "):])
        elif tok[0] == "obj_info":
            obj_info.append(ln.strip()[len("obj_info "):])
        elif tok[0] == "element":
            elements.append([tok[1], int(tok[2]), []])
        elif tok[0] == "property":
            if tok[1] == "list":
                raise ValueError(f"{path}: list properties are not supported")
            elements[-1][2].append((tok[2], _PLY_TYPES[tok[1]]))
    if fmt not in ("binary_little_endian", "binary_big_endian", "ascii"):
        raise ValueError(f"{path}: unknown PLY format {fmt}")
    cols = None
    offset = 0
    text_rows = body.decode("ascii").split("\n") if fmt == "ascii" else None
    row = 0
    for name, count, props in elements:
        if fmt == "ascii":
            vals = np.array([ln.split() for ln in text_rows[row:row + count]], dtype=np.float64).reshape(count, -1)
            row += count
            arr = {p: vals[:, i].astype(t) for i, (p, t) in enumerate(props)}
        else:
            bo = "<" if fmt == "binary_little_endian" else ">"
            dt = np.dtype([(p, bo + t) for p, t in props])
            rec = np.frombuffer(body, dtype=dt, count=count, offset=offset)
            offset += dt.itemsize * count
            arr = {p: rec[p].astype(t) for p, t in props}
        if name == "vertex":
            cols = arr
    if cols is None:
        raise ValueError(f"{path}: no vertex element")
    return cols, obj_info, comments


def _infos(standard_dist, aerial_levels, street_levels):
    return [f"standard_dist {standard_dist:.6f}", f"aerial_levels {aerial_levels:.6f}",
            f"street_levels {street_levels:.6f}"]


def _parse_infos(obj_info):
    out = {}
    for s in obj_info:
        k, v = s.split(" ")[:2]
        out[k] = float(v)
    for k in ("aerial_levels", "street_levels"):
        if k in out:
            out[k] = round(out[k])
    return out


def _np(t):
    return t.detach().float().cpu().numpy() if isinstance(t, torch.Tensor) else np.asarray(t, np.float32)


def _sorted(cols, prefix):
    names = sorted((c for c in cols if c.startswith(prefix)), key=lambda x: int(x.split("_")[-1]))
    if not names:
        return np.zeros((len(cols["x"]), 0), np.float32)
    return np.stack([cols[c].astype(np.float32) for c in names], axis=1)


# --------------------------------------------------------------------- anchor PLY
def save_anchor_ply(path, anchor, level, extra_level, offset, anchor_feat, scaling, rotation, standard_dist,
                    aerial_levels, street_levels):
    """scene/lod_model.py:374-411: offset [A,k,3] is stored as [A,3,k] flattened."""
    a = _np(anchor)
    off = _np(offset)
    off = np.ascontiguousarray(off.transpose(0, 2, 1).reshape(off.shape[0], -1))
    cols = {"x": a[:, 0], "y": a[:, 1], "z": a[:, 2], "level": _np(level).reshape(-1),
            "extra_level": _np(extra_level).reshape(-1)}
    cols.update({f"f_offset_{i}": off[:, i] for i in range(off.shape[1])})
    f = _np(anchor_feat)
    cols.update({f"f_anchor_feat_{i}": f[:, i] for i in range(f.shape[1])})
    s = _np(scaling)
    cols.update({f"scale_{i}": s[:, i] for i in range(s.shape[1])})
    r = _np(rotation)
    cols.update({f"rot_{i}": r[:, i] for i in range(r.shape[1])})
    write_ply(path, {k: v.astype(np.float32) for k, v in cols.items()},
              obj_info=_infos(standard_dist, aerial_levels, street_levels))


def load_anchor_ply(path, device="cuda"):
    """scene/lod_model.py:413-464 -> dict: anchor [A,3], level [A,1] int32 (through int16 as
    the reference), extra_level [A], offset [A,k,3], anchor_feat [A,F], scaling [A,6],
    rotation [A,4] (float32 on `device`), plus the obj_info values."""
    cols, info, _ = read_ply(path)
    A = len(cols["x"])
    anchor = np.stack([cols["x"], cols["y"], cols["z"]], 1).astype(np.float32)
    offs = _sorted(cols, "f_offset_")
    offs = offs.reshape(A, 3, -1).transpose(0, 2, 1)
    t = lambda x, dt=torch.float32: torch.tensor(np.ascontiguousarray(x), dtype=dt, device=device)
    out = dict(anchor=t(anchor), level=t(cols["level"].astype(np.int16)[:, None], torch.int32),
               extra_level=t(cols["extra_level"].astype(np.float32)), offset=t(offs),
               anchor_feat=t(_sorted(cols, "f_anchor_feat")), scaling=t(_sorted(cols, "scale_")),
               rotation=t(_sorted(cols, "rot")))
    out.update(_parse_infos(info))
    return out


# --------------------------------------------------------------------- explicit PLY
def save_explicit_ply(path, xyz, level, extra_level, features_dc, features_rest, opacity, scaling, rotation,
                      standard_dist, aerial_levels, street_levels):
    """scene/lod_model.py:681-771 / merge.py:209-217: features_dc [N,1,3], features_rest
    [N,K-1,3] are stored channel-major (transpose(1,2).flatten)."""
    x = _np(xyz)
    dc = _np(features_dc).reshape(x.shape[0], -1, 3).transpose(0, 2, 1).reshape(x.shape[0], -1)
    rest = _np(features_rest).reshape(x.shape[0], -1, 3).transpose(0, 2, 1).reshape(x.shape[0], -1)
    cols = {"x": x[:, 0], "y": x[:, 1], "z": x[:, 2], "level": _np(level).reshape(-1),
            "extra_level": _np(extra_level).reshape(-1)}
    cols.update({f"f_dc_{i}": dc[:, i] for i in range(dc.shape[1])})
    cols.update({f"f_rest_{i}": rest[:, i] for i in range(rest.shape[1])})
    cols["opacity"] = _np(opacity).reshape(-1)
    s, r = _np(scaling), _np(rotation)
    cols.update({f"scale_{i}": s[:, i] for i in range(s.shape[1])})
    cols.update({f"rot_{i}": r[:, i] for i in range(r.shape[1])})
    write_ply(path, {k: np.ascontiguousarray(v).astype(np.float32) for k, v in cols.items()},
              obj_info=_infos(standard_dist, aerial_levels, street_levels))


def load_explicit_ply(path, device="cuda"):
    """scene/lod_model.py:773-832 -> dict: xyz [N,3], features_dc [N,1,3], features_rest
    [N,K-1,3], opacity [N,1], scaling [N,3], rotation [N,4], level [N,1] int32, extra_level [N]."""
    cols, info, _ = read_ply(path)
    n = len(cols["x"])
    t = lambda x, dt=torch.float32: torch.tensor(np.ascontiguousarray(x), dtype=dt, device=device)
    dc = np.stack([cols[f"f_dc_{i}"] for i in range(3)], 1).reshape(n, 3, 1)
    rest = _sorted(cols, "f_rest_").reshape(n, 3, -1)
    out = dict(xyz=t(np.stack([cols["x"], cols["y"], cols["z"]], 1)), features_dc=t(dc.transpose(0, 2, 1)),
               features_rest=t(rest.transpose(0, 2, 1)), opacity=t(cols["opacity"][:, None]),
               scaling=t(_sorted(cols, "scale_")), rotation=t(_sorted(cols, "rot")),
               level=t(cols["level"].astype(np.int16)[:, None], torch.int32),
               extra_level=t(cols["extra_level"].astype(np.float32)))
    out.update(_parse_infos(info))
    return out


@torch.no_grad()
def export_explicit(path, anchor, level, extra_level, anchor_feat, offset, scaling_raw, mlps, n_offsets, color_dim,
                    standard_dist, aerial_levels, street_levels):
    """save_explicit (scene/lod_model.py:681-771) for a view-independent model (view_dim 0,
    no appearance): every anchor decoded by the fused HIP decode, the opacity > 0 Gaussians
    written with their anchor's level / extra_level."""
    from .decode import decode
    dev = anchor.device
    xyz, _, color, opac, scaling, rot, mask = decode(anchor, anchor_feat, offset, scaling_raw,
                                                     torch.zeros(3, device=dev), mlps, None, 0, n_offsets, color_dim)
    rep = lambda t: t.reshape(anchor.shape[0], -1)[:, :1].repeat_interleave(n_offsets, 0)[mask]
    col = color.reshape(color.shape[0], -1, 3)
    save_explicit_ply(path, xyz, rep(level.float()), rep(extra_level.reshape(-1, 1)), col[:, :1], col[:, 1:], opac,
                      scaling, rot, standard_dist, aerial_levels, street_levels)
    return int(mask.sum())


# --------------------------------------------------------------------- TorchScript MLPs
_HEADS = (("opacity", "opacity_mlp.pt"), ("cov", "cov_mlp.pt"), ("color", "color_mlp.pt"))


def load_mlp_checkpoints(path, device="cuda"):
    """lod_model.py:612-617: TorchScript Linear-ReLU-Linear[-Tanh] heads -> the decode's
    weight dict {opacity,cov,color}_{w1,b1,w2,b2}."""
    w = {}
    for head, fname in _HEADS:
        sd = torch.jit.load(os.path.join(path, fname), map_location="cpu").state_dict()
        keys = sorted({k.split(".")[0] for k in sd if k.endswith(".weight")}, key=int)
        if len(keys) != 2:
            raise NotImplementedError(f"hgsr: {fname} is not a Linear-ReLU-Linear head")
        w[f"{head}_w1"], w[f"{head}_b1"] = sd[f"{keys[0]}.weight"], sd[f"{keys[0]}.bias"]
        w[f"{head}_w2"], w[f"{head}_b2"] = sd[f"{keys[1]}.weight"], sd[f"{keys[1]}.bias"]
    return {k: v.float().to(device).contiguous() for k, v in w.items()}


def save_mlp_checkpoints(path, mlp_opacity, mlp_cov, mlp_color, in_dim):
    """lod_model.py:598-610 (torch.jit.trace of each head on a [1, in_dim] input)."""
    import warnings
    os.makedirs(path, exist_ok=True)
    warnings.filterwarnings("ignore", message=".*torch.jit.trace.*is deprecated", category=DeprecationWarning)
    for (head, fname), m in zip(_HEADS, (mlp_opacity, mlp_cov, mlp_color)):
        p = next(m.parameters())
        torch.jit.trace(m.eval(), torch.rand(1, in_dim, device=p.device, dtype=p.dtype)).save(os.path.join(path, fname))
