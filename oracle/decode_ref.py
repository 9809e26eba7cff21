"""CPU restatement of the anchor -> neural-Gaussian decode (TEST INFRASTRUCTURE ONLY).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline may import this
module; the product path (horizongs_amd.decode) never does.

Follows, line for line in meaning:
  * LoD mask: reference scene/lod_model.py:286-290 (set_anchor_mask) with
    scene/basic_model.py:192-197 (map_to_int_level, dist2level='floor');
  * decode: reference scene/basic_model.py:297-371 (generate_neural_gaussians) with
    the MLP shapes of scene/lod_model.py:67-84 (Linear -> ReLU -> Linear [-> Tanh]),
    appearance_dim = 0, smooth_complement = 1 (dist2level != 'progressive').

Pinned: tests/test_oracle.py checks both functions against tests/golden/decode_{rgb,sh2}.npz,
outputs of the reference module itself (scripts/make_golden.py).  The torch version
(`decode_torch`) is the same restatement in torch ops so autograd gives the reference
gradients the GPU backward is compared with (fp64 on the CPU).
"""
from __future__ import annotations

import math

import numpy as np
import torch


def lod_mask(anchor, level, extra_level, cam_center, res_scale, standard_dist, fork, street_levels):
    """scene/lod_model.py:286-290 + basic_model.py:192-197 (floor)."""
    anchor = np.asarray(anchor, np.float32)
    d = anchor - np.asarray(cam_center, np.float32)[None]
    dist = np.sqrt(np.sum(d * d, axis=1, dtype=np.float32)).astype(np.float32) * np.float32(res_scale)
    pred = (np.log2(np.float32(standard_dist) / dist) / np.float32(math.log2(fork))
            + np.asarray(extra_level, np.float32).reshape(-1)).astype(np.float32)
    il = np.clip(np.floor(pred).astype(np.int32), 0, int(street_levels) - 1)
    return np.asarray(level).reshape(-1) <= il


def _mlp(x, w1, b1, w2, b2):
    h = torch.relu(x @ w1.T + b1)
    return h @ w2.T + b2


def decode_torch(anchor, feat, offset, scaling_raw, cam_center, mlps, view_dim, n_offsets, color_dim):
    """scene/basic_model.py:297-371 on already-visible anchors.

    mlps: dict with opacity_w1/b1/w2/b2, cov_*, color_* tensors (nn.Linear layout [out, in]).
    Returns (xyz, offsets, color, opacity, scaling, rot, mask) exactly like the reference
    (color [M,3] for RGB, [M, color_dim//3, 3] for SH)."""
    grid_scaling = torch.exp(scaling_raw)
    ob_view = anchor - cam_center[None]
    ob_dist = ob_view.norm(dim=1, keepdim=True)
    ob_view = ob_view / ob_dist
    x = torch.cat([feat, ob_view], dim=1) if view_dim > 0 else feat
    m = mlps
    neural_opacity = torch.tanh(_mlp(x, m["opacity_w1"], m["opacity_b1"], m["opacity_w2"], m["opacity_b2"]))
    neural_opacity = neural_opacity.reshape([-1, 1])
    mask = (neural_opacity > 0.0).view(-1)
    opacity = neural_opacity[mask]
    color = _mlp(x, m["color_w1"], m["color_b1"], m["color_w2"], m["color_b2"])
    color = color.reshape([anchor.shape[0] * n_offsets, color_dim])
    scale_rot = _mlp(x, m["cov_w1"], m["cov_b1"], m["cov_w2"], m["cov_b2"]).reshape([anchor.shape[0] * n_offsets, 7])
    offsets = offset.reshape([-1, 3])
    concatenated = torch.cat([grid_scaling, anchor], dim=-1)
    rep = concatenated.repeat_interleave(n_offsets, dim=0)
    allc = torch.cat([rep, color, scale_rot, offsets], dim=-1)
    masked = allc[mask]
    scaling_repeat, repeat_anchor, color, scale_rot, offsets = masked.split([6, 3, color_dim, 7, 3], dim=-1)
    scaling = scaling_repeat[:, 3:] * torch.sigmoid(scale_rot[:, :3])
    rot = torch.nn.functional.normalize(scale_rot[:, 3:7])
    offsets = offsets * scaling_repeat[:, :3]
    xyz = repeat_anchor + offsets
    if color_dim != 3:
        color = color.reshape([color.shape[0], color_dim // 3, 3])
    return xyz, offsets, color, opacity, scaling, rot, mask


def golden_inputs(g, dtype=torch.float64):
    """Unpack a tests/golden/decode_*.npz fixture into decode_torch arguments (visible anchors only)."""
    vm = g["anchor_mask"]
    t = lambda a: torch.from_numpy(np.asarray(a)).to(dtype)
    mlps = {k: t(g[k]) for k in g.files if k.split("_")[0] in ("opacity", "cov", "color") and k[-2] in "wb"}
    view_dim = int(g["view_dim"])
    n_off = g["offset"].shape[1]
    color_dim = g["color_w2"].shape[0] // n_off
    return dict(anchor=t(g["anchor"][vm]), feat=t(g["anchor_feat"][vm]), offset=t(g["offset"][vm]),
                scaling_raw=t(g["scaling"][vm]), cam_center=t(g["cam_center"]), mlps=mlps, view_dim=view_dim,
                n_offsets=n_off, color_dim=color_dim)
