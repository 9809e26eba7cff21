"""Diagnostic: which head / anchors of the decode backward disagree with the oracle."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import numpy as np
import torch
from oracle import decode_ref as D
from test_gpu_decode import _random_model
from horizongs_amd import decode as HD

view_dim, color_dim, n = 0, 27, 700
inputs, mlps = _random_model(n, view_dim, color_dim, seed=5 + n)
vis = torch.rand(n, generator=torch.Generator().manual_seed(77)) < 0.8
names = ("xyz", "offsets", "color", "opacity", "scaling", "rot")
for which in range(6):
    ins = {k: v.double().clone().requires_grad_(True) for k, v in inputs.items()}
    ws = {k: v.double().clone().requires_grad_(True) for k, v in mlps.items()}
    sub = {k: (v[vis] if k != "cam_center" else v) for k, v in ins.items()}
    outs = D.decode_torch(sub["anchor"], sub["feat"], sub["offset"], sub["scaling_raw"], sub["cam_center"], ws,
                          view_dim, 10, color_dim)
    up = torch.randn(outs[which].shape, generator=torch.Generator().manual_seed(3), dtype=torch.float64)
    (outs[which] * up).sum().backward()
    di = {k: v.cuda().clone().requires_grad_(True) for k, v in inputs.items()}
    dw = {k: v.cuda().clone().requires_grad_(True) for k, v in mlps.items()}
    o = HD.decode(di["anchor"], di["feat"], di["offset"], di["scaling_raw"], di["cam_center"], dw, vis.cuda(),
                  view_dim, 10, color_dim)
    (o[which] * up.float().cuda().reshape(o[which].shape)).sum().backward()
    err = (di["feat"].grad.cpu().double() - ins["feat"].grad).abs()
    bad = (err > 1e-3).any(1).nonzero().reshape(-1).tolist()
    vi = torch.nonzero(vis).reshape(-1).tolist()
    pos = [vi.index(b) if b in vi else -1 for b in bad]
    print(names[which], "max err", float(err.max()), "bad anchors", bad[:10], "vis positions", pos[:10],
          "n_vis", len(vi))
    for k in mlps:
        gref = ws[k].grad if ws[k].grad is not None else torch.zeros_like(ws[k])
        e = (dw[k].grad.cpu().double() - gref).abs().max()
        if e > 1e-3:
            print("   weight", k, float(e))
