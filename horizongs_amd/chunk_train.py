"""One chunk stage of the per-chunk pipeline: the child process `chunks.run_chunks` starts.

    python -m horizongs_amd.chunk_train --chunk 0_1 --stage coarse --out DIR [--anchors 20000
           --iters 60 --width 320 --height 180 --views 8] [--dry]

The reference trains each chunk with train.py under chunk_coarse/<m>_<n>.yaml, then
chunk_fine/<m>_<n>.yaml whose pretrained_checkpoint is the coarse output
(preprocess/generate_chunks_config.py:77-104), and saves the anchor PLY + TorchScript MLPs
(scene/lod_model.py:374-411,598-610) and the explicit PLY merge.py reads
(scene/lod_model.py:681-771).  There is no dataset here, so a chunk is a seeded synthetic
one: its anchors (the c4 chunk model: view_dim 0, 10 offsets, SH2 colour head) and a seeded
explicit "ground truth" scene occupy the chunk's own cell of the ground plane, x in
[m S, (m+1) S) and z in [n S, (n+1) S) (S = CELL), padded by OVERLAP on every side as the
partition's overlap expansion pads the chunk's data (preprocess/data_preprocess.py:176-245);
true_bounds() are the unpadded cell, what consolidate_explicit crops to.

coarse: initialise, train `iters` views (the chunk's camera set cycled), save DIR/<chunk>/coarse.
fine:   load DIR/<chunk>/coarse, train `iters` more views, save DIR/<chunk>/fine including
        point_cloud_explicit.ply (export through the fused HIP decode).
--dry:  plumbing only, no device work (the launcher's CPU tests): the same files from the
        seeded initialisation, the explicit PLY holding the anchors themselves.
"""
from __future__ import annotations

import argparse
import math
import os

import numpy as np
import torch

CELL = 4.0      # chunk cell edge on the ground plane (world units)
OVERLAP = 0.5   # padding of a chunk's data beyond its cell
HEIGHT = 2.0    # anchors / ground-truth Gaussians in y in [-HEIGHT/2, HEIGHT/2]


def parse_chunk(cid):
    m, n = (int(x) for x in cid.split("_"))
    return m, n


def true_bounds(cid):
    """(x bounds, z bounds) of the chunk's cell (merge.py crops to these; plane axes 0, 2)."""
    m, n = parse_chunk(cid)
    return ((m * CELL, (m + 1) * CELL), (n * CELL, (n + 1) * CELL))


def _points(count, cid, g):
    (x0, x1), (z0, z1) = true_bounds(cid)
    u = torch.rand(count, 3, generator=g, dtype=torch.float64)
    x = x0 - OVERLAP + u[:, 0] * (x1 - x0 + 2 * OVERLAP)
    y = (u[:, 1] - 0.5) * HEIGHT
    z = z0 - OVERLAP + u[:, 2] * (z1 - z0 + 2 * OVERLAP)
    return torch.stack([x, y, z], 1).float()


def cameras(cid, views, width, height):
    """Aerial views of the chunk's cell: a seeded ring above it looking at its centre."""
    from .synthetic import look_at
    (x0, x1), (z0, z1) = true_bounds(cid)
    c = [(x0 + x1) / 2, 0.0, (z0 + z1) / 2]
    m, n = parse_chunk(cid)
    g = torch.Generator().manual_seed(7000 + 97 * m + n)
    vms = []
    for v in range(views):
        az = 2 * math.pi * (v + float(torch.rand(1, generator=g))) / views
        r = CELL * (0.9 + 0.4 * float(torch.rand(1, generator=g)))
        eye = [c[0] + r * math.cos(az), -(CELL * 1.2), c[2] + r * math.sin(az)]  # y down: above = negative y
        vms.append(look_at(eye, c))
    f = 0.5 * width / math.tan(math.radians(30.0))
    K = torch.tensor([[f, 0.0, width / 2], [0.0, f, height / 2], [0.0, 0.0, 1.0]])
    return torch.stack(vms), K


def init_model(cid, anchors):
    """The c4 chunk model (view_dim 0, 10 offsets, SH2 colour head: scene/lod_model.py:67-84)."""
    m, n = parse_chunk(cid)
    g = torch.Generator().manual_seed(100 * m + n)
    A, k, F = anchors, 10, 32
    p = dict(anchor=_points(A, cid, g), feat=torch.randn(A, F, generator=g) * 0.5,
             offset=torch.randn(A, k, 3, generator=g) * 0.5,
             scaling=(math.log(0.05) + torch.randn(A, 6, generator=g) * 0.1).float())
    torch.manual_seed(100 * m + n + 1)
    mlps = [torch.nn.Sequential(torch.nn.Linear(F, 32), torch.nn.ReLU(True), torch.nn.Linear(32, o))
            for o in (k, 7 * k, 27 * k)]
    return p, mlps


def _paths(out, cid, stage):
    d = os.path.join(out, cid, stage)
    os.makedirs(d, exist_ok=True)
    return d


def save_stage(d, p, mlps):
    from .ply import save_anchor_ply, save_mlp_checkpoints
    A = p["anchor"].shape[0]
    rot = torch.zeros(A, 4)
    rot[:, 0] = 1
    save_anchor_ply(os.path.join(d, "point_cloud.ply"), p["anchor"], torch.zeros(A, 1), torch.zeros(A),
                    p["offset"], p["feat"], p["scaling"], rot, 4.0, 1, 4)
    if mlps is not None:
        save_mlp_checkpoints(d, *mlps, in_dim=32)


def load_stage(d, device):
    from .ply import load_anchor_ply, load_mlp_checkpoints
    a = load_anchor_ply(os.path.join(d, "point_cloud.ply"), device=device)
    p = dict(anchor=a["anchor"], feat=a["anchor_feat"], offset=a["offset"], scaling=a["scaling"])
    w = load_mlp_checkpoints(d, device=device) if os.path.exists(os.path.join(d, "opacity_mlp.pt")) else None
    return p, w


def train(p, weights, cid, iters, width, height, views, seed, lr_scale=1.0):
    """`iters` reference train steps (train.py:150-277) of the chunk model on the device: fused
    LoD-free prefilter -> fused decode -> rasterization(SH2) -> fused loss -> backward -> Adam."""
    from . import decode as HD
    from . import gsplat_api as G
    from .loss import fused_loss
    from .optim import Adam
    from .synthetic import Scene
    dev = torch.device("cuda")
    vms, K = cameras(cid, views, width, height)
    vms, K = vms.to(dev), K.to(dev)
    # the chunk's "images": renders of a seeded explicit scene in the same cell
    m, n = parse_chunk(cid)
    g = torch.Generator().manual_seed(5000 + 100 * m + n)
    nt = 4 * p["anchor"].shape[0]
    gt_sc = Scene(_points(nt, cid, g), torch.nn.functional.normalize(torch.randn(nt, 4, generator=g), dim=-1),
                  torch.exp(math.log(0.02) + torch.randn(nt, 3, generator=g) * 0.3),
                  0.2 + 0.7 * torch.rand(nt, generator=g), torch.rand(nt, 3, generator=g), vms[:1].cpu(), K[None].cpu(),
                  width, height, torch.zeros(1, 3)).to(dev)
    with torch.no_grad():
        gts = [G.rasterization(gt_sc.means, gt_sc.quats, gt_sc.scales, gt_sc.opacities, gt_sc.colors, vms[v:v + 1],
                               K[None], width, height, packed=False)[0][0].permute(2, 0, 1).contiguous()
               for v in range(views)]
    P = {k: v.to(dev).clone().requires_grad_(k != "anchor") for k, v in p.items()}
    W = {k: v.to(dev).clone().requires_grad_(True) for k, v in weights.items()}
    lr = dict(feat=0.0075, offset=0.01, scaling=0.007, opacity=0.002, cov=0.004, color=0.008)
    groups = [{"params": [P[k]], "lr": lr_scale * lr[k]} for k in ("feat", "offset", "scaling")]
    groups += [{"params": [W[k]], "lr": lr_scale * lr[k.split("_")[0]]} for k in W]
    opt = Adam(groups, lr=0.0, eps=1e-15)
    quats = torch.zeros(P["anchor"].shape[0], 4, device=dev)
    quats[:, 0] = 1
    bg = torch.zeros(1, 3, device=dev)
    for it in range(iters):
        v = (it * 7 + seed) % views
        vm = vms[v:v + 1]
        cam = torch.linalg.inv(vm[0].double())[:3, 3].float()
        for t in list(P.values()) + list(W.values()):
            t.grad = None
        with torch.no_grad():
            _, vis = HD.prefilter(P["anchor"], torch.exp(P["scaling"].detach()), quats, vm[0], K, width, height)
        xyz, _, col, op, sc, rot, _ = HD.decode(P["anchor"], P["feat"], P["offset"], P["scaling"], cam, W, vis, 0, 10, 27)
        out, alpha, _ = G.rasterization(xyz, rot, sc, op.reshape(-1), col, vm, K[None], width, height, packed=False,
                                        backgrounds=bg, render_mode="RGB+ED", sh_degree=2)
        img = out[0].permute(2, 0, 1)
        loss = fused_loss(img, gts[v], None, 0.2, alpha[0, ..., 0], 0.0, 0.0, sc, 0.01)[0]
        loss.backward()
        opt.step()
    return {k: t.detach() for k, t in P.items()}, {k: t.detach() for k, t in W.items()}


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--chunk", required=True)
    ap.add_argument("--stage", choices=["coarse", "fine"], required=True)
    ap.add_argument("--out", required=True)
    ap.add_argument("--anchors", type=int, default=20000)
    ap.add_argument("--iters", type=int, default=60)
    ap.add_argument("--width", type=int, default=320)
    ap.add_argument("--height", type=int, default=180)
    ap.add_argument("--views", type=int, default=8)
    ap.add_argument("--lr-scale", type=float, default=1.0, help="every learning rate times this")
    ap.add_argument("--dry", action="store_true", help="plumbing only: no device work")
    a = ap.parse_args(argv)
    d = _paths(a.out, a.chunk, a.stage)
    with open(os.path.join(d, "device.txt"), "w") as f:  # which slot ran this stage
        f.write(os.environ.get("HIP_VISIBLE_DEVICES", ""))
    if a.dry:
        if a.stage == "coarse":
            p, _ = init_model(a.chunk, a.anchors)
            save_stage(d, p, None)
        else:
            p, _ = load_stage(_paths(a.out, a.chunk, "coarse"), "cpu")
            save_stage(d, p, None)
            from .ply import save_explicit_ply
            A = p["anchor"].shape[0]
            save_explicit_ply(os.path.join(d, "point_cloud_explicit.ply"), p["anchor"], torch.zeros(A, 1),
                              torch.zeros(A), p["feat"][:, None, :3], p["feat"][:, 3:27].reshape(A, 8, 3),
                              p["scaling"][:, :1], p["scaling"][:, 3:], torch.ones(A, 4), 4.0, 1, 4)
        return 0
    if not torch.cuda.is_available():
        raise RuntimeError("hgsr chunk_train: no HIP device (HIP_VISIBLE_DEVICES="
                           f"{os.environ.get('HIP_VISIBLE_DEVICES')!r}); --dry runs the plumbing without one")
    if a.stage == "coarse":
        p, mlps = init_model(a.chunk, a.anchors)
        weights = {}
        for h, mlp in zip(("opacity", "cov", "color"), mlps):
            weights[f"{h}_w1"], weights[f"{h}_b1"] = mlp[0].weight.detach(), mlp[0].bias.detach()
            weights[f"{h}_w2"], weights[f"{h}_b2"] = mlp[2].weight.detach(), mlp[2].bias.detach()
        seed = 0
    else:
        p, weights = load_stage(_paths(a.out, a.chunk, "coarse"), "cpu")
        weights = {k: v.cpu() for k, v in weights.items()}
        seed = 3
    p, weights = train(p, weights, a.chunk, a.iters, a.width, a.height, a.views, seed, a.lr_scale)
    mlps = []
    for h in ("opacity", "cov", "color"):
        lin1 = torch.nn.Linear(32, 32)
        lin2 = torch.nn.Linear(32, weights[f"{h}_w2"].shape[0])
        with torch.no_grad():
            lin1.weight.copy_(weights[f"{h}_w1"])
            lin1.bias.copy_(weights[f"{h}_b1"])
            lin2.weight.copy_(weights[f"{h}_w2"])
            lin2.bias.copy_(weights[f"{h}_b2"])
        mlps.append(torch.nn.Sequential(lin1, torch.nn.ReLU(True), lin2))
    save_stage(d, {k: v.cpu() for k, v in p.items()}, mlps)
    if a.stage == "fine":
        from .ply import export_explicit
        A = p["anchor"].shape[0]
        dev = p["anchor"].device
        export_explicit(os.path.join(d, "point_cloud_explicit.ply"), p["anchor"], torch.zeros(A, 1, device=dev),
                        torch.zeros(A, device=dev), p["feat"], p["offset"], p["scaling"], weights, 10, 27, 4.0, 1, 4)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
