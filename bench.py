"""North-star benchmark: train-step views/s (fwd+bwd raster) @ 2M Gaussians / 1080p.

One "step" = one training view through the rasterizer path Horizon-GS runs at
train.py:150-206: gsplat.rasterization(..., packed=False, render_mode="RGB+ED")
(projection -> tile binning + depth sort -> raster forward), the reference loss
head (fused HIP loss), loss.backward() (raster backward -> projection backward)
and the optimizer step (Adam, eps=1e-15, one fused HIP launch), on a synthetic c2 scene
(SURVEY.md §8(d)): 2,000,000 Gaussians at 1920x1080, fp32, inputs resident in HBM.

`--config` selects the workload of the headline line (default c2); the other BASELINE
configs are measured as `secondary` lines of the same JSON object:
  c2          2M explicit Gaussians (the metric's own size), 3DGS
  c2-anchors  configs[1] Block_small coarse: 500k anchors -> LoD + prefilter + fused decode -> 3DGS
  c3          configs[2] Block_small fine: the c2 scene through rasterization_2dgs (+ normal loss)
  c4          configs[3] Block_A per-chunk fine: a 500k-anchor SH2 chunk (color_attr SH2, view_dim 0,
              10 offsets, colour head [32, 270]; config/ours/large_scene/block_A/chunk_fine/*.yaml),
              one chunk per GPU, no collectives
  c5          configs[4] UCGS: 1M anchors (RGB, view_dim 3; config/ours/ucgs/sf/fine.yaml), DDP over views

Multi-GPU: one process per GPU.  `--gpus N` with no WORLD_SIZE in the environment starts
N ranks itself (a torch.distributed.run child process, before this process touches the
GPU); under torchrun it is one rank.  At N > 1 the headline c2 line trains ONE scene
data-parallel over views (each rank renders its own camera; the Gaussian gradients are
reduce-scattered in buckets launched from gradient hooks while the backward runs, each rank
steps Adam on its shard and the parameters are all-gathered, the colours' all-gather left in
flight until the next rasterization reads them: multigpu.ShardedAdamDDP), and the secondary
lines are c2-chunks (the same workload under the per-chunk mapping: each rank trains its own
scene, no collectives), c4 (per chunk -- reference preprocess/generate_chunks_config.py,
merge.py) and c5 (DDP over views, bucketed all-reduce: multigpu.GradientAllReduce).  At N = 1
the DDP modes are the single-GPU step.

Prints ONE JSON line (rank 0) with the metric, a roofline object for the dominant
kernel (HIP-event timed live over the timed region), a CPU baseline (the C oracle on all
host threads, rank 0 at N=1 only) and the secondary lines.
"""
from __future__ import annotations

import argparse
import ctypes as ct
import gc
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))


def _launch_ranks() -> None:
    """--gpus N without WORLD_SIZE: run N ranks under torch.distributed.run in a child process
    (this process has not touched the GPU, and never execs) and exit with its status."""
    import subprocess
    argv = sys.argv[1:]
    n = 1
    for i, a in enumerate(argv):
        if a == "--gpus" and i + 1 < len(argv):
            n = int(argv[i + 1])
        elif a.startswith("--gpus="):
            n = int(a.split("=", 1)[1])
    if n <= 1 or "WORLD_SIZE" in os.environ:
        return
    import socket
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + argv
    sys.exit(subprocess.call(cmd, env=env))


if __name__ == "__main__":
    _launch_ranks()

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

sys.path.insert(0, ROOT)

from horizongs_amd import _native as NAT  # noqa: E402
from horizongs_amd import decode as HD  # noqa: E402
from horizongs_amd import densify as HDn  # noqa: E402
from horizongs_amd import gsplat_api as G  # noqa: E402
from horizongs_amd.activations import activate  # noqa: E402
from horizongs_amd.loss import fused_loss  # noqa: E402
from horizongs_amd.multigpu import GradientAllReduce, ShardedAdamDDP  # noqa: E402
from horizongs_amd.optim import Adam  # noqa: E402
from horizongs_amd.synthetic import camera_set, make_scene  # noqa: E402

METRIC = "train-step views/sec (fwd+bwd raster) @2M Gaussians/1080p; PSNR delta vs ref"
FP32_PEAK_TFLOPS = 157.3   # MI355X fp32 vector (= f32 MFMA) peak, MI355X_MICROARCH.md
HBM_PEAK_GBS = 8000.0      # HBM3E spec
FLOP_PER_PAIR = {"raster3d_fwd": 20.0, "raster3d_bwd": 60.0, "raster2d_fwd": 40.0, "raster2d_bwd": 120.0}
KERNELS = ["project3d_fwd", "isect_count", "isect_emit", "tile_sort", "raster3d_fwd", "raster3d_bwd",
           "project3d_bwd", "project2d_fwd", "raster2d_fwd", "raster2d_bwd", "project2d_bwd", "sh_fwd", "sh_bwd",
           "decode_count", "decode_fwd", "decode_bwd", "loss_fwd", "loss_bwd", "adam", "training_statis", "depth_normal_fwd",
           "depth_normal_bwd", "anchor_prefilter", "explicit_gather"]


CONFIGS = {
    "c2": dict(label=("headline: 2M explicit Gaussians (the metric's own size), 1080p, 3DGS, a seeded 16-view "
                      "camera set cycled per step"), gs="3d", anchors=0, sh_degree=None, mode=None),
    "c2-fixed": dict(label=("c2 on its single identity camera every step (the rounds 1-4 headline: the view with the "
                            "most intersections)"), gs="3d", anchors=0, sh_degree=None, mode=None, cameras=1),
    "c2-anchors": dict(label="configs[1] Block_small coarse: 500k anchors (RGB, view_dim 3), 1080p, 3DGS", gs="3d",
                       anchors=500_000, sh_degree=None, view_dim=3, mode=None),
    "c3": dict(label="configs[2] Block_small fine: 2DGS surfels, depth + normal outputs, 1080p", gs="2d", anchors=0,
               sh_degree=None, mode=None),
    "c2-chunks": dict(label=("c2 under the per-chunk mapping (north_star's first way: each rank trains its own "
                             "2M-Gaussian chunk, seed = rank, no collectives); the headline c2 line at N > 1 is DDP "
                             "over views"), gs="3d", anchors=0, sh_degree=None, mode="chunk"),
    "c4": dict(label=("configs[3] MatrixCity Block_A per-chunk fine: 500k-anchor SH2 chunk (view_dim 0, 10 offsets, "
                      "colour head [32,270]), one chunk per GPU, no collectives"), gs="3d", anchors=500_000,
               sh_degree=2, view_dim=0, mode="chunk"),
    "c5": dict(label=("configs[4] UCGS: 1M anchors (RGB, view_dim 3; ~10M neural Gaussians before the opacity "
                      "mask), DDP over views with RCCL all-reduce"), gs="3d", anchors=1_000_000, sh_degree=None,
               view_dim=3, mode="ddp"),
}


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # 32 = two cycles of the 16-view camera set: every view weighs the same in the mean
    ap.add_argument("--steps", type=int, default=32)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", choices=sorted(CONFIGS), default=None,
                    help="workload of the headline line (default c2; the flags below override it)")
    ap.add_argument("--n", type=int, default=2_000_000)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--gs", choices=["3d", "2d"], default=None)
    ap.add_argument("--mode", choices=["auto", "chunk", "ddp"], default="auto",
                    help="auto: the config's own mapping (c4 per chunk, c5 DDP; c2 / c3 DDP over views at N > 1)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-secondary", action="store_true",
                    help="skip the secondary config lines (N = 1: c2-fixed, c2-anchors, c3, c4, c5; N > 1: c2-chunks, c4, c5)")
    ap.add_argument("--no-timing", action="store_true", help="skip per-kernel HIP events (rocprof runs)")
    ap.add_argument("--no-quality", action="store_true", help="skip the live PSNR-parity measurement (N = 1)")
    ap.add_argument("--freeze", action="store_true",
                    help="diagnostic A/Bs of kernel builds that change the gradients: skip the optimizer step so every "
                         "build sees the same scene (the line is then not the metric)")
    ap.add_argument("--sh-degree", type=int, default=None, choices=[0, 1, 2, 3],
                    help="SH colours: [N,(d+1)^2,3] ~ N(0, 0.3) (explicit), or an SH colour head (anchors)")
    ap.add_argument("--anchors", type=int, default=None,
                    help="decode-inclusive variant (SURVEY 8(d) c2): A anchors -> fused decode -> raster")
    ap.add_argument("--view-dim", type=int, default=None, choices=[0, 3])
    ap.add_argument("--cameras", type=int, default=None,
                    help="training views cycled per step (default 16, c2-fixed 1): the reference picks a camera per "
                         "iteration (train.py:133-148); synthetic.camera_set")
    return ap.parse_args(argv)


def resolve(args, world):
    """Fill gs / anchors / sh_degree / view_dim / mode from --config, explicit flags winning."""
    name = args.config or ("c2-anchors" if args.anchors else ("c3" if args.gs == "2d" else "c2"))
    c = CONFIGS[name]
    args.config = name
    args.gs = args.gs or c["gs"]
    args.anchors = c["anchors"] if args.anchors is None else args.anchors
    if args.sh_degree is None:
        args.sh_degree = c["sh_degree"]
    args.view_dim = c.get("view_dim", 3) if args.view_dim is None else args.view_dim
    args.cameras = c.get("cameras", 16) if args.cameras is None else args.cameras
    if args.mode == "auto":
        args.mode = c["mode"] or ("ddp" if world > 1 else "chunk")
    return args


class Workload:
    def __init__(self, args, rank, dev, world=1):
        self.args = args
        self.dev = dev
        seed = rank if args.mode == "chunk" else 0
        # anchor workloads build their anchors in _init_anchors; the explicit scene needs only a camera
        sc = make_scene(2 if args.anchors else args.n, args.width, args.height, seed=seed, sh_degree=args.sh_degree)
        self.sc = sc
        # the training cameras (train.py:133-148 picks one per iteration): view 0 is the scene's
        # identity camera, the rest a seeded ring / elevation / distance set (synthetic.camera_set);
        # step s of rank r renders view (s * world + r) mod V -- a rank-sharded viewpoint stack
        self.cams = camera_set(args.cameras).to(dev)[:, None] if args.cameras > 1 else sc.viewmats.to(dev)[None]
        self.cam_centers = torch.linalg.inv(self.cams[:, 0].double())[:, :3, 3].float().contiguous()
        self.rank, self.world = rank, (world if args.mode == "ddp" else 1)
        self.n_steps = 0
        self.view_log = []  # (view, intersections, Gaussians in view) of every step
        self.viewmats = self.cams[self.rank % len(self.cams)]
        self.Ks = sc.Ks.to(dev)
        self.bg = torch.zeros(1, 3, device=dev)
        g = torch.Generator().manual_seed(1000 + rank)
        self.target = torch.rand(3, args.height, args.width, generator=g).to(dev)
        if args.anchors:
            groups = self._init_anchors(args, seed, dev)
        else:
            # trained in the 3DGS parametrisation: log scales and opacity logits, activated each step
            self.means = sc.means.to(dev).requires_grad_(True)
            self.quats = sc.quats.to(dev).requires_grad_(True)
            self.log_scales = torch.log(sc.scales).to(dev).requires_grad_(True)
            self.opac_logit = torch.logit(sc.opacities).to(dev).requires_grad_(True)
            self.colors = sc.colors.to(dev).requires_grad_(True)
            self.params = [self.means, self.quats, self.log_scales, self.opac_logit, self.colors]
            # 3DGS per-attribute learning rates for the explicit Gaussians
            groups = [(self.means, 1.6e-4), (self.quats, 1e-3), (self.log_scales, 5e-3), (self.opac_logit, 5e-2),
                      (self.colors, 2.5e-3)]
        # the reference optimizer (scene/lod_model.py:320): Adam(eps=1e-15), one group per tensor,
        # stepped every iteration (train.py:274-277) -- one fused HIP launch here
        self.optimizer = Adam([{"params": [p], "lr": lr} for p, lr in groups], lr=0.0, eps=1e-15)
        # DDP over views: buckets follow the optimizer's current groups (densify surgery safe); the
        # anchor model buckets _offset / _scaling / the cov MLP first: the decode backward hands
        # their gradients over after its first head, so their all-reduce runs under the rest of it
        self.allreduce = GradientAllReduce(self.optimizer, bucket_mb=64.0, order=getattr(self, "ddp_order", None))
        # the explicit-Gaussian step (c2 / c3 at N > 1): every rank produces every gradient and
        # nothing is densified, so the optimizer is sharded instead (ZeRO-1: reduce-scatter ->
        # Adam on this rank's 1/N -> all-gather, multigpu.ShardedAdamDDP)
        self.sharded = None
        self._unhook = None
        if not args.anchors:
            # buckets in the order the backward finishes their gradients: the colours' (the raster
            # backward's) reduce-scatter runs under the projection and activation backwards, the
            # means / quats' under the activation backward.  The colours' all-gather is left in flight
            # by finish() (stepped last) and waited for inside the next rasterization() just before
            # it reads them (gsplat_api parameter-ready hook), under the projection and binning
            # (one bucket per parameter would spare the gradients' copy into the flat buffers, but
            # each collective's fixed cost is larger: c2 1.716 -> 1.821 ms in the one-GPU rehearsal
            # with five buckets, gpurun_out/r05s32; the colours' one-parameter bucket reduces
            # autograd's tensor in place)
            self.sharded = ShardedAdamDDP(self.optimizer, order=[[self.colors], [self.means, self.quats],
                                                                 [self.log_scales, self.opac_logit]],
                                          defer=[self.colors])
            self._unhook = G.register_param_ready_hook(self.sharded.wait_deferred)

    def flush(self):
        """Every parameter whole (the sharded optimizer's deferred colours all-gather waited for)."""
        if self.sharded is not None:
            self.sharded.flush()

    def close(self):
        """Drop the parameter-ready hook (it holds this workload's optimizer and buffers alive)."""
        self.flush()
        if self._unhook is not None:
            self._unhook()
            self._unhook = None

    def _init_anchors(self, args, seed, dev):
        """SURVEY 8(d) decode-inclusive c2: anchors placed like the c2 Gaussians, feat ~ N(0, 0.1),
        offsets ~ N(0, 0.1), _scaling = ln 0.01 + N(0, 0.1), default-initialised MLPs (seed 2),
        feat_dim 32, 10 offsets; view_dim 3 + RGB (Block_small, UCGS) or view_dim 0 + an SH colour
        head of 3 (d+1)^2 outputs per offset (Block_A chunks: SH2, [32, 270]) (scene/lod_model.py:67-84)."""
        A = args.anchors
        k = 10
        self.view_dim = args.view_dim
        self.color_dim = 3 if args.sh_degree is None else 3 * (args.sh_degree + 1) ** 2
        sc = make_scene(A, args.width, args.height, seed=seed)
        g = torch.Generator().manual_seed(2)
        self.anchor = sc.means.to(dev).requires_grad_(True)
        self.feat = (torch.randn(A, 32, generator=g) * 0.1).to(dev).requires_grad_(True)
        self.offset = (torch.randn(A, k, 3, generator=g) * 0.1).to(dev).requires_grad_(True)
        self.scaling_raw = (np.log(0.01) + torch.randn(A, 6, generator=g) * 0.1).float().to(dev).requires_grad_(True)
        torch.manual_seed(2)
        nn = torch.nn
        self.mlps = [nn.Sequential(nn.Linear(32 + self.view_dim, 32), nn.ReLU(True), nn.Linear(32, o)).to(dev)
                     for o in (k, 7 * k, self.color_dim * k)]
        self.cam_center = self.cam_centers[self.rank % len(self.cams)]
        self.params = [self.anchor, self.feat, self.offset, self.scaling_raw] + [
            p for m in self.mlps for p in m.parameters()]
        self.ddp_order = [self.offset, self.scaling_raw, *self.mlps[1].parameters(), self.feat, self.anchor]
        self.anchor_quats = torch.zeros(A, 4, device=dev)
        self.anchor_quats[:, 0] = 1.0  # get_rotation at init (_rotation is not trained)
        # LoD inputs of set_anchor_mask (every synthetic anchor on level 0: the test runs, all pass)
        self.lod = dict(level=torch.zeros(A, dtype=torch.int32, device=dev),
                        extra_level=torch.zeros(A, device=dev), cam_center=self.cam_center, res_scale=1.0,
                        standard_dist=4.0, fork=2, street_levels=4)
        # densification statistics updated every step by training_statis (train.py:258-262)
        self.stats = dict(anchor_opacity_accum=torch.zeros(A, 1, device=dev), anchor_demon=torch.zeros(A, 1, device=dev),
                          offset_gradient_accum=torch.zeros(A * k, 1, device=dev),
                          offset_denom=torch.zeros(A * k, 1, device=dev))
        self.stats_model = type("Stats", (), dict(n_offsets=k, **self.stats))
        self.stats_opt = type("Opt", (), dict(pruning_type="mean", growing_type="mean"))
        # config/base/small_scene/coarse.yaml learning rates (position lr 0: still an Adam group)
        return [(p, lr) for p, lr in zip([self.anchor, self.feat, self.offset, self.scaling_raw] + [
            p for m in self.mlps for p in m.parameters()], [0.0, 0.0075, 0.01, 0.007] + [0.002] * 4 + [0.004] * 4
            + [0.008] * 4)]

    def step(self):
        for p in self.params:
            p.grad = None
        W, H = self.args.width, self.args.height
        view = (self.n_steps * self.world + self.rank) % len(self.cams)
        self.n_steps += 1
        self.viewmats = self.cams[view]
        if self.args.anchors:
            self.cam_center = self.cam_centers[view]
            self.lod["cam_center"] = self.cam_center
        if self.args.anchors:
            # set_anchor_mask + prefilter_voxel (scene/lod_model.py:286-290, gaussian_renderer/render.py
            # :120-197) fused: LoD test AND radius > 0 of the anchors projected with their first three
            # scales, compacted on the device into the visible-anchor index the decode consumes
            with torch.no_grad():
                visible, vis_idx = HD.prefilter(self.anchor.detach(), torch.exp(self.scaling_raw.detach()),
                                                self.anchor_quats, self.viewmats[0], self.Ks[0], W, H, lod=self.lod,
                                                lazy=True)  # Av stays on the device: one sync less
            xyz, _, cols, opac, scales, quats, sel = HD.decode(self.anchor, self.feat, self.offset, self.scaling_raw,
                                                               self.cam_center, self.mlps, vis_idx, self.view_dim, 10,
                                                               self.color_dim)
            opac = opac.reshape(-1)
            self.last_av = sel.numel() // 10  # visible anchors of this view (decode MFMA accounting)
        else:
            xyz, quats, cols = self.means, self.quats, self.colors
            # scaling_activation = exp, opacity_activation = sigmoid: one fused HIP pass each way
            scales, opac = activate(self.log_scales, self.opac_logit)
        self.last_colors = cols
        if self.args.gs == "3d":
            out, alpha, meta = G.rasterization(xyz, quats, scales, opac, cols, self.viewmats, self.Ks, W, H,
                                               packed=False, backgrounds=self.bg, render_mode="RGB+ED",
                                               sh_degree=self.args.sh_degree)
            meta["means2d"].retain_grad()
        else:
            (out, alpha, normals, nfd, distort, median), meta = G.rasterization_2dgs(
                xyz, quats, scales, opac, cols, self.viewmats, self.Ks, W, H,
                packed=False, backgrounds=self.bg, render_mode="RGB+ED", sh_degree=self.args.sh_degree)
        # the reference fine-stage loss head (train.py:153-178, config/base/small_scene/fine.yaml:50-57):
        # 0.8 L1 + 0.2 D-SSIM + 0.01 scale reg + 0.05 sky opacity + 0.05 opacity entropy, all in the fused HIP loss
        # C == 1: reshape/permute are views, so the loss reads the channels-last render in place and
        # its backward writes the full RGB+ED gradient (zero ED channel) with no slice/copy/fill glue
        img = out.reshape(H, W, -1).permute(2, 0, 1)
        # 2DGS adds the normal-consistency term (config/our_2d/*/fine.yaml: lambda_normal 0.05), fused too
        aux = {} if self.args.gs == "3d" else dict(normals=normals.reshape(H, W, 3).permute(2, 0, 1),
                                                 normals_from_depth=nfd.reshape(H, W, 3).permute(2, 0, 1),
                                                 lambda_normal=0.05)
        loss = fused_loss(img, self.target, None, 0.2, alpha.reshape(H, W), 0.05, 0.05, scales, 0.01, **aux)[0]
        ddp = self.args.mode == "ddp" and self.allreduce.active
        red = (self.sharded or self.allreduce) if ddp else None
        if ddp:
            red.begin()  # gradient hooks launch the bucket collectives during the backward
        # the backward's seed dL/dL = 1, allocated once (loss.backward() fills a new one-element
        # tensor with a kernel launch every step)
        if getattr(self, "_seed", None) is None or self._seed.shape != loss.shape:
            self._seed = torch.ones_like(loss)
        loss.backward(self._seed)
        if self.args.anchors:  # densification statistics of this view (train.py:258-262)
            HDn.training_statis(self.stats_model, self.stats_opt,
                                dict(selection_mask=sel, visible_mask=visible, viewspace_points=meta["means2d"],
                                     visibility_filter=meta["radii"][0] > 0, opacity=opac, radii=meta["radii"][0]),
                                W, H)
        if ddp and self.sharded is not None:
            self.sharded.finish()  # per bucket: Adam on this rank's shard, then its all-gather
        elif ddp:
            # train.py:274-277 per bucket: each bucket's Adam launch follows its own all-reduce and
            # overlaps the later buckets' collectives
            self.allreduce.finish(step=self.optimizer.step_params)
        elif not self.args.freeze:
            self.optimizer.step()  # train.py:274-277 (zero_grad(set_to_none) = the grad reset above)
        self.meta = meta
        self.view_log.append((view, meta["flatten_ids"].numel()))
        return loss


def _newest_profile(pattern):
    """profiles/<the newest round's file matching pattern> (rNN-prefixed names sort by round)"""
    import glob
    hits = sorted(glob.glob(os.path.join(ROOT, "profiles", pattern)))
    return os.path.relpath(hits[-1], ROOT) if hits else None


def hbm_kernels(wl, kernels, n_isects):
    """Algorithmic-bytes rate of the HBM-bound kernels of the step (DESIGN.md §4 per-unit
    bytes; unit counts of the last step) against the 8 TB/s HBM3E peak."""
    if not kernels or n_isects is None:
        return None
    N = int(wl.last_colors.shape[0])
    P = wl.args.width * wl.args.height
    n_par = sum(p.numel() for p in wl.params)
    per = {
        "project3d_fwd": 68 * N, "project3d_bwd": 120 * N, "project2d_fwd": 104 * N, "project2d_bwd": 180 * N,
        "tile_sort": 20 * n_isects, "isect_emit": 8 * n_isects + 16 * N,
        "loss_fwd": 60 * 3 * P, "loss_bwd": 72 * 3 * P, "adam": 28 * n_par,
    }
    if wl.args.sh_degree:  # rasterization()'s SH colours (csrc/sh.hip): K coefficient triples per Gaussian
        K = (wl.args.sh_degree + 1) ** 2
        per["sh_fwd"] = (12 + 12 * K + 4 + 12) * N  # means, coefficients, radii in; colours out
        per["sh_bwd"] = (12 + 12 * K + 4 + 12 + 12 * K + 12) * N  # + v_colours in; v_coeffs, v_means out
    out = {}
    for k, nbytes in per.items():
        if k in kernels:
            gbs = nbytes / (kernels[k]["avg_ms"] * 1e-3) / 1e9
            out[k] = {"bytes": nbytes, "GB/s": round(gbs, 1), "frac": round(gbs / HBM_PEAK_GBS, 3)}
    return out


def decode_mfma(wl, kernels):
    """MFMA utilisation of the fused anchor decode (csrc/decode.hip), forward and backward.

    Every MLP product runs on v_mfma_f32_16x16x4_f32 (2,048 FLOP, 32 SIMD-cycles each) on a
    16-anchor wave tile; the counts per wave tile follow the kernels' loops (K1 = 32 + view_dim
    inputs, KS = ceil(K1 / 4) k-steps, output tiles T = ceil(rows / 16) per head):
      forward  : hidden 2 KS per head x 3 + second layer 8 T per head (+ the count pass: the
                 opacity head again, 2 KS + 8);
      backward : per head launch (an RGB colour head in one chunk of <= 5 output tiles) hidden
                 2 KS + recomputed Y (8 x all T, opacity / cov) + dW2 8 nt + dH 8 nt + dW1 and
                 dX 8 ceil(K1 / 16) each; an SH colour head (T > 5) runs as one launch
                 (decode_bwd_color_kernel): hidden 2 KS + dW2 8 T + dH 32 ceil(T / 4) (64-row
                 chunks, padding rows included) + dW1 and dX as above.
    busy = MFMA FLOP / kernel time / 157.3 TFLOP/s (= the f32 MFMA peak at 64 FLOP/clk/SIMD),
    which is SQ_VALU_MFMA_BUSY_CYCLES / (SIMD count x kernel cycles) at the peak clock: the
    r02 PMC pass measured exactly 374 x 32 SIMD-cycles per wave tile for the RGB model."""
    av = getattr(wl, "last_av", None)
    if not av or not kernels:
        return None
    K1 = 32 + wl.view_dim
    KS = (K1 + 3) // 4
    kt = (K1 + 15) // 16
    T = [1, 5, (wl.color_dim * 10 + 15) // 16]  # opacity 10, cov 70, colour color_dim x 10 rows
    fwd = 3 * 2 * KS + 8 * sum(T) + (2 * KS + 8)
    bwd = 0
    col_one = NAT.lib().hgsr_decode_set_color_bwd(-1) != 0 and 5 < T[2] <= 20
    for h in range(3):
        if h == 2 and col_one:
            bwd += 2 * KS + 8 * T[2] + 32 * ((T[2] + 3) // 4) + 16 * kt
            continue
        chunks = [min(5, T[h] - t0) for t0 in range(0, T[h], 5)]
        for nt in chunks:
            bwd += 2 * KS + (8 * T[h] if h < 2 else 0) + 16 * nt + 16 * kt
    tiles = (av + 63) // 64 * 4
    out = {"visible_anchors": av, "mfma_per_wave_tile": {"decode_fwd+count": fwd, "decode_bwd": bwd}}
    for name, n in (("decode_bwd", bwd), ("decode_fwd", fwd)):
        key = name if name in kernels else None
        if key is None:
            continue
        t = kernels[key]["avg_ms"] * 1e-3
        if name == "decode_fwd" and "decode_count" in kernels:
            t += kernels["decode_count"]["avg_ms"] * 1e-3
        tf = tiles * n * 2048 / t / 1e12
        out[name] = {"tflops": round(tf, 2), "busy": round(tf / FP32_PEAK_TFLOPS, 4)}
    return out


def pmc_traffic(args):
    """HBM bytes per launch of each kernel from the newest committed PMC summary
    (profiles/rNN_pmc_traffic.json, written by scripts/profile_summary.py from separate
    rocprofv3 FETCH_SIZE / WRITE_SIZE passes of this bench on the default config,
    gfx950-corrected).  Counters cannot be read inside a timed run, so this is the
    profiled figure for the same command, or {} when no summary matches the config."""
    import glob
    files = sorted(glob.glob(os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles", "r*_pmc_traffic.json")))
    if not files or args.anchors or args.n != 2_000_000 or (args.width, args.height) != (1920, 1080):
        return {}, None
    d = json.load(open(files[-1]))
    out = {}
    for k, v in d["kernels"].get(f"{args.gs}gs", {}).items():
        base = k.split("_kernel")[0]
        if base not in out:
            out[base] = v["hbm_bytes_corrected"]
    return out, os.path.basename(files[-1]) + ": 2*FETCH_SIZE + WRITE_SIZE"


def psnr_quality(args):
    """The "PSNR delta vs ref" half of the metric, measured in this run: the HIP chain of the
    at-scale training-parity problem (tests/test_gpu_training_parity.py: 50k anchors, 480x270,
    500 iterations of the whole train step -- prefilter -> fused decode -> rasterization ->
    fused loss -> HIP Adam; reference train.py:150-277) from the fixture's unperturbed
    initialisation and from the same 1e-6-perturbed initialisations as the reference chain's
    ensemble, against the reference chain's committed results (tests/golden/psnr_scale_*.json;
    the CPU chain takes about an hour per run, scripts/psnr_at_scale.py).  The target render is
    the committed tests/golden/psnr_target_*.npz, so nothing under oracle/ runs here."""
    import statistics

    from scripts import psnr_at_scale as PS
    from tests import pipeline_fit as PF
    out = {}
    for gs, fixture in (("3d", "psnr_scale_3d"), ("2d", "psnr_scale_2d")):
        path = os.path.join(ROOT, "tests", "golden", f"{fixture}.json")
        if not os.path.exists(path) or not os.path.exists(PS.TARGET.format(gs=gs)):
            continue
        gold = json.load(open(path))
        gt, p0, cfg = PS.problem_from_fixture(gold["anchors"], gold["width"], gold["height"], gs)
        ens = {int(k): v for k, v in gold.get("ensemble", {"5": gold["ref_perturbed_1e-6"]}).items()}
        fit = lambda p: PF.fit(p, cfg, gt, gold["iterations"], gs=gs, device="cuda", window=gold["window"],  # noqa
                               lr_scale=gold["lr_scale"])
        t0 = time.perf_counter()
        fin, win, _ = fit(p0)
        hip = [win] + [fit(PS.perturbed(p0, s))[1] for s in sorted(ens)]
        ref = [gold["ref"]["window_db"]] + [ens[s]["window_db"] for s in sorted(ens)]
        full = len(ref) >= 8  # the test's MIN_ENSEMBLE: the delta is then the ensembles' mean difference
        out[f"{gs}gs"] = {
            "psnr_delta_db": round((statistics.mean(hip) - statistics.mean(ref)) if full else (win - gold["ref"]["window_db"]), 4),
            "psnr_delta_kind": "ensemble means" if full else "single draw", "single_draw_delta_db": round(win - gold["ref"]["window_db"], 4),
            "psnr_hip_db": round(win, 4),
            "psnr_ref_db": gold["ref"]["window_db"], "final_iterate_delta_db": round(fin - gold["ref"]["final_db"], 4),
            "ensemble_members": len(ref), "ensemble_mean_delta_db": round(statistics.mean(hip) - statistics.mean(ref), 4),
            "hip_sd_db": round(statistics.stdev(hip), 4), "ref_sd_db": round(statistics.stdev(ref), 4),
            "lr_scale": gold["lr_scale"], "iterations": gold["iterations"], "anchors": gold["anchors"],
            "width": gold["width"], "height": gold["height"], "seconds": round(time.perf_counter() - t0, 1)}
        torch.cuda.empty_cache()
    if not out:
        return None
    head = out.get("3dgs") or out["2dgs"]
    return dict({k: head[k] for k in ("psnr_delta_db", "psnr_delta_kind", "single_draw_delta_db", "psnr_hip_db", "psnr_ref_db",
                                      "ensemble_mean_delta_db")},
                source=("measured in this run: the HIP chain of tests/test_gpu_training_parity.py's at-scale problem "
                        "(window PSNR of the last 50 of 500 iterations), unperturbed and over the reference "
                        "ensemble's 1e-6-perturbation seeds, against the CPU reference chain's committed fixtures "
                        "tests/golden/psnr_scale_{3d,2d}.json (3DGS at 0.1x, 2DGS at 0.3x the fine-stage rates)"),
                **out)


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(args, wl):
    """The C oracle (OpenMP over pixel rows / Gaussians, oracle/hgsr_oracle.c) on one whole
    view of the same workload: projection, tile intersection + sort, raster fwd + bwd over
    every pixel, projection backward.  Threads: the OpenMP default (OMP_NUM_THREADS, else
    every host core)."""
    from oracle import oracle as O
    sc = wl.sc
    W, H = args.width, args.height
    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or os.cpu_count()
    t = {}
    t0 = time.perf_counter()
    r, m2, d, con = O.proj3d_fwd(sc.means.numpy(), sc.quats.numpy(), sc.scales.numpy(), sc.viewmats.numpy(),
                                 sc.Ks.numpy(), W, H)
    t["proj_fwd"] = time.perf_counter() - t0
    tw, th = O.tile_grid(W, H)
    t0 = time.perf_counter()
    tpg, ids, fl = O.isect_tiles(m2, r, d, 16, tw, th)
    offs = O.isect_offsets(ids, 1, tw, th)
    t["isect_sort"] = time.perf_counter() - t0
    cols = np.concatenate([sc.colors.numpy()[None], d[..., None]], -1).astype(np.float32)
    op = sc.opacities.numpy()[None].astype(np.float32)
    t0 = time.perf_counter()
    rc, ra, last = O.raster3d_fwd(m2, con, cols, op, None, W, H, 16, offs, fl)
    t["raster_fwd"] = time.perf_counter() - t0
    g = np.random.default_rng(0)
    vrc = (g.standard_normal(rc.shape) * 1e-6).astype(np.float32)
    vra = np.full(ra.shape, 1e-8, np.float32)
    t0 = time.perf_counter()
    vm2, vcon, vcol, vop = O.raster3d_bwd(m2, con, cols, op, None, W, H, 16, offs, fl, ra, last, vrc, vra)
    t["raster_bwd"] = time.perf_counter() - t0
    t0 = time.perf_counter()
    O.proj3d_bwd(sc.means.numpy(), sc.quats.numpy(), sc.scales.numpy(), sc.viewmats.numpy(), sc.Ks.numpy(), W, H,
                 r, con, vm2, vcol[..., -1].copy(), vcon)
    t["proj_bwd"] = time.perf_counter() - t0
    per_view = sum(t.values())
    return {
        "value": 1.0 / per_view, "unit": "views/s", "cores": threads, "kind": "port",
        "cpu_model": _cpu_model(), "host_cpu_count": os.cpu_count(),
        "sample": (f"one full view of the same workload through the C oracle (oracle/hgsr_oracle.c, OpenMP, "
                   f"{threads} threads): projection, tile intersection + sort (a counting pass over the tile bits, then per-tile sorts spread over the threads), raster fwd + bwd "
                   f"over all {W}x{H} pixels, projection backward, on all {args.n} Gaussians; measured "
                   f"{per_view:.1f}s (no loss head / optimizer: the rasterizer path only)"),
        "breakdown_s": {k: round(v, 3) for k, v in t.items()},
    }


def measure(args, rank, world, dev):
    """Warm up, time exactly args.steps steps (barrier + synchronize on both sides, max over
    ranks), then a per-kernel breakdown pass.  Returns the measurements of this workload."""
    wl = Workload(args, rank, dev, world)
    timing = not args.no_timing
    # live HIP events inside the timed region on the dominant kernel only (the roofline);
    # the per-kernel breakdown comes from a separate pass after it
    dominant = "raster3d_bwd" if args.gs == "3d" else "raster2d_bwd"
    if timing:  # event pool and pair counters created now, not between the warmup and the timed steps
        NAT.call("hgsr_timing_reset")
        NAT.call("hgsr_timing_only", dominant.encode())
        NAT.call("hgsr_timing_pairs", None, 1)  # the backward counts its visited / stepped pairs on the device
    # the objects of the scene setup (and of an earlier workload in this process) are collected
    # before the warmup: no generation-2 pass inside the timed steps, and no idle GPU between
    # the warmup and the timed steps (a collection there left the first timed steps ~10 % slower)
    gc.collect()
    # at N > 1 a progress line on stderr at most once a second (a slow but live run -- a first
    # RCCL collective's setup, gloo in a rehearsal -- is never silent long enough to look hung)
    last = [time.perf_counter()]

    def progress(what, i, n):
        if world > 1:
            now = time.perf_counter()
            if now - last[0] >= 1.0 or i + 1 == n:
                last[0] = now
                print(f"bench rank {rank}: {args.config} {what} step {i + 1}/{n}", file=sys.stderr, flush=True)

    for i in range(args.warmup):
        wl.step()
        progress("warmup", i, args.warmup)
    wl.flush()
    torch.cuda.synchronize(dev)
    # the optimizer moves the scene: intersections before / after the timed steps show the drift
    isects_before = wl.meta["flatten_ids"].numel() if args.warmup else None
    if timing:
        NAT.call("hgsr_timing_enable", 1)
    stats0, log0 = dict(G.isect_stats), len(wl.view_log)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    step_t = [] if os.environ.get("HGSR_BENCH_STEP_TIMES") else None  # (diagnostic: host time per step)
    seg0 = torch.cuda.memory_stats(dev).get("segment.all.allocated") if step_t is not None else None
    for i in range(args.steps):
        wl.step()
        progress("timed", i, args.steps)
        if step_t is not None:
            step_t.append(time.perf_counter())
    wl.flush()  # the last step's deferred all-gather is part of the timed work
    torch.cuda.synchronize(dev)
    if step_t is not None:
        ms = torch.cuda.memory_stats(dev)
        print("step ms:", " ".join(f"{(b - a) * 1e3:.2f}" for a, b in zip([t0] + step_t[:-1], step_t)),
              "| segments allocated", ms.get("segment.all.allocated"), "- before", seg0,
              "| alloc retries", ms.get("num_alloc_retries"), "| gc counts", gc.get_count(), file=sys.stderr)
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    if timing:
        NAT.call("hgsr_timing_enable", 0)
    if world > 1:
        tt = torch.tensor([dt], device=dev, dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
    timed = wl.view_log[log0:]
    res = {"wl": wl, "dt": dt, "kernels": {}, "live": None, "isects_before": isects_before,
           "isects_after": wl.meta["flatten_ids"].numel(), "dominant": dominant,
           "isects_timed": [n for _, n in timed], "views_timed": [v for v, _ in timed],
           "isect_stats": {k: G.isect_stats[k] - stats0[k] for k in stats0}}
    if timing:
        pc, ec = ct.c_ulonglong(0), ct.c_ulonglong(0)
        NAT.call("hgsr_timing_exec_pairs", ct.byref(ec))
        NAT.call("hgsr_timing_pairs", ct.byref(pc), 1)
        res["pairs_timed"], res["exec_pairs_timed"] = pc.value, ec.value
        tot, cnt = NAT.kernel_time(dominant)
        res["live"] = {"avg_ms": round(tot / cnt, 4), "launches": cnt} if cnt else None
        # breakdown pass (outside the timed region): every kernel's events
        NAT.call("hgsr_timing_reset")
        NAT.call("hgsr_timing_only", None)
        NAT.call("hgsr_timing_enable", 1)
        log1 = len(wl.view_log)
        for _ in range(min(args.steps, 10)):
            wl.step()
        wl.flush()
        torch.cuda.synchronize(dev)
        NAT.call("hgsr_timing_enable", 0)
        res["isects_breakdown"] = float(np.mean([n for _, n in wl.view_log[log1:]]))
        for k in KERNELS:
            tot, cnt = NAT.kernel_time(k)
            if cnt:
                res["kernels"][k] = {"avg_ms": round(tot / cnt, 4), "launches": cnt}
    return res


def roofline(args, res):
    """Dominant-kernel roofline: the raster backward is bound by fp32 work on
    (pixel, Gaussian) pairs, so achieved = pairs_evaluated x FLOP per pair / kernel time
    against the fp32 peak (vector = f32 MFMA rate, 157.3 TF).  pairs_evaluated = the
    lane-pairs the kernel actually stepped (every entry of each wave's compacted per-quadrant
    list x 64 lanes), counted on the device over exactly the timed launches.  gsplat's visit
    count (every Gaussian up to each tile's latest contributor x 256 pixels, which includes
    pairs the quadrant culling never evaluates) is kept beside it as a note only."""
    live = res["live"]
    if not live:
        return None
    dom, wl = res["dominant"], res["wl"]
    traffic, traffic_src = pmc_traffic(args)
    n_isects = float(np.mean(res["isects_timed"]))  # mean over the timed steps (the views differ)
    pairs = res["pairs_timed"] // args.steps  # mean over exactly the launches the events time
    epairs = res["exec_pairs_timed"] // args.steps
    avg_s = live["avg_ms"] * 1e-3
    fpp = FLOP_PER_PAIR[dom]
    ach = pairs * fpp / avg_s / 1e12
    ach_x = epairs * fpp / avg_s / 1e12
    roof = {"bound": "valu", "achieved": round(ach_x, 3), "peak": FP32_PEAK_TFLOPS, "unit": "TFLOP/s",
            "frac": round(ach_x / FP32_PEAK_TFLOPS, 4), "traffic": traffic.get(dom), "kernel": dom,
            "pairs_evaluated_per_launch": epairs, "flop_per_pair": fpp,
            "gsplat_visited_pairs_per_launch": pairs, "frac_on_gsplat_visited_pairs": round(ach / FP32_PEAK_TFLOPS, 4),
            "note": (f"fp32-bound compositing (far below the HBM roof): peak = the fp32 rate (vector = f32 MFMA); "
                     f"achieved = {epairs} (pixel, Gaussian) pairs evaluated per launch (each wave's compacted "
                     f"per-quadrant list x 64 lanes, counted on the device over the timed launches) x {fpp:.0f} "
                     f"FLOP/pair (SURVEY 8(d)) / kernel time; frac_on_gsplat_visited_pairs prices gsplat's visit "
                     f"count ({pairs}: every Gaussian up to each tile's latest contributor x 256 pixels, pairs the "
                     f"culling skips included) -- a note, not the roofline; {n_isects:.0f} intersections per view "
                     f"(mean over the timed steps); limiter "
                     f"counters in {_newest_profile('*_pmc_raster*limiters*.txt')}")}
    # aggregate compulsory-bytes figure of SURVEY 8(d): B_step = 384 N + 132 I + 52 P
    b_step = 384 * wl.last_colors.shape[0] + 132 * n_isects + 52 * args.width * args.height
    if roof.get("traffic") is not None:
        roof["traffic_unit"] = "bytes/launch"
        roof["traffic_source"] = traffic_src
    roof["aggregate_hbm_frac"] = round(b_step / (res["dt"] / args.steps) / (HBM_PEAK_GBS * 1e9), 4)
    roof["n_isects"] = round(n_isects)
    roof["n_isects_before_timed"] = res["isects_before"]
    roof["kernel_avg_ms"] = live["avg_ms"]
    roof["timing"] = ("HIP events (no system fence) on the kernel's stream, recorded inside the timed region "
                      "for this kernel only")
    return roof


def camera_summary(args, res):
    """The views of the timed steps: how many cameras the set cycles, their intersection counts
    and the deferred-count outcome of every timed view (gsplat_api.isect_stats: deferred = the
    count was read after the forward was queued; redo = the view overflowed the capacity and was
    re-emitted at the exact size; sync = no history for the camera grid yet)."""
    n = res["isects_timed"]
    out = {"views_in_set": args.cameras, "views_timed": len(set(res["views_timed"])),
           "n_isects_mean": round(float(np.mean(n))), "n_isects_min": int(min(n)), "n_isects_max": int(max(n)),
           "isect_counts_timed": res["isect_stats"]}
    if args.cameras > 1:
        out["note"] = ("synthetic.camera_set: view 0 = the scene's identity camera (its most intersections), the "
                       "others on a ring (yaw +-25 deg, elevation +-15 deg, 0.5-1.5x its distance); view (step * "
                       "world + rank) mod V per step (reference train.py:133-148 picks a camera per iteration)")
    return out


def workload_name(args):
    anchors = (f"LoD mask + anchor prefilter + fused anchor decode ({args.anchors} anchors, view_dim {args.view_dim}, "
               + ("RGB" if args.sh_degree is None else f"SH{args.sh_degree} colour head") + ") + ")
    cams = (f"a {args.cameras}-view camera set cycled per step" if args.cameras > 1 else "one fixed camera")
    return (f"{args.config} {'3DGS' if args.gs == '3d' else '2DGS'} train step on {cams}: "
            + (f"SH{args.sh_degree} colours + " if args.sh_degree is not None and not args.anchors else "")
            + (anchors if args.anchors else "")
            + "rasterization fwd" + (f" (SH degree {args.sh_degree})" if args.sh_degree is not None else "")
            + " + reference loss (L1 + D-SSIM + alpha/scale regs"
            + (" + normal consistency" if args.gs == "2d" else "") + ") + bwd"
            + (" + training_statis" if args.anchors else "") + " + Adam step, RGB+ED")


def parallelism(args, world):
    if args.mode == "chunk":
        return (f"per-chunk: one chunk (seed = rank) per GPU, no collectives (x{world})" if world > 1
                else "single GPU (per-chunk mapping)")
    if world == 1:
        return "single GPU (DDP mapping, no collective at N=1)"
    if args.anchors:
        return (f"DDP over views (x{world}): one scene, a camera per rank, bucketed RCCL all-reduce of every "
                f"gradient launched from backward hooks, per-bucket Adam")
    return (f"DDP over views (x{world}): one scene, a camera per rank, sharded optimizer (ZeRO-1): bucketed RCCL "
            f"reduce-scatter launched from backward hooks, Adam on each rank's 1/{world}, all-gather of the "
            f"updated parameters")


def secondary_names(args, world):
    names = ["c2-chunks", "c4", "c5"] if world > 1 else ["c2-fixed", "c2-anchors", "c3", "c4", "c5"]
    return [n for n in names if n != args.config]


def secondary(args, rank, world, dev):
    """The other BASELINE configs through the same step (each rank runs its part; rank 0
    returns the lines), measured after the headline workload is freed."""
    out = []
    for name in secondary_names(args, world):
        # 16 timed steps = one full cycle of the camera set (10 covered views 3-12 only: a biased mean)
        a = parse(["--config", name, "--steps", str(min(args.steps, 16)), "--warmup", str(min(args.warmup, 3)),
                   "--width", str(args.width), "--height", str(args.height)] + (["--no-timing"] if args.no_timing else []))
        a = resolve(a, world)
        r = measure(a, rank, world, dev)
        if rank == 0:
            roof = roofline(a, r)
            out.append({"config": name, "label": CONFIGS[name]["label"], "workload": workload_name(a),
                        "parallelism": parallelism(a, world), "n_gpus": world,
                        "value": round(world * a.steps / r["dt"], 3), "unit": "views/s",
                        "ms_per_step": round(r["dt"] / a.steps * 1e3, 3), "steps": a.steps, "warmup": a.warmup,
                        "gaussians": int(r["wl"].last_colors.shape[0]), "cameras": camera_summary(a, r),
                        "roofline": None if roof is None else dict(
                            {k: roof[k] for k in ("bound", "kernel", "achieved", "frac", "kernel_avg_ms",
                                                  "pairs_evaluated_per_launch", "gsplat_visited_pairs_per_launch",
                                                  "frac_on_gsplat_visited_pairs")},
                            note=("frac prices the (pixel, Gaussian) pairs the kernel evaluated; the gsplat-visited "
                                  "figure (pairs the per-quadrant culling skips included) is a note only")),
                        "decode_mfma": decode_mfma(r["wl"], r["kernels"]) if a.anchors else None,
                        "kernels": r["kernels"]})
        r["wl"].close()
        del r
        torch.cuda.empty_cache()
    return out


def main():
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    args = resolve(parse(), world)
    # HGSR_BENCH_SHARE_GPU=1 (rehearsal only): the ranks share the visible GPUs round-robin and the
    # collectives go over gloo on device tensors -- the N > 1 code paths on a one-GPU box.  The
    # measured lines are RCCL with one GPU per rank.
    share = os.environ.get("HGSR_BENCH_SHARE_GPU", "0") != "0"
    if share:
        local = local % max(1, torch.cuda.device_count())
    if world > 1 or (os.environ.get("HGSR_DDP_FORCE", "0") != "0" and "WORLD_SIZE" in os.environ):
        torch.cuda.set_device(local)
        if share:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    res = measure(args, rank, world, dev)
    wl, dt = res["wl"], res["dt"]
    roof = roofline(args, res) if rank == 0 else None
    cpu = None
    if (rank == 0 and world == 1 and not args.no_cpu_baseline and args.config == "c2" and args.gs == "3d"
            and args.sh_degree is None and not args.anchors):
        cpu = cpu_baseline(args, wl)
    line = None
    if rank == 0:
        ms = dt / args.steps * 1e3
        line = {
            "metric": METRIC if not args.freeze else "DIAGNOSTIC (--freeze: no optimizer step) " + METRIC,
            "value": round(world * args.steps / dt, 3), "unit": "views/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "fp32",
            "data": "synthetic (seeded scenes of SURVEY 8(d); no dataset in the environment)",
            "config": {"workload": workload_name(args), "config": args.config, "label": CONFIGS[args.config]["label"],
                       "gaussians": int(wl.last_colors.shape[0]), "width": args.width, "height": args.height,
                       "parallelism": parallelism(args, world), "cameras": camera_summary(args, res)},
            "roofline": roof, "cpu_baseline": cpu, "quality": None, "kernels": res["kernels"],
            "kernels_source": "HIP events of every kernel over a separate pass after the timed region",
            "hbm_kernels": hbm_kernels(wl, res["kernels"], res.get("isects_breakdown")),
        }
    wl.close()
    del res, wl
    torch.cuda.empty_cache()
    if not args.no_secondary:
        sec = secondary(args, rank, world, dev)
        if rank == 0:
            line["secondary"] = sec
    if rank == 0 and world == 1 and not args.no_quality:
        line["quality"] = psnr_quality(args)
    if rank == 0:
        print(json.dumps(line))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
