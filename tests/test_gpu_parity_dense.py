"""GPU parity at the tile depths the c2 / c3 workloads actually run.

The toy scenes of test_gpu_parity.py hold <= 93 Gaussians per tile, so they never leave
the first batch of the raster kernels (kFwdBatch = 256, kBwdBatch = 128 in
csrc/raster3d.hip; the same batches in csrc/raster2d.hip).  These tests drive, against the
C oracle (f32 checker + f64 truth, per-element conditioning of oracle/checks.py):

  * dense scenes with >= 1024 Gaussians per tile and a large share of saturated pixels:
    the 2-deep prefetch, the double-buffered staging, the batch-to-batch combine of the
    backward, the `t0 = batch_end - wave_final` trimming, the workgroup early-out vote and
    the exclusive T <= 1e-4 stop;
  * the full c2 scene (2M Gaussians, 1920x1080, ~1,070 intersections per tile) through
    gsplat.rasterization, every image and gradient, and the full c3 2DGS frame (with K13,
    the normals from its expected depth, at 1920x1080).

Each test asserts the depth statistics of its own scene, so it cannot silently become
sparse.  Pixels where the oracle took a discrete decision (alpha vs 1/255, the 0.999 clamp,
the T <= 1e-4 stop, the 2DGS surface / low-pass branch) within a few ulps of its threshold
are reported, bounded in number (oracle/checks.MAX_AMBIGUOUS) and excluded from the value
bar, and carry no upstream gradient: any other correct f32 evaluation order (gsplat itself
evaluates __expf) can take the other branch there.  Reference call site: gaussian_renderer/render.py:40-76.
"""
import numpy as np
import pytest
import torch

from horizongs_amd.synthetic import c2, make_scene
from tests.raster_parity import run_2dgs, run_3dgs

pytestmark = pytest.mark.gpu


def _dense_scene(n=20000, W=128, H=96, seed=5, scale_range=(0.03, 0.18), C=1, opacity_range=(0.02, 0.5)):
    """~1 Gaussian per pixel at c2's on-screen footprint (1,600-2,300 per 16x16 tile); low
    opacities keep the replay deep (>= 1,024) while a large share of pixels still stops."""
    sc = make_scene(n, W, H, seed=seed, scale_range=scale_range, opacity_range=opacity_range)
    if C > 1:
        vms = [sc.viewmats[0]]
        for c in range(1, C):
            th = 0.03 * c
            vm = torch.eye(4)
            vm[:3, :3] = torch.tensor([[np.cos(th), 0, np.sin(th)], [0, 1, 0], [-np.sin(th), 0, np.cos(th)]],
                                      dtype=torch.float32)
            vm[:3, 3] = torch.tensor([0.05 * c, -0.02 * c, 0.1])
            vms.append(vm)
        sc.viewmats = torch.stack(vms)
        sc.Ks = sc.Ks.expand(C, 3, 3).contiguous()
    return sc


@pytest.mark.parametrize("mode", ["RGB+ED", "RGB"])
def test_dense_3dgs_multibatch(mode):
    sc = _dense_scene()
    bg = torch.tensor([[0.1, 0.3, 0.2]])
    (max_tile, replay, sat), _, _ = run_3dgs(sc, mode, bg, count_pairs=True)
    assert max_tile >= 1024, max_tile          # >= 4 forward batches of 256
    assert replay >= 1024, replay              # >= 8 backward batches of 128
    assert sat >= 0.10, sat                    # exclusive T <= 1e-4 stop exercised


def test_dense_3dgs_two_cameras_no_background():
    sc = _dense_scene(C=2, seed=6)
    (max_tile, replay, sat), _, _ = run_3dgs(sc, "RGB+ED", None, seed=1)
    assert max_tile >= 1024 and replay >= 1024 and sat >= 0.10, (max_tile, replay, sat)


@pytest.mark.slow
def test_c2_fullsize_3dgs_vs_oracle():
    """The north-star scene itself: 2M Gaussians, 1920x1080, RGB+ED with a background,
    every output and gradient vs the oracle (about 1,070 intersections per tile)."""
    sc = c2()
    bg = torch.tensor([[0.2, 0.1, 0.3]])
    # count_pairs: bench.py's roofline numerator (the executed-pair counter) pinned at c2
    (max_tile, replay, sat), _, _ = run_3dgs(sc, "RGB+ED", bg, seed=2, count_pairs=True)
    assert max_tile >= 1024 and replay >= 1024 and sat >= 0.10, (max_tile, replay, sat)


def test_dense_2dgs_multibatch():
    sc = _dense_scene(n=24000, seed=7, opacity_range=(0.05, 0.6))
    bg = torch.tensor([[0.2, 0.1, 0.4]])
    (max_tile, replay, sat), _, _ = run_2dgs(sc, "RGB+ED", bg, seed=3)
    assert max_tile >= 1024 and replay >= 1024 and sat >= 0.10, (max_tile, replay, sat)


@pytest.mark.slow
def test_c3_fullsize_2dgs_vs_oracle():
    """c3 (the c2 inputs through rasterization_2dgs), the whole 1920x1080 frame: every image
    and gradient vs the oracle, then K13 -- render_normals_from_depth, the normal-consistency
    input of reference train.py:180-188, computed inside rasterization_2dgs
    (gaussian_renderer/render.py:62-76) -- on this frame's own expected depth against the torch
    restatement of the fork's depth_to_normal in f32 / f64, forward and backward."""
    from horizongs_amd import gsplat_api as G
    from oracle import torch_ref as TR
    from oracle.checks import cond_close
    from tests import parity_report as PR
    sc = c2()
    bg = torch.tensor([[0.2, 0.1, 0.3]])
    (max_tile, replay, sat), _, res = run_2dgs(sc, "RGB+ED", bg, seed=4)
    assert max_tile >= 1024 and replay >= 1024 and sat >= 0.10, (max_tile, replay, sat)
    assert res["r32"].Hr == 1080
    # K13 at full size on the GPU's expected-depth channel (viewmat = I: camera = world frame)
    depth = res["out"].detach()[..., 3:].contiguous()
    c2w = torch.eye(4)[None]
    Ks = sc.Ks
    gup = torch.randn(1, 1080, 1920, 3, generator=torch.Generator().manual_seed(11))
    # f64, then correct f32-level samples: the fork's f32 order, the kernel's (no camera origin),
    # f64 runs with +-u jittered points (oracle/torch_ref.k13_error_samples)
    n64, g64, S = TR.k13_error_samples(depth, c2w, Ks, gup)
    nfd = res["nfd"].detach().cpu().numpy()
    cond_close(nfd, S[0][0], n64, "normals_from_depth (c3 frame)", dilate_axes=(1, 2), alt32=[x[0] for x in S[1:]])
    PR.tensor("normals_from_depth", nfd, S[0][0], S[1][0], n64)
    dg = depth.clone().requires_grad_(True)
    n = G.depth_to_normal(dg, c2w.to(depth.device), Ks.to(depth.device))
    (n * gup.to(depth.device)).sum().backward()
    np.testing.assert_array_equal(n.detach().cpu().numpy(), nfd)  # the same kernel rasterization_2dgs ran
    vd = dg.grad.cpu().numpy()
    cond_close(vd, S[0][1], g64, "v_depth of K13 (c3 frame)", dilate_axes=(1, 2), dilate=5, alt32=[x[1] for x in S[1:]])
    PR.tensor("v_depth(K13)", vd, S[0][1], S[1][1], g64)
