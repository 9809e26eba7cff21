"""GPU parity of K13 (normals from the rendered depth, the 2DGS normal-consistency input) and
of the camera -> world rotation of render_normals, against the torch restatement of the
gsplat fork's depth_to_normal (oracle/torch_ref.py) run on the CPU in f32 and f64.
The central differences of unprojected neighbours cancel to ~1e-3 of the points, so the
check is conditioning-aware (oracle/checks.cond_close): the HIP result (which never adds the
camera origin) must sit within the f32 torch result's own error of the f64 answer."""
import numpy as np
import pytest
import torch

from oracle import torch_ref as TR
from oracle.checks import cond_close

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")


def _cams(C, W, H, seed):
    g = torch.Generator().manual_seed(seed)
    c2w = torch.zeros(C, 4, 4)
    for c in range(C):
        q = torch.nn.functional.normalize(torch.randn(4, generator=g), dim=0)
        w, x, y, z = q.tolist()
        c2w[c, :3, :3] = torch.tensor([[1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y)],
                                       [2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x)],
                                       [2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)]])
        c2w[c, :3, 3] = torch.randn(3, generator=g) * 3.0
        c2w[c, 3, 3] = 1.0
    f = 0.5 * W / np.tan(np.radians(30))
    Ks = torch.tensor([[f, 0, W / 2], [0, f, H / 2], [0, 0, 1]], dtype=torch.float32).repeat(C, 1, 1)
    return c2w, Ks


def _depth(C, H, W, seed):
    g = torch.Generator().manual_seed(seed)
    yy, xx = torch.meshgrid(torch.linspace(0, 1, H), torch.linspace(0, 1, W), indexing="ij")
    base = 3.0 + 1.5 * torch.sin(4 * xx) * torch.cos(3 * yy)
    return (base[None] + 0.05 * torch.randn(C, H, W, generator=g))[..., None].float()


@pytest.mark.parametrize("C,H,W,z_depth", [(1, 48, 64, True), (2, 37, 53, True), (1, 40, 40, False),
                                           (1, 1080, 1920, True)])  # c3's size (1080p)
def test_depth_to_normal_fwd_bwd(C, H, W, z_depth):
    from horizongs_amd import gsplat_api as G
    c2w, Ks = _cams(C, W, H, seed=C * 100 + H)
    depth = _depth(C, H, W, seed=W)
    gup = torch.randn(C, H, W, 3, generator=torch.Generator().manual_seed(7))

    # f64, then correct f32-level samples: the fork's f32 order, the kernel's (no camera origin),
    # f64 runs with +-u jittered points
    n64, g64, S = TR.k13_error_samples(depth, c2w, Ks, gup, z_depth=z_depth)
    n32, g32 = S[0]
    d = depth.to(DEV).requires_grad_(True)
    n = G.depth_to_normal(d, c2w.to(DEV), Ks.to(DEV), z_depth=z_depth)
    (n * gup.to(DEV)).sum().backward()
    # [C,H,W,*]: conditioning is shared with the differenced neighbours (axes 1, 2)
    cond_close(n.detach().cpu().numpy(), n32, n64, "normals_from_depth", dilate_axes=(1, 2),
               alt32=[x[0] for x in S[1:]])
    cond_close(d.grad.cpu().numpy(), g32, g64, "v_depth", dilate_axes=(1, 2), dilate=5, alt32=[x[1] for x in S[1:]])


def test_depth_to_normal_strided_render_channel():
    """the expected-depth channel of a channels-last render, read in place"""
    from horizongs_amd import gsplat_api as G
    C, H, W = 1, 33, 41
    c2w, Ks = _cams(C, W, H, seed=3)
    rc = torch.rand(C, H, W, 4) + 2.0
    rd = rc.to(DEV).requires_grad_(True)
    n = G.depth_to_normal(rd[..., -1:], c2w.to(DEV), Ks.to(DEV))
    n.sum().backward()
    r = rc.clone().requires_grad_(True)
    nr = TR.depth_to_normal(r[..., -1:], c2w, Ks)
    nr.sum().backward()
    r64 = rc.double().requires_grad_(True)
    n64 = TR.depth_to_normal(r64[..., -1:], c2w.double(), Ks.double())
    n64.sum().backward()
    cond_close(n.detach().cpu().numpy(), nr.detach().numpy(), n64.detach().numpy(), "strided normals",
               dilate_axes=(1, 2))
    cond_close(rd.grad.cpu().numpy(), r.grad.numpy(), r64.grad.numpy(), "strided v_render", dilate_axes=(1, 2))
    assert float(rd.grad[..., :3].abs().max()) == 0.0


def test_rotate3_matches_einsum():
    from horizongs_amd import gsplat_api as G
    C, H, W = 2, 17, 23
    c2w, _ = _cams(C, W, H, seed=9)
    R = c2w[:, :3, :3].contiguous()
    v = torch.randn(C, H, W, 3)
    g = torch.randn(C, H, W, 3)
    vd = v.to(DEV).requires_grad_(True)
    out = G._Rotate3.apply(R.to(DEV), vd)
    (out * g.to(DEV)).sum().backward()
    vr = v.double().requires_grad_(True)
    ref = torch.einsum("cij,chwj->chwi", R.double(), vr)
    (ref * g.double()).sum().backward()
    np.testing.assert_allclose(out.detach().cpu().numpy(), ref.detach().numpy(), rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(vd.grad.cpu().numpy(), vr.grad.numpy(), rtol=1e-5, atol=1e-6)


def test_rotate3_viewmat_transpose_and_depth_normal_from_viewmat():
    """rasterization_2dgs passes world -> camera viewmats [C,4,4]: R^T applied in place."""
    from horizongs_amd import gsplat_api as G
    C, H, W = 2, 19, 29
    c2w, Ks = _cams(C, W, H, seed=13)
    vm = torch.linalg.inv(c2w.double()).float()
    v = torch.randn(C, H, W, 3)
    vd = v.to(DEV).requires_grad_(True)
    out = G._Rotate3.apply(vm.to(DEV), vd, True)
    g = torch.randn(C, H, W, 3)
    (out * g.to(DEV)).sum().backward()
    ref = torch.einsum("cij,chwj->chwi", c2w[:, :3, :3].double(), v.double())
    np.testing.assert_allclose(out.detach().cpu().numpy(), ref.numpy(), rtol=1e-5, atol=1e-5)
    gref = torch.einsum("cji,chwj->chwi", c2w[:, :3, :3].double(), g.double())
    np.testing.assert_allclose(vd.grad.cpu().numpy(), gref.numpy(), rtol=1e-5, atol=1e-5)
    depth = _depth(C, H, W, seed=5).to(DEV)
    n_c2w = G.depth_to_normal(depth, c2w.to(DEV), Ks.to(DEV))
    n_vm = G._DepthToNormal.apply(depth, vm.to(DEV), Ks.to(DEV), True, True)
    np.testing.assert_allclose(n_vm.cpu().numpy(), n_c2w.cpu().numpy(), rtol=1e-4, atol=2e-5)
