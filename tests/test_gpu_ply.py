"""GPU: explicit-PLY export through the fused decode (scene/lod_model.py:681-771 save_explicit)
against the oracle decode restatement, then re-loaded."""
import numpy as np
import pytest
import torch

from oracle import decode_ref as D
from oracle.checks import close

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")


def test_export_explicit_matches_decode(tmp_path):
    from horizongs_amd import ply as P
    g = torch.Generator().manual_seed(9)
    A, k, F, cd = 3000, 10, 32, 27
    anchor = torch.randn(A, 3, generator=g) * 5
    feat = torch.randn(A, F, generator=g) * 0.3
    offset = torch.randn(A, k, 3, generator=g) * 0.1
    scaling = np.log(0.01) + torch.randn(A, 6, generator=g) * 0.1
    level = torch.randint(0, 6, (A, 1), generator=g).float()
    extra = torch.randn(A, generator=g) * 0.2
    mlps = {}
    for h, O in (("opacity", k), ("cov", 7 * k), ("color", cd * k)):
        mlps[f"{h}_w1"] = torch.randn(F, F, generator=g) / np.sqrt(F)
        mlps[f"{h}_b1"] = torch.randn(F, generator=g) * 0.1
        mlps[f"{h}_w2"] = torch.randn(O, F, generator=g) / np.sqrt(F)
        mlps[f"{h}_b2"] = torch.randn(O, generator=g) * 0.1
    f = tmp_path / "point_cloud_explicit.ply"
    dv = lambda t: t.to(DEV)
    n = P.export_explicit(f, dv(anchor), dv(level), dv(extra), dv(feat), dv(offset), dv(scaling.float()),
                          {kk: dv(v) for kk, v in mlps.items()}, k, cd, 26.686, 1, 8)
    ref = D.decode_torch(anchor.double(), feat.double(), offset.double(), scaling.double(), torch.zeros(3).double(),
                         {kk: v.double() for kk, v in mlps.items()}, 0, k, cd)
    xyz, _, color, opac, sc, rot, mask = ref
    assert n == int(mask.sum())
    d = P.load_explicit_ply(f, device="cpu")
    close(d["xyz"].numpy(), xyz.numpy(), name="xyz")
    close(d["opacity"].numpy(), opac.numpy(), name="opacity")
    close(d["scaling"].numpy(), sc.numpy(), name="scaling")
    close(d["rotation"].numpy(), rot.numpy(), name="rot")
    close(d["features_dc"].numpy(), color[:, :1].numpy(), name="f_dc")
    close(d["features_rest"].numpy(), color[:, 1:].numpy(), name="f_rest")
    np.testing.assert_array_equal(d["level"].numpy()[:, 0], level.repeat_interleave(k, 0)[mask, 0].int().numpy())
    np.testing.assert_array_equal(d["extra_level"].numpy(), extra.repeat_interleave(k)[mask].numpy())
