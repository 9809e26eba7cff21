"""The deferred intersection count of rasterization() / rasterization_2dgs().

gsplat reads the intersection count on the host between the count pass and the emission
(reference call: gaussian_renderer/render.py:40-76).  gsplat_api instead enqueues the
emission, the per-tile sort and the raster forward into buffers sized from the largest count
of the last views of the same camera grid, and reads the count afterwards.  These tests check that this is
invisible: intersection arrays bit-identical to the synchronous order, renders bit-identical,
gradients equal up to the backward's float-atomic order, and both overflow kinds (more keys
than the capacity, a bin larger than the sort class launched) redone at the exact size."""
import collections

import numpy as np
import pytest
import torch

from horizongs_amd import gsplat_api as G
from horizongs_amd.synthetic import make_scene

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


def _scene(n, W, H, seed):
    return make_scene(n, W, H, seed=seed, scale_range=(0.01, 0.06), depth_range=(2.0, 6.0),
                      opacity_range=(0.2, 0.95))


def _run(sc, gs):
    means, quats, scales, opac, cols, vm, K = (t.to(DEV).contiguous() for t in (
        sc.means, sc.quats, sc.scales, sc.opacities, sc.colors, sc.viewmats, sc.Ks))
    for t in (means, quats, scales, opac, cols):
        t.requires_grad_(True)
    bg = torch.zeros(1, 3, device=DEV)
    if gs == "3d":
        out, alpha, meta = G.rasterization(means, quats, scales, opac, cols, vm, K, sc.width, sc.height,
                                           packed=False, backgrounds=bg, render_mode="RGB+ED")
        imgs = [out, alpha]
    else:
        (out, alpha, nrm, nfd, dist, med), meta = G.rasterization_2dgs(
            means, quats, scales, opac, cols, vm, K, sc.width, sc.height, packed=False, backgrounds=bg,
            render_mode="RGB+ED")
        imgs = [out, alpha, nrm, nfd, dist, med]
    meta["means2d"].retain_grad()
    g = torch.Generator().manual_seed(7)
    loss = sum((im * torch.randn(im.shape, generator=g).to(DEV)).sum() for im in imgs[:4] if im.requires_grad)
    loss.backward()
    torch.cuda.synchronize()
    flat = meta["flatten_ids"]
    deferred = flat.untyped_storage().nbytes() > flat.numel() * 4  # a view of a capacity buffer
    arrays = {k: meta[k].cpu().numpy() for k in ("isect_ids", "flatten_ids", "isect_offsets", "tiles_per_gauss",
                                                  "radii")}
    return ([im.detach().cpu().numpy() for im in imgs], arrays,
            [t.grad.cpu().numpy() for t in (means, quats, scales, opac, cols)] + [meta["means2d"].grad.cpu().numpy()],
            deferred)


def _key(sc):
    return (torch.device(DEV).index or 0, 1, (sc.width + 15) // 16, (sc.height + 15) // 16)


@pytest.mark.parametrize("gs", ["3d", "2d"])
def test_deferred_count_matches_synchronous(gs, monkeypatch):
    sc = _scene(30000, 256, 192, seed=11)
    G._pred.pop(_key(sc), None)  # no prediction for the grid: the synchronous order
    ref_imgs, ref_arr, ref_grads, ref_def = _run(sc, gs)
    assert not ref_def and ref_arr["isect_ids"].size > 50000
    n = ref_arr["isect_ids"].size
    capacity = G._capacity
    mb = int(np.diff(np.append(ref_arr["isect_offsets"].reshape(-1), n)).max())
    cases = {
        # the capacity predicted from this very view: the deferred path proper
        "deferred": lambda: _predict(sc, (n, mb)),
        # predicted from a smaller view: more keys than the capacity -> redone synchronously
        # (capacities come in 256K-key grains, above this scene's count: the headroom is patched)
        "overflow_keys": lambda: (_predict(sc, (n // 4, mb)),
                                  monkeypatch.setattr(G, "_capacity", lambda a, b: (a + 1024, capacity(a, b)[1]))),
        # a bin over the predicted sort class (capacity 16 keys per bin) -> redone
        "overflow_bin": lambda: (_predict(sc, (n, mb)),
                                 monkeypatch.setattr(G, "_capacity", lambda a, b: (n + 1024, 16))),
    }
    for name, setup in cases.items():
        setup()
        redo0 = G.isect_stats["redo"]
        imgs, arr, grads, deferred = _run(sc, gs)
        assert deferred == (name == "deferred"), name
        assert G.isect_stats["redo"] - redo0 == int(name != "deferred"), name  # counted
        assert G._pred[_key(sc)][-1] == (n, mb), name  # the count of this view joins the history
        for k in ref_arr:
            np.testing.assert_array_equal(arr[k], ref_arr[k], err_msg=f"{name}: {k}")
        for i, (a, b) in enumerate(zip(imgs, ref_imgs)):
            np.testing.assert_array_equal(a, b, err_msg=f"{name}: image {i}")  # the forward is atomic-free
        for i, (a, b) in enumerate(zip(grads, ref_grads)):
            # the backward's float atomics sum in a run-dependent order: near-cancelled entries
            # are judged against the tensor's scale
            np.testing.assert_allclose(a, b, rtol=1e-4, atol=1e-5 * float(np.abs(b).max()),
                                       err_msg=f"{name}: grad {i}")
        monkeypatch.setattr(G, "_capacity", capacity)


def _predict(sc, nm):
    G._pred[_key(sc)] = collections.deque([nm], maxlen=G._PRED_VIEWS)


def test_deferred_count_first_view_and_empty():
    """No prediction for a camera grid -> synchronous; a view with no intersection after a
    predicted one composites nothing."""
    sc = _scene(2000, 208, 176, seed=3)  # a grid size no other test uses
    G._pred.pop(_key(sc), None)
    _, arr0, _, d0 = _run(sc, "3d")
    assert not d0 and arr0["isect_ids"].size > 0
    _, arr1, _, d1 = _run(sc, "3d")
    assert d1
    for k in arr0:
        np.testing.assert_array_equal(arr1[k], arr0[k])
    empty = _scene(2000, 208, 176, seed=3)
    empty.means[:, 2] = -5.0  # every Gaussian behind the camera
    imgs, arr, grads, d2 = _run(empty, "3d")
    assert d2 and arr["isect_ids"].size == 0
    assert np.all(imgs[1] == 0) and all(np.all(g == 0) for g in grads[:5])


def test_deferred_capacity_covers_a_camera_cycle():
    """A training loop cycles cameras (train.py:133-148): the capacity is the largest count of
    the grid's recent views, so after one pass over a busy and a quiet view neither is redone
    (with the previous view alone as the prediction, every quiet -> busy change overflowed)."""
    busy = _scene(20000, 224, 160, seed=5)  # a grid size no other test uses
    quiet = _scene(20000, 224, 160, seed=5)
    quiet.means[:, 2] += 12.0  # three times as far: a ninth of the footprint
    G._pred.pop(_key(busy), None)
    counts = []
    for sc in (busy, quiet):
        counts.append(_run(sc, "3d")[1]["isect_ids"].size)
    assert counts[0] > 1.5 * counts[1], counts
    s0 = dict(G.isect_stats)
    for _ in range(3):
        for sc in (quiet, busy):
            assert _run(sc, "3d")[3]
    assert G.isect_stats["redo"] == s0["redo"] and G.isect_stats["deferred"] == s0["deferred"] + 6
    assert max(h[0] for h in G._pred[_key(busy)]) == counts[0]
