"""Shared GPU-vs-oracle raster parity drivers (used by test_gpu_parity.py and
test_gpu_parity_dense.py).  TEST INFRASTRUCTURE.

run_3dgs / run_2dgs: gsplat.rasterization[_2dgs] fwd + bwd on the GPU against the C oracle
(f32 checker + f64 truth) on the same seeded scene: integer outputs bit-exact, images per
pixel with per-element conditioning (oracle/checks.py), every gradient per element.

Pixels whose discrete decisions (alpha vs 1/255, T vs 1e-4, the 0.999 clamp, the 2DGS
surface / low-pass branch) sit within a few ulps of a threshold can legitimately go either
way in any other correct f32 evaluation order.  They are not waved through:

1. value decisions: each such pixel's branch is RESOLVED -- every decision within 0.1 % of its
   threshold in the f32 or the f64 oracle is listed, and the f64 oracle is re-run forced onto
   candidate branches (the f64 outcomes, the f32 outcomes, the f32 outcomes with its closest or
   second-closest call inverted; hgsr_oracle.c decision lists); the GPU pixel must equal one of
   them (its last contributor index exactly, its values within the bar) (`resolve_branches`;
   the counts per branch are printed and returned);
2. gradients: a second backward of the same forward runs WITHOUT zeroing those pixels'
   upstream gradient, against the f32 / f64 oracle forced onto the branch the GPU took at each
   of them.  Only pixels whose sole near-threshold decision switches a
   gradient path and leaves the value unchanged (the 0.999 clamp, the 2DGS surface / low-pass
   branch: invisible in any output) keep a zero upstream gradient there, and are counted.

Reference call site: gaussian_renderer/render.py:40-76.
"""
import numpy as np
import torch

from horizongs_amd import gsplat_api as G
from oracle import pipeline as OP
from oracle.checks import ATOL, DELTA_2D, DELTA_3D, MAX_GRAD_AMBIGUOUS, RTOL, ambiguous, cond_close, image_close
from tests import parity_report as PR

DEV = "cuda:0"
# bare 1e-5 abs / 1e-4 rel pass rate the RGB image must keep against the f32 oracle
RGB_MIN_STRICT = 0.999


def to_dev(*ts):
    return [t.to(DEV).contiguous() for t in ts]


def gpu_last(out):
    """The last-contributor ids [C,H,W] the GPU forward saved for its backward."""
    last = out.grad_fn.saved_tensors[-1]
    assert last.dtype == torch.int32 and last.dim() == 3, (last.dtype, last.shape)
    return last


NEAR_THR = 1e-3  # decisions listed per pixel: margin below 0.1 %


def _merge_lists(pix, src, flip=None):
    """One pixel's decision list: the decisions `src` took within NEAR_THR of their thresholds,
    with its outcomes, optionally with the decision flip = (idx, kind) inverted.  Only src's own
    decisions are forced: a decision src did not list had a margin >= NEAR_THR on src's
    trajectory, so the forced f64 run -- on the same trajectory up to there -- decides it the same
    way by itself.  (Another precision's outcomes must not fill the gaps: once one earlier
    decision differs, its later decisions belong to a different trajectory.)"""
    ent = {}
    n = min(int(src["n"][pix]), src["idx"].shape[1])
    for k in range(n):
        ent[(int(src["idx"][pix, k]), int(src["kind"][pix, k]))] = (int(src["out"][pix, k]), float(src["m"][pix, k]))
    if flip is not None and flip in ent:
        o, m = ent[flip]
        ent[flip] = (1 - o, m)
    return ent


def _closest(pix, lst, j):
    """(idx, kind) of the j-th smallest-margin decision listed for pixel pix, or None"""
    n = min(int(lst["n"][pix]), lst["idx"].shape[1])
    if n <= j:
        return None
    k = int(np.argsort(lst["m"][pix, :n])[j])
    return int(lst["idx"][pix, k]), int(lst["kind"][pix, k])


def resolve_branches(make, r32, r64, amb, vals, last, alt32=None):
    """Branch the GPU took at every near-threshold pixel.

    make(dtype, near, pixmask=None) -> a forwarded oracle of that precision with decision lists
    `near` (None: record mode at NEAR_THR; a dict: force mode, hgsr_oracle.c set_near),
    compositing only the pixels of pixmask when given; vals: list of (GPU
    image [C,rows,W,K], f32 oracle image, f64 oracle image, attribute name of the image on the
    oracle object); last: GPU last ids [C,rows,W] (indices into the f32 oracle's intersection
    list, which the GPU's equals); alt32(near) -> a second correct f32
    evaluation in record mode (2DGS: the plane-form hit the kernels use), or None.

    Every decision within NEAR_THR of its threshold is listed per pixel and evaluation; the
    candidate branches are: the f64 outcomes, the f32 outcomes, and the f32
    outcomes with the closest or second-closest call flipped (and the same three for alt32's
    outcomes) -- each evaluated in f64, forced.
    A pixel matches a candidate when its last contributor is the candidate's and every value is
    within ATOL + RTOL |b| + 3 |b32 - b64|; the first match in preference order wins.  Returns (decision lists
    that reproduce the GPU's branch at every near-threshold pixel, counts)."""
    amb = np.asarray(amb, bool)
    shape = amb.shape
    P, K = int(np.prod(shape)), O_NEAR_K()
    forced = {"n": np.zeros(P, np.int32), "idx": np.full((P, K), -1, np.int64), "kind": np.zeros((P, K), np.int32),
              "out": np.zeros((P, K), np.int32)}
    counts = {"ambiguous": int(amb.sum())}
    if not amb.any():
        return forced, counts
    l32, l64 = make(np.float32, None).decisions, make(np.float64, None).decisions
    srcs = [("f32", l32)] + ([] if alt32 is None else [("f32b", alt32(None).decisions)])
    over = amb.reshape(-1) & ((l64["n"] > K) | np.any([ls["n"] > K for _, ls in srcs], 0))
    counts["list_overflow"] = int(over.sum())
    pixels = np.flatnonzero(amb.reshape(-1) & ~over)
    # (name, the evaluation whose listed outcomes are forced, which of its calls to flip), in
    # order of preference: the evaluation that reproduces the kernels' arithmetic first (alt32:
    # its decisions are the GPU's up to the hardware exp2's last ulp), f64 last.  The first
    # candidate within the value bar wins, not the closest: a keep / skip decision whose
    # contribution is below the value bar cannot be told apart by the render, only by its
    # gradient, so the branch is taken from the evaluation most likely to share it.
    cands = []
    for nm, ls in srcs[::-1]:
        cands += [(nm, ls, None), (nm + "_flip0", ls, 0), (nm + "_flip1", ls, 1)]
    cands.append(("f64", l64, None))
    names = tuple(c[0] for c in cands)
    cand_lists = []
    for _, src, fl in cands:
        lst = {k: v.copy() for k, v in forced.items()}
        for p in pixels:
            ent = _merge_lists(p, src, None if fl is None else _closest(p, src, fl))
            for k, ((idx, kind), (o, _)) in enumerate(sorted(ent.items())[:K]):
                lst["idx"][p, k], lst["kind"][p, k], lst["out"][p, k] = idx, kind, o
            lst["n"][p] = min(len(ent), K)
        cand_lists.append(lst)
    # last contributors compared as Gaussian ids: the f32 and f64 binnings can order the
    # intersection lists differently (the GPU's list is the f32 oracle's, bit for bit)
    last = np.asarray(last)
    gid = r32.flatten_ids[last]
    e32 = [np.abs(np.asarray(b32, np.float64) - b64) for _, b32, b64, _ in vals]

    def err(rv):
        x = np.where(amb & (gid == rv.flatten_ids[rv.last]), 0.0, np.inf)
        for (a, _, _, attr), e in zip(vals, e32):
            b = np.asarray(getattr(rv, attr), np.float64)
            bar = ATOL + RTOL * np.abs(b) + 3.0 * e
            x = np.maximum(x, (np.abs(np.asarray(a, np.float64) - b) / bar).reshape(shape + (-1,)).max(-1))
        return x

    # each candidate forward composites only the near-threshold pixels (the only ones read)
    pm = np.ascontiguousarray(amb.reshape(-1), np.uint8)
    errs = np.stack([err(make(np.float64, lst, pm)) for lst in cand_lists])  # [candidates, C, rows, W]
    fits = errs <= 1.0
    best = np.argmax(fits, 0)  # the first fitting candidate in preference order
    ok = amb & fits.any(0)
    for ci, name in enumerate(names):
        sel = (ok & (best == ci)).reshape(-1)
        counts[name] = int(sel.sum())
        for k in forced:
            forced[k][sel] = cand_lists[ci][k][sel]
    left = amb & ~ok
    counts["unmatched"] = int(left.sum())
    if left.any():
        rows = []
        for p in np.argwhere(left)[:6]:
            p = tuple(p)
            q = int(np.ravel_multi_index(p, shape))
            rows.append(dict(pix=p, gpu_last=int(gid[p]), f64_last=int(r64.flatten_ids[r64.last[p]]),
                             f32_last=int(r32.flatten_ids[r32.last[p]]),
                             err=[float(e[p]) for e in errs], n32=int(l32["n"][q]), n64=int(l64["n"][q]),
                             gpu=np.asarray(vals[0][0])[p].tolist(), f64=np.asarray(vals[0][2])[p].tolist()))
        raise AssertionError(f"{counts['unmatched']} near-threshold pixels match no branch of the oracle: {counts} "
                             f"{rows}")
    return forced, counts


def O_NEAR_K():
    from oracle import oracle as O
    return O.NEAR_K


def depth_stats(ref):
    """(max Gaussians per tile, max backward replay depth of a tile, stopped-pixel fraction).

    Replay depth = the tile's latest contributor over its rasterised rows - tile start + 1,
    i.e. how far back the backward walks.  Stopped = the pixel's list ended at the exclusive
    T <= 1e-4 stop (flag from the oracle forward)."""
    C, th, tw = ref.offsets.shape
    offs = ref.offsets.reshape(-1).astype(np.int64)
    ends = np.append(offs[1:], len(ref.flatten_ids))
    counts = ends - offs
    rows = ref.Hr
    last = np.full((C, th * 16, tw * 16), -1, np.int64)
    last[:, :rows, :ref.W] = ref.last.reshape(C, rows, ref.W)
    tile_last = last.reshape(C, th, 16, tw, 16).max(axis=(2, 4)).reshape(-1)
    replay = np.where(tile_last >= 0, tile_last + 1 - offs, 0)
    return int(counts.max()), int(replay.max()), float(ref.stopped.mean())


def oracle_list_entries(r):
    """The raster3d backward's per-wave compacted-list entries (the bench roofline's executed
    pairs / 64, csrc/raster3d.hip `stepped`), restated from the oracle's forward: for every
    (tile, 8x8 quadrant) the intersections up to the quadrant's latest contributor (the max of
    its pixels' last ids; the kernel's t0 trim) whose record reaches the quadrant -- the
    footprint box |m - q| <= ext + 3.5 with ext = sqrt(2 ln(255 o) Cov_ii) x 1.01 + 0.01
    (rec3.h footprint) and the exact ellipse test: min over the quadrant's pixel-centre
    rectangle of sigma' <= log2(255 o) (+ 1e-3 relative + 1e-3), raster3d.hip
    ellipse_reaches -- evaluated in f64 (the kernels' f32 with hardware log / rcp decide the
    same up to the conservative slack)."""
    C, N = r.means2d.shape[:2]
    fl = r.flatten_ids.astype(np.int64)
    offs = r.offsets.reshape(-1).astype(np.int64)
    n_bins = offs.size
    if fl.size == 0:
        return 0
    ends = np.append(offs[1:], fl.size)
    bin_of = np.repeat(np.arange(n_bins), np.maximum(ends - offs, 0))
    pos = np.arange(fl.size)
    cam = bin_of // (r.tw * r.th)
    tile = bin_of - cam * (r.tw * r.th)
    ty, tx = tile // r.tw, tile % r.tw
    last = np.full((C, r.th * 16, r.tw * 16), -1, np.int64)
    last[:, :r.H, :r.W] = r.last.reshape(C, r.H, r.W)
    qlast = last.reshape(C, r.th, 2, 8, r.tw, 2, 8).max(axis=(3, 6))  # [C, th, 2, tw, 2]
    gi = cam * N + fl
    m2 = r.means2d.reshape(-1, 2).astype(np.float64)[gi]
    cn = r.conics.reshape(-1, 3).astype(np.float32)[gi]
    op = np.asarray(r.opac_c, np.float32).reshape(-1)[gi]
    a32, b32, c32 = cn[:, 0], cn[:, 1], cn[:, 2]
    # the record as pack3 stores it (f32): log2(e)-scaled conic, footprint half-extents
    l2e = np.float32(1.4426950408889634)
    ap, bp, cp = (np.float32(0.5) * l2e * a32).astype(np.float64), (l2e * b32).astype(np.float64), \
        (np.float32(0.5) * l2e * c32).astype(np.float64)
    a, b, c = a32.astype(np.float64), b32.astype(np.float64), c32.astype(np.float64)
    with np.errstate(divide="ignore", invalid="ignore"):
        L = np.log(255.0 * op.astype(np.float64))
        det = a * c - b * b
        ok = (L > 0) & (det > 0)
        k = np.where(ok, 2 * L / np.where(det > 0, det, 1), 0)
        ex = np.where(ok, np.sqrt(np.maximum(k * c, 0)) * 1.01 + 0.01, -1e30)
        ey = np.where(ok, np.sqrt(np.maximum(k * a, 0)) * 1.01 + 0.01, -1e30)
        lim = np.log2(255.0 * op.astype(np.float64))
    total = 0
    for qy in range(2):
        for qx in range(2):
            qcx = tx * 16 + qx * 8 + 4.0
            qcy = ty * 16 + qy * 8 + 4.0
            cx, cy = m2[:, 0] - qcx, m2[:, 1] - qcy
            box = (np.abs(cx) <= ex + 3.5) & (np.abs(cy) <= ey + 3.5)
            x0, x1, y0, y1 = cx - 3.5, cx + 3.5, cy - 3.5, cy + 3.5
            q = lambda dx, dy: ap * dx * dx + bp * dx * dy + cp * dy * dy  # noqa: E731
            with np.errstate(divide="ignore", invalid="ignore"):
                ia, ic = -0.5 / ap, -0.5 / cp
                dya = np.clip(bp * x0 * ic, y0, y1)
                dyb = np.clip(bp * x1 * ic, y0, y1)
                dxa = np.clip(bp * y0 * ia, x0, x1)
                dxb = np.clip(bp * y1 * ia, x0, x1)
                mm = np.minimum(np.minimum(q(x0, dya), q(x1, dyb)), np.minimum(q(dxa, y0), q(dxb, y1)))
            inside = (x0 <= 0) & (x1 >= 0) & (y0 <= 0) & (y1 >= 0)
            mm = np.where(inside, 0.0, mm)
            ell = mm <= lim + 1e-3 * np.abs(lim) + 1e-3
            wf = qlast[cam, ty, qy, tx, qx]
            total += int(np.count_nonzero(box & ell & (pos <= wf)))
    return total


def run_3dgs(sc, mode, bg, rows=None, seed=0, min_strict=RGB_MIN_STRICT, sh=None, train=None, count_pairs=False):
    """rasterization() fwd + bwd on the GPU vs Raster3D f32 / f64; upstream gradients N(0,1)
    on the rasterised rows, zero elsewhere.  count_pairs: the backward's device count of the
    (pixel, Gaussian) pairs it evaluated (bench.py's roofline numerator) is checked against
    oracle_list_entries x 64."""
    kw = dict(backgrounds=bg, render_mode=mode, rows=rows, sh_degree=sh)
    args = (sc.means, sc.quats, sc.scales, sc.opacities, sc.colors, sc.viewmats, sc.Ks, sc.width, sc.height)
    r32 = OP.Raster3D(*args, **kw)
    rc, ra = r32.forward()
    r64 = OP.Raster3D(*args, dtype=np.float64, **kw)
    r64.forward()
    stats = depth_stats(r32)
    rr = r32.Hr
    means, quats, scales, opac, cols, vm, K = to_dev(sc.means, sc.quats, sc.scales, sc.opacities, sc.colors,
                                                     sc.viewmats, sc.Ks)
    gbg = None if bg is None else bg.to(DEV)
    leaves = dict(means=means, quats=quats, scales=scales, opacities=opac, colors=cols)
    train = tuple(leaves) if train is None else train
    for k in train:
        leaves[k].requires_grad_(True)
    out, alpha, meta = G.rasterization(means, quats, scales, opac, cols, vm, K, sc.width, sc.height, packed=False,
                                       backgrounds=gbg, render_mode=mode, sh_degree=sh)
    meta["means2d"].retain_grad()
    np.testing.assert_array_equal(meta["isect_ids"].cpu().numpy(), r32.isect_ids)
    np.testing.assert_array_equal(meta["flatten_ids"].cpu().numpy(), r32.flatten_ids)
    np.testing.assert_array_equal(meta["isect_offsets"].cpu().numpy(), r32.offsets)
    o = out.detach()[:, :rr].cpu().numpy()
    amb = ambiguous(r32, DELTA_3D)                 # value decisions: excluded from the image bar
    gamb = ambiguous(r32, DELTA_3D, gradient=True)  # + gradient-path switches: no upstream gradient
    rates = {}
    Dc = 3 if mode in ("RGB", "RGB+D", "RGB+ED") else 0
    if Dc:
        rates["rgb"], n_amb = image_close(o[..., :Dc], rc[..., :Dc], r64.render_colors[..., :Dc], amb, "render rgb",
                                          min_strict=min_strict)
    if o.shape[-1] > Dc:
        rates["depth"], n_amb = image_close(o[..., Dc:], rc[..., Dc:], r64.render_colors[..., Dc:], amb,
                                            "render depth")
    rates["alpha"], _ = image_close(alpha.detach()[:, :rr].cpu().numpy(), ra, r64.ra, amb, "render alphas")
    rates["ambiguous_px"] = n_amb
    rates["grad_ambiguous_px"] = int(gamb.sum())
    assert gamb.mean() <= MAX_GRAD_AMBIGUOUS, gamb.mean()
    g = torch.Generator().manual_seed(seed)
    keep = torch.from_numpy(~gamb)[..., None].float()  # no gradient flows from ambiguous pixels
    vrc = torch.randn(rc.shape, generator=g) * keep
    vra = torch.randn(ra.shape, generator=g) * keep
    vrc_full = torch.zeros(out.shape)
    vra_full = torch.zeros(alpha.shape)
    vrc_full[:, :rr] = vrc
    vra_full[:, :rr] = vra
    if count_pairs:
        import ctypes as ct
        from horizongs_amd import _native as NAT
        NAT.call("hgsr_timing_reset")
        NAT.call("hgsr_timing_only", b"raster3d_bwd")
        NAT.call("hgsr_timing_pairs", None, 1)
        NAT.call("hgsr_timing_enable", 1)
    try:
        ((out * vrc_full.to(DEV)).sum() + (alpha * vra_full.to(DEV)).sum()).backward(retain_graph=True)
    finally:
        if count_pairs:
            ec = ct.c_ulonglong(0)
            NAT.call("hgsr_timing_exec_pairs", ct.byref(ec))
            NAT.call("hgsr_timing_enable", 0)
            NAT.call("hgsr_timing_only", None)
    if count_pairs:
        want = oracle_list_entries(r32) * 64
        rates["exec_pairs"] = (int(ec.value), want)
        # the kernels' f32 culling (hardware log / rcp) and the f64 restatement may decide the
        # conservative slack differently for a handful of records (r04: 728 extra / 5 missing
        # of 5.7M list entries at c2)
        assert want > 0 and abs(int(ec.value) - want) <= 2e-4 * want + 64 * 8, (ec.value, want)
    gr32 = r32.backward(vrc.numpy(), vra.numpy())
    gr64 = r64.backward(vrc.numpy(), vra.numpy())
    genv = r64.envelope(vrc.numpy(), vra.numpy())
    got = {"means2d": meta["means2d"].grad, **{k: leaves[k].grad for k in train}}
    for k, v in got.items():
        if k == "colors" and not Dc:
            continue
        rates["v_" + k] = cond_close(v.cpu().numpy(), gr32[k], gr64[k], "v_" + k, rel_floor=0, env=genv[k])
    # element-wise report against the gsplat-form f32, the kernel-form f32 (the kernels' alpha
    # arithmetic) and f64 (tests/parity_report.py); images on their unambiguous pixels
    rk = OP.Raster3D(*args, alphaform=1, **kw)
    rk.forward()
    gk32 = rk.backward(vrc.numpy(), vra.numpy())
    px = ~np.asarray(amb, bool)
    for nm, sl in (("render_rgb", slice(0, Dc)), ("render_depth", slice(Dc, o.shape[-1]))):
        if sl.stop > sl.start:
            PR.tensor(nm, o[..., sl], rc[..., sl], rk.render_colors[..., sl], r64.render_colors[..., sl],
                      mask=np.broadcast_to(px[..., None], o[..., sl].shape))
    PR.tensor("render_alpha", alpha.detach()[:, :rr].cpu().numpy(), ra, rk.ra, r64.ra,
              mask=np.broadcast_to(px[..., None], ra.shape))
    for k, v in got.items():
        if k == "colors" and not Dc:
            continue
        PR.tensor("v_" + k, v.cpu().numpy(), gr32[k], gk32[k], gr64[k])
    # near-threshold pixels: resolve the branch the GPU took, then check the gradients again with
    # their upstream gradient kept, against the oracle evaluated on those branches
    def make(dt, near, pixmask=None):
        r = OP.Raster3D(*args, dtype=dt, **kw)
        r.pixmask = pixmask
        if near is None:
            r.record_near(NEAR_THR)
        else:
            r.force_near(near)
        r.forward()
        return r
    vals = [(o, rc, r64.render_colors, "render_colors"),
            (alpha.detach()[:, :rr].cpu().numpy(), ra, r64.ra, "ra")]

    def make_k(near):  # the kernels' alpha form (log2(e)-scaled conic, FMAs, exp2), f32
        r = OP.Raster3D(*args, alphaform=1, **kw)
        r.record_near(NEAR_THR)
        r.forward()
        return r
    forced, counts = resolve_branches(make, r32, r64, amb, vals, gpu_last(out)[:, :rr].cpu().numpy(), alt32=make_k)
    gonly = gamb & ~amb  # a gradient-path switch only (the 0.999 clamp): invisible in every output
    rates["branches"] = counts
    rates["grad_only_ambiguous_px"] = int(gonly.sum())
    if amb.any():
        got = {k: v.clone() for k, v in got.items()}
        g2 = torch.Generator().manual_seed(seed + 1000)
        keep2 = torch.from_numpy(~gonly)[..., None].float()
        vrc2 = torch.randn(rc.shape, generator=g2) * keep2
        vra2 = torch.randn(ra.shape, generator=g2) * keep2
        vrc_full.zero_()
        vra_full.zero_()
        vrc_full[:, :rr] = vrc2
        vra_full[:, :rr] = vra2
        meta["means2d"].grad = None
        for k in train:
            leaves[k].grad = None
        ((out * vrc_full.to(DEV)).sum() + (alpha * vra_full.to(DEV)).sum()).backward()
        rv = {}
        for dt in (np.float32, np.float64):  # both precisions forced onto the GPU's branches
            rv[dt] = OP.Raster3D(*args, dtype=dt, **kw)
            rv[dt].force_near(forced)
            rv[dt].forward()
        gv32 = rv[np.float32].backward(vrc2.numpy(), vra2.numpy())
        gv64 = rv[np.float64].backward(vrc2.numpy(), vra2.numpy())
        genv2 = rv[np.float64].envelope(vrc2.numpy(), vra2.numpy())
        got2 = {"means2d": meta["means2d"].grad, **{k: leaves[k].grad for k in train}}
        for k, v in got2.items():
            if k == "colors" and not Dc:
                continue
            rates["v2_" + k] = cond_close(v.cpu().numpy(), gv32[k], gv64[k], "v2_" + k + " (resolved branches)",
                                          rel_floor=0, env=genv2[k], env_k=ENV_K_RESOLVED)
    print("strict 1e-5/1e-4 pass rates:", {k: (round(float(v), 6) if not isinstance(v, (dict, tuple)) else v)
                                           for k, v in rates.items()}, "stats", stats)
    return stats, rates, dict(out=out, alpha=alpha, meta=meta, r32=r32, r64=r64, grads=got, gr32=gr32, gr64=gr64)


# Envelope multiple of the resolved-branch re-check (gradients with the near-threshold pixels'
# upstream kept, the oracle forced onto the GPU's branches).  E sums the per-step roundings in
# quadrature (an RMS estimate, oracle Raster*.envelope), so its tail grows with the element
# count: over the 6M colour gradients of the full c3 frame the worst element needs 5.9 u E
# (profiles/r04_parity_strict.txt), the 1080-row band of round 3 needed < 2.
ENV_K_RESOLVED = 8.0


def run_2dgs(sc, mode, bg, rows=None, seed=0, min_strict=RGB_MIN_STRICT):
    kw = dict(backgrounds=bg, render_mode=mode, rows=rows)
    args = (sc.means, sc.quats, sc.scales, sc.opacities, sc.colors, sc.viewmats, sc.Ks, sc.width, sc.height)
    r32 = OP.Raster2D(*args, **kw)
    rc, ra, rn = r32.forward()
    r64 = OP.Raster2D(*args, dtype=np.float64, **kw)
    r64.forward()
    # the plane-form hit (what the kernels evaluate) is a second correct f32 evaluation:
    # near edge-on surfels the two forms differ far beyond an ulp (the hit's z cancels)
    r32b = OP.Raster2D(*args, hitform=1, **kw)
    r32b.forward()
    stats = depth_stats(r32)
    rr = r32.Hr
    means, quats, scales, opac, cols, vm, K = to_dev(sc.means, sc.quats, sc.scales, sc.opacities, sc.colors,
                                                     sc.viewmats, sc.Ks)
    gbg = None if bg is None else bg.to(DEV)
    for t in (means, quats, scales, opac, cols):
        t.requires_grad_(True)
    (out, alpha, normals, nfd, distort, median), meta = G.rasterization_2dgs(
        means, quats, scales, opac, cols, vm, K, sc.width, sc.height, packed=False, backgrounds=gbg,
        render_mode=mode)
    np.testing.assert_array_equal(meta["isect_ids"].cpu().numpy(), r32.isect_ids)
    np.testing.assert_array_equal(meta["flatten_ids"].cpu().numpy(), r32.flatten_ids)
    o = out.detach()[:, :rr].cpu().numpy()
    # either form's decisions near a threshold, or the two forms ending a pixel differently
    split = (r32.last != r32b.last) | (r32.stopped != r32b.stopped)
    amb = ambiguous(r32, DELTA_2D) | ambiguous(r32b, DELTA_2D) | split
    gamb = ambiguous(r32, DELTA_2D, gradient=True) | ambiguous(r32b, DELTA_2D, gradient=True) | split
    rates = {}
    rb = r32b.render_colors
    rates["rgb"], n_amb = image_close(o[..., :3], rc[..., :3], r64.render_colors[..., :3], amb, "2dgs rgb",
                                      min_strict=min_strict, margin=r32.margin, alt32=rb[..., :3])
    rates["depth"], _ = image_close(o[..., 3:], rc[..., 3:], r64.render_colors[..., 3:], amb, "2dgs depth",
                                    alt32=rb[..., 3:])
    rates["alpha"], _ = image_close(alpha.detach()[:, :rr].cpu().numpy(), ra, r64.ra, amb, "2dgs alphas",
                                    alt32=r32b.ra)
    # viewmat = I: the world-frame normals are the camera-frame ones
    # normals keep factor 3: at c3 one element of 6.2M (an edge-on surfel, where the normal's
    # direction is the cross product of two nearly parallel tangent axes) sits 2.2e-3 further
    # from f64 than either f32 hit form (profiles/r04_parity_strict.txt)
    rates["normals"], _ = image_close(normals.detach()[:, :rr].cpu().numpy(), rn, r64.rn, amb, "2dgs normals",
                                      alt32=r32b.rn, factor=3.0)
    rates["ambiguous_px"] = n_amb
    rates["grad_ambiguous_px"] = int(gamb.sum())
    assert gamb.mean() <= MAX_GRAD_AMBIGUOUS, gamb.mean()
    g = torch.Generator().manual_seed(seed)
    keep = torch.from_numpy(~gamb)[..., None].float()  # no gradient flows from ambiguous pixels
    vrc = torch.randn(rc.shape, generator=g) * keep
    vra = torch.randn(ra.shape, generator=g) * keep
    vrn = torch.randn(rn.shape, generator=g) * keep
    full = [torch.zeros(t.shape) for t in (out, alpha, normals)]
    for f, v in zip(full, (vrc, vra, vrn)):
        f[:, :rr] = v
    ((out * full[0].to(DEV)).sum() + (alpha * full[1].to(DEV)).sum()
     + (normals * full[2].to(DEV)).sum()).backward(retain_graph=True)
    gr32 = r32.backward(vrc.numpy(), vra.numpy(), vrn.numpy())
    gr32b = r32b.backward(vrc.numpy(), vra.numpy(), vrn.numpy())
    gr64 = r64.backward(vrc.numpy(), vra.numpy(), vrn.numpy())
    genv = r64.envelope(vrc.numpy(), vra.numpy(), vrn.numpy())
    leaves = {"opacities": opac, "colors": cols, "means": means, "quats": quats, "scales": scales}
    got = {"densify": meta["gradient_2dgs"].grad, **{k: v.grad for k, v in leaves.items()}}
    for k, v in got.items():
        rates["v_" + k] = cond_close(v.cpu().numpy(), gr32[k], gr64[k], "v_" + k, rel_floor=0, env=genv[k],
                                     alt32=gr32b[k])
    # element-wise report: gsplat-form (per-pixel cross product) f32, kernel-form (plane-form
    # hit) f32 and f64 (tests/parity_report.py); images on their unambiguous pixels
    px = ~np.asarray(amb, bool)
    for nm, a, b, k, c in (("render_rgb", o[..., :3], rc[..., :3], rb[..., :3], r64.render_colors[..., :3]),
                           ("render_depth", o[..., 3:], rc[..., 3:], rb[..., 3:], r64.render_colors[..., 3:]),
                           ("render_alpha", alpha.detach()[:, :rr].cpu().numpy(), ra, r32b.ra, r64.ra),
                           ("render_normals", normals.detach()[:, :rr].cpu().numpy(), rn, r32b.rn, r64.rn)):
        PR.tensor(nm, a, b, k, c, mask=np.broadcast_to(px[..., None], a.shape))
    for k, v in got.items():
        PR.tensor("v_" + k, v.cpu().numpy(), gr32[k], gr32b[k], gr64[k])
    # near-threshold pixels: resolve the GPU's branch, then the gradients again with their upstream kept

    def make(dt, near, pixmask=None):
        r = OP.Raster2D(*args, dtype=dt, **kw)
        r.pixmask = pixmask
        if near is None:
            r.record_near(NEAR_THR)
        else:
            r.force_near(near)
        r.forward()
        return r
    # the f32 error of each value: the larger of the two hit forms' (the kernels use the plane form)
    vals = [(o, np.where(np.abs(rb - r64.render_colors) > np.abs(rc - r64.render_colors), rb, rc),
             r64.render_colors, "render_colors"),
            (alpha.detach()[:, :rr].cpu().numpy(), np.where(np.abs(r32b.ra - r64.ra) > np.abs(ra - r64.ra), r32b.ra, ra),
             r64.ra, "ra"),
            (normals.detach()[:, :rr].cpu().numpy(), np.where(np.abs(r32b.rn - r64.rn) > np.abs(rn - r64.rn), r32b.rn,
                                                              rn), r64.rn, "rn")]
    def make_b(near):  # the plane-form hit the kernels evaluate, f32
        r = OP.Raster2D(*args, hitform=1, **kw)
        r.record_near(NEAR_THR)
        r.forward()
        return r
    forced, counts = resolve_branches(make, r32, r64, amb, vals, gpu_last(out)[:, :rr].cpu().numpy(), alt32=make_b)
    # gradient-path switches only (the 0.999 clamp; the surface / low-pass branch of sigma =
    # min(g3, g2)/2, continuous in value): invisible in every output, so unresolvable
    gonly = gamb & ~amb
    rates["branches"] = counts
    rates["grad_only_ambiguous_px"] = int(gonly.sum())
    if amb.any():
        got = {k: v.clone() for k, v in got.items()}
        g2 = torch.Generator().manual_seed(seed + 1000)
        keep2 = torch.from_numpy(~gonly)[..., None].float()
        ups = [torch.randn(t.shape, generator=g2) * keep2 for t in (rc, ra, rn)]
        for f, v in zip(full, ups):
            f.zero_()
            f[:, :rr] = v
        meta["gradient_2dgs"].grad = None
        for t in leaves.values():
            t.grad = None
        ((out * full[0].to(DEV)).sum() + (alpha * full[1].to(DEV)).sum() + (normals * full[2].to(DEV)).sum()).backward()
        rv = {}
        for key, dt, hf in (("32", np.float32, 0), ("32b", np.float32, 1), ("64", np.float64, 0)):
            rv[key] = OP.Raster2D(*args, dtype=dt, hitform=hf, **kw)
            rv[key].force_near(forced)
            rv[key].forward()
        un = [u.numpy() for u in ups]
        gv = {k: r.backward(*un) for k, r in rv.items()}
        genv2 = rv["64"].envelope(*un)
        got2 = {"densify": meta["gradient_2dgs"].grad, **{k: v.grad for k, v in leaves.items()}}
        for k, v in got2.items():
            rates["v2_" + k] = cond_close(v.cpu().numpy(), gv["32"][k], gv["64"][k], "v2_" + k + " (resolved branches)",
                                          rel_floor=0, env=genv2[k], env_k=ENV_K_RESOLVED, alt32=gv["32b"][k])
    print("strict 1e-5/1e-4 pass rates:", {k: (round(float(v), 6) if not isinstance(v, (dict, tuple)) else v)
                                           for k, v in rates.items()}, "stats", stats)
    return stats, rates, dict(out=out, alpha=alpha, normals=normals, nfd=nfd, distort=distort, median=median,
                              meta=meta, r32=r32, r64=r64)
