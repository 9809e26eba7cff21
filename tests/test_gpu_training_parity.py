"""Training parity (BASELINE "PSNR delta vs ref"): the same small
synthetic scene is fitted for the same number of Adam iterations through (a) the HIP
rasterizer (horizongs_amd.gsplat_api.rasterization) + the fused HIP Adam and (b) the autograd torch
restatement of gsplat's rasterization (oracle/torch_ref.py, CPU, fp32), from the same
perturbed initialisation towards the same ground-truth render.  The two final PSNRs
must agree within 0.05 dB.  The measured numbers are written to
gpurun_out/psnr_parity.json (copied into profiles/ and quoted by bench.py)."""
import json
import math
import os

import numpy as np
import pytest
import torch

from horizongs_amd.synthetic import make_scene
from oracle import torch_ref as TR

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")


def _params(sc, seed):
    g = torch.Generator().manual_seed(seed)
    z = sc.means[:, 2:3]
    fx = float(sc.Ks[0, 0, 0])
    jitter = torch.cat([torch.randn(sc.means.shape[0], 2, generator=g) * 2.0 * z / fx,
                        torch.zeros(sc.means.shape[0], 1)], 1)  # ~2 px
    return dict(means=sc.means + jitter, log_scales=torch.log(sc.scales * 1.5), quats=sc.quats.clone(),
                opac_logit=torch.full((sc.means.shape[0],), -0.5), colors=torch.full_like(sc.colors, 0.5))


def _fit(render, p0, gt, iters):
    """Fit with the reference optimizer (torch.optim.Adam) on CPU tensors and with the
    fused HIP Adam (horizongs_amd.optim.Adam) on device tensors."""
    p = {k: v.clone().requires_grad_(True) for k, v in p0.items()}
    lr = dict(means=1e-3, log_scales=1e-2, quats=1e-2, opac_logit=5e-2, colors=2e-2)
    if next(iter(p.values())).is_cuda:
        from horizongs_amd.optim import Adam
    else:
        Adam = torch.optim.Adam
    opt = Adam([{"params": [p[k]], "lr": lr[k]} for k in p])
    for _ in range(iters):
        opt.zero_grad()
        loss = (render(p) - gt).abs().mean()
        loss.backward()
        opt.step()
    with torch.no_grad():
        mse = ((render(p) - gt) ** 2).mean().item()
    return 10 * math.log10(1.0 / mse)


def test_psnr_parity_3dgs():
    from horizongs_amd import gsplat_api as G
    W, H, N, iters = 128, 96, 300, 200
    sc = make_scene(N, W, H, seed=11)
    vm, K = sc.viewmats[0], sc.Ks[0]

    def render_cpu(p):
        m2, con, dep, rad = TR.project3d(p["means"], p["quats"], torch.exp(p["log_scales"]), vm, K, W, H)
        img, _ = TR.raster3d(m2, con, p["colors"], torch.sigmoid(p["opac_logit"]), dep, rad, W, H)
        return img

    vmd, Kd = sc.viewmats.cuda(), sc.Ks.cuda()

    def render_gpu(p):
        out, _, _ = G.rasterization(p["means"], p["quats"], torch.exp(p["log_scales"]), torch.sigmoid(p["opac_logit"]),
                                    p["colors"], vmd, Kd, W, H, packed=False)
        return out[0]

    with torch.no_grad():
        gt_cpu = render_cpu(dict(means=sc.means, quats=sc.quats, log_scales=torch.log(sc.scales),
                                 opac_logit=torch.logit(sc.opacities), colors=sc.colors))
    p0 = _params(sc, seed=12)
    psnr_init = 10 * math.log10(1.0 / ((render_cpu(p0).detach() - gt_cpu) ** 2).mean().item())
    psnr_cpu = _fit(render_cpu, p0, gt_cpu, iters)
    psnr_gpu = _fit(render_gpu, {k: v.cuda() for k, v in p0.items()}, gt_cpu.cuda(), iters)
    res = dict(psnr_init_db=round(psnr_init, 4), psnr_ref_db=round(psnr_cpu, 4), psnr_hip_db=round(psnr_gpu, 4),
               psnr_delta_db=round(psnr_gpu - psnr_cpu, 4), iterations=iters, gaussians=N, width=W, height=H,
               reference="oracle/torch_ref.py autograd restatement of gsplat rasterization (CPU, fp32)")
    os.makedirs("gpurun_out", exist_ok=True)
    with open(os.path.join("gpurun_out", "psnr_parity.json"), "w") as f:
        json.dump(res, f)
    print(res)
    assert psnr_cpu > psnr_init + 3.0  # the fit actually fits
    assert abs(psnr_gpu - psnr_cpu) <= 0.05, res


def test_psnr_parity_2dgs():
    from horizongs_amd import gsplat_api as G
    W, H, N, iters = 128, 96, 300, 200
    sc = make_scene(N, W, H, seed=13)
    vm, K = sc.viewmats[0], sc.Ks[0]

    def render_cpu(p):
        m2, rt, dep, nrm, rad = TR.project2d(p["means"], p["quats"], torch.exp(p["log_scales"]), vm, K)
        img, _, _ = TR.raster2d(m2, rt, p["colors"], torch.sigmoid(p["opac_logit"]), nrm, dep, rad, W, H)
        return img

    vmd, Kd = sc.viewmats.cuda(), sc.Ks.cuda()

    def render_gpu(p):
        (out, *_), _ = G.rasterization_2dgs(p["means"], p["quats"], torch.exp(p["log_scales"]),
                                            torch.sigmoid(p["opac_logit"]), p["colors"], vmd, Kd, W, H, packed=False)
        return out[0]

    with torch.no_grad():
        gt_cpu = render_cpu(dict(means=sc.means, quats=sc.quats, log_scales=torch.log(sc.scales),
                                 opac_logit=torch.logit(sc.opacities), colors=sc.colors))
    p0 = _params(sc, seed=14)
    psnr_init = 10 * math.log10(1.0 / ((render_cpu(p0).detach() - gt_cpu) ** 2).mean().item())
    psnr_cpu = _fit(render_cpu, p0, gt_cpu, iters)
    psnr_gpu = _fit(render_gpu, {k: v.cuda() for k, v in p0.items()}, gt_cpu.cuda(), iters)
    res = dict(psnr_init_db=round(psnr_init, 4), psnr_ref_db=round(psnr_cpu, 4), psnr_hip_db=round(psnr_gpu, 4),
               psnr_delta_db=round(psnr_gpu - psnr_cpu, 4), iterations=iters, gaussians=N, width=W, height=H,
               reference="oracle/torch_ref.py autograd restatement of gsplat rasterization_2dgs (CPU, fp32)")
    with open(os.path.join("gpurun_out", "psnr_parity_2dgs.json"), "w") as f:
        json.dump(res, f)
    print(res)
    assert psnr_cpu > psnr_init + 3.0
    assert abs(psnr_gpu - psnr_cpu) <= 0.05, res


# ----------------------------------------------------------------------------- anchor pipeline
def _pipeline_parity(gs):
    """200 equal Adam iterations of the whole reference train step on an anchor model
    (5k anchors, 160x120; tests/pipeline_fit.py): prefilter -> decode -> rasterization ->
    loss head -> backward -> Adam, HIP chain vs the CPU chain whose decode and loss stages are
    pinned to the reference's own goldens, at the fine-stage learning rates x PF.LR_SCALE (0.3:
    below the chain's chaotic regime, pipeline_fit docstring).  The PSNR of the last 50
    iterations' renders against the same target must agree within 0.05 dB.  The final-iterate PSNRs are recorded
    too, next to the chain's own sensitivity: the CPU chain rerun from an initialisation
    perturbed by 1e-6 (relative) -- a single final iterate differs by about that much between
    ANY two f32 evaluations of this chaotic training (tests/pipeline_fit.py)."""
    import torch as _t
    from tests import pipeline_fit as PF
    A, W, H, iters = 5000, 160, 120, 200
    gt = PF.target(40000, W, H, seed=31, gs=gs)
    p0, cfg = PF.anchor_model(A, W, H, seed=32, param_seed=200)
    with torch.no_grad():
        psnr_init = PF.psnr(PF.cpu_render(p0, cfg, gs)[0], gt)
    ls = PF.LR_SCALE
    fin_cpu, win_cpu, loss_cpu = PF.fit(p0, cfg, gt, iters, gs=gs, lr_scale=ls)
    fin_gpu, win_gpu, loss_gpu = PF.fit(p0, cfg, gt, iters, gs=gs, device="cuda", lr_scale=ls)
    pert = {k: (v * (1 + 1e-6 * _t.randn(v.shape, generator=_t.Generator().manual_seed(5))) if k != "anchor" else v)
            for k, v in p0.items()}
    fin_self, win_self, _ = PF.fit(pert, cfg, gt, iters, gs=gs, lr_scale=ls)
    res = dict(psnr_init_db=round(psnr_init, 4), psnr_ref_db=round(win_cpu, 4), psnr_hip_db=round(win_gpu, 4),
               psnr_delta_db=round(win_gpu - win_cpu, 4), psnr_metric="mean MSE of the last 50 iterations' renders",
               final_iterate={"ref_db": round(fin_cpu, 4), "hip_db": round(fin_gpu, 4),
                              "delta_db": round(fin_gpu - fin_cpu, 4),
                              "ref_perturbed_1e-6_delta_db": round(fin_self - fin_cpu, 4)},
               window_ref_perturbed_delta_db=round(win_self - win_cpu, 4),
               iterations=iters, anchors=A, width=W, height=H, lr_scale=ls,
               loss_first=[round(loss_cpu[0], 6), round(loss_gpu[0], 6)],
               loss_last=[round(loss_cpu[-1], 6), round(loss_gpu[-1], 6)],
               reference=("CPU chain: oracle/decode_ref.decode_torch (pinned to tests/golden/decode_*.npz) -> "
                          f"C-oracle rasterization{'_2dgs' if gs == '2d' else ''} (oracle/autograd.py) -> "
                          "oracle/loss_ref.loss (pinned to tests/golden/losses.npz) -> torch.optim.Adam(eps=1e-15); "
                          "fine-stage loss weights (config/base/small_scene/fine.yaml), its learning rates x "
                          f"{ls}"))
    os.makedirs("gpurun_out", exist_ok=True)
    with open(os.path.join("gpurun_out", f"psnr_pipeline_{gs}gs.json"), "w") as f:
        json.dump(res, f)
    print(res)
    # the first losses see identical parameters: the two chains agree before any divergence
    assert abs(loss_gpu[0] - loss_cpu[0]) <= 1e-5 + 1e-4 * abs(loss_cpu[0]), res
    assert win_cpu > psnr_init + 10.0  # the fit actually fits
    # the chain's own noise floor (a 1e-6 perturbation of its initialisation) is below the bar
    assert abs(win_self - win_cpu) <= 0.05, res
    assert abs(win_gpu - win_cpu) <= 0.05, res


def test_psnr_parity_pipeline_3dgs():
    _pipeline_parity("3d")


def test_psnr_parity_pipeline_2dgs():
    _pipeline_parity("2d")


@pytest.mark.parametrize("gs", ["3d", "2d"])
def test_pipeline_step_gradients(gs):
    """One step of the PSNR-parity pipeline (tests/pipeline_fit.py) at its initial parameters: the
    loss and the gradient of every trained tensor (anchor features, offsets, scalings, the twelve
    MLP tensors) of the HIP chain against the CPU chain in f32 (checker) and f64 (truth), per
    element with conditioning (oracle/checks.cond_close).  The per-step statement behind the
    equal-iteration PSNR comparison."""
    from oracle.checks import cond_close
    from tests import pipeline_fit as PF
    W, H = 160, 120
    gt = PF.target(40000, W, H, seed=31, gs=gs)
    p0, cfg = PF.anchor_model(5000, W, H, seed=32, param_seed=200)
    res = {}
    for name, dev, dt in (("gpu", "cuda", None), ("f32", "cpu", torch.float32), ("f64", "cpu", torch.float64)):
        p = {k: v.to(dev).clone().requires_grad_(k != "anchor") for k, v in p0.items()}
        c = dict(cfg)
        if dt is not None:
            c["dtype"] = dt
        loss = (PF.gpu_loss if dev == "cuda" else PF.cpu_loss)(p, c, gt.to(dev), gs)[0]
        loss.backward()
        res[name] = (float(loss), {k: v.grad.detach().cpu().double().numpy() for k, v in p.items() if k != "anchor"})
    cond_close(np.array([res["gpu"][0]]), np.array([res["f32"][0]]), np.array([res["f64"][0]]), "loss")
    for k in res["gpu"][1]:
        cond_close(res["gpu"][1][k], res["f32"][1][k], res["f64"][1][k], "d_" + k)


# ----------------------------------------------------------------------------- at scale
MIN_ENSEMBLE = 8  # reference-chain members (unperturbed + 1e-6-perturbed draws) a fixed bar needs


def _hip_fit(p0, cfg, gt, iters, gs, gold):
    from tests import pipeline_fit as PF
    return PF.fit(p0, cfg, gt, iters, gs=gs, device="cuda", window=gold["window"], lr_scale=gold["lr_scale"])


def _parity_at_scale(gs, fixture=None, chaotic=False):
    """PSNR parity at scale: 50k anchors at 480x270, 500 iterations of the whole train step
    (reference train.py:150-277; PSNR as utils/image_utils.py:18-20 over the renders of the last
    50 iterations) at the fixture's multiple of the fine-stage learning rates.  The CPU reference
    chain takes ~3-7 s per iteration, so its results are committed fixtures
    (tests/golden/psnr_scale_{gs}[_lrNN].json, scripts/psnr_at_scale.py with the same seeds).

    Both chains are f32 evaluations of a chaotic map: any rounding difference, a 1e-6
    perturbation of the initialisation or a different summation order, moves the final PSNR by
    a draw of the chain's own spread.  So the comparison is between ENSEMBLES: the reference
    chain's unperturbed run and its runs from initialisations perturbed by 1e-6 with seeds
    5..12 (scripts/psnr_ensemble_run.sh + scripts/psnr_ensemble.py: "ensemble" in the fixture),
    and the HIP chain from the same initialisations, here.  Since round 6 the HIP chain is
    bit-reproducible (deterministic raster backwards), so its ensemble is a fixed fact of the
    code, not a random draw per run.
    The window PSNR has a heavy lower tail: a transient loss spike inside the 50-iteration window
    (Adam overshooting on a few Gaussians, recovered within ~20 iterations) costs a draw up to
    ~0.8 dB (2DGS seed 12: window MSE 5.0e-5 -> 1.08e-4 at iteration 451, back by 470,
    gpurun_out/seedtrace12.json; its final iterate is unaffected, 43.30 dB).  One such draw
    dominates a 9-member mean and sd, so the ensembles are compared by ROBUST statistics:
      * the ensemble medians must agree within 0.05 dB -- a fixed bar, not widened by either
        chain's noise (this is the PSNR delta the metric states);
      * the HIP chain's robust spread (1.4826 x the median absolute deviation) must stay within
        3x the reference chain's + 0.01 dB (a 6x more sensitive chain fails);
      * at most one HIP draw may sit more than 0.3 dB below the reference median (the reference
        ensembles span <= 0.08 dB): a chain that spikes systematically fails;
      * means and sds are recorded beside them;
      * the unperturbed pair is one draw of each chain: its delta is recorded against the
        reference ensemble's spread, not bounded -- with the chains' own spreads at 0.02-0.04 dB
        (2DGS) a single draw sits outside 0.05 dB of another in a sizeable fraction of runs
        whichever implementation produced it.
    A fixture without a full ensemble (>= MIN_ENSEMBLE members) keeps the single-draw bar
    (0.05 dB, or twice the reference chain's own 1e-6 floor when that is larger).
    chaotic (the unscaled learning rates, where a 1e-6 perturbation moves the reference chain's
    window PSNR by ~1 dB): a fixed 0.05 dB bar on the medians is below what 8 draws of either
    chain can resolve, so the medians must agree within 3 standard errors of the difference
    computed from the REFERENCE ensemble's sd (3 x 1.2533 sd_ref sqrt(1/n_ref + 1/n_hip), the
    median's standard error); the spreads are compared by the two-sided 1% F-test of equal
    variances on the classical sds (sd_hip / sd_ref <= sqrt(F_0.995(n_hip - 1, n_ref - 1)), 2.98 at
    8 + 8 members), since the draws there are a wide distribution, not a narrow one with rare
    spikes, and the median-absolute-deviation spread of 8 such draws is too noisy an estimate
    for a 3x bar (the reference's own: 0.57 dB robust vs 0.97 dB classical); no outlier count
    applies (draws 1 dB apart are that chain's nature)."""
    import statistics

    from scripts import psnr_at_scale as PS
    fixture = fixture or f"psnr_scale_{gs}"
    gold = json.load(open(os.path.join(os.path.dirname(__file__), "golden", f"{fixture}.json")))
    A, W, H, iters = gold["anchors"], gold["width"], gold["height"], gold["iterations"]
    assert gold["seeds"] == PS.SEEDS
    gt, p0, cfg, _ = PS.problem(A, W, H, gs)
    fin_gpu, win_gpu, loss_gpu = _hip_fit(p0, cfg, gt, iters, gs, gold)
    ref = gold["ref"]
    ens = {int(k): v for k, v in gold.get("ensemble", {"5": gold["ref_perturbed_1e-6"]}).items()}
    hip_ens = {}
    # a fixture without a reference ensemble (the unscaled rates) still gets the HIP chain's full
    # spread over seeds 5..12: its sensitivity is then a measured sd, not one draw
    hip_seeds = sorted(ens) if len(ens) > 1 else list(range(5, 13))
    for seed in hip_seeds:
        _, w, _ = _hip_fit(PS.perturbed(p0, seed), cfg, gt, iters, gs, gold)
        hip_ens[seed] = round(w, 4)
    ref_w = [ref["window_db"]] + [ens[s]["window_db"] for s in sorted(ens)]
    hip_w = [win_gpu] + [hip_ens[s] for s in hip_seeds]
    full = len(ref_w) >= MIN_ENSEMBLE
    sd_ref, sd_hip = statistics.stdev(ref_w), statistics.stdev(hip_w)
    mean_delta = statistics.mean(hip_w) - statistics.mean(ref_w)
    med_ref, med_hip = statistics.median(ref_w), statistics.median(hip_w)
    med_delta = med_hip - med_ref
    rsd_ref = 1.4826 * statistics.median([abs(x - med_ref) for x in ref_w])
    rsd_hip = 1.4826 * statistics.median([abs(x - med_hip) for x in hip_w])
    n_low = sum(1 for x in hip_w if x < med_ref - 0.3)
    mean_bar = 0.05
    spread, spread_bar, spread_kind = rsd_hip, 3.0 * rsd_ref + 0.01, "robust sd hip"
    if chaotic:
        from scipy.stats import f as fdist
        assert full, "the chaotic case needs the reference ensemble"
        mean_bar = 3.0 * 1.2533 * sd_ref * math.sqrt(1.0 / len(ref_w) + 1.0 / len(hip_w))
        spread, spread_kind = sd_hip / sd_ref, "sd ratio hip / ref (F-test 1%)"
        spread_bar = math.sqrt(fdist.ppf(0.995, len(hip_w) - 1, len(ref_w) - 1))
    if full:
        bar_single = None  # the single pair is recorded, the ensembles are bounded
    else:
        bar_single = max(0.05, 2.0 * abs(gold["noise_floor_window_db"]))
    res = dict(psnr_init_db=gold["psnr_init_db"], psnr_ref_db=ref["window_db"], psnr_hip_db=round(win_gpu, 4),
               psnr_delta_db=round(win_gpu - ref["window_db"], 4), psnr_metric="mean MSE of the last 50 iterations' renders",
               ensemble={"members": len(ref_w), "seeds": sorted(ens), "hip_seeds": hip_seeds, "ref_window_db": ref_w,
                         "hip_window_db": hip_w,
                         "ref_mean_db": round(statistics.mean(ref_w), 4), "hip_mean_db": round(statistics.mean(hip_w), 4),
                         "mean_delta_db": round(mean_delta, 4), "ref_sd_db": round(sd_ref, 4),
                         "hip_sd_db": round(sd_hip, 4), "ref_median_db": round(med_ref, 4),
                         "hip_median_db": round(med_hip, 4), "median_delta_db": round(med_delta, 4),
                         "ref_robust_sd_db": round(rsd_ref, 4), "hip_robust_sd_db": round(rsd_hip, 4),
                         "hip_draws_0p3_below_ref_median": n_low, "median_bar_db": round(mean_bar, 4),
                         "median_bar_kind": ("3 x the median's standard error of the difference from the reference sd"
                                             if chaotic else "fixed"),
                         "spread_kind": spread_kind, "spread": round(spread, 4), "spread_bar": round(spread_bar, 4)},
               final_iterate={"ref_db": ref["final_db"], "hip_db": round(fin_gpu, 4),
                              "delta_db": round(fin_gpu - ref["final_db"], 4)},
               bar_db=(round(mean_bar, 4) if full else round(bar_single, 4)),
               bar_source=(("ensemble medians within 3 standard errors of their difference; sd_hip / sd_ref within "
                            "the two-sided 1% F-test bound; means / robust sds and the unperturbed pair recorded")
                           if chaotic else
                           "ensemble medians within 0.05 dB; HIP robust sd <= 3 x the reference's + 0.01 dB; <= 1 HIP "
                           "draw 0.3 dB below the reference median; means / sds and the unperturbed pair recorded"
                           if full else "single reference draw: 2 x its 1e-6 floor (0.05 dB at least)"),
               single_pair_vs_ref_ensemble_sd=(round((win_gpu - ref["window_db"]) / sd_ref, 2) if sd_ref > 0 else None),
               iterations=iters, anchors=A, width=W, height=H, lr_scale=gold["lr_scale"],
               loss_first=[round(ref["loss_first"], 6), round(loss_gpu[0], 6)],
               loss_last=[round(ref["loss_last"], 6), round(loss_gpu[-1], 6)],
               reference=f"tests/golden/{fixture}.json (scripts/psnr_at_scale.py: the CPU chain of "
                         "tests/pipeline_fit.py, reference-pinned decode + loss, C-oracle rasterizer, torch Adam)")
    os.makedirs("gpurun_out", exist_ok=True)
    with open(os.path.join("gpurun_out", f"{fixture}_{gs}gs.json".replace(f"psnr_scale_{gs}_", "psnr_scale_")), "w") as f:
        json.dump(res, f)
    print(res)
    # the first line of every failure states the numbers and the bars (the driver keeps a tail)
    head = (f"{fixture}: median delta {med_delta:+.4f} dB (bar {mean_bar:.4f}); {spread_kind} {spread:.4f} (bar "
            f"{spread_bar:.4f}; robust sd ref {rsd_ref:.4f}); hip draws 0.3 dB low {n_low} (bar {'-' if chaotic else 1}); mean "
            f"delta {mean_delta:+.4f}, sd hip / ref {sd_hip:.4f} / {sd_ref:.4f}; single pair "
            f"{win_gpu - ref['window_db']:+.4f} dB{'' if full else f' (bar {bar_single:.4f})'}; first loss "
            f"{loss_gpu[0]:.6f} vs {ref['loss_first']:.6f}\n")
    # identical parameters at the first step: the chains agree before any divergence
    assert abs(loss_gpu[0] - ref["loss_first"]) <= 1e-5 + 1e-4 * abs(ref["loss_first"]), head + str(res)
    assert ref["window_db"] > gold["psnr_init_db"] + 5.0 and win_gpu > gold["psnr_init_db"] + 5.0, head  # both fit
    if full:
        assert abs(med_delta) <= mean_bar, head + str(res)
        assert spread <= spread_bar, head + str(res)
        if not chaotic:
            assert n_low <= 1, head + str(res)
    else:
        assert abs(win_gpu - ref["window_db"]) <= bar_single, head + str(res)


@pytest.mark.slow
def test_psnr_parity_at_scale_3dgs():
    _parity_at_scale("3d")


@pytest.mark.slow
def test_psnr_parity_at_scale_2dgs():
    _parity_at_scale("2d")


@pytest.mark.slow
def test_psnr_parity_at_scale_3dgs_lr03():
    """The 3DGS chain at 0.3x the fine-stage learning rates, against a 9-member reference ensemble
    (unperturbed + 1e-6 perturbations, seeds 5-12: window sd 0.053 dB, scripts/psnr_ensemble_lr03.sh)
    with the full-ensemble bars of _parity_at_scale."""
    _parity_at_scale("3d", "psnr_scale_3d_lr03")


@pytest.mark.slow
def test_psnr_parity_at_scale_3dgs_unscaled():
    """The unscaled fine-stage learning rates: the 3DGS chain is chaotic -- the reference
    chain's 8-member ensemble (unperturbed + 1e-6 perturbations, seeds 5-11) spreads 0.97 dB sd
    in window PSNR and 2.0 dB in the final iterate -- so the ensemble means are compared at 3
    standard errors of their difference (from the reference sd: ~1.8 dB with 8 + 8 members) and
    the spreads by the two-sided 1% F-test (sd ratio <= 2.98; gpurun_out/psnr_scale_lr1_3dgs.json:
    medians 42.985 / 42.968 dB, sds 1.82 / 0.97 dB, the HIP chain being bit-reproducible these
    are fixed numbers of the code).
    The tight fixed 0.05 dB bar is on the 0.1x and 0.3x fixtures, where the chains are not chaotic."""
    _parity_at_scale("3d", "psnr_scale_3d_lr1", chaotic=True)
