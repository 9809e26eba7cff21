"""Limiter breakdown of the raster backwards from a gpu_r04_prof.sh run (developer tool).

usage: python scripts/limiter_summary.py gpurun_out/r05prof gpurun_out/<suite>/bench.json r05 > profiles/r05_pmc_raster_limiters.txt
Reads the l3 / l2 PMC summaries (scripts/pmc_summary.py output), profiles/<tag>_pmc_traffic.json,
the LDS-pipe passes d3 / d2 when the run has them and the bench line's evaluated-pair counter.  SQ_WAVE_CYCLES / SQ_WAIT_* count quad-cycles
(MI355X_MICROARCH.md, PMC table); kernel cycles = GRBM_GUI_ACTIVE / 8 XCDs.
"""
import json
import os
import subprocess
import sys

root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
src, bench = sys.argv[1], sys.argv[2]
tag = sys.argv[3] if len(sys.argv) > 3 else "r04"
b = json.loads(open(bench).read().strip().splitlines()[-1])
roof = b["roofline"]
steps = roof["pairs_evaluated_per_launch"] / 64
nis = roof["n_isects"]


def counters(d, kernel_has="bwd"):
    """pmc_summary.py's averages for the kernel whose name contains kernel_has"""
    out = subprocess.run([sys.executable, os.path.join(root, "scripts", "pmc_summary.py"), d], capture_output=True,
                         text=True).stdout
    L, cur = {}, None
    for line in out.splitlines():
        if not line.startswith(" "):
            cur = line.split()[0] if line.strip() else None
            continue
        p = line.split()
        if len(p) == 2 and cur and kernel_has in cur:
            L[p[0]] = float(p[1])
    return L, out


pm = json.load(open(os.path.join(root, "profiles", f"{tag}_pmc_traffic.json")))["kernels"]
lines = [f"{tag} limiter breakdown of the raster backwards (scripts/gpu_{tag}_prof.sh: rocprofv3 --pmc SQ_WAVES "
         "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_LDS "
         "GRBM_GUI_ACTIVE, one pass per config; FETCH_SIZE / WRITE_SIZE from separate passes, "
         f"profiles/{tag}_pmc_traffic.json).  SQ_WAVE_CYCLES / SQ_WAIT_* count quad-cycles; kernel cycles = "
         "GRBM_GUI_ACTIVE / 8 XCDs.", ""]
raw = ["", "raw counters (per launch):"]
P = 1920 * 1080
for ptag, gs, name, occ, rows_mb, alg in (
        ("l3", "3dgs", "raster3d_bwd, c2 (2M Gaussians, 1080p)", "7 (72 VGPRs, 22 KB LDS)",
         2e6 * (48 if tag == "r04" else 64) / 1e6, (44 * nis + 28 * P) / 1e6 if tag < "r06" else
         (56 * nis + 28 * P + 65 * steps) / 1e6),
        ("l2", "2dgs", "raster2d_bwd (transposed inputs), c3", "5 (96 VGPRs, 29 KB LDS)", 2e6 * 96 / 1e6, None)):
    L, txt = counters(os.path.join(src, ptag))
    raw += txt.splitlines()
    kname = [k for k in pm[gs] if k.startswith(name.split(",")[0].split(" ")[0])]
    kname = [k for k in kname if "bwd" in k][0]
    k = pm[gs][kname]
    t_us = k["avg_us"]
    cyc = L["GRBM_GUI_ACTIVE"] / 8
    wc = L["SQ_WAVE_CYCLES"]
    lines.append(f"== {name} [{kname}]: {t_us:.1f} us under rocprofv3, effective clock {cyc / (t_us * 1e-6) / 1e9:.2f} GHz")
    lines.append(f"   waves / SIMD: compiled occupancy {occ}; resident on average {wc * 4 / (1024 * cyc):.2f}")
    lines.append(f"   SQ_INSTS_VALU {L['SQ_INSTS_VALU']:.4g} per launch = {L['SQ_INSTS_VALU'] / t_us / 1e3:.0f} G "
                 f"wave-instr/s ({L['SQ_INSTS_VALU'] / t_us / 1e3 / 935:.2f} of the 935 G/s v_fma_f32 issue ceiling)")
    if gs == "3dgs":
        lines.append(f"   per wave-step: {L['SQ_INSTS_VALU'] / steps:.1f} VALU, {L['SQ_INSTS_LDS'] / steps:.2f} LDS "
                     f"instructions ({steps / 1e6:.2f}M wave-steps = evaluated pairs / 64)")
    lines.append(f"   wave time: parked on s_waitcnt / barrier (SQ_WAIT_ANY) {L['SQ_WAIT_ANY'] / wc:.1%}, issue-stalled "
                 f"(SQ_WAIT_INST_ANY) {L['SQ_WAIT_INST_ANY'] / wc:.1%}, issuing {1 - (L['SQ_WAIT_ANY'] + L['SQ_WAIT_INST_ANY']) / wc:.1%}")
    lines.append(f"   HBM: 2 x FETCH_SIZE {2 * k['fetch_size_raw_bytes'] / 1e6:.1f} MB + WRITE_SIZE {k['write_size_bytes'] / 1e6:.1f} MB"
                 f" = {k['hbm_bytes_corrected'] / 1e6:.1f} MB / launch"
                 + (f" against {alg:.0f} MB algorithmic ({k['hbm_bytes_corrected'] / 1e6 / alg:.2f}x)" if alg else ""))
    if tag < "r06":
        lines.append(f"   WRITE_SIZE {k['write_size_bytes'] / 1e6:.1f} MB vs {rows_mb:.0f} MB of accumulator rows "
                     f"({k['write_size_bytes'] / 1e6 / rows_mb:.1f}x: float atomics of every (wave, Gaussian) group meet in L2)")
    elif gs == "3dgs":
        # round 6: one plain 64-B gradient-slot row + a flag byte per wave-list entry (no atomics);
        # algorithmic above = 56 B of each 64-B record per intersection + 28 B per pixel + those rows
        lines.append(f"   WRITE_SIZE {k['write_size_bytes'] / 1e6:.1f} MB vs {65 * steps / 1e6:.0f} MB of gradient-slot rows "
                     f"and flags ({k['write_size_bytes'] / 1e6 / (65 * steps / 1e6):.2f}x); reads "
                     f"{2 * k['fetch_size_raw_bytes'] / 1e6:.0f} MB vs {(56 * nis + 28 * P) / 1e6:.0f} MB of records and pixels "
                     f"({2 * k['fetch_size_raw_bytes'] / (56 * nis + 28 * P):.2f}x)")
    dpass = os.path.join(src, "d3" if gs == "3dgs" else "d2")
    if os.path.isdir(dpass):
        D, dtxt = counters(dpass)
        raw += dtxt.splitlines()
        if "SQ_LDS_IDX_ACTIVE" in D:
            dc = D["GRBM_GUI_ACTIVE"] / 8
            lines.append(f"   LDS (separate pass): array busy "
                         f"{D['SQ_LDS_IDX_ACTIVE'] / (256 * dc):.2f} of capacity, bank-conflict cycles "
                         f"{D['SQ_LDS_BANK_CONFLICT'] / D['SQ_LDS_IDX_ACTIVE']:.2f} of them")
print("\n".join(lines + raw))
