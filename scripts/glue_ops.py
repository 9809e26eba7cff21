"""Attribute the torch (non-hgsr) device work of one bench train step to the Python lines that
launch it: torch.profiler over a few steps of bench.Workload, printing every aten op that ran a
device kernel with its kernel count and the innermost repo stack frame.
Usage (GPU box): python scripts/glue_ops.py [--gs 3d|2d] [--config c2|c2-anchors|...]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
from torch.profiler import ProfilerActivity, profile  # noqa: E402

import bench  # noqa: E402


def main():
    args = bench.resolve(bench.parse(sys.argv[1:] + ["--no-secondary", "--no-timing"]), 1)
    dev = torch.device("cuda", 0)
    wl = bench.Workload(args, 0, dev)
    for _ in range(3):
        wl.step()
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
        for _ in range(2):
            wl.step()
        torch.cuda.synchronize()
    rows = {}
    for ev in prof.events():
        if ev.device_type.name != "CPU" or not ev.name.startswith("aten::"):
            continue
        kern = [k for k in ev.kernels] if hasattr(ev, "kernels") else []
        if not kern:
            continue
        frames = [f for f in (ev.stack or []) if ROOT in f and "glue_ops.py" not in f]
        where = frames[0].replace(ROOT + "/", "") if frames else ""
        # inside the backward there is no Python stack: name the autograd node / parent ops
        par, chain = ev.cpu_parent, []
        while par is not None and len(chain) < 3:
            chain.append(par.name.replace("autograd::engine::evaluate_function: ", "bwd:"))
            par = par.cpu_parent
        where = (where + " " + " < ".join(chain)).strip() or "?"
        key = (ev.name, where)
        r = rows.setdefault(key, [0, 0.0, set()])
        r[0] += len(kern)
        r[1] += sum(k.duration for k in kern)
        r[2].update(k.name[:60] for k in kern)
    for (name, where), (n, us, ks) in sorted(rows.items(), key=lambda kv: -kv[1][1]):
        print(f"{us / 2:8.1f} us/step  {n / 2:4.1f} kernels/step  {name:28s} {where}  [{'; '.join(sorted(ks))[:120]}]")


if __name__ == "__main__":
    main()
