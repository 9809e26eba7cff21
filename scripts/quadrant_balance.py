"""How evenly the four waves of a raster3d_bwd workgroup share a batch (GPU; diagnostics).

The backward walks each tile's list in 128-record batches with two workgroup barriers per batch;
wave w steps only the records the forward's culling marked for its 8x8 quadrant (the qmask
bits).  A batch lasts as long as its longest wave list, so sum(mean) / sum(max) over batches is
the fraction of the waves' batch time spent stepping rather than waiting at the barrier for a
sibling.  Lists are counted in 4-step groups (the backward's pass-2 granularity) and over each
tile's whole bin (the backward's further trim to the latest contributor is ignored).

usage: python scripts/quadrant_balance.py > gpurun_out/quadrant_balance.jsonl
"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from horizongs_amd import gsplat_api as G  # noqa: E402
from horizongs_amd.synthetic import camera_set, make_scene  # noqa: E402

NB = 128  # kBwdBatch (csrc/raster3d.hip)


def main():
    dev = "cuda:0"
    W, H = 1920, 1080
    sc = make_scene(2_000_000, W, H, seed=0)
    cams = camera_set(16).to(dev)
    Ks = sc.Ks.to(dev)
    ps = [t.to(dev).clone().requires_grad_(True) for t in (sc.means, sc.quats, sc.scales, sc.opacities, sc.colors)]
    for v in range(0, 16, 3):
        rc, ra, meta = G.rasterization(*ps, cams[v][None], Ks, W, H, packed=False, render_mode="RGB+ED")
        node = rc.grad_fn
        while node is not None and not hasattr(node, "qmask"):
            node = node.next_functions[0][0] if node.next_functions else None
        qm = node.qmask.cpu().numpy()
        offs = meta["isect_offsets"].reshape(-1).long().cpu().numpy()
        n = int(meta["flatten_ids"].numel())
        nb = offs.size
        cnt = np.diff(np.append(offs, n))
        order_b = 2 * ((nb * 4 + 255) // 256 * 256)  # tile_order_bytes: [order | tile_end]
        words = qm[order_b:].view(np.uint64)
        qstride = words.size // 4
        bits = np.unpackbits(words[:4 * qstride].reshape(4, qstride).view(np.uint8), axis=1, bitorder="little")
        binid = np.repeat(np.arange(nb), cnt)
        rel = np.arange(n) - offs[binid]
        word0 = (offs + 63) // 64 + np.arange(nb) + 2  # qmask_word0(start, bin)
        bit_idx = word0[binid] * 64 + rel
        batch = (cnt[binid] - 1 - rel) // NB  # the backward walks each list from its end
        key = binid.astype(np.int64) * 4096 + batch
        uk, inv = np.unique(key, return_inverse=True)
        c = np.stack([np.bincount(inv, weights=bits[w, bit_idx], minlength=uk.size) for w in range(4)])
        g = np.ceil(c / 4.0) * 4.0  # 4-step groups
        used = g.sum(axis=0) > 0
        g = g[:, used]
        rec = {"view": v, "isects": n, "batches": int(used.sum()),
               "wave_steps_mean_over_max": round(float(g.mean(axis=0).sum() / g.max(axis=0).sum()), 4),
               "steps_per_batch_mean": round(float(g.mean()), 2),
               "batches_with_an_idle_wave": round(float((g.min(axis=0) == 0).mean()), 4)}
        print(json.dumps(rec), flush=True)
        del rc, ra, meta, node


if __name__ == "__main__":
    main()
