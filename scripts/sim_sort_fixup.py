"""CPU design study for tile_sort's 32-bit path (isect.hip sort32_and_emit): sort each bin by
(depth bits >> SHIFT, emission index), then count the odd-even transposition passes (even +
odd phase) needed to reach the exact (depth, flatten id) order, on the seeded c2 scene.
Result on the c2 scene (SHIFT 10, 21-bit depth): at most 2 passes in every sampled bin."""
import sys

import numpy as np

sys.path.insert(0, ".")
from horizongs_amd.synthetic import make_scene  # noqa: E402
from oracle import oracle as O  # noqa: E402

sc = make_scene(2_000_000, 1920, 1080, seed=0)
r, m2, d, _ = O.proj3d_fwd(sc.means.numpy(), sc.quats.numpy(), sc.scales.numpy(), sc.viewmats.numpy(),
                           sc.Ks.numpy(), 1920, 1080)
tw, th = O.tile_grid(1920, 1080)
_, ids, fl = O.isect_tiles(m2, r, d, 16, tw, th)
offs = O.isect_offsets(ids, 1, tw, th).reshape(-1)
db = d.reshape(-1).view(np.uint32)
rng = np.random.default_rng(0)
for shift in (8, 9, 10, 11):
    passes = []
    for b in rng.choice(len(offs) - 1, 400, replace=False):
        f = fl[offs[b]:offs[b + 1]].astype(np.int64)
        perm = rng.permutation(len(f))  # emission order inside a bin is arbitrary
        fk = ((db[f].astype(np.int64) << 32) | f)[perm]
        k32 = ((db[f[perm]].astype(np.int64) >> shift) << 11) | np.arange(len(f))
        seq = fk[np.argsort(k32, kind="stable")]
        p = 0
        while not np.all(seq[:-1] < seq[1:]) and p <= 20:
            for st in (0, 1):
                a, bb = seq[st:-1:2].copy(), seq[st + 1::2][: len(seq[st:-1:2])].copy()
                sw = a > bb
                seq[st:-1:2][: len(a)] = np.where(sw, bb, a)
                seq[st + 1::2][: len(a)] = np.where(sw, a, bb)
            p += 1
        passes.append(p)
    passes = np.array(passes)
    print(f"shift {shift} ({31 - shift}-bit depth): passes mean {passes.mean():.2f} max {passes.max()}")
