"""Design study (CPU, oracle forward): backward wave-steps of the 3DGS raster for different
pixel-block shapes per list.  For every tile of the c2 scene and every pixel block B of a
candidate partition, list(B) = the tile's Gaussians t with t <= max last contributor over B
and alpha >= 1/255 somewhere on B; a wave processing several blocks side by side steps
max_B |list(B) within a 128-record batch| per batch.

    python scripts/sim_lists.py [n_gaussians]
"""
import sys
import time

import numpy as np

sys.path.insert(0, ".")
from horizongs_amd.synthetic import make_scene  # noqa: E402
from oracle.pipeline import Raster3D  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 2_000_000
W, H, TS = 1920, 1080, 16
sc = make_scene(n, W, H, seed=0)
t0 = time.time()
r = Raster3D(sc.means.numpy(), sc.quats.numpy(), sc.scales.numpy(), sc.opacities.numpy(), sc.colors.numpy(),
             sc.viewmats.numpy(), sc.Ks.numpy(), W, H, backgrounds=np.zeros((1, 3), np.float32))
r.forward()
print(f"oracle forward {time.time() - t0:.1f}s", flush=True)
offs = r.offsets.reshape(-1).astype(np.int64)
n_is = r.flatten_ids.shape[0]
tw, th = r.tw, r.th
nt = tw * th
ends = np.append(offs[1:], n_is)
tile_of = np.repeat(np.arange(nt), ends - offs)
g = r.flatten_ids.astype(np.int64) % n
m2 = r.means2d.reshape(-1, 2)[g]
con = r.conics.reshape(-1, 3)[g]
op = r.opac_c.reshape(-1)[g]
last = r.last.reshape(H, W).astype(np.int64)
lim = np.log(255.0 * op)  # alpha >= 1/255  <=>  sigma <= ln(255 o)
ty, tx = tile_of // tw, tile_of % tw
# per 4x4 block reach flags (16 per tile) and block finals
B4 = 4
reach = np.zeros((16, n_is), bool)
lastp = np.full((th * TS, tw * TS), -1, np.int64)
lastp[:H, :W] = last
fin4 = lastp.reshape(th * 4, B4, tw * 4, B4).max(axis=(1, 3))  # [th*4, tw*4]
a, b, c = con[:, 0], con[:, 1], con[:, 2]


def minsig(x0, x1, y0, y1):
    """min over the pixel-centre rectangle of 0.5 a dx^2 + b dx dy + 0.5 c dy^2 (dx = x - mx)."""
    q = lambda dx, dy: 0.5 * a * dx * dx + b * dx * dy + 0.5 * c * dy * dy  # noqa: E731
    dya = np.clip(-b * x0 / c, y0, y1)
    dyb = np.clip(-b * x1 / c, y0, y1)
    dxa = np.clip(-b * y0 / a, x0, x1)
    dxb = np.clip(-b * y1 / a, x0, x1)
    m = np.minimum(np.minimum(q(x0, dya), q(x1, dyb)), np.minimum(q(dxa, y0), q(dxb, y1)))
    inside = (x0 <= 0) & (x1 >= 0) & (y0 <= 0) & (y1 >= 0)
    return np.where(inside, 0.0, m)


t0 = time.time()
for by in range(4):
    for bx in range(4):
        px0 = tx * TS + bx * 4 + 0.5
        py0 = ty * TS + by * 4 + 0.5
        x0, x1 = px0 - m2[:, 0], px0 + 3 - m2[:, 0]
        y0, y1 = py0 - m2[:, 1], py0 + 3 - m2[:, 1]
        reach[by * 4 + bx] = minsig(x0, x1, y0, y1) <= lim
print(f"reach {time.time() - t0:.1f}s", flush=True)
tidx = np.arange(n_is, dtype=np.int64)
# block finals per intersection
fin = np.stack([fin4[ty * 4 + by, tx * 4 + bx] for by in range(4) for bx in range(4)])  # [16, n_is]
ok4 = reach & (tidx[None] <= fin)  # item t is stepped by the 4x4 block


def union(blocks):
    return np.any(np.stack([reach[k] for k in blocks]), 0) & (tidx <= np.max(np.stack([fin[k] for k in blocks]), 0))


quads = [[0, 1, 4, 5], [2, 3, 6, 7], [8, 9, 12, 13], [10, 11, 14, 15]]
ok8 = [union(q) for q in quads]
halves_h = [[0, 1], [4, 5], [2, 3], [6, 7], [8, 9], [12, 13], [10, 11], [14, 15]]  # 8 wide x 4 tall
ok84 = [union(h) for h in halves_h]
halves_v = [[0, 4], [1, 5], [2, 6], [3, 7], [8, 12], [9, 13], [10, 14], [11, 15]]  # 4 wide x 8 tall
ok48 = [union(h) for h in halves_v]
# tile-level effective end: max final over the tile
tile_fin = lastp.reshape(th, TS, tw, TS).max(axis=(1, 3)).reshape(-1)
end_eff = np.minimum(ends, tile_fin + 1)
batch = np.where(tidx[None] >= 0, (end_eff[tile_of] - 1 - tidx) // 128, 0)[0]
key = tile_of * 64 + np.clip(batch, 0, 63)
nk = nt * 64


def steps_group(oks):
    """wave-steps when the blocks in `oks` share one wave: sum over (tile, batch) of the max count."""
    cnt = np.stack([np.bincount(key[o], minlength=nk) for o in oks])
    return cnt.max(0).sum()


s8 = sum(int(o.sum()) for o in ok8)
s84 = sum(steps_group([ok84[2 * w], ok84[2 * w + 1]]) for w in range(4))
s48 = sum(steps_group([ok48[2 * w], ok48[2 * w + 1]]) for w in range(4))
s44 = sum(steps_group([ok4[k] for k in q]) for q in quads)
s44_sum = int(ok4.sum())
print(f"intersections {n_is}  (tile mean {n_is / nt:.0f})")
print(f"8x8 per wave (current):         wave-steps {s8 / 1e6:.2f} M")
print(f"2 x (8 wide x 4 tall) per wave: wave-steps {s84 / 1e6:.2f} M  ({s84 / s8:.3f})")
print(f"2 x (4 wide x 8 tall) per wave: wave-steps {s48 / 1e6:.2f} M  ({s48 / s8:.3f})")
print(f"4 x (4x4) per wave:             wave-steps {s44 / 1e6:.2f} M  ({s44 / s8:.3f});  sum of 4x4 lists {s44_sum / 1e6:.2f} M")
