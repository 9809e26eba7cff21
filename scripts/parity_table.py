"""Element-wise strict parity table from a GPU-suite run (TEST INFRASTRUCTURE: reads the JSON
lines tests/parity_report.py appends during the raster parity tests).

usage: python scripts/parity_table.py gpurun_out/<tag>/parity_strict.jsonl > profiles/r04_parity_strict.txt

Prints every tensor row, then the exceptions to "the GPU is worse than the gsplat-form f32
oracle on <= 1e-3 of the elements" with the mirror figure (the oracle worse than the GPU) and
the kernel-form comparison next to each, which is what explains them.
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tests.parity_report import table  # noqa: E402

rows = [json.loads(line) for line in open(sys.argv[1])]
print(table(rows))
print()
exc = [r for r in rows if r["worse_g32"] > 1e-3]
print(f"{len(exc)} of {len(rows)} tensors have worse_g32 > 1e-3 (all gradients; no image, depth, alpha or "
      f"normal map does):")
print(f"{'test':40s} {'tensor':16s} {'worse_g32':>10s} {'better_g32':>10s} {'worse_k32':>10s} {'better_k32':>10s}")
for r in exc:
    print(f"{r['test'][:40]:40s} {r['tensor'][:16]:16s} {r['worse_g32']:10.6f} {r.get('better_g32', float('nan')):10.6f} "
          f"{r['worse_k32']:10.6f} {r.get('better_k32', float('nan')):10.6f}")
imgs = [r for r in rows if not r["tensor"].startswith("v_")]
grads = [r for r in rows if r["tensor"].startswith("v_")]
print()
print(f"images / maps: max worse_g32 {max(r['worse_g32'] for r in imgs):.2e}, "
      f"max worse_k32 {max(r['worse_k32'] for r in imgs):.2e} over {len(imgs)} tensors")
if grads and all("better_g32" in r for r in grads):
    wg = sum(r["worse_g32"] * r["n"] for r in grads) / sum(r["n"] for r in grads)
    bg = sum(r["better_g32"] * r["n"] for r in grads) / sum(r["n"] for r in grads)
    wk = sum(r["worse_k32"] * r["n"] for r in grads) / sum(r["n"] for r in grads)
    bk = sum(r["better_k32"] * r["n"] for r in grads) / sum(r["n"] for r in grads)
    print(f"gradients, element-weighted over {len(grads)} tensors: GPU worse than gsplat-f32 on {wg:.4f}, "
          f"gsplat-f32 worse than GPU on {bg:.4f}; GPU worse than kernel-form f32 on {wk:.4f}, "
          f"kernel-form worse than GPU on {bk:.4f}")
