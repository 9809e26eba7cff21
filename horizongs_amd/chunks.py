"""Per-chunk training on N GPUs: the launcher and the merge (SURVEY.md §8(e) mapping 1).

The reference trains a large scene as m x n independent chunks
(preprocess/generate_chunks_config.py:50-104 writes chunk_coarse/<m>_<n>.yaml and
chunk_fine/<m>_<n>.yaml, the fine config's pretrained_checkpoint pointing at the chunk's own
coarse output, :89-94); the user runs train.py once per chunk config and merge.py joins the
chunks' explicit PLYs (merge.py:132-217, consolidate_lod).  Nothing crosses chunks during
training, so the GPU mapping is one chunk per GPU with no collectives.

* `run_chunks`  the parent: a work queue of chunks over device slots.  Each chunk runs its stages
  (coarse, then fine) as separate child processes on one slot, with HIP_VISIBLE_DEVICES set to
  that slot's device; a free slot takes the next chunk.  The parent never touches the GPU (no
  device call initialises the HIP runtime in it, and it never execs): every device process is a
  fresh child, which is what the reference's one-train.py-per-chunk invocation is.
* `consolidate_explicit`  merge.py:132-217: each chunk's explicit Gaussians cropped to its
  true_bounds on the two ground-plane axes (x / scale within the bounds, inclusive), then
  concatenated in chunk order into one explicit PLY.
"""
from __future__ import annotations

import os
import queue
import subprocess
import threading
import time
from typing import Callable, Dict, List, Sequence, Tuple


def chunk_ids(n_width: int, n_height: int) -> List[str]:
    """generate_chunks_config.py:76-79: "m_n" for m in range(n_width), n in range(n_height)."""
    return [f"{m}_{n}" for m in range(n_width) for n in range(n_height)]


def run_chunks(chunks: Sequence[str], devices: Sequence[str], command: Callable[[str, str], List[str]],
               stages: Sequence[str] = ("coarse", "fine"), env: Dict[str, str] | None = None,
               log_dir: str | None = None, timeout: float | None = None) -> Dict[str, dict]:
    """Train every chunk: command(chunk, stage) -> argv of one child process.

    devices: one entry per concurrent slot, the HIP_VISIBLE_DEVICES value of that slot (a
    device may appear twice to run two chunks on it).  A chunk's stages run in order in its
    slot; a stage that fails skips the chunk's later stages.  Returns {chunk: {"device",
    "returncodes" {stage: rc}, "seconds"}}; raises RuntimeError listing the failed chunks once
    every slot has drained."""
    if not devices:
        raise ValueError("run_chunks: no device slots")
    base = dict(os.environ if env is None else env)
    base.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    todo: "queue.Queue[str]" = queue.Queue()
    for c in chunks:
        todo.put(c)
    results: Dict[str, dict] = {}
    lock = threading.Lock()
    if log_dir:
        os.makedirs(log_dir, exist_ok=True)

    def slot(dev: str) -> None:
        while True:
            try:
                c = todo.get_nowait()
            except queue.Empty:
                return
            rec = {"device": dev, "returncodes": {}, "seconds": 0.0}
            t0 = time.time()
            try:
                for st in stages:
                    e = dict(base)
                    e["HIP_VISIBLE_DEVICES"] = str(dev)
                    try:
                        out = open(os.path.join(log_dir, f"{c}_{st}.log"), "w") if log_dir else subprocess.DEVNULL
                        try:
                            rc = subprocess.call(command(c, st), env=e, stdout=out, stderr=subprocess.STDOUT,
                                                 timeout=timeout)
                        finally:
                            if log_dir:
                                out.close()
                    except subprocess.TimeoutExpired:
                        rc = -9
                    except Exception as ex:  # a command() error, a missing executable, an unwritable log
                        rc = -1
                        rec["error"] = f"{st}: {type(ex).__name__}: {ex}"
                    rec["returncodes"][st] = rc
                    if rc != 0:
                        break
            finally:
                # recorded whatever happened, so a chunk never silently drops out of the results
                rec["seconds"] = round(time.time() - t0, 3)
                with lock:
                    results[c] = rec

    threads = [threading.Thread(target=slot, args=(d,), daemon=True) for d in devices]
    for t in threads:
        t.start()
    for t in threads:
        t.join()
    missing = [c for c in chunks if c not in results]
    failed = [c for c, r in results.items() if any(v != 0 for v in r["returncodes"].values())
              or len(r["returncodes"]) < len(stages)]
    if failed or missing:
        raise RuntimeError(f"run_chunks: chunks failed: {sorted(failed)}, never run: {sorted(missing)} "
                           f"({ {c: results[c] for c in failed} })")
    return results


def crop_mask(xyz, true_bounds: Tuple[Tuple[float, float], Tuple[float, float]], plane_index: Sequence[int],
              scale: float = 1.0):
    """merge.py:165-171: inside the chunk's true bounds on the two ground-plane axes."""
    (x0, x1), (y0, y1) = true_bounds
    a, b = xyz[:, plane_index[0]], xyz[:, plane_index[1]]
    return (a >= x0 / scale) & (a <= x1 / scale) & (b >= y0 / scale) & (b <= y1 / scale)


def consolidate_explicit(parts: Sequence[Tuple[str, str, tuple]], plane_index: Sequence[int], out_path: str,
                         scale: float = 1.0) -> Dict[str, int]:
    """merge.py:132-217 for explicit PLYs: parts = [(chunk id, point_cloud_explicit.ply, true_bounds)]
    in merge order.  Writes the merged explicit PLY (the obj_info LoD values of the last chunk,
    as the reference writes those of its last loaded model) and returns {chunk: kept count}."""
    import numpy as np

    from .ply import read_ply, write_ply
    merged, kept, info = None, {}, []
    for cid, path, bounds in parts:
        cols, info, _ = read_ply(path)
        xyz = np.stack([cols["x"], cols["y"], cols["z"]], 1)
        m = crop_mask(xyz, bounds, plane_index, scale)
        kept[cid] = int(m.sum())
        if merged is None:
            merged = {k: [] for k in cols}
        if list(merged) != list(cols):
            raise ValueError(f"consolidate_explicit: {path} has properties {list(cols)}, expected {list(merged)}")
        for k in cols:
            merged[k].append(cols[k][m])
    if merged is None:
        raise ValueError("consolidate_explicit: no parts")
    write_ply(out_path, {k: np.concatenate(v).astype(np.float32) for k, v in merged.items()}, obj_info=info)
    return kept

