"""Extract the reference's rasterizer call sites into tests/golden/render_calls.json.

Run in the build container (the reference is not on the GPU box):
    python scripts/extract_render_calls.py [/root/reference]

Parses reference gaussian_renderer/render.py with `ast` (nothing is imported or executed) and
records, for every call of the gsplat surface (gsplat.rasterization, gsplat.rasterization_2dgs,
fully_fused_projection, fully_fused_projection_2dgs):
  * the line, the callee, each positional argument's source text and each keyword's name and
    source text (render.py:40-76, 149-186);
  * how the result is unpacked (the assignment target's tuple nesting, following a plain name
    to the statement that unpacks it, e.g. `proj_results` at render.py:189);
plus the module imports of the gsplat surface and the meta-dict keys the caller reads
(info["radii"], info["means2d"]).  tests/test_boundary.py binds every recorded call against
horizongs_amd.gsplat_api with inspect.signature; tests/test_gpu_parity.py calls each one with
tensors and unpacks the result the recorded way.
"""
from __future__ import annotations

import ast
import json
import os
import sys

SURFACE = {"rasterization", "rasterization_2dgs", "fully_fused_projection", "fully_fused_projection_2dgs"}


def _callee(node):
    f = node.func
    if isinstance(f, ast.Attribute) and isinstance(f.value, ast.Name):
        return f"{f.value.id}.{f.attr}", f.attr
    if isinstance(f, ast.Name):
        return f.id, f.id
    return None, None


def _shape(t):
    """Assignment target -> nested list of names."""
    if isinstance(t, (ast.Tuple, ast.List)):
        return [_shape(e) for e in t.elts]
    return ast.unparse(t)


def extract(ref_root):
    path = os.path.join(ref_root, "gaussian_renderer", "render.py")
    src = open(path).read()
    tree = ast.parse(src)
    imports, calls, meta_keys = [], [], set()
    unpack_of = {}  # name -> unpack shape of a later `a, b, ... = name`
    for node in ast.walk(tree):
        if isinstance(node, ast.Import):
            imports += [{"line": node.lineno, "module": a.name} for a in node.names if "gsplat" in a.name]
        elif isinstance(node, ast.ImportFrom) and node.module and "gsplat" in node.module:
            imports.append({"line": node.lineno, "module": node.module, "names": [a.name for a in node.names]})
        elif isinstance(node, ast.Assign) and isinstance(node.value, ast.Name) and isinstance(node.targets[0], ast.Tuple):
            unpack_of[node.value.id] = {"line": node.lineno, "shape": _shape(node.targets[0])}
        elif isinstance(node, ast.Subscript) and isinstance(node.value, ast.Name) and node.value.id == "info":
            if isinstance(node.slice, ast.Constant) and isinstance(node.slice.value, str):
                meta_keys.add(node.slice.value)
    for node in ast.walk(tree):
        if not isinstance(node, ast.Assign) or not isinstance(node.value, ast.Call):
            continue
        full, name = _callee(node.value)
        if name not in SURFACE:
            continue
        tgt = node.targets[0]
        shape = _shape(tgt)
        entry = {"line": node.lineno, "end_line": node.value.end_lineno, "callee": full, "function": name,
                 "args": [ast.unparse(a) for a in node.value.args],
                 "kwargs": {k.arg: ast.unparse(k.value) for k in node.value.keywords}, "target": shape}
        if isinstance(tgt, ast.Name) and tgt.id in unpack_of:
            entry["unpacked_at"] = unpack_of[tgt.id]
        calls.append(entry)
    calls.sort(key=lambda c: c["line"])
    return {"source": "gaussian_renderer/render.py", "imports": sorted(imports, key=lambda i: i["line"]),
            "calls": calls, "meta_keys_read": sorted(meta_keys)}


def main():
    ref = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
    out = extract(ref)
    dst = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden",
                       "render_calls.json")
    with open(dst, "w") as f:
        json.dump(out, f, indent=1)
    print(f"{len(out['calls'])} calls, meta keys {out['meta_keys_read']} -> {dst}")


if __name__ == "__main__":
    main()
