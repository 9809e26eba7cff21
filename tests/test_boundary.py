"""CPU tests of the drop-in boundary: the C-ABI library loads and exports every symbol
include/hgsr.h declares (no compute calls: there is no GPU here), the ctypes binding
covers the whole header, the gsplat import paths used by the reference resolve, and
the product path refuses CPU tensors instead of falling back."""
import ctypes
import os
import re
import subprocess

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "hgsr.h")


def header_symbols():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(hgsr_[a-z0-9_]+)\s*\(", txt)))


@pytest.fixture(scope="module")
def lib():
    from horizongs_amd import _native
    if not os.path.exists(_native.LIB_PATH):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "horizongs_amd", "csrc")], check=True)
    return _native.lib()


def test_header_symbols_exported(lib):
    syms = header_symbols()
    assert len(syms) >= 20
    for s in syms:
        assert hasattr(lib, s), f"libhgsr.so does not export {s}"


def test_ctypes_binding_covers_header():
    from horizongs_amd import _native
    assert set(header_symbols()) == set(_native.EXPORTED)


def test_ctypes_arity_matches_header():
    """Every binding declares exactly as many arguments as its prototype in hgsr.h."""
    from horizongs_amd import _native
    txt = re.sub(r"/\*.*?\*/", "", open(HEADER).read(), flags=re.S)
    for name, (_, args) in _native._SIGS.items():
        m = re.search(r"\b" + name + r"\((.*?)\);", txt, flags=re.S)
        assert m, name
        params = [a for a in m.group(1).split(",") if a.strip() and a.strip() != "void"]
        assert len(params) == len(args), f"{name}: header {len(params)} args, binding {len(args)}"


def test_pure_host_entry_points(lib):
    from horizongs_amd import _native
    assert lib.hgsr_version() == 1
    # workspace queries are host-only arithmetic
    assert _native.size_query("hgsr_isect_ws1_bytes", 1, 2_000_000, 120, 68) > 0
    assert _native.size_query("hgsr_isect_ws2_bytes", 1000, 10) >= 8000
    assert _native.size_query("hgsr_isect_ws2_bytes", 1000, 5000) >= 16000
    # raster backwards' gradient slots: 3DGS 4 flags + 4 partial rows of 64 B per intersection,
    # 2DGS (waves merged in LDS) 1 flag + one 80-B row; per Gaussian the slot index (seg, base)
    # and, unless reused, the packed record
    assert _native.size_query("hgsr_raster3d_bwd_ws_bytes", 1, 100, 4, 500, 0) >= 500 * 4 * (1 + 64) + 100 * (12 + 48)
    assert _native.size_query("hgsr_raster3d_bwd_ws_bytes", 1, 100, 4, 500, 1) >= 500 * 4 * (1 + 64) + 100 * 12
    assert _native.size_query("hgsr_raster2d_bwd_ws_bytes", 1, 100, 4, 500, 0) >= 500 * (1 + 80) + 100 * (12 + 96)


def test_invalid_args_return_status(lib):
    # bad dimensions are rejected before any device work
    st = lib.hgsr_raster3d_fwd(1, 10, 9, None, None, None, None, None, 64, 64, 16, 4, 4, None, 0, None, None,
                               None, None, None, 0, None)
    assert st == -1
    assert b"channels" in lib.hgsr_last_error()
    st = lib.hgsr_sh_fwd(7, 64, 10, None, None, None, None, None)
    assert st == -1 and b"degree" in lib.hgsr_last_error()


def test_gsplat_alias_import_paths():
    import gsplat
    from gsplat.cuda._wrapper import fully_fused_projection, fully_fused_projection_2dgs  # noqa: F401
    assert callable(gsplat.rasterization) and callable(gsplat.rasterization_2dgs)


def test_no_cpu_fallback():
    from horizongs_amd import gsplat_api as G
    n = 4
    with pytest.raises(RuntimeError, match="HIP device"):
        G.fully_fused_projection(torch.zeros(n, 3), None, torch.ones(n, 4), torch.ones(n, 3),
                                 torch.eye(4)[None], torch.eye(3)[None], 8, 8)


def test_unsupported_options_raise():
    from horizongs_amd import gsplat_api as G
    with pytest.raises(NotImplementedError):
        G.rasterization(torch.zeros(1, 3), torch.ones(1, 4), torch.ones(1, 3), torch.ones(1), torch.ones(1, 3),
                        torch.eye(4)[None], torch.eye(3)[None], 8, 8, packed=True)


def _render_calls():
    import json
    with open(os.path.join(os.path.dirname(__file__), "golden", "render_calls.json")) as f:
        return json.load(f)


def test_reference_call_sites_bind():
    """Every gsplat call of the reference's renderer (tests/golden/render_calls.json, extracted
    from gaussian_renderer/render.py:40-76,149-186 by scripts/extract_render_calls.py) binds to the
    drop-in surface: the same positional arity and keyword names, through the same import paths."""
    import importlib
    import inspect
    rc = _render_calls()
    assert len(rc["calls"]) == 4 and rc["meta_keys_read"] == ["means2d", "radii"]
    for imp in rc["imports"]:  # `import gsplat`, `from gsplat.cuda._wrapper import ...`
        mod = importlib.import_module(imp["module"])
        for n in imp.get("names", []):
            assert callable(getattr(mod, n)), (imp, n)
    import gsplat
    from gsplat.cuda import _wrapper
    for c in rc["calls"]:
        fn = getattr(gsplat, c["function"]) if c["callee"].startswith("gsplat.") else getattr(_wrapper, c["function"])
        ba = inspect.signature(fn).bind(*c["args"], **c["kwargs"])  # raises TypeError on any mismatch
        assert set(ba.arguments) >= set(c["kwargs"]), c["line"]


def test_reference_call_site_unpack_shapes():
    """The recorded result structures (render.py:40 -> 3 names; :56 -> ((6 names), info); the
    prefilter's 5-way unpack at :189) are the ones gsplat_api returns (GPU side:
    tests/test_gpu_parity.py::test_reference_call_sites_run)."""
    shapes = {c["function"]: c.get("unpacked_at", {}).get("shape", c["target"]) for c in _render_calls()["calls"]}
    assert len(shapes["rasterization"]) == 3
    assert len(shapes["rasterization_2dgs"]) == 2 and len(shapes["rasterization_2dgs"][0]) == 6
    assert len(shapes["fully_fused_projection"]) == 5 and len(shapes["fully_fused_projection_2dgs"]) == 5
