"""gsplat-compatible call surface backed by the hgsr HIP kernels.

Mirrors the gsplat (< 1.5, FantasticOven2 2DGS fork) functions that Horizon-GS
calls, so reference gaussian_renderer/render.py runs unchanged through the
`gsplat` alias package:

  * rasterization()              render.py:40-54  (3DGS, packed=False)
  * rasterization_2dgs()         render.py:62-76  (2DGS, nested 6-tuple return)
  * fully_fused_projection()     render.py:149-165 (anchor prefilter)
  * fully_fused_projection_2dgs() render.py:171-186 (fork signature with densifications)
plus the lower-level ops gsplat exposes (isect_tiles, isect_offset_encode,
rasterize_to_pixels[_2dgs], spherical_harmonics).

Argument meaning, shapes, defaults and the returned meta dict follow gsplat;
unsupported options (packed=True, antialiased mode, covars, tile masks,
non-pinhole cameras, sparse grads, distributed) raise NotImplementedError
rather than silently diverging.  Errors from the native layer surface as
RuntimeError, as gsplat's TORCH_CHECKs do.
"""
from __future__ import annotations

import collections
import ctypes as ct
import math
import threading
from typing import Optional, Tuple


import torch
import torch.nn.functional as F

from . import _native as N
from . import gradbuf
from ._native import ptr

_MAX_CH = 4  # channels per raster kernel call


def _f32(t):
    return t.contiguous() if t.dtype == torch.float32 else t.float().contiguous()


def _check_cuda(*ts):
    for t in ts:
        if t is not None and not t.is_cuda:
            raise RuntimeError("hgsr: inputs must be HIP device tensors (no CPU fallback)")


def _unsupported(flag, what):
    if flag:
        raise NotImplementedError(f"hgsr: {what} is not supported (Horizon-GS never requests it)")


# =========================================================================
# projection
# =========================================================================
def _grads_or_zeros(grads, lead, tails, like):
    """Output gradients of a projection (materialize_grads off): zeros for unused outputs."""
    out = []
    for g, t in zip(grads, tails):
        if g is None:
            shape = lead + (() if t is None else (t if isinstance(t, tuple) else (t,)))
            g = torch.zeros(shape, dtype=torch.float32, device=like.device)
        out.append(g)
    return out


class GradSink:
    """Hand-off of a second gradient of the projection's `scales` ("glue").

    The reference loss head regularises the same activated scales the rasterizer projects
    (train.py:163-167), so autograd would sum the loss's gradient and the projection's with a
    separate add kernel.  The projection's forward (when a backward can follow) hangs a sink
    on its scales tensor; the fused loss, seeing it on the tensor it regularises, puts its
    gradient there instead of returning it, and the projection backward -- which by the graph's
    order runs after the loss backward -- adds it inside its own kernel (v_scales_in).  A put
    after the projection backward took the sink (a second backward) is refused, and the loss
    then returns its gradient through autograd as usual."""
    __slots__ = ("value", "closed")

    def __init__(self):
        self.value, self.closed = None, False

    def put(self, g):
        if self.closed:
            return False
        self.value = g if self.value is None else self.value + g
        return True

    def take(self):
        self.closed = True
        v, self.value = self.value, None
        return v


# The folded glue (DESIGN.md §8 "Round 4: the deferred intersection count and the folded glue"):
# the loss's scale gradient through a GradSink, and rasterization_2dgs' world-frame normals + K13
# inside the fused raster Function.  Module constants, not knobs: tests/test_gpu_glue.py flips
# them to compare against the unfolded composition they replace.
_GRAD_SINK = True
_FUSE_FRAME = True


def _attach_sink(ctx, scales, grad_mode, idx):
    """Hang a fresh sink on `scales` for this projection.  If the tensor still carries an OPEN
    sink -- a second projection of the same scales before the first one's backward ran, e.g. a
    render whose graph is never backpropagated -- the loss could not tell which projection's
    backward will take its gradient: both sinks are closed (a put is refused, so the loss
    returns its gradient through autograd) and this projection gets none."""
    ctx.sink = None
    if not (_GRAD_SINK and grad_mode and ctx.needs_input_grad[idx]):
        return
    prev = getattr(scales, "_hgsr_grad_sink", None)
    if prev is not None and not prev.closed:
        prev.closed = True
        scales._hgsr_grad_sink = None
        return
    ctx.sink = GradSink()
    scales._hgsr_grad_sink = ctx.sink


def _sink_grad(ctx, like):
    """The gradient handed over through the sink (contiguous fp32 like `like`), or None."""
    v = None if ctx.sink is None else ctx.sink.take()
    return None if v is None else _f32(v.reshape(like.shape))


class _Project3D(torch.autograd.Function):
    @staticmethod
    def forward(ctx, means, quats, scales, viewmats, Ks, width, height, eps2d, near_plane, far_plane,
                radius_clip, grad_mode=False, means_sink=None):
        C, Ng = viewmats.shape[0], means.shape[0]
        dev = means.device
        radii = torch.empty((C, Ng), dtype=torch.int32, device=dev)
        means2d = torch.empty((C, Ng, 2), dtype=torch.float32, device=dev)
        depths = torch.empty((C, Ng), dtype=torch.float32, device=dev)
        conics = torch.empty((C, Ng, 3), dtype=torch.float32, device=dev)
        N.call("hgsr_project3d_fwd", C, Ng, ptr(means), ptr(quats), ptr(scales), ptr(viewmats), ptr(Ks),
               width, height, eps2d, near_plane, far_plane, radius_clip, ptr(radii), ptr(means2d), ptr(depths),
               ptr(conics), N.stream(dev))
        ctx.save_for_backward(means, quats, scales, viewmats, Ks, radii, conics)
        ctx.cfg = (width, height, eps2d)
        _attach_sink(ctx, scales, grad_mode, 2)
        # the SH colour step's means gradient, handed over by _SHColors' backward (which runs
        # first: it is later in the graph) and added in this backward's kernel (v_means_in)
        ctx.msink = means_sink if ctx.needs_input_grad[0] else None
        ctx.mark_non_differentiable(radii)
        ctx.set_materialize_grads(False)  # no zero-filled int grad for radii per step
        return radii, means2d, depths, conics

    @staticmethod
    def backward(ctx, v_radii, v_means2d, v_depths, v_conics):
        means, quats, scales, viewmats, Ks, radii, conics = ctx.saved_tensors
        width, height, eps2d = ctx.cfg
        C, Ng = viewmats.shape[0], means.shape[0]
        v_means = gradbuf.alloc(means)  # in place in a DDP bucket when one is registered
        v_quats = gradbuf.alloc(quats)
        v_scales = torch.empty_like(scales)
        v_means2d, v_depths, v_conics = (_f32(g) for g in _grads_or_zeros((v_means2d, v_depths, v_conics), (C, Ng),
                                                                           (2, None, 3), means))
        v_in = _sink_grad(ctx, scales)
        vm_in = None if ctx.msink is None else ctx.msink.take()
        vm_in = None if vm_in is None else _f32(vm_in.reshape(means.shape))
        N.call("hgsr_project3d_bwd", C, Ng, ptr(means), ptr(quats), ptr(scales), ptr(viewmats), ptr(Ks), width,
               height, eps2d, ptr(radii), ptr(conics), ptr(v_means2d), ptr(v_depths), ptr(v_conics), ptr(v_means),
               ptr(v_quats), ptr(v_scales), ptr(v_in), ptr(vm_in), N.stream(means.device))
        if ctx.needs_input_grad[3]:
            raise NotImplementedError("hgsr: gradients w.r.t. viewmats are not supported")
        return v_means, v_quats, v_scales, None, None, None, None, None, None, None, None, None, None


def fully_fused_projection(means, covars, quats, scales, viewmats, Ks, width, height, eps2d=0.3,
                           packed=False, near_plane=0.01, far_plane=1e10, radius_clip=0.0,
                           sparse_grad=False, calc_compensations=False, camera_model="pinhole"):
    """gsplat.cuda._wrapper.fully_fused_projection -> (radii, means2d, depths, conics, compensations)."""
    return _projection(means, covars, quats, scales, viewmats, Ks, width, height, eps2d, packed, near_plane,
                       far_plane, radius_clip, sparse_grad, calc_compensations, camera_model)


def _projection(means, covars, quats, scales, viewmats, Ks, width, height, eps2d, packed, near_plane, far_plane,
                radius_clip, sparse_grad, calc_compensations, camera_model, means_sink=None):
    _unsupported(covars is not None, "covars input")
    _unsupported(packed, "packed=True")
    _unsupported(sparse_grad, "sparse_grad")
    _unsupported(calc_compensations, "calc_compensations")
    _unsupported(camera_model != "pinhole", f"camera_model={camera_model}")
    _check_cuda(means, quats, scales, viewmats, Ks)
    Ng = means.shape[0]
    assert means.shape == (Ng, 3) and quats.shape == (Ng, 4) and scales.shape == (Ng, 3), "bad Gaussian shapes"
    assert viewmats.dim() == 3 and viewmats.shape[1:] == (4, 4) and Ks.shape == (viewmats.shape[0], 3, 3)
    radii, means2d, depths, conics = _Project3D.apply(
        _f32(means), _f32(quats), _f32(scales), _f32(viewmats), _f32(Ks), int(width), int(height),
        float(eps2d), float(near_plane), float(far_plane), float(radius_clip), torch.is_grad_enabled(), means_sink)
    return radii, means2d, depths, conics, None


class _Project2D(torch.autograd.Function):
    @staticmethod
    def forward(ctx, means, quats, scales, viewmats, Ks, width, height, near_plane, far_plane, radius_clip,
                grad_mode=False):
        C, Ng = viewmats.shape[0], means.shape[0]
        dev = means.device
        radii = torch.empty((C, Ng), dtype=torch.int32, device=dev)
        means2d = torch.empty((C, Ng, 2), dtype=torch.float32, device=dev)
        depths = torch.empty((C, Ng), dtype=torch.float32, device=dev)
        rt = torch.empty((C, Ng, 3, 3), dtype=torch.float32, device=dev)
        normals = torch.empty((C, Ng, 3), dtype=torch.float32, device=dev)
        N.call("hgsr_project2d_fwd", C, Ng, ptr(means), ptr(quats), ptr(scales), ptr(viewmats), ptr(Ks),
               width, height, near_plane, far_plane, radius_clip, ptr(radii), ptr(means2d), ptr(depths), ptr(rt),
               ptr(normals), N.stream(dev))
        ctx.save_for_backward(means, quats, scales, viewmats, Ks, radii, rt)
        ctx.cfg = (width, height)
        _attach_sink(ctx, scales, grad_mode, 2)
        ctx.mark_non_differentiable(radii)
        ctx.set_materialize_grads(False)  # no zero-filled int grad for radii per step
        return radii, means2d, depths, rt, normals

    @staticmethod
    def backward(ctx, v_radii, v_means2d, v_depths, v_rt, v_normals):
        means, quats, scales, viewmats, Ks, radii, rt = ctx.saved_tensors
        width, height = ctx.cfg
        C, Ng = viewmats.shape[0], means.shape[0]
        v_means = gradbuf.alloc(means)  # in place in a DDP bucket when one is registered
        v_quats = gradbuf.alloc(quats)
        v_scales = torch.empty_like(scales)
        v_means2d, v_depths, v_rt, v_normals = (_f32(g) for g in _grads_or_zeros(
            (v_means2d, v_depths, v_rt, v_normals), (C, Ng), (2, None, (3, 3), 3), means))
        v_in = _sink_grad(ctx, scales)
        N.call("hgsr_project2d_bwd", C, Ng, ptr(means), ptr(quats), ptr(scales), ptr(viewmats), ptr(Ks), width,
               height, ptr(radii), ptr(rt), ptr(v_means2d), ptr(v_depths), ptr(v_rt), ptr(v_normals), ptr(v_means),
               ptr(v_quats), ptr(v_scales), ptr(v_in), N.stream(means.device))
        if ctx.needs_input_grad[3]:
            raise NotImplementedError("hgsr: gradients w.r.t. viewmats are not supported")
        return v_means, v_quats, v_scales, None, None, None, None, None, None, None, None


def fully_fused_projection_2dgs(means, quats, scales, viewmats, densifications, Ks, width, height, eps2d=0.3,
                                packed=False, near_plane=0.01, far_plane=1e10, radius_clip=0.0,
                                sparse_grad=False):
    """Fork signature (render.py:171-186): (..., viewmats, densifications, Ks, ...) ->
    (radii, means2d, depths, ray_transforms, normals).  `densifications` [C,N,2] (zeros)
    only carries the densification-gradient proxy; the projection values ignore it."""
    _unsupported(packed, "packed=True")
    _unsupported(sparse_grad, "sparse_grad")
    _check_cuda(means, quats, scales, viewmats, Ks)
    Ng = means.shape[0]
    assert means.shape == (Ng, 3) and quats.shape == (Ng, 4) and scales.shape == (Ng, 3), "bad Gaussian shapes"
    return _Project2D.apply(_f32(means), _f32(quats), _f32(scales), _f32(viewmats), _f32(Ks), int(width),
                            int(height), float(near_plane), float(far_plane), float(radius_clip),
                            torch.is_grad_enabled())


# =========================================================================
# spherical harmonics
# =========================================================================
class _SH(torch.autograd.Function):
    @staticmethod
    def forward(ctx, degree, dirs, coeffs, masks):
        n = dirs.shape[0]
        K = coeffs.shape[1]
        colors = torch.empty((n, 3), dtype=torch.float32, device=dirs.device)
        N.call("hgsr_sh_fwd", degree, K, n, ptr(dirs), ptr(coeffs), ptr(masks), ptr(colors), N.stream(dirs.device))
        ctx.save_for_backward(dirs, coeffs, masks)
        ctx.degree = degree
        return colors

    @staticmethod
    def backward(ctx, v_colors):
        dirs, coeffs, masks = ctx.saved_tensors
        n, K = coeffs.shape[0], coeffs.shape[1]
        v_coeffs = torch.empty_like(coeffs)
        v_dirs = torch.zeros_like(dirs) if ctx.needs_input_grad[1] else None
        vc = _f32(v_colors)
        N.call("hgsr_sh_bwd", ctx.degree, K, n, ptr(dirs), ptr(coeffs), ptr(masks), ptr(vc), ptr(v_coeffs),
               ptr(v_dirs), N.stream(dirs.device))
        return None, v_dirs, v_coeffs, None


class _SHColors(torch.autograd.Function):
    """rasterization()'s SH colour path (dirs = means - campos, masked SH evaluation,
    clamp_min(+0.5, 0)) as one native call each way: hgsr_sh_rgb_{fwd,bwd}.  viewmats (instead
    of campos): the kernels compute the camera centres -R^T t themselves."""

    @staticmethod
    def forward(ctx, degree, means, campos, coeffs, radii, viewmats=None, means_sink=None):
        C, Ng = radii.shape
        K = coeffs.shape[-2]
        shared = coeffs.dim() == 3
        colors = torch.empty((C, Ng, 3), dtype=torch.float32, device=means.device)
        N.call("hgsr_sh_rgb_fwd", degree, C, Ng, K, ptr(means), ptr(campos), ptr(viewmats), ptr(coeffs), int(shared),
               ptr(radii), ptr(colors), N.stream(means.device))
        ctx.save_for_backward(means, campos, coeffs, radii, viewmats)
        ctx.degree = degree
        ctx.msink = means_sink
        return colors

    @staticmethod
    def backward(ctx, v_colors):
        means, campos, coeffs, radii, viewmats = ctx.saved_tensors
        C, Ng = radii.shape
        v_coeffs = torch.empty_like(coeffs)
        v_means = torch.empty_like(means) if ctx.needs_input_grad[1] else None
        vc = _f32(v_colors)
        N.call("hgsr_sh_rgb_bwd", ctx.degree, C, Ng, coeffs.shape[-2], ptr(means), ptr(campos), ptr(viewmats),
               ptr(coeffs), int(coeffs.dim() == 3), ptr(radii), ptr(vc), ptr(v_coeffs), ptr(v_means),
               N.stream(means.device))
        if v_means is not None and ctx.msink is not None and ctx.msink.put(v_means):
            v_means = None  # added by the projection backward (refused once it has run: autograd sums)
        return None, v_means, None, v_coeffs, None, None, None


def spherical_harmonics(degrees_to_use: int, dirs: torch.Tensor, coeffs: torch.Tensor,
                        masks: Optional[torch.Tensor] = None) -> torch.Tensor:
    """gsplat spherical_harmonics: dirs [..., 3], coeffs [..., K, 3] -> colors [..., 3] (degree <= 3)."""
    _check_cuda(dirs, coeffs)
    assert coeffs.shape[-1] == 3 and dirs.shape[-1] == 3
    K = coeffs.shape[-2]
    assert (degrees_to_use + 1) ** 2 <= K, "not enough SH coefficients"
    batch = dirs.shape[:-1]
    d = _f32(dirs.reshape(-1, 3))
    c = _f32(coeffs.reshape(-1, K, 3))
    if masks is None:
        m = None
    else:  # bool -> uint8 is a free view (same bytes), any other dtype a converting copy
        m = masks.reshape(-1).contiguous()
        m = m.view(torch.uint8) if m.dtype == torch.bool else m.to(torch.uint8)
    out = _SH.apply(int(degrees_to_use), d, c, m)
    return out.reshape(batch + (3,))


# =========================================================================
# tile intersection
# =========================================================================
def _tile_grid(width, height, tile_size):
    return math.ceil(width / tile_size), math.ceil(height / tile_size)


_pinned = threading.local()
# Deferred intersection count: rasterization() enqueues the emission, the sort
# and the raster forward into capacity-sized buffers BEFORE it reads the count, so the one
# host wait of a view lands behind queued work instead of draining the queue.  The capacity
# is the largest count of the last _PRED_VIEWS views of the same camera grid (+ headroom): a
# training loop cycles cameras (train.py:133-148) whose intersection counts differ widely, and
# the previous view alone under-predicts every view busier than it.  An overflow (detected on
# the device: the kernels then write nothing) is redone at the exact size; the first view of a
# grid takes the synchronous order (count -> host -> emit), as gsplat does it.
_PRED_VIEWS = 64
_pred = {}  # (device, C, tile_w, tile_h) -> deque of (n_isects, largest bin) of the last views
_CAP_GRAIN = 1 << 18  # capacities in steps of 256K keys: stable sizes for the caching allocator
# views through the binned intersection: deferred (count read after the forward was queued),
# redone (deferred over capacity, re-emitted at the exact size), synchronous (no prediction yet)
isect_stats = {"deferred": 0, "redo": 0, "sync": 0}


def _capacity(n, max_bin):
    """(key capacity, largest-bin capacity) for a view predicted to have n keys: 12.5 % + 64K of
    headroom; bins sort in classes (<= 2048 keys: one launch, <= 4096: the big-bin launch, more:
    merge scratch), so the bin capacity is the class of the predicted largest bin."""
    cap = (int(n * 1.125) + 65536 + _CAP_GRAIN - 1) // _CAP_GRAIN * _CAP_GRAIN
    m = int(max_bin * 1.125) + 64
    return cap, (2048 if m <= 2048 else (4096 if m <= 4096 else 1 << 30))


def _host_info_buffer():
    """Per-thread pinned 2 x int64 landing buffer for the intersection count."""
    buf = getattr(_pinned, "buf", None)
    if buf is None:
        buf = _pinned.buf = torch.empty(2, dtype=torch.int64, pin_memory=True)
    return buf


@torch.no_grad()
def _isect_count(means2d, radii, tile_size, tile_width, tile_height, depths):
    """Stage 1 of the binned intersection: launches the count pass and an async copy of
    {n_isects, largest bin} to pinned host memory.  Work enqueued before _isect_finish()
    runs on the device while the host waits for that copy."""
    C, Ng = radii.shape
    dev = means2d.device
    m2 = _f32(means2d.detach())
    dep = _f32(depths.detach())
    radii = radii.contiguous()
    tpg = torch.empty((C, Ng), dtype=torch.int32, device=dev)
    offsets = torch.empty((C, tile_height, tile_width), dtype=torch.int32, device=dev)
    info = torch.empty(3, dtype=torch.int64, device=dev)  # {n_isects, largest bin, overflow (deferred)}
    ws1_b = N.size_query("hgsr_isect_ws1_bytes", C, Ng, tile_width, tile_height)
    ws1 = torch.empty(max(ws1_b, 1), dtype=torch.uint8, device=dev)
    s = N.stream(dev)
    N.call("hgsr_isect_count", C, Ng, ptr(m2), ptr(radii), tile_size, tile_width, tile_height, ptr(tpg),
           ptr(offsets), ptr(info), ptr(ws1), ws1_b, s)
    host = _host_info_buffer()
    host.copy_(info[:2], non_blocking=True)
    ev = torch.cuda.Event()
    ev.record(torch.cuda.current_stream(dev))
    return (m2, dep, radii, tpg, offsets, ws1, ws1_b, host, ev, info, tile_size, tile_width, tile_height)


def _isect_count_host(st):
    """Wait for the count's copy (not for the queue behind it) -> (n_isects, largest bin);
    remembered as the next view's capacity prediction."""
    m2, radii, host, ev, tw, th = st[0], st[2], st[7], st[8], st[11], st[12]
    ev.synchronize()
    n_isects, max_bin = int(host[0]), int(host[1])
    key = (m2.device.index, radii.shape[0], tw, th)
    if key not in _pred:
        _pred[key] = collections.deque(maxlen=_PRED_VIEWS)
    _pred[key].append((n_isects, max_bin))
    return n_isects, max_bin


@torch.no_grad()
def _isect_finish(st):
    """Stage 2, synchronous: wait for the count (gsplat's host sync), then emit + sort ->
    (tiles_per_gauss, isect_ids, flatten_ids, isect_offsets)."""
    m2, dep, radii, tpg, offsets, ws1, ws1_b, host, ev, info, tile_size, tile_width, tile_height = st
    C, Ng = radii.shape
    dev = m2.device
    s = N.stream(dev)
    n_isects, max_bin = _isect_count_host(st)
    isect_ids = torch.empty(n_isects, dtype=torch.int64, device=dev)
    flatten_ids = torch.empty(n_isects, dtype=torch.int32, device=dev)
    if n_isects > 0:
        ws2_b = N.size_query("hgsr_isect_ws2_bytes", n_isects, max_bin)
        ws2 = torch.empty(ws2_b, dtype=torch.uint8, device=dev)
        N.call("hgsr_isect_emit_sorted", C, Ng, ptr(m2), ptr(radii), ptr(dep), tile_size, tile_width,
               tile_height, ptr(offsets), n_isects, max_bin, ptr(isect_ids), ptr(flatten_ids), ptr(ws1), ws1_b,
               ptr(ws2), ws2_b, None, s)
    return tpg, isect_ids, flatten_ids, offsets


class _Deferred:
    """Capacity-sized intersection arrays of a deferred count; n is set by _isect_resolve."""
    __slots__ = ("ids", "flat", "ws2", "info", "cap", "mbcap", "n")


@torch.no_grad()
def _isect_emit_deferred(st):
    """Stage 2 enqueued before the count is read (None without a prediction for this camera
    grid: the first view takes the synchronous path)."""
    m2, dep, radii, tpg, offsets, ws1, ws1_b, host, ev, info, tile_size, tile_width, tile_height = st
    C, Ng = radii.shape
    hist = _pred.get((m2.device.index, C, tile_width, tile_height))
    if not hist:
        isect_stats["sync"] += 1
        return None
    dev = m2.device
    d = _Deferred()
    d.cap, d.mbcap = _capacity(max(h[0] for h in hist), max(h[1] for h in hist))
    d.ids = torch.empty(d.cap, dtype=torch.int64, device=dev)
    d.flat = torch.empty(d.cap, dtype=torch.int32, device=dev)
    ws2_b = N.size_query("hgsr_isect_ws2_bytes", d.cap, d.mbcap)
    d.ws2 = torch.empty(ws2_b, dtype=torch.uint8, device=dev)
    d.info, d.n = info, None
    N.call("hgsr_isect_emit_sorted", C, Ng, ptr(m2), ptr(radii), ptr(dep), tile_size, tile_width, tile_height,
           ptr(offsets), d.cap, d.mbcap, ptr(d.ids), ptr(d.flat), ptr(ws1), ws1_b, ptr(d.ws2), ws2_b, ptr(info),
           N.stream(dev))
    return d


def _isect_resolve(st, d):
    """After the raster forward is enqueued: read the count (its copy finished long ago, so the
    host does not drain the queue).  True when it fit the capacities; d.n = n_isects."""
    n_isects, max_bin = _isect_count_host(st)
    d.ws2 = d.info = None  # the sort scratch and the count are the queued kernels' alone now
    if n_isects > d.cap or max_bin > d.mbcap:
        isect_stats["redo"] += 1
        return False  # the kernels wrote nothing: the caller redoes it at the exact size
    isect_stats["deferred"] += 1
    d.n = n_isects
    return True


def _isect_binned(means2d, radii, tile_size, tile_width, tile_height, depths):
    """Binned tile intersection: (tiles_per_gauss, isect_ids, flatten_ids, isect_offsets)."""
    return _isect_finish(_isect_count(means2d, radii, tile_size, tile_width, tile_height, depths))


@torch.no_grad()
def isect_tiles(means2d, radii, depths, tile_size, tile_width, tile_height, sort=True, packed=False,
                n_cameras=None, camera_ids=None, gaussian_ids=None):
    """gsplat isect_tiles (non-packed) -> (tiles_per_gauss [C,N], isect_ids [I], flatten_ids [I])."""
    _unsupported(packed, "packed=True")
    _check_cuda(means2d, radii, depths)
    if sort:
        tpg, ids, fl, _ = _isect_binned(means2d, radii, int(tile_size), int(tile_width), int(tile_height), depths)
        return tpg, ids, fl
    C, Ng = radii.shape
    dev = means2d.device
    m2, dep, radii = _f32(means2d.detach()), _f32(depths.detach()), radii.contiguous()
    tpg, _, _, _ = _isect_binned(m2, radii, int(tile_size), int(tile_width), int(tile_height), dep)
    cum = torch.cumsum(tpg.reshape(-1).to(torch.int64), 0)
    n = int(cum[-1].item()) if cum.numel() else 0
    ids = torch.empty(n, dtype=torch.int64, device=dev)
    fl = torch.empty(n, dtype=torch.int32, device=dev)
    if n:
        N.call("hgsr_isect_emit_unsorted", C, Ng, ptr(m2), ptr(radii), ptr(dep), int(tile_size), int(tile_width),
               int(tile_height), ptr(cum), ptr(ids), ptr(fl), N.stream(dev))
    return tpg, ids, fl


@torch.no_grad()
def isect_offset_encode(isect_ids, n_cameras, tile_width, tile_height):
    """gsplat isect_offset_encode -> offsets [C, tile_height, tile_width] int32."""
    _check_cuda(isect_ids)
    out = torch.empty((n_cameras, tile_height, tile_width), dtype=torch.int32, device=isect_ids.device)
    ids = isect_ids.contiguous()
    N.call("hgsr_isect_offset_encode", ids.numel(), ptr(ids) if ids.numel() else None, int(n_cameras),
           int(tile_width), int(tile_height), ptr(out), N.stream(isect_ids.device))
    return out


# =========================================================================
# rasterization (3DGS)
# =========================================================================
class _Raster3D(torch.autograd.Function):
    @staticmethod
    def forward(ctx, means2d, conics, colors, opacities, backgrounds, width, height, tile_size, isect_offsets,
                flatten_ids, absgrad):
        C = isect_offsets.shape[0]
        Ng = means2d.shape[1]
        D = colors.shape[-1]
        th, tw = isect_offsets.shape[1:]
        dev = means2d.device
        rc = torch.empty((C, height, width, D), dtype=torch.float32, device=dev)
        ra = torch.empty((C, height, width, 1), dtype=torch.float32, device=dev)
        last = torch.empty((C, height, width), dtype=torch.int32, device=dev)
        ws_b = N.size_query("hgsr_raster3d_fwd_ws_bytes", C, Ng, D)
        ws = torch.empty(max(ws_b, 1), dtype=torch.uint8, device=dev)
        N.call("hgsr_raster3d_fwd", C, Ng, D, ptr(means2d), ptr(conics), ptr(colors), ptr(opacities),
               ptr(backgrounds), width, height, tile_size, tw, th, ptr(isect_offsets), flatten_ids.numel(),
               ptr(flatten_ids) if flatten_ids.numel() else None, ptr(rc), ptr(ra), ptr(last), ptr(ws), ws_b,
               N.stream(dev))
        ctx.save_for_backward(means2d, conics, colors, opacities, backgrounds, isect_offsets, flatten_ids, ra, last)
        ctx.cfg = (width, height, tile_size, absgrad)
        ctx.fwd_ws = ws  # packed raster records, reused by the backward
        return rc, ra

    @staticmethod
    def backward(ctx, v_rc, v_ra):
        means2d, conics, colors, opacities, backgrounds, offsets, flatten_ids, ra, last = ctx.saved_tensors
        width, height, tile_size, absgrad = ctx.cfg
        C, Ng, D = means2d.shape[0], means2d.shape[1], colors.shape[-1]
        th, tw = offsets.shape[1:]
        dev = means2d.device
        # the kernels overwrite every gradient element
        v_means2d = torch.empty_like(means2d)
        v_conics = torch.empty_like(conics)
        v_colors = torch.empty_like(colors)
        v_opac = torch.empty_like(opacities)
        v_abs = torch.empty_like(means2d) if absgrad else None
        fwd_ws = ctx.fwd_ws
        ws_b = N.size_query("hgsr_raster3d_bwd_ws_bytes", C, Ng, D, flatten_ids.numel(), int(fwd_ws is not None))
        ws = torch.empty(max(ws_b, 1), dtype=torch.uint8, device=dev)
        v_rc = _f32(v_rc)
        v_ra = _f32(v_ra)
        N.call("hgsr_raster3d_bwd", C, Ng, D, ptr(means2d), ptr(conics), ptr(colors), ptr(opacities),
               ptr(backgrounds), width, height, tile_size, tw, th, ptr(offsets), flatten_ids.numel(),
               ptr(flatten_ids) if flatten_ids.numel() else None, ptr(ra), ptr(last), ptr(v_rc), ptr(v_ra),
               ptr(v_means2d), ptr(v_conics), ptr(v_colors), ptr(v_opac), ptr(v_abs), ptr(fwd_ws), ptr(ws), ws_b,
               N.stream(dev))
        if absgrad:
            means2d.absgrad = v_abs
        v_bg = None
        if backgrounds is not None and ctx.needs_input_grad[4]:
            v_bg = (v_rc * (1.0 - ra)).sum(dim=(1, 2))
        return v_means2d, v_conics, v_colors, v_opac, v_bg, None, None, None, None, None, None


def _bwd_ws(size_fn, ctx, C, Ng, D, n_isects, dev, grad_mode):
    """The raster backward's workspace (records reused), allocated by the forward when a
    backward can follow: the forward kernel clears its gradient-slot flags while it composites,
    so the backward needs no memset (hgsr_raster{3,2}d_fwd_packed bwd_ws).  n_isects: the
    intersection arrays' size (a deferred count's capacity).  grad_mode is the
    CALLER's torch.is_grad_enabled() (inside forward() grad mode is always off, and
    needs_input_grad follows requires_grad only): an evaluation render under no_grad()
    allocates and clears nothing."""
    ctx.bwd_ws = None
    if not grad_mode or not any(ctx.needs_input_grad):
        return None
    ws_b = N.size_query(size_fn, C, Ng, D, n_isects, 1)
    ctx.bwd_ws = torch.empty(max(ws_b, 1), dtype=torch.uint8, device=dev)
    return ctx.bwd_ws


def _take_bwd_ws(ctx, ws_b, dev):
    """(workspace, slot flags already zero) for the backward: the forward's pre-cleared one once,
    else a fresh one the backward clears itself (a second backward through the same graph)."""
    ws = getattr(ctx, "bwd_ws", None)
    ctx.bwd_ws = None
    if ws is not None and ws.numel() >= ws_b:
        return ws, 1
    return torch.empty(max(ws_b, 1), dtype=torch.uint8, device=dev), 0


class _Raster3DFused(torch.autograd.Function):
    """rasterization()'s colour assembly + rasterize_to_pixels + ED normalisation as one
    native call each way (hgsr_raster3d_{fwd,bwd}_fused): colours shared over cameras or
    per camera, the depth channel, shared opacities and expected depth are handled in the
    kernels instead of torch cat / repeat / divide (gsplat rendering.py does those in torch)."""

    @staticmethod
    def pack(means2d, conics, colors, depths, opacities, radii=None, tiles=(0, 0, 0), areas=None):
        """Raster records for forward(records=...): launched before the intersection
        count is read back, so the packing overlaps the host sync.  radii (when a backward will
        follow; tiles = (tile_size, tile_width, tile_height)): the records also carry their
        gradient slots -- pass the same radii to forward().  areas (optional): tiles_per_gauss of
        the intersection count of these radii, read by the slot prefix's row sums."""
        C, Ng = means2d.shape[:2]
        Dc = 0 if colors is None else colors.shape[-1]
        D = Dc + (0 if depths is None else 1)
        ws_b = N.size_query("hgsr_raster3d_fwd_ws_bytes", C, Ng, D)
        ws = torch.empty(max(ws_b, 1), dtype=torch.uint8, device=means2d.device)
        N.call("hgsr_raster3d_pack_fused", C, Ng, Dc, ptr(means2d), ptr(conics), ptr(colors),
               int(colors is not None and colors.dim() == 2), ptr(depths), ptr(opacities), int(opacities.dim() == 1),
               ptr(radii), ptr(areas), *tiles, ptr(ws), ws_b, N.stream(means2d.device))
        return ws

    @staticmethod
    def forward(ctx, means2d, conics, colors, depths, opacities, backgrounds, width, height, tile_size,
                isect_offsets, flatten_ids, expected_depth, absgrad, records=None, grad_mode=True, deferred=None,
                radii=None):
        """deferred (_Deferred): flatten_ids is its capacity-sized array, the count device-resident.
        radii: the projection's radii the lists were emitted from (the backward's gradient slots
        follow their tile rectangles; without them the backward finds the rectangles in the lists);
        records packed with the same radii carry the slots already."""
        C, Ng = means2d.shape[:2]
        Dc = 0 if colors is None else colors.shape[-1]
        D = Dc + (0 if depths is None else 1)
        col_shared = colors is not None and colors.dim() == 2
        op_shared = opacities.dim() == 1
        th, tw = isect_offsets.shape[1:]
        dev = means2d.device
        rc = torch.empty((C, height, width, D), dtype=torch.float32, device=dev)
        ra = torch.empty((C, height, width, 1), dtype=torch.float32, device=dev)
        last = torch.empty((C, height, width), dtype=torch.int32, device=dev)
        qmask = None
        if records is not None:
            ws = records
            # the forward's per-quadrant culling bits, read back by the backward
            q_b = N.size_query("hgsr_raster3d_qmask_bytes", C, tw, th, flatten_ids.numel())
            qmask = torch.empty(q_b, dtype=torch.uint8, device=dev)
            # the backward's workspace, its gradient-slot flags cleared by this forward launch
            bwd_ws = _bwd_ws("hgsr_raster3d_bwd_ws_bytes", ctx, C, Ng, D, flatten_ids.numel(), dev, grad_mode)
            N.call("hgsr_raster3d_fwd_packed", C, Ng, Dc, int(depths is not None), int(expected_depth),
                   ptr(backgrounds), width, height, tile_size, tw, th, ptr(isect_offsets), flatten_ids.numel(),
                   ptr(flatten_ids) if flatten_ids.numel() else None, ptr(rc), ptr(ra), ptr(last), ptr(ws),
                   ws.numel(), ptr(qmask), q_b, ptr(bwd_ws), 0 if bwd_ws is None else bwd_ws.numel(),
                   None if deferred is None else ptr(deferred.info), N.stream(dev))
        else:
            ws_b = N.size_query("hgsr_raster3d_fwd_ws_bytes", C, Ng, D)
            ws = torch.empty(max(ws_b, 1), dtype=torch.uint8, device=dev)
            N.call("hgsr_raster3d_fwd_fused", C, Ng, Dc, ptr(means2d), ptr(conics), ptr(colors), int(col_shared),
                   ptr(depths), int(expected_depth), ptr(opacities), int(op_shared), ptr(backgrounds), width,
                   height, tile_size, tw, th, ptr(isect_offsets), flatten_ids.numel(),
                   ptr(flatten_ids) if flatten_ids.numel() else None, ptr(rc), ptr(ra), ptr(last), ptr(ws), ws_b,
                   N.stream(dev))
        ctx.save_for_backward(means2d, conics, colors, depths, opacities, backgrounds, isect_offsets, flatten_ids,
                              rc, ra, last)
        ctx.cfg = (width, height, tile_size, expected_depth, absgrad, Dc, col_shared, op_shared)
        ctx.fwd_ws = ws  # packed raster records, reused by the backward
        ctx.qmask = qmask
        ctx.deferred = deferred
        ctx.radii = None if radii is None else radii.detach().contiguous()
        ctx.fwd_slots = records is not None and radii is not None  # pack(radii=...) filled the slots
        return rc, ra

    @staticmethod
    def backward(ctx, v_rc, v_ra):
        means2d, conics, colors, depths, opacities, backgrounds, offsets, flatten_ids, rc, ra, last = ctx.saved_tensors
        width, height, tile_size, expected_depth, absgrad, Dc, col_shared, op_shared = ctx.cfg
        C, Ng = means2d.shape[:2]
        D = Dc + (0 if depths is None else 1)
        th, tw = offsets.shape[1:]
        dev = means2d.device
        v_means2d = torch.empty_like(means2d)
        v_conics = torch.empty_like(conics)
        v_colors = None if colors is None else torch.empty_like(colors)
        v_depths = None if depths is None else torch.empty_like(depths)
        v_opac = torch.empty_like(opacities)
        v_abs = torch.empty_like(means2d) if absgrad else None
        fwd_ws = ctx.fwd_ws
        n_is = flatten_ids.numel() if ctx.deferred is None else ctx.deferred.n  # exact once resolved
        ws_b = N.size_query("hgsr_raster3d_bwd_ws_bytes", C, Ng, D, n_is, int(fwd_ws is not None))
        ws, zeroed = _take_bwd_ws(ctx, ws_b, dev)
        v_rc, v_ra = _f32(v_rc), _f32(v_ra)
        N.call("hgsr_raster3d_bwd_fused", C, Ng, Dc, ptr(means2d), ptr(conics), ptr(colors), int(col_shared),
               ptr(depths), int(expected_depth), ptr(opacities), int(op_shared), ptr(backgrounds), width, height,
               tile_size, tw, th, ptr(offsets), n_is, ptr(flatten_ids) if n_is else None, ptr(rc), ptr(ra), ptr(last), ptr(v_rc), ptr(v_ra),
               ptr(v_means2d), ptr(v_conics), ptr(v_colors), ptr(v_depths), ptr(v_opac), ptr(v_abs), ptr(fwd_ws),
               ptr(ws), ws_b, ptr(ctx.qmask), 0 if ctx.qmask is None else ctx.qmask.numel(), zeroed,
               ptr(ctx.radii), int(ctx.fwd_slots), N.stream(dev))
        if absgrad:
            means2d.absgrad = v_abs
        v_bg = None
        if backgrounds is not None and ctx.needs_input_grad[5]:
            v_bg = (v_rc[..., :Dc] * (1.0 - ra)).sum(dim=(1, 2))
        return (v_means2d, v_conics, v_colors, v_depths, v_opac, v_bg, None, None, None, None, None, None, None,
                None, None, None, None)


def rasterize_to_pixels(means2d, conics, colors, opacities, image_width, image_height, tile_size, isect_offsets,
                        flatten_ids, backgrounds=None, masks=None, packed=False, absgrad=False):
    """gsplat rasterize_to_pixels (non-packed): colors [C,N,D] -> (render_colors [C,H,W,D], alphas [C,H,W,1])."""
    _unsupported(masks is not None, "tile masks")
    _unsupported(packed, "packed=True")
    _check_cuda(means2d, conics, colors, opacities, isect_offsets, flatten_ids)
    C, Ng = means2d.shape[:2]
    D = colors.shape[-1]
    assert colors.shape[:2] == (C, Ng) and opacities.shape == (C, Ng)
    args = (_f32(means2d), _f32(conics), None, _f32(opacities))
    outs, alphas = [], None
    for c0 in range(0, D, _MAX_CH):
        c1 = min(D, c0 + _MAX_CH)
        col = _f32(colors[..., c0:c1])
        bg = None if backgrounds is None else _f32(backgrounds[..., c0:c1])
        rc, ra = _Raster3D.apply(args[0], args[1], col, args[3], bg, int(image_width), int(image_height),
                                 int(tile_size), isect_offsets.contiguous(), flatten_ids.contiguous(), absgrad)
        outs.append(rc)
        if alphas is None:
            alphas = ra
    render_colors = outs[0] if len(outs) == 1 else torch.cat(outs, dim=-1)
    return render_colors, alphas


# =========================================================================
# rasterization (2DGS)
# =========================================================================
class _Raster2D(torch.autograd.Function):
    @staticmethod
    def forward(ctx, means2d, rt, colors, opacities, normals, densify, backgrounds, width, height, tile_size,
                isect_offsets, flatten_ids):
        C = isect_offsets.shape[0]
        Ng = means2d.shape[1]
        D = colors.shape[-1]
        th, tw = isect_offsets.shape[1:]
        dev = means2d.device
        rc = torch.empty((C, height, width, D), dtype=torch.float32, device=dev)
        ra = torch.empty((C, height, width, 1), dtype=torch.float32, device=dev)
        rn = torch.empty((C, height, width, 3), dtype=torch.float32, device=dev)
        rd = torch.empty((C, height, width, 1), dtype=torch.float32, device=dev)
        rm = torch.empty((C, height, width, 1), dtype=torch.float32, device=dev)
        last = torch.empty((C, height, width), dtype=torch.int32, device=dev)
        med = torch.empty((C, height, width), dtype=torch.int32, device=dev)
        ws_b = N.size_query("hgsr_raster2d_fwd_ws_bytes", C, Ng, D)
        ws = torch.empty(max(ws_b, 1), dtype=torch.uint8, device=dev)
        N.call("hgsr_raster2d_fwd", C, Ng, D, ptr(means2d), ptr(rt), ptr(colors), ptr(opacities), ptr(normals),
               ptr(backgrounds), width, height, tile_size, tw, th, ptr(isect_offsets), flatten_ids.numel(),
               ptr(flatten_ids) if flatten_ids.numel() else None, ptr(rc), ptr(ra), ptr(rn), ptr(rd), ptr(rm),
               ptr(last), ptr(med), ptr(ws), ws_b, N.stream(dev))
        ctx.save_for_backward(means2d, rt, colors, opacities, normals, backgrounds, isect_offsets, flatten_ids,
                              ra, last)
        ctx.cfg = (width, height, tile_size)
        ctx.fwd_ws = ws  # packed surfel records, reused by the backward
        ctx.mark_non_differentiable(rd, rm)
        ctx.set_materialize_grads(False)  # no zero-filled image grads for distort / median per step
        ctx.out_shapes = (rc.shape, ra.shape, rn.shape)
        return rc, ra, rn, rd, rm

    @staticmethod
    def backward(ctx, v_rc, v_ra, v_rn, v_rd, v_rm):
        means2d, rt, colors, opacities, normals, backgrounds, offsets, flatten_ids, ra, last = ctx.saved_tensors
        width, height, tile_size = ctx.cfg
        C, Ng, D = means2d.shape[0], means2d.shape[1], colors.shape[-1]
        th, tw = offsets.shape[1:]
        dev = means2d.device
        # the kernels overwrite every gradient element
        v_means2d = torch.empty_like(means2d)
        v_rt = torch.empty_like(rt)
        v_colors = torch.empty_like(colors)
        v_opac = torch.empty_like(opacities)
        v_normals = torch.empty_like(normals)
        v_dens = torch.empty_like(means2d)
        fwd_ws = ctx.fwd_ws
        ws_b = N.size_query("hgsr_raster2d_bwd_ws_bytes", C, Ng, D, flatten_ids.numel(), int(fwd_ws is not None))
        ws = torch.empty(max(ws_b, 1), dtype=torch.uint8, device=dev)
        v_rc, v_ra, v_rn = (_f32(g if g is not None else torch.zeros(sh, dtype=torch.float32, device=dev))
                            for g, sh in zip((v_rc, v_ra, v_rn), ctx.out_shapes))
        N.call("hgsr_raster2d_bwd", C, Ng, D, ptr(means2d), ptr(rt), ptr(colors), ptr(opacities), ptr(normals),
               ptr(backgrounds), width, height, tile_size, tw, th, ptr(offsets), flatten_ids.numel(),
               ptr(flatten_ids) if flatten_ids.numel() else None, ptr(ra), ptr(last), ptr(v_rc), ptr(v_ra),
               ptr(v_rn), ptr(v_means2d), ptr(v_rt), ptr(v_colors), ptr(v_opac), ptr(v_normals), ptr(v_dens),
               ptr(fwd_ws), ptr(ws), ws_b, N.stream(dev))
        v_bg = None
        if backgrounds is not None and ctx.needs_input_grad[6]:
            v_bg = (v_rc * (1.0 - ra)).sum(dim=(1, 2))
        return v_means2d, v_rt, v_colors, v_opac, v_normals, v_dens, v_bg, None, None, None, None, None


class _Raster2DFused(torch.autograd.Function):
    """rasterization_2dgs()'s colour assembly + rasterize_to_pixels_2dgs + ED as one
    native call each way (hgsr_raster2d_{fwd,bwd}_fused); see _Raster3DFused."""

    @staticmethod
    def pack(means2d, rt, colors, depths, opacities, normals, radii=None, tiles=(0, 0, 0), areas=None):
        """Surfel records for forward(records=...), packed while the host reads the count; with
        radii (a backward will follow) they carry their gradient slots (_Raster3DFused.pack)."""
        C, Ng = means2d.shape[:2]
        Dc = 0 if colors is None else colors.shape[-1]
        D = Dc + (0 if depths is None else 1)
        ws_b = N.size_query("hgsr_raster2d_fwd_ws_bytes", C, Ng, D)
        ws = torch.empty(max(ws_b, 1), dtype=torch.uint8, device=means2d.device)
        N.call("hgsr_raster2d_pack_fused", C, Ng, Dc, ptr(means2d), ptr(rt), ptr(colors),
               int(colors is not None and colors.dim() == 2), ptr(depths), ptr(opacities), int(opacities.dim() == 1),
               ptr(normals), ptr(radii), ptr(areas), *tiles, ptr(ws), ws_b, N.stream(means2d.device))
        return ws

    @staticmethod
    def forward(ctx, means2d, rt, colors, depths, opacities, normals, densify, backgrounds, width, height,
                tile_size, isect_offsets, flatten_ids, expected_depth, records=None, grad_mode=True, deferred=None,
                frame=None, radii=None):
        """frame = (viewmats [C,4,4], Ks [C,3,3], normals_from_depth) with records: render_normals
        come out in world frame (the kernels apply R^T) and, with normals_from_depth, K13 runs on
        the depth channel here and is a sixth output whose gradient the raster backward adds to
        the depth channel's (no rotate / slice / sum kernels in torch)."""
        C, Ng = means2d.shape[:2]
        Dc = 0 if colors is None else colors.shape[-1]
        D = Dc + (0 if depths is None else 1)
        col_shared = colors is not None and colors.dim() == 2
        op_shared = opacities.dim() == 1
        th, tw = isect_offsets.shape[1:]
        dev = means2d.device
        rc = torch.empty((C, height, width, D), dtype=torch.float32, device=dev)
        ra = torch.empty((C, height, width, 1), dtype=torch.float32, device=dev)
        rn = torch.empty((C, height, width, 3), dtype=torch.float32, device=dev)
        rd = torch.empty((C, height, width, 1), dtype=torch.float32, device=dev)
        rm = torch.empty((C, height, width, 1), dtype=torch.float32, device=dev)
        last = torch.empty((C, height, width), dtype=torch.int32, device=dev)
        med = torch.empty((C, height, width), dtype=torch.int32, device=dev)
        qmask = None
        if records is not None:
            ws = records
            # the forward's per-quadrant culling bits, read back by the backward
            q_b = N.size_query("hgsr_raster3d_qmask_bytes", C, tw, th, flatten_ids.numel())
            qmask = torch.empty(q_b, dtype=torch.uint8, device=dev)
            # the backward's workspace, its gradient-slot flags cleared by this forward launch
            bwd_ws = _bwd_ws("hgsr_raster2d_bwd_ws_bytes", ctx, C, Ng, D, flatten_ids.numel(), dev, grad_mode)
            N.call("hgsr_raster2d_fwd_packed", C, Ng, Dc, int(depths is not None), int(expected_depth),
                   ptr(backgrounds), width, height, tile_size, tw, th, ptr(isect_offsets), flatten_ids.numel(),
                   ptr(flatten_ids) if flatten_ids.numel() else None, ptr(rc), ptr(ra), ptr(rn), ptr(rd), ptr(rm),
                   ptr(last), ptr(med), ptr(ws), ws.numel(), ptr(qmask), q_b, ptr(bwd_ws),
                   0 if bwd_ws is None else bwd_ws.numel(), None if deferred is None else ptr(deferred.info),
                   None if frame is None else ptr(frame[0]), N.stream(dev))
        else:
            assert frame is None, "frame needs the packed records"
            ws_b = N.size_query("hgsr_raster2d_fwd_ws_bytes", C, Ng, D)
            ws = torch.empty(max(ws_b, 1), dtype=torch.uint8, device=dev)
            N.call("hgsr_raster2d_fwd_fused", C, Ng, Dc, ptr(means2d), ptr(rt), ptr(colors), int(col_shared),
                   ptr(depths), int(expected_depth), ptr(opacities), int(op_shared), ptr(normals),
                   ptr(backgrounds), width, height, tile_size, tw, th, ptr(isect_offsets), flatten_ids.numel(),
                   ptr(flatten_ids) if flatten_ids.numel() else None, ptr(rc), ptr(ra), ptr(rn), ptr(rd), ptr(rm),
                   ptr(last), ptr(med), ptr(ws), ws_b, N.stream(dev))
        ctx.save_for_backward(means2d, rt, colors, depths, opacities, normals, backgrounds, isect_offsets,
                              flatten_ids, rc, ra, last)
        ctx.cfg = (width, height, tile_size, expected_depth, Dc, col_shared, op_shared)
        ctx.fwd_ws = ws  # packed surfel records, reused by the backward
        ctx.qmask = qmask  # the forward's quadrant culling bits, reused by the backward
        ctx.deferred = deferred
        ctx.frame = frame
        ctx.radii = None if radii is None else radii.detach().contiguous()
        ctx.fwd_slots = records is not None and radii is not None  # pack(radii=...) filled the slots
        nfd = None
        if frame is not None and frame[2] and depths is not None:
            # K13 on the rendered depth channel (read in place through its strides), world frame
            dch = rc[..., D - 1]
            st = (ct.c_int64 * 3)(*dch.stride())
            nfd = torch.empty((C, height, width, 3), dtype=torch.float32, device=dev)
            N.call("hgsr_depth_normal_fwd", C, height, width, dch.data_ptr(), ct.cast(st, ct.c_void_p),
                   ptr(frame[0]), ptr(frame[1]), 1, 1, ptr(nfd), N.stream(dev))
        ctx.mark_non_differentiable(rd, rm)
        ctx.set_materialize_grads(False)  # no zero-filled image grads for distort / median per step
        ctx.out_shapes = (rc.shape, ra.shape, rn.shape)
        return rc, ra, rn, rd, rm, nfd

    @staticmethod
    def backward(ctx, v_rc, v_ra, v_rn, v_rd, v_rm, v_nfd=None):
        (means2d, rt, colors, depths, opacities, normals, backgrounds, offsets, flatten_ids, rc, ra,
         last) = ctx.saved_tensors
        width, height, tile_size, expected_depth, Dc, col_shared, op_shared = ctx.cfg
        C, Ng = means2d.shape[:2]
        D = Dc + (0 if depths is None else 1)
        th, tw = offsets.shape[1:]
        dev = means2d.device
        v_means2d = torch.empty_like(means2d)
        v_rt = torch.empty_like(rt)
        v_colors = None if colors is None else torch.empty_like(colors)
        v_depths = None if depths is None else torch.empty_like(depths)
        v_opac = torch.empty_like(opacities)
        v_normals = torch.empty_like(normals)
        v_dens = torch.empty_like(means2d)
        fwd_ws = ctx.fwd_ws
        n_is = flatten_ids.numel() if ctx.deferred is None else ctx.deferred.n  # exact once resolved
        ws_b = N.size_query("hgsr_raster2d_bwd_ws_bytes", C, Ng, D, n_is, int(fwd_ws is not None))
        ws, zeroed = _take_bwd_ws(ctx, ws_b, dev)
        v_rc, v_ra, v_rn = (_f32(g if g is not None else torch.zeros(sh, dtype=torch.float32, device=dev))
                            for g, sh in zip((v_rc, v_ra, v_rn), ctx.out_shapes))
        frame, v_dep = ctx.frame, None
        if v_nfd is not None:  # K13 backward: its depth gradient goes into the raster backward
            dch = rc[..., D - 1]
            st = (ct.c_int64 * 3)(*dch.stride())
            v_dep = torch.empty((C, height, width), dtype=torch.float32, device=dev)
            N.call("hgsr_depth_normal_bwd", C, height, width, dch.data_ptr(), ct.cast(st, ct.c_void_p),
                   ptr(frame[0]), ptr(frame[1]), 1, 1, ptr(_f32(v_nfd)), ptr(v_dep), N.stream(dev))
        N.call("hgsr_raster2d_bwd_fused", C, Ng, Dc, ptr(means2d), ptr(rt), ptr(colors), int(col_shared),
               ptr(depths), int(expected_depth), ptr(opacities), int(op_shared), ptr(normals), ptr(backgrounds),
               width, height, tile_size, tw, th, ptr(offsets), n_is, ptr(flatten_ids) if n_is else None, ptr(rc), ptr(ra), ptr(last), ptr(v_rc), ptr(v_ra),
               ptr(v_rn), ptr(v_means2d), ptr(v_rt), ptr(v_colors), ptr(v_depths), ptr(v_opac), ptr(v_normals),
               ptr(v_dens), ptr(fwd_ws), ptr(ws), ws_b, ptr(ctx.qmask), 0 if ctx.qmask is None else ctx.qmask.numel(),
               zeroed, None if frame is None else ptr(frame[0]), ptr(v_dep), ptr(ctx.radii), int(ctx.fwd_slots),
               N.stream(dev))
        v_bg = None
        if backgrounds is not None and ctx.needs_input_grad[7]:
            v_bg = (v_rc[..., :Dc] * (1.0 - ra)).sum(dim=(1, 2))
        return (v_means2d, v_rt, v_colors, v_depths, v_opac, v_normals, v_dens, v_bg, None, None, None, None, None,
                None, None, None, None, None, None)


def rasterize_to_pixels_2dgs(means2d, ray_transforms, colors, opacities, normals, densify, image_width,
                             image_height, tile_size, isect_offsets, flatten_ids, backgrounds=None, masks=None,
                             packed=False, absgrad=False, distloss=False):
    """gsplat rasterize_to_pixels_2dgs -> (colors, alphas, normals, distort, median).

    The last colour channel must be the depth (RGB+ED/RGB+D).  The distortion
    map is computed but, as in gsplat with distloss=False, not differentiated."""
    _unsupported(masks is not None, "tile masks")
    _unsupported(packed, "packed=True")
    _unsupported(absgrad, "absgrad for 2DGS")
    _unsupported(distloss, "distloss backward")
    _check_cuda(means2d, ray_transforms, colors, opacities, normals, isect_offsets, flatten_ids)
    C, Ng = means2d.shape[:2]
    D = colors.shape[-1]
    if D > _MAX_CH:
        raise NotImplementedError("hgsr: 2DGS rasterization supports at most 4 channels (RGB+depth)")
    if densify is None:
        densify = torch.zeros_like(means2d)
    rc, ra, rn, rd, rm = _Raster2D.apply(
        _f32(means2d), _f32(ray_transforms.reshape(C, Ng, 9)), _f32(colors), _f32(opacities), _f32(normals),
        densify, None if backgrounds is None else _f32(backgrounds), int(image_width), int(image_height),
        int(tile_size), isect_offsets.contiguous(), flatten_ids.contiguous())
    return rc, ra, rn, rd, rm


# =========================================================================
# high-level entry points
# =========================================================================
def _colors_for_raster(means, colors, viewmats, radii, sh_degree, C, means_sink=None):
    """Colours per raster call: [N,D] (shared over cameras) or [C,N,D]."""
    if sh_degree is None:
        return colors
    # gsplat: dirs = means - campos, spherical_harmonics(masks = radii > 0), clamp_min(+0.5, 0),
    # fused into one native call each way (no dirs tensor, no elementwise glue)
    _check_cuda(means, colors, viewmats)
    K = colors.shape[-2]
    assert colors.shape[-1] == 3 and colors.dim() in (3, 4) and (sh_degree + 1) ** 2 <= K, "bad SH coefficients"
    # the camera centres -R^T t are computed in the SH kernels from the view matrices
    return _SHColors.apply(int(sh_degree), _f32(means), None, _f32(colors), radii.contiguous(),
                           _f32(viewmats.detach().reshape(-1, 4, 4)), means_sink)


def _with_depth(colors, backgrounds, depths, render_mode, C):
    if render_mode in ("RGB+D", "RGB+ED"):
        colors = torch.cat((colors, depths[..., None]), dim=-1)
        if backgrounds is not None:
            backgrounds = torch.cat([backgrounds, torch.zeros(C, 1, device=backgrounds.device)], dim=-1)
    elif render_mode in ("D", "ED"):
        colors = depths[..., None]
        if backgrounds is not None:
            backgrounds = torch.zeros(C, 1, device=backgrounds.device)
    return colors, backgrounds


# Parameter-ready hooks: called by rasterization() / rasterization_2dgs() with the colour
# tensor right before the first kernel that reads it (after the projection and the intersection
# count are queued).  multigpu.ShardedAdamDDP(defer=[colours]) registers its wait_deferred here,
# so the colours' all-gather of the previous step lands under this step's first kernels.
_READY_HOOKS = []


def register_param_ready_hook(fn):
    """fn(*tensors) before rasterization reads the colours; returns a remover."""
    _READY_HOOKS.append(fn)
    return lambda: _READY_HOOKS.remove(fn) if fn in _READY_HOOKS else None


def _params_ready(*tensors):
    for fn in tuple(_READY_HOOKS):
        fn(*tensors)


def rasterization(means, quats, scales, opacities, colors, viewmats, Ks, width, height, near_plane=0.01,
                  far_plane=1e10, radius_clip=0.0, eps2d=0.3, sh_degree=None, packed=True, tile_size=16,
                  backgrounds=None, render_mode="RGB", sparse_grad=False, absgrad=False,
                  rasterize_mode="classic", channel_chunk=32, distributed=False, camera_model="pinhole",
                  covars=None):
    """gsplat.rasterization (3DGS) -> (render_colors [C,H,W,D], render_alphas [C,H,W,1], meta)."""
    assert render_mode in ("RGB", "D", "ED", "RGB+D", "RGB+ED"), render_mode
    _unsupported(packed, "packed=True (pass packed=False as Horizon-GS does)")
    _unsupported(rasterize_mode != "classic", f"rasterize_mode={rasterize_mode}")
    _unsupported(distributed, "distributed=True")
    C = viewmats.shape[0]
    # SH colours: their means gradient goes to the projection backward's kernel (GradSink)
    msink = (GradSink() if _GRAD_SINK and sh_degree is not None and torch.is_grad_enabled() and means.requires_grad
             else None)
    radii, means2d, depths, conics, _ = _projection(
        means, covars, quats, scales, viewmats, Ks, width, height, eps2d, False, near_plane, far_plane, radius_clip,
        sparse_grad, False, camera_model, msink)
    tw, th = _tile_grid(width, height, tile_size)
    isect_state = _isect_count(means2d, radii, int(tile_size), tw, th, depths)
    _params_ready(colors)
    cols = _colors_for_raster(means, colors, viewmats, radii, sh_degree, C, msink)
    with_depth = render_mode in ("RGB+D", "RGB+ED", "D", "ED")
    rgb = render_mode in ("RGB", "RGB+D", "RGB+ED")
    Dc = cols.shape[-1] if rgb else 0
    if Dc + int(with_depth) <= _MAX_CH:
        # one fused native call each way: no cat / repeat / ED divide in torch; the raster
        # records are packed while the host waits for the intersection count
        r_in = (_f32(means2d), _f32(conics), _f32(cols) if rgb else None, _f32(depths) if with_depth else None,
                _f32(opacities))
        ed, grad_mode = render_mode in ("ED", "RGB+ED"), torch.is_grad_enabled()
        # a backward will follow: the records carry their gradient slots (the same radii go to
        # the Function, whose backward then finds them there)
        slot_radii = radii.contiguous() if grad_mode and any(t is not None and t.requires_grad for t in r_in) else None
        records = _Raster3DFused.pack(*(t.detach() if t is not None else None for t in r_in), radii=slot_radii,
                                      tiles=(int(tile_size), tw, th), areas=isect_state[3])
        bgs = None if (backgrounds is None or not rgb) else _f32(backgrounds)
        args = (bgs, int(width), int(height), int(tile_size))
        tpg, isect_offsets = isect_state[3], isect_state[4]
        d = _isect_emit_deferred(isect_state)
        if d is not None:  # emission, sort and forward queued; then the count is read
            render_colors, render_alphas = _Raster3DFused.apply(*r_in, *args, isect_offsets, d.flat, ed, absgrad,
                                                                records, grad_mode, d, slot_radii)
            if _isect_resolve(isect_state, d):
                isect_ids, flatten_ids = d.ids[:d.n], d.flat[:d.n]
            else:
                d = None  # over capacity: nothing was emitted or composited; redo at the exact size
        if d is None:
            tpg, isect_ids, flatten_ids, isect_offsets = _isect_finish(isect_state)
            render_colors, render_alphas = _Raster3DFused.apply(*r_in, *args, isect_offsets, flatten_ids, ed,
                                                                absgrad, records, grad_mode, None, slot_radii)
        opac = opacities.expand(C, -1)
    else:
        tpg, isect_ids, flatten_ids, isect_offsets = _isect_finish(isect_state)
        opac = opacities.repeat(C, 1)
        if cols.dim() == 2:
            cols = cols.expand(C, -1, -1)
        cols, bgs = _with_depth(cols, backgrounds, depths, render_mode, C)
        render_colors, render_alphas = rasterize_to_pixels(
            means2d, conics, cols, opac, width, height, tile_size, isect_offsets, flatten_ids, backgrounds=bgs,
            absgrad=absgrad)
        if render_mode in ("ED", "RGB+ED"):
            render_colors = torch.cat([render_colors[..., :-1],
                                       render_colors[..., -1:] / render_alphas.clamp(min=1e-10)], dim=-1)
    meta = {
        "camera_ids": None, "gaussian_ids": None, "radii": radii, "means2d": means2d, "depths": depths,
        "conics": conics, "opacities": opac, "tile_width": tw, "tile_height": th,
        "tiles_per_gauss": tpg, "isect_ids": isect_ids, "flatten_ids": flatten_ids,
        "isect_offsets": isect_offsets, "width": width, "height": height, "tile_size": tile_size,
        "n_cameras": C,
    }
    return render_colors, render_alphas, meta


class _DepthToNormal(torch.autograd.Function):
    """K13 on the device (hgsr_depth_normal_{fwd,bwd}); gradient to the depth map only."""

    @staticmethod
    def forward(ctx, depths, camtoworlds, Ks, z_depth, from_viewmat=False):
        C, H, W = depths.shape[0], depths.shape[-3], depths.shape[-2]
        d = depths.reshape(C, H, W, -1)[..., 0] if depths.dim() == 4 else depths
        if d.dtype != torch.float32:
            d = d.float()
        st = (ct.c_int64 * 3)(*d.stride())
        c2w, K = _f32(camtoworlds), _f32(Ks)
        out = torch.empty((C, H, W, 3), dtype=torch.float32, device=d.device)
        N.call("hgsr_depth_normal_fwd", C, H, W, d.data_ptr(), ct.cast(st, ct.c_void_p), ptr(c2w), ptr(K),
               int(z_depth), int(from_viewmat), ptr(out), N.stream(d.device))
        ctx.save_for_backward(d, c2w, K)
        ctx.cfg = (z_depth, depths.shape, from_viewmat)
        return out

    @staticmethod
    def backward(ctx, v_normals):
        d, c2w, K = ctx.saved_tensors
        z_depth, shape, from_viewmat = ctx.cfg
        C, H, W = d.shape
        st = (ct.c_int64 * 3)(*d.stride())
        v_depth = torch.empty((C, H, W), dtype=torch.float32, device=d.device)
        vn = _f32(v_normals)
        N.call("hgsr_depth_normal_bwd", C, H, W, d.data_ptr(), ct.cast(st, ct.c_void_p), ptr(c2w), ptr(K),
               int(z_depth), int(from_viewmat), ptr(vn), ptr(v_depth), N.stream(d.device))
        return v_depth.reshape(shape), None, None, None, None


def depth_to_normal(depths, camtoworlds, Ks, z_depth=True):
    """K13: central-difference normals of the unprojected depth map [C,H,W,1] -> [C,H,W,3]
    (the gsplat fork's depth_to_normal; HIP kernels, gradient to the depth map)."""
    _check_cuda(depths, camtoworlds, Ks)
    _unsupported(camtoworlds.requires_grad or Ks.requires_grad, "depth_to_normal gradients w.r.t. the cameras")
    return _DepthToNormal.apply(depths, camtoworlds.detach(), Ks.detach(), bool(z_depth))


class _Rotate3(torch.autograd.Function):
    """vectors [C,...,3] -> R_c v (hgsr_rotate3); the vjp applies R_c^T.  R ([C,3,3], or [C,4,4]
    whose rotation block is used) carries no gradient; transpose=True applies R_c^T forward
    (camera -> world from world -> camera viewmats)."""

    @staticmethod
    def forward(ctx, R, v, transpose=False):
        C = v.shape[0]
        vc = _f32(v)
        out = torch.empty_like(vc)
        Rc = _f32(R)
        cs, rs = (16, 4) if Rc.shape[-1] == 4 else (9, 3)
        N.call("hgsr_rotate3", C, vc.numel() // (3 * C), ptr(Rc), cs, rs, int(transpose), ptr(vc), ptr(out),
               N.stream(v.device))
        ctx.save_for_backward(Rc)
        ctx.cfg = (cs, rs, transpose)
        return out

    @staticmethod
    def backward(ctx, g):
        (Rc,) = ctx.saved_tensors
        cs, rs, transpose = ctx.cfg
        C = g.shape[0]
        gc = _f32(g)
        out = torch.empty_like(gc)
        N.call("hgsr_rotate3", C, gc.numel() // (3 * C), ptr(Rc), cs, rs, int(not transpose), ptr(gc), ptr(out),
               N.stream(g.device))
        return None, out, None


def rasterization_2dgs(means, quats, scales, opacities, colors, viewmats, Ks, width, height, near_plane=0.01,
                       far_plane=1e10, radius_clip=0.0, eps2d=0.3, sh_degree=None, packed=False, tile_size=16,
                       backgrounds=None, render_mode="RGB", sparse_grad=False, absgrad=False, distloss=False,
                       depth_mode="expected"):
    """gsplat.rasterization_2dgs in the fork's nesting (render.py:56-76):
    ((colors, alphas, normals, normals_from_depth, distort, median), meta).

    Decisions where the fork is unverifiable here: rendered normals
    and depth normals are in world frame; normals_from_depth uses the expected
    (or, depth_mode="median", the median) depth; means2d's gradient is the exact
    chain-rule gradient and the densification proxy goes to meta["gradient_2dgs"].grad."""
    assert render_mode in ("RGB", "D", "ED", "RGB+D", "RGB+ED"), render_mode
    _unsupported(packed, "packed=True")
    _unsupported(distloss, "distloss backward")
    C, Ng = viewmats.shape[0], means.shape[0]
    densifications = torch.zeros((C, Ng, 2), dtype=means.dtype, device=means.device, requires_grad=True)
    radii, means2d, depths, ray_transforms, normals = fully_fused_projection_2dgs(
        means, quats, scales, viewmats, densifications, Ks, width, height, eps2d=eps2d, packed=False,
        near_plane=near_plane, far_plane=far_plane, radius_clip=radius_clip, sparse_grad=sparse_grad)
    tw, th = _tile_grid(width, height, tile_size)
    isect_state = _isect_count(means2d, radii, int(tile_size), tw, th, depths)
    _params_ready(colors)
    cols = _colors_for_raster(means, colors, viewmats, radii, sh_degree, C)
    with_depth = render_mode in ("RGB+D", "RGB+ED", "D", "ED")
    rgb = render_mode in ("RGB", "RGB+D", "RGB+ED")
    Dc = cols.shape[-1] if rgb else 0
    if Dc + int(with_depth) <= _MAX_CH and not absgrad:
        # one fused native call each way: no cat / repeat / ED divide in torch; the surfel
        # records are packed while the host waits for the intersection count
        r_in = (_f32(means2d), _f32(ray_transforms.reshape(C, Ng, 9)), _f32(cols) if rgb else None,
                _f32(depths) if with_depth else None, _f32(opacities), _f32(normals))
        ed, grad_mode = render_mode in ("ED", "RGB+ED"), torch.is_grad_enabled()
        # a backward will follow: the records carry their gradient slots (same radii to the Function)
        slot_radii = radii.contiguous() if grad_mode and (densifications.requires_grad or any(
            t is not None and t.requires_grad for t in r_in)) else None
        records = _Raster2DFused.pack(*(t.detach() if t is not None else None for t in r_in), radii=slot_radii,
                                      tiles=(int(tile_size), tw, th), areas=isect_state[3])
        bgs = None if (backgrounds is None or not rgb) else _f32(backgrounds)
        opac = opacities.expand(C, -1)
        args = (densifications, bgs, int(width), int(height), int(tile_size))
        # world-frame normals and (expected / raw depth channel) K13 inside the fused Function
        _unsupported(viewmats.requires_grad or Ks.requires_grad, "rasterization_2dgs gradients w.r.t. the cameras")
        frame = (_f32(viewmats.detach()), _f32(Ks.detach()),
                 render_mode in ("RGB+ED", "RGB+D") and depth_mode != "median") if _FUSE_FRAME else None
        tpg, isect_offsets = isect_state[3], isect_state[4]
        d = _isect_emit_deferred(isect_state)
        if d is not None:  # emission, sort and forward queued; then the count is read
            outs = _Raster2DFused.apply(*r_in, *args, isect_offsets, d.flat, ed, records, grad_mode, d, frame,
                                        slot_radii)
            if _isect_resolve(isect_state, d):
                isect_ids, flatten_ids = d.ids[:d.n], d.flat[:d.n]
            else:
                d = None  # over capacity: redo at the exact size
        if d is None:
            tpg, isect_ids, flatten_ids, isect_offsets = _isect_finish(isect_state)
            outs = _Raster2DFused.apply(*r_in, *args, isect_offsets, flatten_ids, ed, records, grad_mode, None, frame,
                                        slot_radii)
        render_colors, render_alphas, render_normals, render_distort, render_median, nfd_fused = outs
        fused_frame = frame is not None
    else:
        tpg, isect_ids, flatten_ids, isect_offsets = _isect_finish(isect_state)
        opac = opacities.repeat(C, 1)
        if cols.dim() == 2:
            cols = cols.expand(C, -1, -1)
        cols, bgs = _with_depth(cols, backgrounds, depths, render_mode, C)
        render_colors, render_alphas, render_normals, render_distort, render_median = rasterize_to_pixels_2dgs(
            means2d, ray_transforms, cols, opac, normals, densifications, width, height, tile_size, isect_offsets,
            flatten_ids, backgrounds=bgs, absgrad=absgrad, distloss=distloss)
        if render_mode in ("ED", "RGB+ED"):
            render_colors = torch.cat([render_colors[..., :-1],
                                       render_colors[..., -1:] / render_alphas.clamp(min=1e-10)], dim=-1)
        fused_frame, nfd_fused = False, None
    # camera -> world rotations straight from the viewmats (R_c2w = R^T), no c2w tensor built
    _unsupported(viewmats.requires_grad or Ks.requires_grad, "rasterization_2dgs gradients w.r.t. the cameras")
    vm = _f32(viewmats.detach())
    render_normals_from_depth = nfd_fused
    if render_mode in ("RGB+ED", "RGB+D") and render_normals_from_depth is None:
        dmap = render_median if depth_mode == "median" else render_colors[..., -1:]
        _check_cuda(dmap, vm, Ks)
        render_normals_from_depth = _DepthToNormal.apply(dmap, vm, Ks.detach(), True, True)
    if not fused_frame:
        render_normals = _Rotate3.apply(vm, render_normals, True)  # camera -> world frame
    meta = {
        "camera_ids": None, "gaussian_ids": None, "radii": radii, "means2d": means2d, "depths": depths,
        "ray_transforms": ray_transforms, "normals": normals, "opacities": opac, "tile_width": tw,
        "tile_height": th, "tiles_per_gauss": tpg, "isect_ids": isect_ids, "flatten_ids": flatten_ids,
        "isect_offsets": isect_offsets, "width": width, "height": height, "tile_size": tile_size,
        "n_cameras": C, "gradient_2dgs": densifications,
    }
    return (render_colors, render_alphas, render_normals, render_normals_from_depth, render_distort,
            render_median), meta
