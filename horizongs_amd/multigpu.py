"""Multi-GPU mapping of the rasterizer path.

Two ways the path shards, one process per GPU (torch.distributed; backend "nccl"
is RCCL over xGMI on MI355X):

1. per-chunk (no collectives): the reference splits a large scene into m x n
   chunks (preprocess/generate_chunks_config.py:50-104) trained independently and
   joined only by merge.py (merge.py:132-217).  `chunks_for_rank` deals chunk
   configs to ranks; each rank trains its chunks alone.
2. data-parallel over views: every rank renders a different camera of one scene;
   after backward the Gaussian/anchor gradients are averaged with bucketed
   all-reduces (`GradientAllReduce`) and the densification statistics are
   reduced only at densify steps (`reduce_densify_stats`: sums, and max for the
   max-mode fields, reference scene/basic_model.py:96-144).  Every rank then runs the
   deterministic anchor_growing / prune on the same reduced statistics, so no parameters
   are broadcast; `assert_replicas_agree` checks that with a digest per rank (SURVEY.md
   §8(e): "verify with a hash").
"""
from __future__ import annotations

import os
from typing import Dict, Iterable, List, Sequence

import torch
import torch.distributed as dist

from . import gradbuf


def chunks_for_rank(chunks: Sequence[str], rank: int, world: int) -> List[str]:
    """Round-robin deal of chunk ids (e.g. '0_0'..'3_1' for Block_A) to ranks."""
    if world < 1 or not (0 <= rank < world):
        raise ValueError(f"bad rank/world {rank}/{world}")
    return [c for i, c in enumerate(chunks) if i % world == rank]


_FORCE = os.environ.get("HGSR_DDP_FORCE", "0") != "0"


class GradientAllReduce:
    """Bucketed gradient averaging across ranks, overlapped with the backward.

    * Buckets (~`bucket_mb` MiB of fp32: few, large collectives -- xGMI rings are per-link
      bound, so fewer calls of larger messages amortise the latency) are built from the
      optimizer's CURRENT param_groups and rebuilt whenever the parameter set changes, so
      densification surgery (cat_tensors_to_optimizer / prune, reference
      scene/lod_model.py:487-596) that replaces the Parameter objects is picked up.
    * A post-accumulate-grad hook copies each gradient, pre-scaled by 1 / world, into its
      bucket slice and makes that slice the parameter's .grad (no copy back after the
      collective).  A bucket's async all-reduce is launched as soon as all its parameters
      have a gradient -- i.e. while the backward is still running -- and buckets are always
      launched in bucket order, so every rank issues the same collectives in the same order.
    * Each bucket carries one presence slot per parameter: after the reduction a parameter
      no rank produced a gradient for keeps grad = None (torch.optim.Adam then skips it, as
      single-GPU training would), while one that some ranks did not reach averages their
      zeros in (the reference's mean over the views of a batch).

    * ``finish(step=...)`` applies the optimizer bucket by bucket: bucket b's parameters are
      stepped (one fused HIP Adam launch over just them) as soon as b's collective completes,
      while the collectives of the later buckets are still running on RCCL's stream -- the
      optimizer overlaps the communication instead of waiting for all of it.  Adam is
      elementwise, so the per-bucket launches give bit-identical parameters to one launch
      over everything (tests/test_multigpu_gloo.py).

    * Early gradients: between begin() and finish() the fused anchor decode's backward hands over
      the gradients that are final after its first (cov) head -- _offset, _scaling and the cov
      MLP -- through decode.set_early_grad_hook, so their buckets are all-reduced while the
      opacity and colour heads still run; `order` puts those parameters in the first buckets
      (buckets launch in bucket order on every rank).

    Usage per step: ``red.begin()`` before backward, ``loss.backward()``, then either
    ``red.finish()`` + ``optimizer.step()`` or ``red.finish(step=optimizer.step_params)``.
    Exactly ONE backward may run between begin() and finish(): a gradient that arrives for a
    bucket already in flight raises.  ``red()`` = begin-less synchronous form for grads
    already computed.

    order: parameters in the order they should be bucketed (those not listed follow, in reverse
    registration order) -- the order their gradients become final, e.g. (offset, scaling, cov MLP,
    feat, anchor, opacity MLP, colour MLP) for the anchor model."""

    def __init__(self, params_or_optimizer, bucket_mb: float = 64.0, group=None, order=None):
        self.source = params_or_optimizer
        self.group = group
        self.order = order
        self.cap = max(1, int(bucket_mb * (1 << 20) // 4))
        self._key = None
        self._hooks = []
        self.buckets: List[dict] = []
        self._in_step = False  # between begin() and finish(): the hooks copy into buckets

    # ---------------------------------------------------------------- setup
    def _params(self) -> List[torch.Tensor]:
        src = self.source
        if hasattr(src, "param_groups"):
            ps = [p for g in src.param_groups for p in g["params"]]
        else:
            ps = list(src)
        return [p for p in ps if p.requires_grad]

    def _active(self) -> bool:
        # HGSR_DDP_FORCE=1: a one-rank group runs the whole bucket / hook / RCCL path anyway (a
        # single-GPU rehearsal of the multi-GPU step; the all-reduce of one rank is the identity)
        return dist.is_initialized() and (dist.get_world_size(self.group) > 1 or _FORCE)

    def _bind(self) -> None:
        """(Re)build the buckets when the parameter objects changed.  Buckets follow the
        reverse parameter order, the order a backward usually produces the gradients."""
        params = self._params()
        key = tuple(id(p) for p in params) + tuple(p.numel() for p in params)
        if key == self._key:
            return
        for h in self._hooks:
            h.remove()
        self._hooks = []
        self.buckets = []
        cur, size = [], 0
        seq = list(reversed(params))
        if self.order is not None:
            ids = {id(p) for p in params}
            first = [p for p in self.order if id(p) in ids]
            fid = {id(p) for p in first}
            seq = first + [p for p in seq if id(p) not in fid]
        for p in seq:
            n = p.numel()
            if cur and size + n > self.cap:
                self.buckets.append(cur)
                cur, size = [], 0
            cur.append(p)
            size += n
        if cur:
            self.buckets.append(cur)
        self.buckets = [self._make_bucket(b) for b in self.buckets]
        self._where = {}
        for bi, b in enumerate(self.buckets):
            for k, p in enumerate(b["params"]):
                self._where[id(p)] = (bi, k)
                self._hooks.append(p.register_post_accumulate_grad_hook(self._on_grad))
        self._key = key

    @staticmethod
    def _make_bucket(params):
        offs, o = [], 0
        for p in params:
            offs.append(o)
            o += p.numel()
        dev = params[0].device
        # flat = [grads of every parameter | one presence slot per parameter]
        flat = torch.empty(o + len(params), dtype=torch.float32, device=dev)
        return {"params": params, "offs": offs, "n": o, "flat": flat, "ready": [False] * len(params),
                "early": [None] * len(params), "work": None, "launched": False}

    # ---------------------------------------------------------------- per step
    def begin(self) -> None:
        if not self._active():
            return
        self._bind()
        self.world = dist.get_world_size(self.group)
        self._next = 0
        for b in self.buckets:
            b["ready"] = [False] * len(b["params"])
            b["early"] = [None] * len(b["params"])
            b["work"], b["launched"] = None, False
        self._in_step = True
        from . import decode
        decode.set_early_grad_hook(self.early)

    def early(self, pairs) -> None:
        """Gradients final before the backward ends ([(parameter, gradient)], decode backward):
        copied into their buckets now, and the buckets that became complete are launched.

        The handed-over tensor must be the very gradient the caller's backward then returns
        for the parameter, and the only one: _on_grad checks that autograd's accumulated
        gradient IS that tensor (a second consumer of the parameter would have made autograd
        sum a new one, whose extra part the early collective never saw) and raises otherwise."""
        if not self._in_step:
            return
        for p, g in pairs:
            loc = self._where.get(id(p))
            if loc is None or g is None:
                continue
            b = self.buckets[loc[0]]
            k = loc[1]
            if b["launched"] or b["ready"][k]:
                raise RuntimeError("hgsr GradientAllReduce: an early gradient arrived for a parameter whose gradient "
                                   "is already in its bucket this step (exactly one backward, and one hand-off, "
                                   "between begin() and finish())")
            dst = b["flat"][b["offs"][k]:b["offs"][k] + p.numel()].view_as(p)
            torch.mul(g.reshape(p.shape), 1.0 / self.world, out=dst)
            b["ready"][k] = True
            # the storage address only: holding the tensor would make autograd copy it instead of
            # adopting it as .grad, and the check below relies on the adoption
            b["early"][k] = g.data_ptr()
        self._launch_ready()

    def _on_grad(self, p) -> None:
        # hooks stay registered between steps: a backward outside begin()/finish() (e.g. before
        # the synchronous red()) leaves the gradient alone
        if not self._in_step or not self._active() or p.grad is None:
            return
        bi, k = self._where[id(p)]
        b = self.buckets[bi]
        if b["early"][k] is not None:  # handed over by early(): autograd's adoption of it arrives now
            handed, b["early"][k] = b["early"][k], None
            if p.grad.data_ptr() != handed:
                raise RuntimeError(
                    "hgsr GradientAllReduce: the gradient autograd accumulated for a parameter differs from the one "
                    "the decode backward handed over early (another consumer of the parameter in this graph, or a "
                    "create_graph backward): its all-reduce already left with the decode's part only.  Train such "
                    "graphs without the early hand-off (decode.set_early_grad_hook(None) after begin()).")
            p.grad = b["flat"][b["offs"][k]:b["offs"][k] + p.numel()].view_as(p)
            return
        if b["launched"] or b["ready"][k]:
            raise RuntimeError("hgsr GradientAllReduce: a second gradient arrived for a parameter in this step (its "
                               "bucket's all-reduce may already be in flight); exactly one backward is allowed "
                               "between begin() and finish()")
        n = p.numel()
        dst = b["flat"][b["offs"][k]:b["offs"][k] + n].view_as(p)
        torch.mul(p.grad, 1.0 / self.world, out=dst)
        p.grad = dst  # the bucket slice is the gradient: no copy back after the collective
        b["ready"][k] = True
        self._launch_ready()

    def _launch(self, b) -> None:
        # presence slots written once per bucket on the device (a per-parameter Python scalar
        # store is a host-to-device copy, issued from inside the backward's hooks)
        if all(b["ready"]):
            b["flat"][b["n"]:].fill_(1.0)
        else:
            for k, p in enumerate(b["params"]):  # parameters this rank never reached: zeros, absent
                n = p.numel()
                if not b["ready"][k]:
                    b["flat"][b["offs"][k]:b["offs"][k] + n].zero_()
                b["flat"][b["n"] + k:b["n"] + k + 1].fill_(1.0 if b["ready"][k] else 0.0)
        b["work"] = dist.all_reduce(b["flat"], op=dist.ReduceOp.SUM, group=self.group, async_op=True)
        b["launched"] = True

    def _launch_ready(self) -> None:
        while self._next < len(self.buckets) and all(self.buckets[self._next]["ready"]):
            self._launch(self.buckets[self._next])
            self._next += 1

    @property
    def active(self) -> bool:
        return self._active()

    def finish(self, step=None) -> None:
        """Launch what the backward left (in bucket order), wait, set the averaged grads.
        step(params): optional per-bucket optimizer step, issued on the current stream right
        after each bucket's collective (overlapping the remaining ones)."""
        if not self._active():
            if step is not None:
                step(self._params())
            return
        self._in_step = False  # later gradients (a backward outside begin()/finish()) are not bucketed
        from . import decode
        decode.set_early_grad_hook(None)
        while self._next < len(self.buckets):
            self._launch(self.buckets[self._next])
            self._next += 1
        for b in self.buckets:
            b["work"].wait()  # NCCL/RCCL: the current stream waits for the collective; the host does not
            pres = b["flat"][b["n"]:].tolist() if not all(b["ready"]) else None
            for k, p in enumerate(b["params"]):
                n = p.numel()
                if pres is not None and pres[k] == 0.0:
                    p.grad = None  # no rank produced a gradient
                elif not b["ready"][k]:
                    p.grad = b["flat"][b["offs"][k]:b["offs"][k] + n].view_as(p)
            if step is not None:
                step(b["params"])

    def __call__(self) -> None:
        """Synchronous form: average gradients that are already in place (no overlap)."""
        if not self._active():
            return
        self.begin()
        for b in self.buckets:
            for p in b["params"]:
                if p.grad is not None:
                    self._on_grad(p)
        self.finish()


def _hip_adam(descs, betas, eps, device):
    """One fused HIP Adam launch over (param, grad, exp_avg, exp_avg_sq, numel, lr, step)
    segments (csrc/optim.hip, the kernel horizongs_amd.optim.Adam launches)."""
    import ctypes as ct

    from . import _native as NAT
    from .optim import _AdamTensor
    if not descs:
        return
    arr = (_AdamTensor * len(descs))(*[_AdamTensor(p.data_ptr(), g.data_ptr(), m.data_ptr(), v.data_ptr(), p.numel(),
                                                   lr, step) for p, g, m, v, lr, step in descs])
    NAT.call("hgsr_adam_step", len(descs), ct.cast(arr, ct.c_void_p), betas[0], betas[1], eps, NAT.stream(device))


class ShardedAdamDDP:
    """DDP over views with the optimizer state and step sharded across ranks (ZeRO stage 1),
    for the explicit-Gaussian step (bench c2 at N > 1).

    GradientAllReduce all-reduces every gradient and then every rank runs Adam over all of the
    parameters: 2 (N-1)/N S bytes per GPU on the links, then 28 B per parameter of HBM on every
    rank.  Here each bucket's gradients are reduce-scattered (each rank receives the sum over
    ranks of its 1/N shard), each rank runs Adam on its shard only (its exp_avg / exp_avg_sq
    shards live here, 1/N of the optimizer state), and the updated parameter shards are
    all-gathered back into every rank's parameters: the same link bytes as the all-reduce
    ((N-1)/N S each way), Adam's HBM traffic and state memory divided by N, and the all-gather of
    bucket b overlaps the optimizer step and collectives of the later buckets.

    * Buckets (~bucket_mb MiB) follow the optimizer's param_groups in reverse registration order
      (the order a backward produces gradients); every parameter of a bucket becomes a view into
      the bucket's flat parameter buffer (its values copied in), so the all-gather writes the
      parameters in place.  Bucket data is padded to a multiple of the world size.
    * Each gradient lands in its bucket's flat gradient buffer: begin() registers the buffer's
      slices as the parameters' gradient destinations (gradbuf), so the projection and
      activation backwards write into them and autograd adopts them as `.grad` without a copy;
      a gradient produced elsewhere is copied in by the post-accumulate-grad hook, which then
      drops `.grad`.  A complete bucket's reduce-scatter is launched during the backward,
      buckets in bucket order on every rank, and the 1/world of the mean is applied to the
      reduced shard (exact for power-of-two worlds).
    * Every rank must produce a gradient for every parameter in every step (the explicit
      Gaussians' step always does): a missing one raises instead of desynchronising the
      collectives.  Densification (new Parameter objects) is not supported under the sharded
      state and raises; use GradientAllReduce for the anchor model.
    * Adam: torch's single-tensor order of operations per element (the HIP kernel of
      optim.Adam), per-parameter learning rates from the groups, one step counter per
      parameter kept here (state that exists in the optimizer when the buckets are built --
      exp_avg / exp_avg_sq / step -- is taken over shard by shard).
    adam_fn(descs, betas, eps, device): the optimizer kernel over segments (default: the HIP
    launch); tests pass a CPU restatement.
    order (optional): the buckets themselves, a list of parameter lists in launch order (every
    trainable parameter exactly once; bucket_mb is then unused) -- e.g. the gradients the
    backward produces first in the first bucket.
    defer (optional): parameters whose bucket's all-gather finish() leaves in flight.  The next
    step may run kernels that do not read them (projection, binning) while it lands;
    wait_deferred() -- which rasterization() calls through gsplat_api's parameter-ready hooks
    before it first reads the colours, and begin() calls as a backstop -- makes the current
    stream wait for it.  A deferred parameter must not be read between finish() and that wait."""

    def __init__(self, optimizer, bucket_mb: float = 64.0, group=None, adam_fn=None, order=None, defer=None):
        self.opt = optimizer
        self.group = group
        self.cap = max(1, int(bucket_mb * (1 << 20) // 4))
        self.adam_fn = adam_fn or _hip_adam
        self.order = [list(b) for b in order] if order is not None else None
        self.defer_ids = {id(p) for p in (defer or ())}
        self._deferred = []
        self._key = None
        self._hooks = []
        self.buckets: List[dict] = []
        self._in_step = False
        self.copies = 0

    def _active(self) -> bool:
        return dist.is_initialized() and (dist.get_world_size(self.group) > 1 or _FORCE)

    @property
    def active(self) -> bool:
        return self._active()

    def _bind(self) -> None:
        entries = [(p, g) for g in self.opt.param_groups for p in g["params"] if p.requires_grad]
        key = tuple(id(p) for p, _ in entries) + tuple(p.numel() for p, _ in entries)
        if key == self._key:
            return
        if self._key is not None:
            raise NotImplementedError("hgsr ShardedAdamDDP: the parameter set changed (densification); the sharded "
                                      "optimizer state cannot follow it -- use GradientAllReduce")
        world = dist.get_world_size(self.group)
        rank = dist.get_rank(self.group)
        if self.order is not None:
            gof = {id(p): g for p, g in entries}
            listed = [id(p) for b in self.order for p in b]
            if sorted(listed) != sorted(gof) or len(set(listed)) != len(listed):
                raise ValueError("hgsr ShardedAdamDDP: order must list every trainable parameter exactly once")
            groups = [[(p, gof[id(p)]) for p in b] for b in self.order if b]
        else:
            cur, size, groups = [], 0, []
            for p, g in reversed(entries):
                if cur and size + p.numel() > self.cap:
                    groups.append(cur)
                    cur, size = [], 0
                cur.append((p, g))
                size += p.numel()
            if cur:
                groups.append(cur)
        for members in groups:
            d = [id(p) in self.defer_ids for p, _ in members]
            if any(d) and not all(d):
                raise ValueError("hgsr ShardedAdamDDP: a deferred parameter must share its bucket only with "
                                 "deferred parameters (pass order=)")
        self.buckets, self._where = [], {}
        for bi, members in enumerate(groups):
            n = sum(p.numel() for p, _ in members)
            L = (n + world - 1) // world
            dev, dt = members[0][0].device, members[0][0].dtype
            pflat = torch.zeros(world * L, dtype=dt, device=dev)
            offs, o = [], 0
            lo, hi = rank * L, rank * L + L
            m = torch.zeros(L, dtype=dt, device=dev)
            v = torch.zeros(L, dtype=dt, device=dev)
            steps = []
            for k, (p, g) in enumerate(members):
                nk = p.numel()
                with torch.no_grad():
                    pflat[o:o + nk].copy_(p.detach().reshape(-1))
                    p.data = pflat[o:o + nk].view_as(p)
                st = self.opt.state.get(p, {})
                steps.append(int(float(st["step"])) if "step" in st else 0)
                a, z = max(o, lo), min(o + nk, hi)
                if a < z and "exp_avg" in st:  # take the existing state's shard over
                    m[a - lo:z - lo].copy_(st["exp_avg"].reshape(-1)[a - o:z - o])
                    v[a - lo:z - lo].copy_(st["exp_avg_sq"].reshape(-1)[a - o:z - o])
                self.opt.state.pop(p, None)
                self._where[id(p)] = (bi, k)
                self._hooks.append(p.register_post_accumulate_grad_hook(self._on_grad))
                offs.append(o)
                o += nk
            # a one-parameter bucket whose size divides by the world reduce-scatters the gradient
            # tensor autograd produced, in place of a scaled copy into gflat (the 1/N goes onto
            # this rank's shard after the reduction: exact for power-of-two worlds)
            direct = len(members) == 1 and n == world * L
            self.buckets.append({"members": members, "offs": offs, "n": n, "L": L, "pflat": pflat,
                                 "direct": direct, "gsrc": None,
                                 "gflat": None if direct else torch.zeros(world * L, dtype=dt, device=dev),
                                 "gshard": torch.empty(L, dtype=dt, device=dev), "m": m, "v": v, "steps": steps,
                                 "ready": [False] * len(members), "work": None, "launched": False})
        self.rank, self.world = rank, world
        self._key = key

    def wait_deferred(self, *_tensors) -> None:
        """The current stream waits for the all-gathers finish() left in flight."""
        works, self._deferred = self._deferred, []
        for w in works:
            w.wait()

    def flush(self) -> None:
        """Make every parameter whole again: wait for the deferred all-gathers.  finish() returns
        with the colours' all-gather still writing p.data (rasterization()'s parameter-ready hook
        and the next begin() wait for it); call this before any other read of the parameters --
        a checkpoint or PLY save, replica_digest / assert_replicas_agree, an evaluation render
        outside gsplat_api."""
        self.wait_deferred()

    def begin(self) -> None:
        if not self._active():
            return
        self.wait_deferred()  # backstop: the next backward / Adam touch the deferred buffers
        self._bind()
        self._next = 0
        self.copies = 0  # gradients of this step the hook had to copy into a bucket (0: all in place)
        for b in self.buckets:
            b["ready"] = [False] * len(b["members"])
            b["work"], b["launched"], b["gsrc"] = None, False, None
            if not b["direct"]:  # the producing backward writes straight into the flat buffer
                for (p, _), o in zip(b["members"], b["offs"]):
                    gradbuf.set_dest(p, b["gflat"][o:o + p.numel()].view_as(p))
        self._in_step = True

    def _on_grad(self, p) -> None:
        if not self._in_step or p.grad is None:
            return
        bi, k = self._where[id(p)]
        b = self.buckets[bi]
        if b["launched"] or b["ready"][k]:
            raise RuntimeError("hgsr ShardedAdamDDP: a second gradient arrived for a parameter in this step; "
                               "exactly one backward is allowed between begin() and finish()")
        o, n = b["offs"][k], p.numel()
        g = p.grad
        if b["direct"] and g.is_contiguous() and g.dtype == b["pflat"].dtype:
            b["gsrc"] = g.reshape(-1)  # held until the reduce-scatter is waited for
        else:
            if b["gflat"] is None:
                b["gflat"] = torch.zeros(self.world * b["L"], dtype=b["pflat"].dtype, device=b["pflat"].device)
            dst = b["gflat"][o:o + n]
            if g.data_ptr() != dst.data_ptr() or not g.is_contiguous():  # produced elsewhere: copy it in
                dst.copy_(g.reshape(-1))
                self.copies += 1
            b["gsrc"] = None
        p.grad = None  # the reduced gradient exists only as this rank's shard
        b["ready"][k] = True
        while self._next < len(self.buckets) and all(self.buckets[self._next]["ready"]):
            self._launch(self.buckets[self._next])
            self._next += 1

    def _launch(self, b) -> None:
        if not all(b["ready"]):
            miss = [tuple(p.shape) for (p, _), r in zip(b["members"], b["ready"]) if not r]
            raise RuntimeError(f"hgsr ShardedAdamDDP: no gradient this step for parameters {miss}; every rank must "
                               "produce every gradient (use GradientAllReduce for partial graphs)")
        src = b["gsrc"] if b["gsrc"] is not None else b["gflat"]
        b["work"] = dist.reduce_scatter_tensor(b["gshard"], src, op=dist.ReduceOp.SUM, group=self.group,
                                               async_op=True)
        b["launched"] = True

    def finish(self) -> None:
        """Launch what the backward left, then per bucket: wait for its reduce-scatter, Adam on
        this rank's shard, launch the all-gather of the updated shard (which overlaps the later
        buckets); finally the current stream waits for every all-gather but the deferred ones.
        The deferred buckets are stepped and gathered last, whatever their place in `order`: the
        collectives of one group run in issue order, so an all-gather left in flight must not sit
        in front of one that is waited for (a deferred bucket may still come first in `order`, so
        that its reduce-scatter starts while the backward is still running)."""
        if not self._active():
            self.opt.step()
            return
        self._in_step = False
        while self._next < len(self.buckets):
            self._launch(self.buckets[self._next])
            self._next += 1
        gathers = []
        lo = self.rank
        deferred = [id(b["members"][0][0]) in self.defer_ids for b in self.buckets]
        gradbuf.clear()  # destinations no backward took
        for b in [b for b, d in zip(self.buckets, deferred) if not d] + [b for b, d in zip(self.buckets, deferred) if d]:
            b["work"].wait()
            b["gsrc"] = None
            if self.world > 1:  # reduced unscaled: the mean over ranks on the shard only
                b["gshard"].mul_(1.0 / self.world)
            L = b["L"]
            s0, s1 = lo * L, lo * L + L
            descs = {}
            for k, ((p, g), o) in enumerate(zip(b["members"], b["offs"])):
                b["steps"][k] += 1
                a, z = max(o, s0), min(o + p.numel(), s1)
                if a >= z:
                    continue
                key = (tuple(g["betas"]), float(g["eps"]))
                descs.setdefault(key, []).append((b["pflat"][a:z], b["gshard"][a - s0:z - s0], b["m"][a - s0:z - s0],
                                                  b["v"][a - s0:z - s0], float(g["lr"]), b["steps"][k]))
            for (betas, eps), dl in descs.items():
                self.adam_fn(dl, betas, eps, b["pflat"].device)
            w = dist.all_gather_into_tensor(b["pflat"], b["pflat"][s0:s1], group=self.group, async_op=True)
            (self._deferred if id(b["members"][0][0]) in self.defer_ids else gathers).append(w)
        for w in gathers:
            w.wait()

    def state_shard(self):
        """This rank's optimizer state: [(bucket, shard range, exp_avg, exp_avg_sq, steps)]."""
        return [(i, (self.rank * b["L"], self.rank * b["L"] + b["L"]), b["m"], b["v"], list(b["steps"]))
                for i, b in enumerate(self.buckets)]


MAX_FIELDS = ("max_radii2D",)


def reduce_densify_stats(stats: Dict[str, torch.Tensor], max_fields: Sequence[str] = MAX_FIELDS,
                         group=None) -> Dict[str, torch.Tensor]:
    """In-place cross-rank reduction of densification accumulators at a densify step:
    sums for the accumulators/denominators, max for the max-mode fields (and for
    offset_gradient_accum when growing_type == 'max', pass it in max_fields)."""
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return stats
    for k in sorted(stats):
        op = dist.ReduceOp.MAX if k in max_fields else dist.ReduceOp.SUM
        dist.all_reduce(stats[k], op=op, group=group)
    return stats


def replica_digest(tensors: Iterable[torch.Tensor]) -> torch.Tensor:
    """Order-sensitive 64-bit digest of the tensors' bytes, computed on their device
    (int64 arithmetic: bit-exact on every rank that holds identical tensors, whatever the
    reduction order).  Each tensor contributes its shape and its 32-bit words weighted by
    position; a one-bit difference anywhere changes the digest."""
    dev = None
    acc = None
    for i, t in enumerate(tensors):
        t = t.detach().contiguous()
        dev = t.device
        w = t.reshape(-1).view(torch.uint8)
        pad = (-w.numel()) % 4
        if pad:
            w = torch.cat([w, w.new_zeros(pad)])
        x = w.view(torch.int32).to(torch.int64)
        pos = torch.arange(1, x.numel() + 1, device=dev, dtype=torch.int64)
        h = ((x + (i + 1) * 0x9E3779B1) * (pos * 0x5BD1E995 + 0x27D4EB2F)).sum()
        h = h + (i + 1) * 1000003 * x.numel() + sum((k + 7) * int(n) for k, n in enumerate(t.shape))
        acc = h if acc is None else acc * 31 + h
    if acc is None:
        return torch.zeros((), dtype=torch.int64)
    return acc


def assert_replicas_agree(tensors: Sequence[torch.Tensor], group=None, what: str = "parameters") -> int:
    """Raise on every rank if the ranks' `tensors` differ (digest all-gather; after a densify
    step every rank must have grown / pruned the same anchors).  Returns the digest."""
    d = replica_digest(tensors)
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return int(d)
    dev = d.device if dist.get_backend(group) != "gloo" else torch.device("cpu")
    mine = d.reshape(1).to(dev)
    allv = [torch.zeros_like(mine) for _ in range(dist.get_world_size(group))]
    dist.all_gather(allv, mine, group=group)
    vals = [int(v) for v in allv]
    if len(set(vals)) != 1:
        raise RuntimeError(f"hgsr multigpu: the ranks' {what} differ after a replicated update (digests {vals})")
    return vals[0]

