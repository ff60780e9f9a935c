"""Data parallelism for the multimodal train step (new capability; the reference is a
single CPU process).

One process per GPU; the (image, report) minibatch is sharded across ranks (weak scaling),
every rank holds a full replica, and the only exchange per step is the gradient
all-reduce: fp32 gradients are packed into ~64 MB buckets and reduced with
`torch.distributed.all_reduce` — RCCL over xGMI with the "nccl" backend on ROCm, gloo in
the CPU tests — then averaged.  Buckets are launched as soon as backward has produced
them: each bucket's all-reduce runs asynchronously (work handles) so RCCL moves bucket i
while the next is packed; `finish()` waits and scatters the averaged gradients back.
BatchNorm keeps per-replica batch statistics (DDP semantics, no SyncBN); clip_grad_norm_
runs after the all-reduce, so every rank clips identically.
"""
from __future__ import annotations

import os
import sys
import time
import weakref

import torch
import torch.distributed as dist

from .trace import rng

BUCKET_BYTES = 64 << 20
# whole flat gradient buffers below this travel in the packed buckets (see _launch)
SMALL_ARENA_BYTES = 16 << 20

# MMDX_DP_TRACE=1: per step, the collectives issued (kind, elements, dtype) and the host time
# of launch() / finish(); the 8th step's record is printed to stderr (tools/lab/r05_rccl.sh)
_TRACE = ({"calls": [], "host": [], "step": 0}
          if os.environ.get("MMDX_DP_TRACE", "0") == "1" else None)


def _trace_step():
    _TRACE["step"] += 1
    if _TRACE["step"] == 8:
        print("[dp-trace] collectives:", _TRACE["calls"], file=sys.stderr)
        print("[dp-trace] host ms:", [(k, round(v * 1e3, 3)) for k, v in _TRACE["host"]],
              file=sys.stderr)
    _TRACE["calls"], _TRACE["host"] = [], []


class GradAllReducer:
    """Mean all-reduce of `.grad` over the ranks.

    `launch(params)` starts the asynchronous all-reduce of those parameters' gradients as
    soon as they are final — from the stream that produced them, so RCCL runs beside the
    rest of the backward (the text tower's and fusion head's gradients while the image trunk
    is still in its backward).  `finish()` waits for every launched collective on the
    current stream and writes the averages back.  `reduce()` = launch(all not yet
    launched) + finish().

    Gradients that are views covering one whole flat buffer (the ResNet trunk's gradient
    arena, resnet._TrunkFn) are reduced in place on that buffer — no pack/unpack copies;
    the rest are packed into `bucket_bytes` buckets.
    """

    def __init__(self, params, world_size: int | None = None, bucket_bytes: int = BUCKET_BYTES,
                 group=None, bucket_dtype: torch.dtype | None = None, rehearse: bool = False,
                 small_arena_bytes: int = SMALL_ARENA_BYTES):
        self.params = [p for p in params if p.requires_grad]
        self.world = world_size or dist.get_world_size(group)
        # rehearse: run every collective even in a 1-rank group (RCCL on one GPU exercises
        # the comm stream, the plan events and the write-back of the multi-GPU path)
        self.active = self.world > 1 or rehearse
        # RCCL averages inside the collective (ncclAvg): no separate 1/world pass over the
        # ~160 MB of fp32 gradients afterwards; gloo has no AVG (sum, then scale)
        self._avg = (self.active and dist.is_initialized()
                     and dist.get_backend(group) == "nccl")
        self.bucket_bytes = bucket_bytes
        self.small_arena_bytes = small_arena_bytes
        self.group = group
        # packed buckets may travel in bf16 (MMDX_DP_BUCKET_DTYPE=bf16: half the xGMI bytes
        # for C5's ~800 MB of per-tensor gradients; RCCL sums in bf16, the mean is taken in
        # fp32 after the cast back).  The trunk arena always reduces in fp32.
        if bucket_dtype is None and os.environ.get("MMDX_DP_BUCKET_DTYPE", "fp32") == "bf16":
            bucket_dtype = torch.bfloat16
        self.bucket_dtype = bucket_dtype
        self._pending = []
        self._launched = set()
        # flat buffer (keyed by its storage) -> [(lo, hi)] already launched by launch_region
        self._regions = {}
        self._comm = None
        # id(param) -> (weakref to the bucket view finish() rebound as its .grad, bucket kind):
        # a gradient that is still that view next step (accumulated, zero_grad(set_to_none=
        # False)) stays on the packed-bucket path of its kind, although the views together
        # tile one whole storage like an arena would
        self._rebound = {}

    def trunk_hook(self, grads, regions):
        """resnet.TRUNK_GRAD_HOOK: start the all-reduce of each layer's slice of the trunk's
        gradient arena from that layer's plan event (layers 4, 3, 2 in backward order)."""
        for lo, hi, ev in regions:
            self.launch_region(grads, lo, hi, ev)

    def trunk_segment(self, buf, lo: int, hi: int):
        """resnet.TRUNK_SEGMENT_HOOK: all-reduce buf[lo:hi] in place, issued from the current
        stream right after the last writer of the slice was enqueued on it.  With RCCL the
        collective's stream waits on the current stream, so it starts when the slice is
        final while the rest of the backward keeps running; no comm stream, no event, no
        copy (nothing reads or writes the slice again before finish())."""
        if not self.active or hi <= lo:
            return
        part = buf[lo:hi]
        with rng("mmdx/allreduce/trunk_segment"):
            work = self._all_reduce(part, "segment")
        self._pending.append((None, part, work, None))
        off = buf.storage_offset()
        self._regions.setdefault(_store_key(buf), []).append((off + lo, off + hi))

    def launch_region(self, buf, lo: int, hi: int, event=None):
        """Start the all-reduce of the slice buf[lo:hi] of a flat gradient buffer once
        `event` (a torch.cuda.Event recorded after the slice is final) has fired; the rest of
        the buffer is reduced by the next launch().  Used for the ResNet trunk's layers 4..2
        (resnet.TRUNK_GRAD_HOOK): ~90 % of the trunk's gradient bytes move over xGMI while
        the earlier layers' backward still runs.  With RCCL the host never waits: the comm
        stream waits on the event, the collectives queue on it in issue order."""
        if not self.active or hi <= lo:
            return
        view = buf[lo:hi]
        # reduced in a private copy, written back by finish() on the caller's stream: nothing
        # else ever sees the slice half-reduced (the backward is still running when this is
        # issued), and a backend's in-place write into a view never races a reader
        if event is not None and buf.is_cuda:
            if self._comm is None:
                self._comm = torch.cuda.Stream(device=buf.device)
            with torch.cuda.stream(self._comm):
                self._comm.wait_event(event)
                tmp = view.clone()
                work = self._all_reduce(tmp, "region")
            tmp.record_stream(torch.cuda.current_stream(buf.device))
        else:
            tmp = view.clone()
            work = self._all_reduce(tmp, "region")
        self._pending.append((None, tmp, work, view))
        off = buf.storage_offset()
        self._regions.setdefault(_store_key(buf), []).append((off + lo, off + hi))

    def _buckets(self, pairs):
        plan, cur, size = [], [], 0
        # reverse parameter order ~ order in which backward produces the gradients
        for p, g in reversed(pairs):
            cur.append((p, g))
            size += g.numel() * g.element_size()
            if size >= self.bucket_bytes:
                plan.append(cur)
                cur, size = [], 0
        if cur:
            plan.append(cur)
        return plan

    def launch(self, params=None):
        """Start the all-reduce of these parameters' gradients (default: all remaining)."""
        if not self.active:
            return
        t0 = time.perf_counter()
        with rng("mmdx/allreduce/launch"):
            self._launch(params)
        if _TRACE is not None:
            _TRACE["host"].append(("launch", time.perf_counter() - t0))

    def _launch(self, params):
        ps = self.params if params is None else [p for p in params if p.requires_grad]
        pairs = []
        loose = {"t": [], "a": []}   # per-tensor gradients / small whole arenas
        for p in ps:
            if id(p) in self._launched or p.grad is None:
                continue
            self._launched.add(id(p))
            r = self._rebound.get(id(p))
            if r is not None and r[0]() is p.grad:
                loose[r[1]].append((p, p.grad))
                continue
            pairs.append((p, p.grad))
        # Gradients that together tile one whole flat buffer (the ResNet trunk's gradient
        # arena, the encoder stacks') are reduced in place on that buffer, minus what
        # launch_region already started.  They are found by their shared STORAGE: autograd
        # stores a returned view detached (.grad._base is None), so the view relation itself
        # does not survive.  Small flat buffers (the BiLSTM's per-layer weight and bias
        # pairs, a few MB each) join the packed bucket instead: one collective per ~64 MB,
        # not one per buffer (each costs ~20 us of host issue at the end of the backward).
        # Small arenas keep fp32 in their bucket whatever bucket_dtype says: they were whole
        # fp32 buffers reduced in place before they joined the packed path.
        by_store = {}
        for p, g in pairs:
            by_store.setdefault(_store_key(g), []).append((p, g))
        for key, pgs in by_store.items():
            gs = [g for _, g in pgs]
            # a buffer that launch_region already started is the trunk's arena even when
            # frozen parameters leave gaps in it (their slots are reduced too, unused): the
            # rest must not also travel through the packed buckets
            started = key in self._regions
            flat = _whole_buffer(gs, allow_gaps=started)
            if flat is None:
                loose["t"] += pgs
                continue
            if not started and flat.numel() * flat.element_size() < self.small_arena_bytes:
                loose["a"] += pgs
                continue
            for a, z in _complement(self._regions.get(key, []), flat.numel()):
                part = flat[a:z]   # what launch_region left
                work = self._all_reduce(part, "arena")
                self._pending.append((None, part, work, None))
        if self.bucket_dtype is None:   # one dtype: one packed path
            loose["t"] += loose.pop("a")
        for kind in loose:
            for bucket in self._buckets(loose[kind]):
                flat = torch._utils._flatten_dense_tensors([g for _, g in bucket])
                if (kind == "t" and self.bucket_dtype is not None
                        and flat.dtype != self.bucket_dtype):
                    flat = flat.to(self.bucket_dtype)
                work = self._all_reduce(flat, f"bucket{'' if kind == 't' else '-arena'}"
                                              f"[{len(bucket)}]")
                self._pending.append((bucket, flat, work, None, kind))

    def _all_reduce(self, t, kind):
        if _TRACE is not None:
            _TRACE["calls"].append((kind, t.numel(), str(t.dtype)))
        return dist.all_reduce(t, op=self._op(t), group=self.group, async_op=True)

    def _op(self, t):
        # averaged in the collective for fp32 with RCCL; bf16 buckets sum in bf16 and take
        # the mean in fp32 after the cast back
        avg = self._avg and t.dtype == torch.float32
        return dist.ReduceOp.AVG if avg else dist.ReduceOp.SUM

    def finish(self):
        t0 = time.perf_counter()
        with rng("mmdx/allreduce/finish"):
            self._finish()
        if _TRACE is not None:
            _TRACE["host"].append(("finish", time.perf_counter() - t0))
            _trace_step()

    def _finish(self):
        inv = 1.0 / self.world
        cur = None
        for bucket, flat, work, dest, *kind in self._pending:
            work.wait()
            if flat.is_cuda:
                # the buffer may have been allocated on another stream (launch() issued from
                # the text stream): keep the allocator from reusing it before this stream's
                # reads below have run
                cur = cur or torch.cuda.current_stream(flat.device)
                flat.record_stream(cur)
            averaged = self._op(flat) == dist.ReduceOp.AVG
            if flat.dtype != torch.float32:
                flat = flat.float()
            if not averaged:
                flat.mul_(inv)
            if dest is not None:
                dest.copy_(flat)
            if bucket is not None:
                # the averaged bucket becomes the gradients: each .grad is rebound to its view
                # of `flat` (no copy back; the foreach copy it replaces was ~70 us of the
                # stream's tail at C4, after every other backward kernel)
                views = torch._utils._unflatten_dense_tensors(flat, [g for _, g in bucket])
                for (p, _), v in zip(bucket, views):
                    p.grad = v
                    self._rebound[id(p)] = (weakref.ref(v), kind[0])
        self._pending = []
        self._launched = set()
        self._regions = {}

    def reduce(self):
        """All-reduce (mean) every existing .grad across ranks, in place."""
        if not self.active:
            return
        self.launch()
        self.finish()


def _store_key(t):
    return (t.device.type, t.device.index, t.untyped_storage().data_ptr())


def _whole_buffer(gs, allow_gaps=False):
    """The flat 1-D tensor over the storage `gs` share when they are >= 2 contiguous,
    same-dtype tensors whose sizes add up to the whole storage (views of one arena, disjoint
    by construction), else None.  allow_gaps: a known arena (launch_region used it) whose
    views cover only part of it (frozen parameters' slots get no gradient)."""
    if len(gs) < 2 and not (allow_gaps and gs):
        return None
    g0 = gs[0]
    if any(g.dtype != g0.dtype or not g.is_contiguous() for g in gs):
        return None
    st = g0.untyped_storage()
    n = st.nbytes() // g0.element_size()
    if sum(g.numel() for g in gs) != n and not allow_gaps:
        return None
    return torch.empty(0, dtype=g0.dtype, device=g0.device).set_(st, 0, (n,), (1,))


def _complement(intervals, n):
    """[0, n) minus the union of the half-open `intervals`, as sorted (a, z) pieces."""
    out, cur = [], 0
    for lo, hi in sorted(intervals):
        if lo > cur:
            out.append((cur, lo))
        cur = max(cur, hi)
    if cur < n:
        out.append((cur, n))
    return out


def init_distributed(backend: str, local_rank: int, timeout_s: float = 300.0):
    """init_process_group with fail-fast semantics for the data-parallel step:
    RCCL's async errors are polled by torch's ProcessGroupNCCL watchdog
    (ncclCommGetAsyncError); TORCH_NCCL_ASYNC_ERROR_HANDLING=1 makes it tear the process
    down on an error or on a collective exceeding `timeout_s`, so a lost peer ends the job
    with a non-zero exit instead of hanging the node."""
    from datetime import timedelta
    os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
    if backend == "nccl":
        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank),
                                timeout=timedelta(seconds=timeout_s))
    else:
        dist.init_process_group(backend, timeout=timedelta(seconds=timeout_s))


def shard_batch(batch_size: int, rank: int, world: int):
    """Contiguous [start, stop) of the global batch owned by `rank` (global batch must
    divide evenly: C4 = 1024 over 8 ranks = 128 each)."""
    if batch_size % world:
        raise ValueError(f"global batch {batch_size} not divisible by world size {world}")
    per = batch_size // world
    return rank * per, (rank + 1) * per
