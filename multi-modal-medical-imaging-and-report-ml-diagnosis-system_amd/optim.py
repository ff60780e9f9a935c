"""Fused AdamW + global-norm clipping on the mmdx kernels.

`AdamW` is a drop-in for the `torch.optim.AdamW` that the reference's `build_optimizer`
methods instantiate (training_pipeline.py:238-269, 408-432) and the fusion loop builds
(TP:1018-1023): same param-group API, same defaults, same update rule — executed as ONE
kernel over every tensor of every group (device-side descriptor table + device step
counter, so the step replays inside a hipGraph).  `clip_grad_norm_` mirrors
torch.nn.utils.clip_grad_norm_ (TP:1058); `AdamW.step(grad_scale=...)` folds the clip
coefficient into the update instead of a separate in-place pass.
"""
from __future__ import annotations

import ctypes as C

import os

import numpy as np
import torch

from . import _lib as L
from ._lib import call, ptr, stream


# elements per workgroup descriptor (MMDX_ADAMW_CHUNK for A/B runs).  16K: C5's 196 M
# parameters in 64K chunks were ~3000 blocks, 1.5 rounds of the 2048 resident slots (a
# half-empty tail); 16K / 8K chunks +0.3 % on C5 and C4, paired (profiles/r04_adamw_ab.txt)
CHUNK = int(os.environ.get("MMDX_ADAMW_CHUNK", str(1 << 14)))

# Pinned staging buffers cannot be allocated while a stream is capturing a graph, so the
# eager path keeps a few spares (at most _MAX_SPARES, the largest kept) for a later capture.
_PINNED_SPARES: list = []
_MAX_SPARES = 4


def _reserve_spare(nbytes: int):
    if sum(t.numel() >= nbytes for t in _PINNED_SPARES) >= 2:  # AdamW + grad-norm tables
        return
    _PINNED_SPARES.append(torch.empty(nbytes, dtype=torch.uint8, pin_memory=True))
    _PINNED_SPARES.sort(key=lambda t: -t.numel())
    del _PINNED_SPARES[_MAX_SPARES:]


def _pinned(nbytes: int) -> torch.Tensor:
    if torch.cuda.is_current_stream_capturing():
        for i, t in enumerate(_PINNED_SPARES):
            if t.numel() >= nbytes:
                return _PINNED_SPARES.pop(i)
        raise RuntimeError("mmdx AdamW: no pinned staging buffer reserved for graph capture; "
                           "run one eager step before capturing")
    _reserve_spare(nbytes)
    return torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)


# mirrors struct mmdx_adamw_tensor (include/mmdx.h): 4 pointers, long n, long off, 2 floats
_DESC = np.dtype([("p", "<u8"), ("g", "<u8"), ("m", "<u8"), ("v", "<u8"), ("n", "<i8"),
                  ("off", "<i8"), ("lr", "<f4"), ("wd", "<f4")])
assert _DESC.itemsize == C.sizeof(L.AdamWTensor)

_CAPTURED: list = []  # staging buffers referenced by captured graphs: they must stay alive


class _Plan:
    """Chunk table of one parameter set: every tensor split into <= CHUNK-element pieces,
    one workgroup each.  The table lives on the device; everything but the gradient pointers
    is fixed when it is built.  Per step only the gradient column changes (the gradient
    buffers move between steps): mmdx_adamw_patch_grads rewrites it in stream order from
    kernel arguments, skipped when no gradient moved.  (A per-step hipMemcpyAsync of the table
    from pinned memory blocked the issuing thread until the stream reached it: 2.2 ms of host
    time per C4 step in the r03h host profile, and an idle GPU queue behind it.)  A learning-
    rate / weight-decay change re-uploads the whole table through pinned staging buffers."""

    RING = 3

    def __init__(self, params, ms, vs, lrs, wds, device):
        tidx, boff, rows = [], [], []
        for i, (p, m, v, lr, wd) in enumerate(zip(params, ms, vs, lrs, wds)):
            n = p.numel()
            pp, mp, vp = ptr(p), ptr(m), ptr(v)
            for o in range(0, n, CHUNK):
                c = min(CHUNK, n - o)
                tidx.append(i)
                boff.append(4 * o)
                rows.append((pp + 4 * o, 0, mp + 4 * o, vp + 4 * o, c, o, lr, wd))
        self.desc = np.array(rows, dtype=_DESC)
        self.tidx = np.asarray(tidx, dtype=np.int64)
        self.boff = np.asarray(boff, dtype=np.uint64)
        self.n = len(rows)
        self.ntensors = len(params)
        self.nbytes = self.desc.nbytes
        self.dev = torch.empty(self.nbytes, dtype=torch.uint8, device=device)
        self.row_tensor = torch.from_numpy(self.tidx.astype(np.int32)).to(device)
        self.ring = [torch.empty(self.nbytes, dtype=torch.uint8, pin_memory=True)
                     for _ in range(self.RING)]
        self.events = [None] * self.RING
        self.k = 0
        self.last = None
        self.full = True   # the device table needs a whole upload (new, or lr/wd changed)
        self.hyper = (tuple(lrs), tuple(wds))
        _reserve_spare(self.nbytes)

    def set_hyper(self, lrs, wds):
        """A learning-rate / weight-decay change (scheduler, param_group edit) rewrites the
        table's lr/wd columns in place; the next upload ships the whole table."""
        hyper = (tuple(lrs), tuple(wds))
        if hyper == self.hyper:
            return
        self.hyper = hyper
        self.desc["lr"] = np.asarray(lrs, dtype=np.float32)[self.tidx]
        self.desc["wd"] = np.asarray(wds, dtype=np.float32)[self.tidx]
        self.full = True

    def upload(self, grads):
        gp = np.fromiter((g.data_ptr() for g in grads), dtype=np.uint64, count=len(grads))
        capturing = torch.cuda.is_current_stream_capturing()
        if not self.full:
            if not capturing and self.last is not None and np.array_equal(gp, self.last):
                return
            self.desc["g"] = gp[self.tidx] + self.boff
            arr = (C.c_void_p * len(gp))(*gp.tolist())
            call("mmdx_adamw_patch_grads", self.n, ptr(self.dev), ptr(self.row_tensor),
                 self.ntensors, arr, stream())
            self.last = None if capturing else gp
            return
        self.desc["g"] = gp[self.tidx] + self.boff
        if capturing:  # the graph keeps reading this buffer: never reuse it
            host = _pinned(self.nbytes)
            _CAPTURED.append(host)
            self.last = None
        else:
            host = self.ring[self.k]
            if self.events[self.k] is not None:
                self.events[self.k].synchronize()  # its previous copy has been consumed
            self.last = gp
        host.numpy()[: self.nbytes] = self.desc.view(np.uint8)
        self.dev.copy_(host, non_blocking=True)
        if not capturing:
            ev = torch.cuda.Event()
            ev.record()
            self.events[self.k] = ev
            self.k = (self.k + 1) % self.RING
            self.full = False


def _plan_for(cache: dict, params, ms, vs, lrs, wds, device):
    """The table is keyed on the storage the kernel writes (p, exp_avg, exp_avg_sq data
    pointers): a load_state_dict that swaps in new moment tensors, or a moved parameter,
    builds a new table; lr/wd changes only rewrite two columns (_Plan.set_hyper)."""
    key = (tuple(p.data_ptr() for p in params), tuple(m.data_ptr() for m in ms),
           tuple(v.data_ptr() for v in vs), tuple(p.numel() for p in params))
    plan = cache.get(key)
    if plan is None:
        if len(cache) > 8:
            cache.clear()
        plan = cache[key] = _Plan(params, ms, vs, lrs, wds, device)
    plan.set_hyper(lrs, wds)
    return plan


class AdamW(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2,
                 amsgrad=False):
        if amsgrad:
            raise NotImplementedError("amsgrad is not used by the reference")
        defaults = dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay)
        super().__init__(params, defaults)
        self._tables = {}
        self._step_t = None

    def load_state_dict(self, state_dict):
        """torch.optim.Optimizer.load_state_dict, then re-bind the fused kernel: the loaded
        exp_avg / exp_avg_sq tensors replace the old ones (new descriptor table) and the
        shared device step counter restarts from the loaded 'step'."""
        super().load_state_dict(state_dict)
        self._tables.clear()
        self._step_t = None
        # one device step counter drives every parameter's bias correction: a state whose
        # per-parameter steps differ (torch.optim.AdamW keeps one each) cannot be represented
        steps = {float(st["step"].item() if torch.is_tensor(st["step"]) else st["step"])
                 for st in self.state.values() if "step" in st}
        if len(steps) > 1:
            raise ValueError(f"mmdx AdamW keeps one step count for all parameters; the loaded "
                             f"state has per-parameter steps {sorted(steps)}")
        step = steps.pop() if steps else None
        if step is not None:
            dev = next((st["exp_avg"].device for st in self.state.values() if "exp_avg" in st),
                       None)
            self._step_t = torch.full((1,), step, dtype=torch.float32, device=dev)
            for st in self.state.values():
                if "exp_avg" in st:
                    st["step"] = self._step_t
                    for k in ("exp_avg", "exp_avg_sq"):
                        if not st[k].is_contiguous():
                            st[k] = st[k].contiguous()

    @torch.no_grad()
    def step(self, closure=None, grad_scale: torch.Tensor | None = None,
             found_inf: torch.Tensor | None = None):
        """torch.optim.AdamW.step.  grad_scale (device scalar) multiplies every gradient
        (clip coefficient, and / or 1/loss_scale); found_inf (device scalar, GradScaler) skips
        the whole update — step count included — when non-zero."""
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        params, grads, ms, vs, lrs, wds = [], [], [], [], [], []
        dev = None
        b1 = b2 = eps = None
        for group in self.param_groups:
            gb1, gb2 = group["betas"]
            if b1 is None:
                b1, b2, eps = gb1, gb2, group["eps"]
            elif (gb1, gb2, group["eps"]) != (b1, b2, eps):
                raise NotImplementedError("param groups with different betas/eps")
            for p in group["params"]:
                if p.grad is None:
                    continue
                if p.grad.is_sparse or p.dtype != torch.float32:
                    raise TypeError("fused AdamW expects dense fp32 params/grads")
                st = self.state[p]
                if not st:
                    if self._step_t is not None:
                        # torch would start this parameter's own step count at 1; the one
                        # shared device counter cannot, so refuse rather than mis-correct
                        raise ValueError(
                            "mmdx AdamW: a parameter received its first gradient after the "
                            "optimizer had already stepped; every parameter must get a "
                            "gradient from the first step on (one shared step count)")
                    st["exp_avg"] = torch.zeros_like(p, memory_format=torch.contiguous_format)
                    st["exp_avg_sq"] = torch.zeros_like(p,
                                                        memory_format=torch.contiguous_format)
                g = p.grad
                if not g.is_contiguous():
                    g = p.grad = g.contiguous()
                params.append(p)
                grads.append(g)
                ms.append(st["exp_avg"])
                vs.append(st["exp_avg_sq"])
                lrs.append(float(group["lr"]))
                wds.append(float(group["weight_decay"]))
                dev = p.device
        if not params:
            return loss
        L.require_device(params[0])
        if self._step_t is None:
            self._step_t = torch.zeros(1, dtype=torch.float32, device=dev)
            for p in params:
                self.state[p]["step"] = self._step_t
        plan = _plan_for(self._tables, params, ms, vs, lrs, wds, dev)
        plan.upload(grads)
        call("mmdx_adamw_multi_amp", plan.n, ptr(plan.dev), float(b1), float(b2), float(eps),
             ptr(self._step_t), ptr(grad_scale), ptr(found_inf), stream())
        return loss


_clip_cache: dict = {}


@torch.no_grad()
def grad_norm(parameters, max_norm: float = 0.0, apply: bool = False, loss_scale=None,
              unscale_first: bool = False, found_inf=None):
    """Return (total_norm, clip_scale) as device scalars; optionally scale grads in place.
    With `loss_scale` (device scalar, GradScaler) the gradients hold loss_scale * g:
    clip_scale also carries 1/loss_scale and `found_inf` (device scalar) is set to 1 when
    any gradient is inf/NaN (mmdx_grad_norm_amp)."""
    if isinstance(parameters, torch.Tensor):
        parameters = [parameters]
    ps = [p for p in parameters if p.grad is not None]
    if not ps:
        z = torch.zeros((), dtype=torch.float32)
        return z, torch.ones((), dtype=torch.float32)
    dev = ps[0].device
    tab = _plan_for(_clip_cache, ps, ps, ps, [0.0] * len(ps), [0.0] * len(ps), dev)
    tab.upload([p.grad for p in ps])
    norm = torch.empty((), dtype=torch.float32, device=dev)
    scale = torch.empty((), dtype=torch.float32, device=dev)
    ws_n = L.lib().mmdx_grad_norm_workspace_size(tab.n)
    ws = L.workspace(ws_n, dev)
    call("mmdx_grad_norm_amp", tab.n, ptr(tab.dev), float(max_norm), ptr(loss_scale),
         int(bool(unscale_first)), ptr(norm), ptr(scale), ptr(found_inf), ptr(ws), ws_n,
         stream())
    if apply:
        call("mmdx_scale_grads", tab.n, ptr(tab.dev), ptr(scale), stream())
    return norm, scale


def clip_grad_norm_(parameters, max_norm: float, norm_type: float = 2.0):
    """torch.nn.utils.clip_grad_norm_ (L2 only), grads scaled in place on the device."""
    if norm_type != 2.0:
        raise NotImplementedError("only the L2 norm (the reference's default) is fused")
    norm, _ = grad_norm(parameters, max_norm, apply=True)
    return norm
