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

import torch

from . import _lib as L
from ._lib import call, ptr, stream


CHUNK = 1 << 16  # elements per workgroup descriptor

# Pinned staging buffers cannot be allocated while a stream is capturing a graph, so every
# eagerly built table leaves a spare of its size behind for a later capture to take.
_PINNED_SPARES: list = []


def _pinned(nbytes: int) -> torch.Tensor:
    if torch.cuda.is_current_stream_capturing():
        for i, t in enumerate(_PINNED_SPARES):
            if t.numel() >= nbytes:
                return _PINNED_SPARES.pop(i)
        raise RuntimeError("mmdx AdamW: no pinned staging buffer reserved for graph capture; "
                           "run one eager step before capturing")
    while sum(t.numel() >= nbytes for t in _PINNED_SPARES) < 2:  # AdamW + grad-norm tables
        _PINNED_SPARES.append(torch.empty(nbytes, dtype=torch.uint8, pin_memory=True))
    return torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)


class _Table:
    """Device copy of an mmdx_adamw_tensor[] chunk table (kept alive with its pinned host
    source): every tensor split into <= CHUNK-element pieces, one workgroup each."""

    def __init__(self, entries, device):
        descs = []
        total = 0
        for p, g, m, v, lr, wd in entries:
            n = p.numel()
            pp, gp, mp, vp = ptr(p), ptr(g), ptr(m), ptr(v)
            for o in range(0, n, CHUNK):
                c = min(CHUNK, n - o)
                b = 4 * o
                descs.append((pp + b, gp + b, mp + b, vp + b, c, o, float(lr), float(wd)))
            total += n
        n = len(descs)
        arr = (L.AdamWTensor * n)()
        for i, d in enumerate(descs):
            arr[i] = L.AdamWTensor(*d)
        nbytes = C.sizeof(arr)
        self.host = _pinned(nbytes)
        C.memmove(self.host.data_ptr(), C.addressof(arr), nbytes)
        self.dev = torch.empty(nbytes, dtype=torch.uint8, device=device)
        self.dev.copy_(self.host, non_blocking=True)
        self.n, self.total = n, total


_CAPTURED: list = []  # tables referenced by captured graphs: their host/device copies must live


def _table_for(cache: dict, entries, device):
    key = tuple((ptr(p), ptr(g), float(lr), float(wd)) for p, g, _, _, lr, wd in entries)
    t = cache.get(key)
    if t is None:
        if len(cache) > 8:
            cache.clear()
        t = cache[key] = _Table(entries, device)
        if torch.cuda.is_current_stream_capturing():
            _CAPTURED.append(t)
    return t


class AdamW(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2,
                 amsgrad=False):
        if amsgrad:
            raise NotImplementedError("amsgrad is not used by the reference")
        defaults = dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay)
        super().__init__(params, defaults)
        self._tables = {}
        self._step_t = None

    @torch.no_grad()
    def step(self, closure=None, grad_scale: torch.Tensor | None = None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        entries = []
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
                    st["exp_avg"] = torch.zeros_like(p, memory_format=torch.contiguous_format)
                    st["exp_avg_sq"] = torch.zeros_like(p,
                                                        memory_format=torch.contiguous_format)
                g = p.grad
                if not g.is_contiguous():
                    g = p.grad = g.contiguous()
                entries.append((p, g, st["exp_avg"], st["exp_avg_sq"], group["lr"],
                                group["weight_decay"]))
                dev = p.device
        if not entries:
            return loss
        L.require_device(entries[0][0])
        if self._step_t is None:
            self._step_t = torch.zeros(1, dtype=torch.float32, device=dev)
            for e in entries:
                self.state[e[0]]["step"] = self._step_t
        tab = _table_for(self._tables, entries, dev)
        call("mmdx_adamw_multi", tab.n, ptr(tab.dev), float(b1), float(b2), float(eps),
             ptr(self._step_t), ptr(grad_scale), stream())
        return loss


_clip_cache: dict = {}


@torch.no_grad()
def grad_norm(parameters, max_norm: float = 0.0, apply: bool = False):
    """Return (total_norm, clip_scale) as device scalars; optionally scale grads in place."""
    if isinstance(parameters, torch.Tensor):
        parameters = [parameters]
    ps = [p for p in parameters if p.grad is not None]
    if not ps:
        z = torch.zeros((), dtype=torch.float32)
        return z, torch.ones((), dtype=torch.float32)
    dev = ps[0].device
    entries = [(p, p.grad, p, p, 0.0, 0.0) for p in ps]
    tab = _table_for(_clip_cache, entries, dev)
    norm = torch.empty((), dtype=torch.float32, device=dev)
    scale = torch.empty((), dtype=torch.float32, device=dev)
    ws_n = L.lib().mmdx_grad_norm_workspace_size(tab.n)
    ws = L.workspace(ws_n, dev)
    call("mmdx_grad_norm", tab.n, ptr(tab.dev), float(max_norm), ptr(norm), ptr(scale),
         ptr(ws), ws_n, stream())
    if apply:
        call("mmdx_scale_grads", tab.n, ptr(tab.dev), ptr(scale), stream())
    return norm, scale


def clip_grad_norm_(parameters, max_norm: float, norm_type: float = 2.0):
    """torch.nn.utils.clip_grad_norm_ (L2 only), grads scaled in place on the device."""
    if norm_type != 2.0:
        raise NotImplementedError("only the L2 norm (the reference's default) is fused")
    norm, _ = grad_norm(parameters, max_norm, apply=True)
    return norm
