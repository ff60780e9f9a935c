"""Loss scaling for the fp16 path: `GradScaler` with torch.amp.GradScaler's semantics.

The reference's fusion loop enables AMP whenever it runs on a GPU (TP:1025-1026:
`use_amp = device.type == "cuda"`, `GradScaler(enabled=use_amp)`) and drives it as

    scaler.scale(loss).backward()                               # TP:1056
    torch.nn.utils.clip_grad_norm_(params, 1.0)                 # TP:1058 (on SCALED grads)
    scaler.step(optim); scaler.update()                         # TP:1060-1061

Everything stays on the device (no host sync per step): the scale and the growth tracker
are device scalars, `found_inf` comes out of the same pass that computes the gradient norm
(mmdx_grad_norm_amp: a per-chunk non-finite flag beside the sum of squares), the unscale rides
in AdamW's `grad_scale`, an overflowed step is skipped inside the AdamW launch
(mmdx_adamw_multi_amp: no update, no step count), and `update()` is one tiny kernel
(mmdx_amp_update_scale = torch._amp_update_scale_).
"""
from __future__ import annotations

import warnings

import torch

from . import _lib as L
from ._lib import call, ptr, stream
from .optim import grad_norm


class _ScaleFn(torch.autograd.Function):
    """loss * scale (device scalar), backward d * scale — mmdx_mul_dev_scalar."""

    @staticmethod
    def forward(ctx, x, s):
        xf = x.detach().float().contiguous()
        out = torch.empty_like(xf)
        call("mmdx_mul_dev_scalar", ptr(xf), xf.numel(), ptr(s), ptr(out), stream())
        ctx.save_for_backward(s)
        ctx.dtype = x.dtype
        return out

    @staticmethod
    def backward(ctx, d):
        (s,) = ctx.saved_tensors
        df = d.float().contiguous()
        out = torch.empty_like(df)
        call("mmdx_mul_dev_scalar", ptr(df), df.numel(), ptr(s), ptr(out), stream())
        return out.to(ctx.dtype), None


class GradScaler:
    """torch.amp.GradScaler("cuda", init_scale, growth_factor, backoff_factor,
    growth_interval, enabled) for mmdx optimizers.

    * `scale(loss)` multiplies by the current scale.
    * `unscale_(opt)` divides opt's gradients by the scale in place and records found_inf
      (then a `clip_grad_norm_` sees true gradients: the order torch documents).
    * `step(opt)` skips the update when a gradient overflowed; otherwise unscales inside the
      fused AdamW (or, after `unscale_`, steps plainly).
    * `update()` backs the scale off after an overflow, grows it every `growth_interval`
      clean steps.
    * `clip_and_step(opt, max_norm, unscale_first=False)` is the fused form of
      clip_grad_norm_ + step: one norm pass yields the clip coefficient, 1/scale and
      found_inf, and AdamW applies them; `unscale_first=False` clips the scaled norm, exactly
      as the reference's TP:1058 call does before `scaler.step`.
    """

    def __init__(self, device="cuda", init_scale=2.0 ** 16, growth_factor=2.0,
                 backoff_factor=0.5, growth_interval=2000, enabled=True):
        if growth_factor <= 1.0 or not (0.0 < backoff_factor < 1.0):
            raise ValueError("growth_factor must be > 1 and backoff_factor in (0, 1)")
        self._enabled = bool(enabled)
        self._init_scale = float(init_scale)
        self._growth = float(growth_factor)
        self._backoff = float(backoff_factor)
        self._interval = int(growth_interval)
        self._device = device
        self._scale = None
        self._tracker = None
        self._init_tracker = 0
        self._found_inf = None       # the combined overflow flag of the last update()
        self._opt_inf = {}           # id(optimizer) -> its own found_inf device scalar
        self._step_infs = {}         # the optimizers checked since the last update()
        self._unscaled = {}
        self._noop = False           # a clip_and_step since the last update() found no grads
        self._warned_noop = False

    def is_enabled(self):
        return self._enabled

    def _lazy(self, dev):
        if self._scale is None:
            self._scale = torch.full((1,), self._init_scale, dtype=torch.float32, device=dev)
            self._tracker = torch.full((1,), self._init_tracker, dtype=torch.int32, device=dev)
            self._found_inf = torch.zeros((1,), dtype=torch.float32, device=dev)

    def _inf_for(self, optimizer, dev):
        """optimizer's own found_inf (written by this step's norm pass), recorded for update():
        with several optimizers the scale backs off if ANY of them overflowed (torch.amp)."""
        self._lazy(dev)
        fi = self._opt_inf.get(id(optimizer))
        if fi is None:
            fi = self._opt_inf[id(optimizer)] = torch.zeros((1,), dtype=torch.float32,
                                                           device=dev)
        self._step_infs[id(optimizer)] = fi
        return fi

    def get_scale(self):
        """Current scale as a Python float (host sync), or 1.0 when disabled."""
        if not self._enabled:
            return 1.0
        return self._init_scale if self._scale is None else float(self._scale.item())

    @property
    def found_inf(self):
        return self._found_inf

    def scale(self, outputs):
        if not self._enabled:
            return outputs
        L.require_device(outputs)
        self._lazy(outputs.device)
        return _ScaleFn.apply(outputs, self._scale)

    @staticmethod
    def _params(optimizer):
        return [p for g in optimizer.param_groups for p in g["params"] if p.grad is not None]

    def unscale_(self, optimizer):
        if not self._enabled:
            return
        if id(optimizer) in self._unscaled:
            raise RuntimeError("unscale_() has already been called on this optimizer since "
                               "the last update().")
        ps = self._params(optimizer)
        if not ps:
            return
        fi = self._inf_for(optimizer, ps[0].device)
        grad_norm(ps, 0.0, apply=True, loss_scale=self._scale, unscale_first=True, found_inf=fi)
        self._unscaled[id(optimizer)] = True

    def step(self, optimizer, *args, **kwargs):
        if not self._enabled:
            return optimizer.step(*args, **kwargs)
        ps = self._params(optimizer)
        if not ps:
            # torch.amp.GradScaler.step's behaviour: gradients that never reached the
            # optimizer (a detached graph, a wrong param list) are an error, not a skipped step
            raise AssertionError("No inf checks were recorded for this optimizer.")
        if id(optimizer) in self._unscaled:
            return optimizer.step(*args, found_inf=self._opt_inf[id(optimizer)], **kwargs)
        fi = self._inf_for(optimizer, ps[0].device)
        _, inv = grad_norm(ps, 0.0, loss_scale=self._scale, found_inf=fi)
        return optimizer.step(*args, grad_scale=inv, found_inf=fi, **kwargs)

    def clip_and_step(self, optimizer, max_norm=1.0, unscale_first=False, params=None):
        """clip_grad_norm_(params, max_norm) + step(optimizer) in one norm pass; returns the
        gradient norm (device scalar; unscaled iff unscale_first)."""
        ps = params if params is not None else self._params(optimizer)
        ps = [p for p in ps if p.grad is not None]
        if not ps:   # no gradients: nothing to clip or step (clip_grad_norm_ returns 0)
            if not self._warned_noop:
                warnings.warn("GradScaler.clip_and_step: no parameter has a gradient; the "
                              "step is skipped and the loss scale kept", RuntimeWarning)
                self._warned_noop = True
            self._noop = True
            return torch.zeros(())
        if not self._enabled:
            norm, s = grad_norm(ps, max_norm)
            optimizer.step(grad_scale=s)
            return norm
        fi = self._inf_for(optimizer, ps[0].device)
        norm, s = grad_norm(ps, max_norm, loss_scale=self._scale, unscale_first=unscale_first,
                            found_inf=fi)
        optimizer.step(grad_scale=s, found_inf=fi)
        return norm

    def update(self, new_scale=None):
        if not self._enabled or self._scale is None:
            return
        if new_scale is not None:
            self._scale.fill_(float(new_scale))
        else:
            infs = list(self._step_infs.values())
            if not infs:
                if self._noop:   # the steps since the last update() had no gradients: the
                    self._noop = False   # scale and the growth tracker stay as they are
                    self._unscaled.clear()
                    return
                raise AssertionError("No inf checks were recorded prior to update.")
            # any optimizer's overflow backs the scale off (torch.amp.GradScaler.update)
            self._found_inf = infs[0] if len(infs) == 1 else torch.stack(infs).amax(0)
            call("mmdx_amp_update_scale", ptr(self._scale), ptr(self._tracker),
                 ptr(self._found_inf), self._growth, self._backoff, self._interval, stream())
        self._step_infs = {}
        self._unscaled.clear()
        self._noop = False

    def state_dict(self):
        if not self._enabled:
            return {}
        return {"scale": self.get_scale(), "growth_factor": self._growth,
                "backoff_factor": self._backoff, "growth_interval": self._interval,
                "_growth_tracker": 0 if self._tracker is None else int(self._tracker.item())}

    def load_state_dict(self, sd):
        if not self._enabled:
            return
        self._init_scale = float(sd["scale"])
        self._growth = float(sd["growth_factor"])
        self._backoff = float(sd["backoff_factor"])
        self._interval = int(sd["growth_interval"])
        # kept for a scaler whose device state does not exist yet (_lazy starts from it)
        self._init_tracker = int(sd.get("_growth_tracker", 0))
        if self._scale is not None:
            self._scale.fill_(self._init_scale)
            self._tracker.fill_(self._init_tracker)
