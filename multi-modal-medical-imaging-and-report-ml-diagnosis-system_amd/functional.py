"""Autograd functions over the HIP kernels (the only compute path; no fallback).

Every forward/backward here is a sequence of C-ABI calls on torch's current HIP stream,
so a whole train step (forward, backward, optimizer) can be captured into one hipGraph.
Parameters stay fp32 (PyTorch layouts, state_dict-identical to the reference); the
compute dtype of activations is fp32 (parity path) or bf16 (throughput path).
"""
from __future__ import annotations

import os

import torch

from . import _lib as L
from ._lib import call, ptr, stream

__all__ = [
    "gemm", "cast", "linear", "fusion_linear", "layer_norm", "dropout", "bce_with_logits",
    "masked_mean", "embed_mean",
]


class _NoTimer:
    def __call__(self, flops):
        return self

    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


# bench.py installs a HIP-event timer here to measure the dense GEMM launches (C5 roofline).
GEMM_TIMER = _NoTimer()


def attn_flash(T) -> bool:
    """The flash-style attention path (mmdx_attention_fwd_lse / _bwd_lse: row log-sum-exp
    saved, P recomputed in the backward) for the 16-bit compute dtypes; MMDX_ATTN_FLASH=0
    saves P [B,H,L,L] fp32 instead (the previous path, kept for A/B runs)."""
    return T != torch.float32 and os.environ.get("MMDX_ATTN_FLASH", "1") != "0"


def attention_fwd(qkv, mask, B, Ls, H, scale, p_drop, seed, counter, out, keep):
    """Self-attention forward of the eager per-layer nodes (BERT, ViT): returns what
    attention_bwd needs besides qkv / out — (lse, rng) on the flash-style path, (probs,)
    otherwise ((None,) when nothing is kept for a backward)."""
    T = qkv.dtype
    dev = qkv.device
    if keep and attn_flash(T):
        lse = torch.empty((B, H, Ls), dtype=torch.float32, device=dev)
        rng = torch.empty(1, dtype=torch.int64, device=dev)
        call("mmdx_attention_fwd_lse", L.dtype_code(T), ptr(qkv), ptr(mask), B, Ls, H,
             float(scale), float(p_drop), seed, ptr(counter), ptr(out), ptr(lse), ptr(rng),
             stream())
        return (lse, rng)
    probs = torch.empty((B, H, Ls, Ls), dtype=torch.float32, device=dev) if keep else None
    call("mmdx_attention_fwd", L.dtype_code(T), ptr(qkv), ptr(mask), B, Ls, H, float(scale),
         float(p_drop), seed, ptr(counter), ptr(out), ptr(probs), stream())
    return (probs,)


def attention_bwd(qkv, saved, out, dout, mask, B, Ls, H, scale, p_drop, dqkv):
    T = qkv.dtype
    dc = L.dtype_code(T)
    if len(saved) == 2:
        n = L.lib().mmdx_attention_lse_workspace_size(dc, B, Ls, H)
        w = torch.empty(max(1, n), dtype=torch.uint8, device=qkv.device)
        call("mmdx_attention_bwd_lse", dc, ptr(qkv), ptr(out), ptr(saved[0]), ptr(saved[1]),
             ptr(dout), ptr(mask), B, Ls, H, float(scale), float(p_drop), ptr(dqkv), ptr(w), n,
             stream())
        return
    n = L.lib().mmdx_attention_workspace_size(dc, B, Ls, H)
    w = torch.empty(max(1, n), dtype=torch.uint8, device=qkv.device)
    call("mmdx_attention_bwd", dc, ptr(qkv), ptr(saved[0]), ptr(dout), ptr(mask), B, Ls, H,
         float(scale), float(p_drop), ptr(dqkv), ptr(w), n, stream())


def gemm_cost(M, N, K, dt, c_dt, beta=0.0, act=L.ACT_NONE, preact=None):
    """LaunchCost of one GEMM: 2MNK FLOPs; A, B read once, C written (read too when
    beta != 0), the pre-activation written (GELU) or read (GELU backward)."""
    from .resnet import LaunchCost
    e = 4 if dt == L.F32 else 2
    ce = 4 if c_dt == L.F32 else 2
    b = (M * K + N * K) * e + M * N * ce * (2 if beta else 1)
    if preact is not None:
        b += M * N * ce
    return LaunchCost("gemm", 2 * M * N * K, b, f"{M}x{N}x{K}")


# ----------------------------------------------------------------------------- primitives
def gemm(A, lda, a_kmajor, B, ldb, b_kmajor, M, N, K, Cout, ldc, *, bias=None, addend=None,
         act=L.ACT_NONE, alpha=1.0, beta=0.0, preact=None, compute_dtype=None, residual=None):
    """C[M,N] = act(alpha * A.B^T + bias) + beta*C (+ residual) on the MFMA implicit-GEMM
    core."""
    dt = L.dtype_code(compute_dtype if compute_dtype is not None else A.dtype)
    ws_n = L.lib().mmdx_gemm_workspace_size(dt, M, N, K)
    ws = L.workspace(ws_n, Cout.device)
    cost = gemm_cost(M, N, K, dt, L.dtype_code(Cout.dtype),
                     1.0 if residual is not None else beta, act, preact)
    with GEMM_TIMER(cost):
        if residual is not None:
            call("mmdx_gemm_res", dt, M, N, K, ptr(A), lda, int(a_kmajor), ptr(B), ldb,
                 int(b_kmajor), ptr(Cout), ldc, L.dtype_code(Cout.dtype), ptr(bias),
                 ptr(addend), act, float(alpha), float(beta), ptr(preact), ptr(residual),
                 ptr(ws), ws_n, stream())
        else:
            call("mmdx_gemm", dt, M, N, K, ptr(A), lda, int(a_kmajor), ptr(B), ldb,
                 int(b_kmajor), ptr(Cout), ldc, L.dtype_code(Cout.dtype), ptr(bias),
                 ptr(addend), act, float(alpha), float(beta), ptr(preact), ptr(ws), ws_n,
                 stream())
    return Cout


def gemm_wgrad_bias(dY, ldy, X, ldx, M, N, K, dW, ldw, db, *, compute_dtype=None):
    """dW[M,N] = dY^T X (both R-major: dY [K][ldy], X [K][ldx]) and db[M] = column sums of
    dY, in one launch sequence (mmdx_gemm_bias_grad)."""
    dt = L.dtype_code(compute_dtype if compute_dtype is not None else dY.dtype)
    ws_n = L.lib().mmdx_gemm_bias_grad_workspace_size(dt, M, N, K)
    ws = L.workspace(ws_n, dW.device)
    with GEMM_TIMER(gemm_cost(M, N, K, dt, L.dtype_code(dW.dtype), 0.0, L.ACT_NONE, None)):
        call("mmdx_gemm_bias_grad", dt, M, N, K, ptr(dY), ldy, ptr(X), ldx, ptr(dW), ldw,
             L.dtype_code(dW.dtype), ptr(db), ptr(ws), ws_n, stream())
    return dW, db


def cast(x: torch.Tensor, dtype: torch.dtype) -> torch.Tensor:
    """Device cast through the mmdx kernel (fp32 master weights -> compute dtype)."""
    if x.dtype == dtype:
        return x
    L.require_device(x)
    y = torch.empty(x.shape, dtype=dtype, device=x.device)
    call("mmdx_cast", L.dtype_code(dtype), L.dtype_code(x.dtype), ptr(x), x.numel(), ptr(y),
         stream())
    return y


def _bias_grad(dy, M, N, out):
    ws_n = L.lib().mmdx_bias_grad_workspace_size(M, N)
    ws = L.workspace(ws_n, dy.device)
    call("mmdx_bias_grad", L.dtype_code(dy.dtype), ptr(dy), M, N, ptr(out), 0.0, ptr(ws), ws_n,
         stream())
    return out


def _gelu_bwd(pre, dy):
    dx = torch.empty_like(dy)
    call("mmdx_gelu_bwd", L.dtype_code(dy.dtype), ptr(pre), ptr(dy), dy.numel(), ptr(dx),
         stream())
    return dx


# ----------------------------------------------------------------------------- Linear
class _LinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, act, out_dtype):
        L.require_device(x, w, b)
        M, K = x.shape
        N = w.shape[0]
        T = x.dtype
        wc = cast(w, T)
        y = torch.empty((M, N), dtype=out_dtype, device=x.device)
        pre = torch.empty((M, N), dtype=out_dtype, device=x.device) if act == L.ACT_GELU else None
        gemm(x, K, True, wc, K, True, M, N, K, y, N, bias=b, act=act, preact=pre,
             compute_dtype=T)
        ctx.save_for_backward(x, wc, pre if pre is not None else y)
        ctx.act, ctx.has_b, ctx.T = act, b is not None, T
        return y

    @staticmethod
    def backward(ctx, dy):
        x, wc, saved = ctx.saved_tensors
        T = ctx.T
        M, K = x.shape
        N = wc.shape[0]
        dy = dy.contiguous()
        if ctx.act == L.ACT_GELU:
            dy = _gelu_bwd(saved, dy)
        elif ctx.act == L.ACT_RELU:
            raise NotImplementedError("relu epilogue backward is fused in the trunk, not here")
        dy = cast(dy, T)
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            dx = torch.empty((M, K), dtype=T, device=x.device)
            gemm(dy, N, True, wc, K, False, M, K, N, dx, K, compute_dtype=T)
        if ctx.needs_input_grad[1]:
            dw = torch.empty((N, K), dtype=torch.float32, device=x.device)
            gemm(dy, N, False, x, K, False, N, K, M, dw, K, compute_dtype=T)
        if ctx.has_b and ctx.needs_input_grad[2]:
            db = torch.empty((N,), dtype=torch.float32, device=x.device)
            _bias_grad(dy, M, N, db)
        return dx, dw, db, None, None


def linear(x, weight, bias=None, act=L.ACT_NONE, out_dtype=None):
    """y = act(x @ W^T + b); x in the compute dtype, W/b fp32 masters."""
    return _LinearFn.apply(x, weight, bias, act, out_dtype or x.dtype)


class _FusionLinearFn(torch.autograd.Function):
    """fusion_mlp[0] on cat([z_img, z_txt]) without materialising the concat (TP:586-589):
    y = act(z_img W[:, :Di]^T + z_txt W[:, Di:]^T + b) as two accumulating GEMMs."""

    @staticmethod
    def forward(ctx, za, zb, w, b, act):
        L.require_device(za, zb, w, b)
        M, Da = za.shape
        Db = zb.shape[1]
        N, Kt = w.shape
        assert Kt == Da + Db, "fusion weight must be [N, d_img + d_txt]"
        T = za.dtype
        wc = cast(w, T)
        y = torch.empty((M, N), dtype=T, device=za.device)
        pre = torch.empty((M, N), dtype=T, device=za.device) if act == L.ACT_GELU else None
        # acc = za Wa^T (fp32), then y = act(zb Wb^T + b + acc) in the second epilogue
        acc = torch.empty((M, N), dtype=torch.float32, device=za.device)
        gemm(za, Da, True, wc, Kt, True, M, N, Da, acc, N, compute_dtype=T)
        gemm(zb, Db, True, wc[:, Da:], Kt, True, M, N, Db, y, N, bias=b, addend=acc, act=act,
             preact=pre, compute_dtype=T)
        ctx.save_for_backward(za, zb, wc, pre if pre is not None else y)
        ctx.act, ctx.T, ctx.Da = act, T, Da
        return y

    @staticmethod
    def backward(ctx, dy):
        za, zb, wc, saved = ctx.saved_tensors
        T, Da = ctx.T, ctx.Da
        M, N = dy.shape
        Kt = wc.shape[1]
        Db = Kt - Da
        dy = dy.contiguous()
        if ctx.act == L.ACT_GELU:
            dy = _gelu_bwd(saved, dy)
        dy = cast(dy, T)
        dza = torch.empty((M, Da), dtype=T, device=dy.device)
        dzb = torch.empty((M, Db), dtype=T, device=dy.device)
        gemm(dy, N, True, wc, Kt, False, M, Da, N, dza, Da, compute_dtype=T)
        gemm(dy, N, True, wc[:, Da:], Kt, False, M, Db, N, dzb, Db, compute_dtype=T)
        dw = torch.empty((N, Kt), dtype=torch.float32, device=dy.device)
        gemm(dy, N, False, za, Da, False, N, Da, M, dw, Kt, compute_dtype=T)
        gemm(dy, N, False, zb, Db, False, N, Db, M, dw[:, Da:], Kt, compute_dtype=T)
        db = torch.empty((N,), dtype=torch.float32, device=dy.device)
        _bias_grad(dy, M, N, db)
        return dza, dzb, dw, db, None


def fusion_linear(z_img, z_txt, weight, bias, act=L.ACT_GELU):
    return _FusionLinearFn.apply(z_img, z_txt, weight, bias, act)


# ----------------------------------------------------------------------------- LayerNorm
class _LayerNormFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, residual, gamma, beta, eps):
        L.require_device(x, residual, gamma, beta)
        D = x.shape[-1]
        rows = x.numel() // D
        y = torch.empty_like(x)
        xs = torch.empty_like(x)
        mean = torch.empty(rows, dtype=torch.float32, device=x.device)
        rstd = torch.empty(rows, dtype=torch.float32, device=x.device)
        call("mmdx_layernorm_fwd", L.dtype_code(x.dtype), ptr(x), ptr(residual), rows, D,
             ptr(gamma), ptr(beta), float(eps), ptr(y), ptr(xs), ptr(mean), ptr(rstd),
             stream())
        ctx.save_for_backward(xs, gamma, mean, rstd)
        ctx.has_res = residual is not None
        return y

    @staticmethod
    def backward(ctx, dy):
        xs, gamma, mean, rstd = ctx.saved_tensors
        D = xs.shape[-1]
        rows = xs.numel() // D
        dy = cast(dy.contiguous(), xs.dtype)
        dx = torch.empty_like(xs)
        dg = torch.empty(D, dtype=torch.float32, device=xs.device)
        db = torch.empty(D, dtype=torch.float32, device=xs.device)
        ws_n = L.lib().mmdx_layernorm_workspace_size(rows, D)
        ws = L.workspace(ws_n, xs.device)
        call("mmdx_layernorm_bwd", L.dtype_code(xs.dtype), ptr(xs), ptr(dy), rows, D,
             ptr(gamma), ptr(mean), ptr(rstd), ptr(dx), ptr(dg), ptr(db), 0.0, ptr(ws), ws_n,
             stream())
        return dx, (dx if ctx.has_res else None), dg, db, None


def layer_norm(x, gamma, beta, eps, residual=None):
    return _LayerNormFn.apply(x, residual, gamma, beta, eps)


# ----------------------------------------------------------------------------- Dropout
_DROPOUT_SEED = [0x5EED]


class _DropoutFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, p, seed, offset):
        y = torch.empty_like(x)
        mask = torch.empty(x.shape, dtype=torch.uint8, device=x.device)
        call("mmdx_dropout_fwd", L.dtype_code(x.dtype), ptr(x), x.numel(), float(p), seed,
             offset, ptr(L.rng_counter(x.device)), ptr(y), ptr(mask), stream())
        ctx.save_for_backward(mask)
        ctx.p = p
        return y

    @staticmethod
    def backward(ctx, dy):
        (mask,) = ctx.saved_tensors
        dy = dy.contiguous()
        dx = torch.empty_like(dy)
        call("mmdx_dropout_bwd", L.dtype_code(dy.dtype), ptr(dy), ptr(mask), dy.numel(),
             float(ctx.p), ptr(dx), stream())
        return dx, None, None, None


def dropout(x, p, training):
    if not training or p == 0.0:
        return x
    # the device counter (L.rng_counter) advances per launch; the host seed stays fixed so
    # the call is graph-replayable
    return _DropoutFn.apply(x, p, L.dropout_seed(_DROPOUT_SEED[0]), 0)


# ----------------------------------------------------------------------------- BCE
class _BCEFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, target):
        L.require_device(logits, target)
        if logits.dtype != torch.float32 or target.dtype != torch.float32:
            raise TypeError("BCEWithLogitsLoss kernel takes fp32 logits and targets")
        B, Cn = logits.shape
        loss = torch.empty((), dtype=torch.float32, device=logits.device)
        call("mmdx_bce_logits_fwd", ptr(logits), ptr(target), B, Cn, ptr(loss), stream())
        ctx.save_for_backward(logits, target)
        return loss

    @staticmethod
    def backward(ctx, dloss):
        logits, target = ctx.saved_tensors
        B, Cn = logits.shape
        dloss = dloss.contiguous().float()
        dz = torch.empty_like(logits)
        call("mmdx_bce_logits_bwd", ptr(logits), ptr(target), B, Cn, ptr(dloss), ptr(dz),
             stream())
        return dz, None


def bce_with_logits(logits, target):
    return _BCEFn.apply(logits.contiguous(), target.contiguous())


# ----------------------------------------------------------------------------- pooling
class _MaskedMeanFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, h, mask):
        L.require_device(h, mask)
        B, Ls, D = h.shape
        out = torch.empty((B, D), dtype=h.dtype, device=h.device)
        call("mmdx_masked_mean_fwd", L.dtype_code(h.dtype), ptr(h), ptr(mask), B, Ls, D,
             ptr(out), stream())
        ctx.save_for_backward(mask)
        ctx.shape = (B, Ls, D)
        ctx.dt = h.dtype
        return out

    @staticmethod
    def backward(ctx, dout):
        (mask,) = ctx.saved_tensors
        B, Ls, D = ctx.shape
        dout = cast(dout.contiguous(), ctx.dt)
        dh = torch.empty((B, Ls, D), dtype=ctx.dt, device=dout.device)
        call("mmdx_masked_mean_bwd", L.dtype_code(ctx.dt), ptr(dout), ptr(mask), B, Ls, D,
             ptr(dh), stream())
        return dh, None


def masked_mean(h, mask):
    """TextEncoderTransformer.mean_pool (TP:452-459) with an int64 attention mask."""
    return _MaskedMeanFn.apply(h.contiguous(), mask.contiguous())


class _EmbedMeanFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, ids, mask, table, dt):
        L.require_device(ids, mask, table)
        B, Ls = ids.shape
        D = table.shape[1]
        out = torch.empty((B, D), dtype=dt, device=ids.device)
        call("mmdx_embed_mean_fwd", L.dtype_code(dt), ptr(ids), ptr(mask), B, Ls, D, ptr(table),
             ptr(out), stream())
        ctx.save_for_backward(ids, mask)
        ctx.tshape = table.shape
        ctx.dt = dt
        return out

    @staticmethod
    def backward(ctx, dout):
        ids, mask = ctx.saved_tensors
        B, Ls = ids.shape
        dout = cast(dout.contiguous(), ctx.dt)
        dtab = torch.zeros(ctx.tshape, dtype=torch.float32, device=dout.device)
        call("mmdx_embed_mean_bwd", L.dtype_code(ctx.dt), ptr(ids), ptr(mask), B, Ls,
             ctx.tshape[1], ptr(dout), ptr(dtab), stream())
        return None, None, dtab, None


def embed_mean(ids, mask, table, dt):
    return _EmbedMeanFn.apply(ids.contiguous(), mask.contiguous(), table, dt)
