"""ViT-B/16 image tower on the mmdx kernels (build-defined backbone name "vit_b_16", SURVEY
§8 a1 / BASELINE config C5), state_dict-identical to torchvision's `vit_b_16()` minus the
classification head: conv_proj, class_token, encoder.pos_embedding,
encoder.layers.encoder_layer_{i}.{ln_1, self_attention.{in_proj_weight, in_proj_bias,
out_proj}, ln_2, mlp.{0,3}}, encoder.ln.

Forward semantics (torchvision VisionTransformer, dropout 0): patch embedding Conv2d(3, 768,
16, stride 16) -> prepend class token -> + pos_embedding -> 12 pre-LN blocks
{x = x + MHA(LN1(x)); x = x + MLP(LN2(x))} (LN eps 1e-6, exact GELU) -> encoder.ln ->
class-token row (the [B, 768] feature the image encoder's `proj` consumes).

Kernels: patchify + one GEMM for the patch embedding, token assembly, per block the fused
QKV GEMM, attention core (no key mask), out-proj GEMM, LayerNorm with the residual sum
fused in (it emits both x + attn and LN2 of it), MLP GEMMs with the GELU in the epilogue
and the second residual accumulated in the GEMM epilogue (beta = 1).
"""
from __future__ import annotations

import math
from collections import OrderedDict

import torch
import torch.nn as nn

from . import _lib as L
from . import functional as F
from ._lib import call, ptr, stream
from .layers import LayerNorm, Linear

D_MODEL, HEADS, MLP_DIM, LAYERS, PATCH, IMG = 768, 12, 3072, 12, 16, 224
EPS = 1e-6


def _ln(x, res, g, b, want_sum):
    """LayerNorm(x (+res)) over the last dim; returns (y, sum or None, mean, rstd)."""
    D = x.shape[-1]
    rows = x.numel() // D
    y = torch.empty_like(x)
    s = torch.empty_like(x) if want_sum else None
    mean = torch.empty(rows, dtype=torch.float32, device=x.device)
    rstd = torch.empty(rows, dtype=torch.float32, device=x.device)
    call("mmdx_layernorm_fwd", L.dtype_code(x.dtype), ptr(x), ptr(res), rows, D, ptr(g), ptr(b),
         float(EPS), ptr(y), ptr(s), ptr(mean), ptr(rstd), stream())
    return y, s, mean, rstd


def _ln_bwd(xs, dy, g, mean, rstd, addin=None):
    """LayerNorm backward; addin: a residual branch's gradient added to dx (one pass)."""
    D = xs.shape[-1]
    rows = xs.numel() // D
    dx = torch.empty_like(xs)
    dg = torch.empty(D, dtype=torch.float32, device=xs.device)
    db = torch.empty(D, dtype=torch.float32, device=xs.device)
    n = L.lib().mmdx_layernorm_workspace_size(rows, D)
    w = L.workspace(n, xs.device)
    if addin is not None:
        call("mmdx_layernorm_bwd_residual", L.dtype_code(xs.dtype), ptr(xs), ptr(dy), rows, D,
             ptr(g), ptr(mean), ptr(rstd), ptr(addin), ptr(dx), ptr(dg), ptr(db), 0.0, ptr(w),
             n, stream())
    else:
        call("mmdx_layernorm_bwd", L.dtype_code(xs.dtype), ptr(xs), ptr(dy), rows, D, ptr(g),
             ptr(mean), ptr(rstd), ptr(dx), ptr(dg), ptr(db), 0.0, ptr(w), n, stream())
    return dx, dg, db


def _add(x, y):
    out = torch.empty_like(x)
    call("mmdx_add", L.dtype_code(x.dtype), x.numel(), ptr(x), ptr(y), ptr(out), stream())
    return out


def _copy(x):
    out = torch.empty_like(x)
    dt = L.dtype_code(x.dtype)
    call("mmdx_cast", dt, dt, ptr(x), x.numel(), ptr(out), stream())
    return out


def _colsum(t, M, N):
    return F._bias_grad(t, M, N, torch.empty(N, dtype=torch.float32, device=t.device))


class _PatchTokensFn(torch.autograd.Function):
    """images [N,3,224,224] fp32 -> tokens [N,197,768] (class token + patches + pos)."""

    @staticmethod
    def forward(ctx, x, w, b, cls, pos, T):
        L.require_device(x)
        N, C, H, W = x.shape
        S = (H // PATCH) * (W // PATCH)
        K = C * PATCH * PATCH
        D = w.shape[0]
        dev = x.device
        patches = torch.empty((N * S, K), dtype=T, device=dev)
        call("mmdx_patchify", L.dtype_code(T), ptr(x.contiguous()), N, C, H, W, PATCH,
             ptr(patches), stream())
        wc = F.cast(w.reshape(D, K), T)
        emb = torch.empty((N * S, D), dtype=T, device=dev)
        F.gemm(patches, K, True, wc, K, True, N * S, D, K, emb, D, bias=b, compute_dtype=T)
        tok = torch.empty((N, S + 1, D), dtype=T, device=dev)
        call("mmdx_vit_tokens_fwd", L.dtype_code(T), ptr(emb), ptr(cls), ptr(pos), N, S + 1, D,
             ptr(tok), stream())
        ctx.save_for_backward(patches)
        ctx.dims = (N, S, K, D, tuple(w.shape))
        return tok

    @staticmethod
    def backward(ctx, dtok):
        (patches,) = ctx.saved_tensors
        N, S, K, D, wshape = ctx.dims
        T = patches.dtype
        dev = patches.device
        dtok = F.cast(dtok.contiguous(), T)
        demb = torch.empty((N * S, D), dtype=T, device=dev)
        call("mmdx_vit_tokens_bwd", L.dtype_code(T), ptr(dtok), N, S + 1, D, ptr(demb), stream())
        dpos = _colsum(dtok, N, (S + 1) * D)
        dcls = torch.empty(D, dtype=torch.float32, device=dev)
        call("mmdx_axpby", D, 1.0, ptr(dpos), 0.0, None, ptr(dcls), stream())
        dW = torch.empty((D, K), dtype=torch.float32, device=dev)
        F.gemm(demb, D, False, patches, K, False, D, K, N * S, dW, K, compute_dtype=T)
        db = _colsum(demb, N * S, D)
        return (None, dW.reshape(wshape), db, dcls.reshape(1, 1, D),
                dpos.reshape(1, S + 1, D), None)


class _VitBlockFn(torch.autograd.Function):
    """One torchvision EncoderBlock (pre-LN): x += MHA(LN1 x); x += MLP(LN2 x)."""

    @staticmethod
    def forward(ctx, h, heads, g1, b1, w_in, b_in, w_out, b_out, g2, b2, w1, bb1, w2, bb2):
        N, S, D = h.shape
        T = h.dtype
        dev = h.device
        M = N * S
        I = w1.shape[0]
        x = h.reshape(M, D)
        u1, _, mu1, rs1 = _ln(x, None, g1, b1, False)
        wqkv = F.cast(w_in, T)
        qkv = torch.empty((M, 3 * D), dtype=T, device=dev)
        F.gemm(u1, D, True, wqkv, D, True, M, 3 * D, D, qkv, 3 * D, bias=b_in, compute_dtype=T)
        keep = any(ctx.needs_input_grad)
        scale = 1.0 / math.sqrt(D // heads)
        att = torch.empty((M, D), dtype=T, device=dev)
        ctx.attn = F.attention_fwd(qkv, None, N, S, heads, scale, 0.0, 0, None, att, keep)
        woc = F.cast(w_out, T)
        o = torch.empty((M, D), dtype=T, device=dev)
        F.gemm(att, D, True, woc, D, True, M, D, D, o, D, bias=b_out, compute_dtype=T)
        # a = x + o and u2 = LN2(a) in one pass
        u2, a, mu2, rs2 = _ln(o, x, g2, b2, True)
        w1c = F.cast(w1, T)
        f = torch.empty((M, I), dtype=T, device=dev)
        pre = torch.empty((M, I), dtype=T, device=dev)
        F.gemm(u2, D, True, w1c, D, True, M, I, D, f, I, bias=bb1, act=L.ACT_GELU, preact=pre,
               compute_dtype=T)
        w2c = F.cast(w2, T)
        out = torch.empty_like(a)  # out = a + f W2^T + b2 (the residual read by the epilogue)
        F.gemm(f, I, True, w2c, I, True, M, D, I, out, D, bias=bb2, residual=a, compute_dtype=T)
        if keep:
            ctx.save_for_backward(x, u1, mu1, rs1, g1, wqkv, qkv, att, woc, a, u2, mu2,
                                  rs2, g2, w1c, pre, f, w2c)
        ctx.dims = (N, S, D, I, heads, scale)
        return out.reshape(N, S, D)

    @staticmethod
    def backward(ctx, dout):
        (x, u1, mu1, rs1, g1, wqkv, qkv, att, woc, a, u2, mu2, rs2, g2, w1c, pre, f,
         w2c) = ctx.saved_tensors
        N, S, D, I, heads, scale = ctx.dims
        T = x.dtype
        dev = x.device
        M = N * S
        dO = F.cast(dout.contiguous().reshape(M, D), T)
        # dpre = (dO W2) * gelu'(pre): the GELU backward in the GEMM epilogue
        dpre = torch.empty((M, I), dtype=T, device=dev)
        F.gemm(dO, D, True, w2c, I, False, M, I, D, dpre, I, act=L.ACT_GELU_BWD, preact=pre,
               compute_dtype=T)
        dW2 = torch.empty((D, I), dtype=torch.float32, device=dev)
        dbb2 = torch.empty(D, dtype=torch.float32, device=dev)
        F.gemm_wgrad_bias(dO, D, f, I, D, I, M, dW2, I, dbb2, compute_dtype=T)
        dW1 = torch.empty((I, D), dtype=torch.float32, device=dev)
        dbb1 = torch.empty(I, dtype=torch.float32, device=dev)
        F.gemm_wgrad_bias(dpre, I, u2, D, I, D, M, dW1, D, dbb1, compute_dtype=T)
        du2 = torch.empty((M, D), dtype=T, device=dev)
        F.gemm(dpre, I, True, w1c, D, False, M, D, I, du2, D, compute_dtype=T)
        from .xplan import VIT_LN_ADDIN
        if VIT_LN_ADDIN:   # dO + LN2'(du2) in one pass (xplan._build_vit's choice)
            da, dg2, db2 = _ln_bwd(a, du2, g2, mu2, rs2, addin=dO)
        else:
            da_ln, dg2, db2 = _ln_bwd(a, du2, g2, mu2, rs2)
            da = _add(dO, da_ln)
        datt = torch.empty((M, D), dtype=T, device=dev)
        F.gemm(da, D, True, woc, D, False, M, D, D, datt, D, compute_dtype=T)
        dWo = torch.empty((D, D), dtype=torch.float32, device=dev)
        dbo = torch.empty(D, dtype=torch.float32, device=dev)
        F.gemm_wgrad_bias(da, D, att, D, D, D, M, dWo, D, dbo, compute_dtype=T)
        dqkv = torch.empty((M, 3 * D), dtype=T, device=dev)
        F.attention_bwd(qkv, ctx.attn, att, datt, None, N, S, heads, scale, 0.0, dqkv)
        dWqkv = torch.empty((3 * D, D), dtype=torch.float32, device=dev)
        dbqkv = torch.empty(3 * D, dtype=torch.float32, device=dev)
        F.gemm_wgrad_bias(dqkv, 3 * D, u1, D, 3 * D, D, M, dWqkv, D, dbqkv, compute_dtype=T)
        du1 = torch.empty((M, D), dtype=T, device=dev)
        F.gemm(dqkv, 3 * D, True, wqkv, D, False, M, D, 3 * D, du1, D, compute_dtype=T)
        if VIT_LN_ADDIN:
            dx, dg1, db1 = _ln_bwd(x, du1, g1, mu1, rs1, addin=da)
        else:
            dx_ln, dg1, db1 = _ln_bwd(x, du1, g1, mu1, rs1)
            dx = _add(da, dx_ln)
        return (dx.reshape(N, S, D), None, dg1, db1, dWqkv, dbqkv, dWo, dbo, dg2, db2, dW1,
                dbb1, dW2, dbb2)


class _ClassTokenLNFn(torch.autograd.Function):
    """encoder.ln applied to the class-token rows only (the only rows the tower returns)."""

    @staticmethod
    def forward(ctx, h, g, b):
        N, S, D = h.shape
        T = h.dtype
        rows = torch.empty((N, D), dtype=T, device=h.device)
        call("mmdx_rows_copy", L.dtype_code(T), ptr(h), S * D, ptr(rows), D, N, D, stream())
        y, _, mean, rstd = _ln(rows, None, g, b, False)
        ctx.save_for_backward(rows, g, mean, rstd)
        ctx.S = S
        return y

    @staticmethod
    def backward(ctx, dy):
        rows, g, mean, rstd = ctx.saved_tensors
        N, D = rows.shape
        S = ctx.S
        T = rows.dtype
        drow, dg, db = _ln_bwd(rows, F.cast(dy.contiguous(), T), g, mean, rstd)
        dh = torch.zeros((N, S, D), dtype=T, device=rows.device)
        call("mmdx_rows_copy", L.dtype_code(T), ptr(drow), D, ptr(dh), S * D, N, D, stream())
        return dh, dg, db


# ----------------------------------------------------------------------------- modules
class EncoderBlock(nn.Module):
    def __init__(self):
        super().__init__()
        self.ln_1 = LayerNorm(D_MODEL, eps=EPS)
        self.self_attention = nn.MultiheadAttention(D_MODEL, HEADS, batch_first=True)
        self.ln_2 = LayerNorm(D_MODEL, eps=EPS)
        self.mlp = nn.Sequential(OrderedDict([
            ("0", Linear(D_MODEL, MLP_DIM)), ("1", nn.GELU()), ("2", nn.Dropout(0.0)),
            ("3", Linear(MLP_DIM, D_MODEL)), ("4", nn.Dropout(0.0))]))
        for m in (self.mlp[0], self.mlp[3]):  # torchvision MLPBlock init
            nn.init.xavier_uniform_(m.weight)
            nn.init.normal_(m.bias, std=1e-6)

    def forward(self, h):
        at = self.self_attention
        return _VitBlockFn.apply(h, HEADS, self.ln_1.weight, self.ln_1.bias, at.in_proj_weight,
                                 at.in_proj_bias, at.out_proj.weight, at.out_proj.bias,
                                 self.ln_2.weight, self.ln_2.bias, self.mlp[0].weight,
                                 self.mlp[0].bias, self.mlp[3].weight, self.mlp[3].bias)


class Encoder(nn.Module):
    def __init__(self, seq_len, layers=LAYERS):
        super().__init__()
        self.pos_embedding = nn.Parameter(torch.empty(1, seq_len, D_MODEL).normal_(std=0.02))
        self.dropout = nn.Dropout(0.0)
        self.layers = nn.Sequential(OrderedDict(
            (f"encoder_layer_{i}", EncoderBlock()) for i in range(layers)))
        self.ln = LayerNorm(D_MODEL, eps=EPS)


class VitTrunk(nn.Module):
    """torchvision vit_b_16 without `heads`; forward -> class-token features [B, 768]."""

    def __init__(self, layers=LAYERS):
        super().__init__()
        self.conv_proj = nn.Conv2d(3, D_MODEL, PATCH, PATCH)
        fan_in = 3 * PATCH * PATCH
        nn.init.trunc_normal_(self.conv_proj.weight, std=math.sqrt(1 / fan_in))
        nn.init.zeros_(self.conv_proj.bias)
        self.class_token = nn.Parameter(torch.zeros(1, 1, D_MODEL))
        self.encoder = Encoder((IMG // PATCH) ** 2 + 1, layers)
        self.feat_dim = D_MODEL
        self.compute_dtype = torch.float32

    def forward(self, x):
        T = self.compute_dtype
        if x.dim() != 4 or x.shape[1] != 3:
            raise ValueError("expected images [B,3,H,W]")
        h = _PatchTokensFn.apply(x.float(), self.conv_proj.weight, self.conv_proj.bias,
                                 self.class_token, self.encoder.pos_embedding, T)
        from . import xplan
        params = []
        for blk in self.encoder.layers:
            at = blk.self_attention
            params += [blk.ln_1.weight, blk.ln_1.bias, at.in_proj_weight, at.in_proj_bias,
                       at.out_proj.weight, at.out_proj.bias, blk.ln_2.weight, blk.ln_2.bias,
                       blk.mlp[0].weight, blk.mlp[0].bias, blk.mlp[3].weight, blk.mlp[3].bias]
        # the 12 blocks as one native launch plan per direction (xplan); the eager per-block
        # nodes when gradients are off or a block parameter is frozen
        cfg = type("VitCfg", (), dict(heads=HEADS, eps=EPS))
        out = xplan.run_stack("vit", h, None, cfg, self.encoder, params) if params else None
        if out is not None:
            h = out
        else:
            for blk in self.encoder.layers:
                h = blk(h)
        return _ClassTokenLNFn.apply(h, self.encoder.ln.weight, self.encoder.ln.bias)
