"""T5 report head on the mmdx kernels.

The reference builds `report_model = T5ForConditionalGeneration` (training_pipeline.py:545,
t5-small) and drives only its DECODER: the encoder is replaced by K = 4 synthetic tokens
`cond_proj(z_fuse)` (TP:553-558, 574-578); training feeds `labels` (teacher forcing,
decoder_input_ids = shift_right(labels), CrossEntropyLoss(ignore_index=-100), TP:983-991,
1049-1053); predict beam-searches (TP:613-618, IP:190-196).

`T5Head` executes a transformers `T5ForConditionalGeneration`'s decoder + tied lm_head from
its own parameters (so `report_model.*` state_dict keys, dtype handling and the bundle format
are untouched) on HIP kernels: one autograd node per decoder block (RMSNorm, fused QKV GEMM,
causal self-attention with the relative-position bias, cross-attention over the condition
tokens, ReLU FFN, dropout), the final RMSNorm + lm_head (alpha = d_model^-0.5, fp32 logits)
+ cross-entropy in one more node.  Beam search (`generate`) restates transformers'
vectorised `_beam_search` on the host (numpy, float32) over decoder forwards on the GPU.
"""
from __future__ import annotations

import math

import numpy as np
import torch

from . import _lib as L
from . import functional as F
from ._lib import call, ptr, stream


def _cat_cast(ws, T, dev):
    rows = sum(w.shape[0] for w in ws)
    out = torch.empty((rows,) + tuple(ws[0].shape[1:]), dtype=T, device=dev)
    o = 0
    for w in ws:
        n = w.shape[0]
        call("mmdx_cast", L.dtype_code(T), L.F32, ptr(w), w.numel(), ptr(out[o:o + n]), stream())
        o += n
    return out


def _mm(a, w, M, N, K, out, act=L.ACT_NONE, alpha=1.0, beta=0.0):
    """out[M,N] = act(alpha * a[M,K] @ w[N,K]^T) + beta * out."""
    return F.gemm(a, K, True, w, K, True, M, N, K, out, N, act=act, alpha=alpha, beta=beta,
                  compute_dtype=a.dtype)


def _mm_dx(dy, w, M, N, K, out, beta=0.0):
    """out[M,K] = dy[M,N] @ w[N,K] (+ beta * out)."""
    return F.gemm(dy, N, True, w, K, False, M, K, N, out, K, beta=beta, compute_dtype=dy.dtype)


def _mm_dw(dy, x, M, N, K):
    """dW[N,K] = dy[M,N]^T @ x[M,K] (fp32)."""
    dw = torch.empty((N, K), dtype=torch.float32, device=dy.device)
    F.gemm(dy, N, False, x, K, False, N, K, M, dw, K, compute_dtype=dy.dtype)
    return dw


def _rms(x, w, eps):
    D = x.shape[-1]
    rows = x.numel() // D
    y = torch.empty_like(x)
    r = torch.empty(rows, dtype=torch.float32, device=x.device)
    call("mmdx_rmsnorm_fwd", L.dtype_code(x.dtype), ptr(x), rows, D, ptr(w), float(eps), ptr(y),
         ptr(r), stream())
    return y, r


def _rms_bwd(x, dy, w, r, dx_acc):
    """dx_acc += d rms(x) / dx . dy (in place); returns dw."""
    D = x.shape[-1]
    rows = x.numel() // D
    dw = torch.empty(D, dtype=torch.float32, device=x.device)
    n = L.lib().mmdx_rmsnorm_workspace_size(rows, D)
    ws = L.workspace(n, x.device)
    call("mmdx_rmsnorm_bwd", L.dtype_code(x.dtype), ptr(x), ptr(dy), rows, D, ptr(w), ptr(r),
         ptr(dx_acc), 1.0, ptr(dw), 0.0, ptr(ws), n, stream())
    return dw


def _add(a, b):
    out = torch.empty_like(a)
    call("mmdx_add", L.dtype_code(a.dtype), a.numel(), ptr(a), ptr(b), ptr(out), stream())
    return out


def _dropout(x, p, training, seed):
    if not training or p <= 0.0:
        return x, None
    y = torch.empty_like(x)
    m = torch.empty(x.shape, dtype=torch.uint8, device=x.device)
    call("mmdx_dropout_fwd", L.dtype_code(x.dtype), ptr(x), x.numel(), float(p),
         L.dropout_seed(seed), 0, ptr(L.rng_counter(x.device)), ptr(y), ptr(m), stream())
    return y, m


def _dropout_bwd(dy, m, p):
    if m is None:
        return dy
    dx = torch.empty_like(dy)
    call("mmdx_dropout_bwd", L.dtype_code(dy.dtype), ptr(dy), ptr(m), dy.numel(), float(p),
         ptr(dx), stream())
    return dx


_SEED = [0x7A5]


class _BlockCfg:
    def __init__(self, H, eps, p, training, nb, maxd):
        self.H, self.eps, self.p, self.training, self.nb, self.maxd = H, eps, p, training, nb, maxd


class _T5BlockFn(torch.autograd.Function):
    """One transformers T5Block of the decoder (T5LayerSelfAttention, T5LayerCrossAttention,
    T5LayerFF; modeling_t5.py), forward and hand-sequenced backward.  `table` is the shared
    relative_attention_bias.weight: every block returns its share of d(table)."""

    @staticmethod
    def forward(ctx, h, enc, table, bias, cfg, ln0, wq, wk, wv, wo, ln1, wq2, wk2, wv2, wo2, ln2,
                wi, wo3):
        B, Ls, D = h.shape
        Kc = enc.shape[1]
        H = cfg.H
        T = h.dtype
        dev = h.device
        M = B * Ls
        x = h.reshape(M, D)
        tr = cfg.training
        keep = any(ctx.needs_input_grad)
        # --- self-attention: x + dropout(o(attn(rms(x))))
        n1, r1 = _rms(x, ln0, cfg.eps)
        wqkv = _cat_cast([wq, wk, wv], T, dev)
        qkv = _mm(n1, wqkv, M, 3 * D, D, torch.empty((M, 3 * D), dtype=T, device=dev))
        att = torch.empty((M, D), dtype=T, device=dev)
        probs = torch.empty((B, H, Ls, Ls), dtype=torch.float32, device=dev) if keep else None
        pa = cfg.p if tr else 0.0
        if pa > 0:
            _SEED[0] += 1
        call("mmdx_attention_fwd_ex", L.dtype_code(T), ptr(qkv), None, ptr(bias), 1, B, Ls, H,
             1.0, float(pa), L.dropout_seed(_SEED[0]) if pa > 0 else 0,
             ptr(L.rng_counter(dev)), ptr(att), ptr(probs), stream())
        woc = F.cast(wo, T)
        a = _mm(att, woc, M, D, D, torch.empty((M, D), dtype=T, device=dev))
        _SEED[0] += 1
        a, m1 = _dropout(a, cfg.p, tr, _SEED[0])
        h1 = _add(x, a)
        # --- cross-attention over the condition tokens
        n2, r2 = _rms(h1, ln1, cfg.eps)
        wq2c = F.cast(wq2, T)
        q2 = _mm(n2, wq2c, M, D, D, torch.empty((M, D), dtype=T, device=dev))
        e2 = enc.reshape(B * Kc, D)
        wkv2 = _cat_cast([wk2, wv2], T, dev)
        kv = _mm(e2, wkv2, B * Kc, 2 * D, D, torch.empty((B * Kc, 2 * D), dtype=T, device=dev))
        xatt = torch.empty((M, D), dtype=T, device=dev)
        xprobs = torch.empty((B, H, Ls, Kc), dtype=torch.float32, device=dev) if keep else None
        if pa > 0:
            _SEED[0] += 1
        call("mmdx_xattn_fwd", L.dtype_code(T), ptr(q2), D, ptr(kv), B, Ls, Kc, H, 1.0,
             float(pa), L.dropout_seed(_SEED[0]) if pa > 0 else 0, ptr(L.rng_counter(dev)),
             ptr(xatt), ptr(xprobs), stream())
        wo2c = F.cast(wo2, T)
        c = _mm(xatt, wo2c, M, D, D, torch.empty((M, D), dtype=T, device=dev))
        _SEED[0] += 1
        c, m2 = _dropout(c, cfg.p, tr, _SEED[0])
        h2 = _add(h1, c)
        # --- FFN: h2 + dropout(wo(dropout(relu(wi(rms(h2))))))
        n3, r3 = _rms(h2, ln2, cfg.eps)
        I = wi.shape[0]
        wic = F.cast(wi, T)
        f = _mm(n3, wic, M, I, D, torch.empty((M, I), dtype=T, device=dev), act=L.ACT_RELU)
        _SEED[0] += 1
        fd, m3 = _dropout(f, cfg.p, tr, _SEED[0])
        wo3c = F.cast(wo3, T)
        g = _mm(fd, wo3c, M, D, I, torch.empty((M, D), dtype=T, device=dev))
        _SEED[0] += 1
        g, m4 = _dropout(g, cfg.p, tr, _SEED[0])
        h3 = _add(h2, g)
        if keep:
            ctx.save_for_backward(x, n1, r1, wqkv, qkv, probs, att, woc, h1, n2, r2, wq2c, q2,
                                  e2, wkv2, kv, xprobs, xatt, wo2c, h2, n3, r3, wic, f, fd, wo3c,
                                  ln0, ln1, ln2)
            ctx.masks = (m1, m2, m3, m4)
            ctx.cfg, ctx.pa = cfg, pa
            ctx.dims = (B, Ls, D, Kc, I)
        return h3.reshape(B, Ls, D)

    @staticmethod
    def backward(ctx, dh3):
        (x, n1, r1, wqkv, qkv, probs, att, woc, h1, n2, r2, wq2c, q2, e2, wkv2, kv, xprobs, xatt,
         wo2c, h2, n3, r3, wic, f, fd, wo3c, ln0, ln1, ln2) = ctx.saved_tensors
        m1, m2, m3, m4 = ctx.masks
        cfg, pa = ctx.cfg, ctx.pa
        B, Ls, D, Kc, I = ctx.dims
        H = cfg.H
        T = x.dtype
        dev = x.device
        M = B * Ls
        dh = F.cast(dh3.contiguous().reshape(M, D), T).clone()   # running residual gradient
        # FFN
        dg = _dropout_bwd(dh, m4, cfg.p)
        dWo3 = _mm_dw(dg, fd, M, D, I)
        dfd = _mm_dx(dg, wo3c, M, D, I, torch.empty((M, I), dtype=T, device=dev))
        df = _dropout_bwd(dfd, m3, cfg.p)
        dpre = torch.empty_like(df)
        call("mmdx_relu_bwd", L.dtype_code(T), ptr(f), ptr(df), df.numel(), ptr(dpre), stream())
        dWi = _mm_dw(dpre, n3, M, I, D)
        dn3 = _mm_dx(dpre, wic, M, I, D, torch.empty((M, D), dtype=T, device=dev))
        dln2 = _rms_bwd(h2, dn3, ln2, r3, dh)
        # cross-attention
        dc = _dropout_bwd(dh, m2, cfg.p)
        dWo2 = _mm_dw(dc, xatt, M, D, D)
        dxatt = _mm_dx(dc, wo2c, M, D, D, torch.empty((M, D), dtype=T, device=dev))
        dq2 = torch.empty((M, D), dtype=T, device=dev)
        dkv = torch.empty((B * Kc, 2 * D), dtype=T, device=dev)
        n = L.lib().mmdx_xattn_workspace_size(B, Ls, Kc, H)
        ws = L.workspace(n, dev)
        call("mmdx_xattn_bwd", L.dtype_code(T), ptr(q2), D, ptr(kv), ptr(xprobs), ptr(dxatt), B,
             Ls, Kc, H, 1.0, float(pa), ptr(dq2), D, ptr(dkv), ptr(ws), n, stream())
        dWq2 = _mm_dw(dq2, n2, M, D, D)
        dn2 = _mm_dx(dq2, wq2c, M, D, D, torch.empty((M, D), dtype=T, device=dev))
        dWkv2 = _mm_dw(dkv, e2, B * Kc, 2 * D, D)
        denc = _mm_dx(dkv, wkv2, B * Kc, 2 * D, D, torch.empty((B * Kc, D), dtype=T, device=dev))
        dln1 = _rms_bwd(h1, dn2, ln1, r2, dh)
        # self-attention
        da = _dropout_bwd(dh, m1, cfg.p)
        dWo = _mm_dw(da, att, M, D, D)
        datt = _mm_dx(da, woc, M, D, D, torch.empty((M, D), dtype=T, device=dev))
        dqkv = torch.empty((M, 3 * D), dtype=T, device=dev)
        n = L.lib().mmdx_attention_workspace_size(L.dtype_code(T), B, Ls, H)
        ws = L.workspace(n, dev)
        call("mmdx_attention_bwd", L.dtype_code(T), ptr(qkv), ptr(probs), ptr(datt), None, B, Ls,
             H, 1.0, float(pa), ptr(dqkv), ptr(ws), n, stream())
        dtable = torch.empty((cfg.nb, H), dtype=torch.float32, device=dev)
        LP = (Ls + 31) // 32 * 32
        call("mmdx_t5_position_bias_bwd", L.dtype_code(T), ptr(ws), B, H, Ls, LP, cfg.nb,
             cfg.maxd, ptr(dtable), 0.0, stream())
        dWqkv = _mm_dw(dqkv, n1, M, 3 * D, D)
        dn1 = _mm_dx(dqkv, wqkv, M, 3 * D, D, torch.empty((M, D), dtype=T, device=dev))
        dln0 = _rms_bwd(x, dn1, ln0, r1, dh)
        return (dh.reshape(B, Ls, D), denc.reshape(B, Kc, D), dtable, None, None, dln0,
                dWqkv[:D], dWqkv[D:2 * D], dWqkv[2 * D:], dWo, dln1, dWq2, dWkv2[:D], dWkv2[D:],
                dWo2, dln2, dWi, dWo3)


class _EmbedFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, ids, table, T):
        B, Ls = ids.shape
        D = table.shape[1]
        out = torch.empty((B, Ls, D), dtype=T, device=ids.device)
        call("mmdx_embed_gather", L.dtype_code(T), ptr(ids), B * Ls, D, ptr(table), ptr(out),
             stream())
        ctx.save_for_backward(ids)
        ctx.tshape = table.shape
        return out

    @staticmethod
    def backward(ctx, dout):
        (ids,) = ctx.saved_tensors
        B, Ls = ids.shape
        dtab = torch.zeros(ctx.tshape, dtype=torch.float32, device=dout.device)
        call("mmdx_embed_scatter", L.dtype_code(dout.dtype), ptr(ids), B * Ls, ctx.tshape[1],
             ptr(dout.contiguous()), ptr(dtab), stream())
        return None, dtab, None


class _HeadFn(torch.autograd.Function):
    """final_layer_norm -> dropout -> * d_model^-0.5 -> tied lm_head (fp32 logits) ->
    CrossEntropyLoss(ignore_index=-100) (T5ForConditionalGeneration.forward)."""

    @staticmethod
    def forward(ctx, h, shared, lnf, labels, eps, p, training, scale):
        B, Ls, D = h.shape
        T = h.dtype
        dev = h.device
        M = B * Ls
        V = shared.shape[0]
        hf, rf = _rms(h.reshape(M, D), lnf, eps)
        _SEED[0] += 1
        hd, md = _dropout(hf, p, training, _SEED[0])
        wc = F.cast(shared, T)
        logits = torch.empty((M, V), dtype=torch.float32, device=dev)
        _mm(hd, wc, M, V, D, logits, alpha=scale)
        loss = count = ws = None
        if labels is not None:
            loss = torch.empty((), dtype=torch.float32, device=dev)
            count = torch.empty((), dtype=torch.float32, device=dev)
            n = L.lib().mmdx_cross_entropy_workspace_size(M)
            ws = L.workspace(n, dev)
            call("mmdx_cross_entropy_fwd", ptr(logits), ptr(labels), M, V, ptr(loss), ptr(count),
                 ptr(ws), n, stream())
        ctx.save_for_backward(h, hd, rf, wc, logits, labels, lnf, count, ws)
        ctx.md, ctx.p, ctx.eps, ctx.scale = md, p, eps, scale
        ctx.set_materialize_grads(False)
        return (loss if loss is not None else torch.zeros((), device=dev)), logits.view(B, Ls, V)

    @staticmethod
    def backward(ctx, dloss, dlogits_ext):
        h, hd, rf, wc, logits, labels, lnf, count, ws = ctx.saved_tensors
        B, Ls, D = h.shape
        T = h.dtype
        dev = h.device
        M = B * Ls
        V = wc.shape[0]
        if labels is not None and dloss is not None:
            dlog = torch.empty((M, V), dtype=T, device=dev)
            call("mmdx_cross_entropy_bwd", L.dtype_code(T), ptr(logits), ptr(labels), M, V,
                 ptr(dloss.contiguous()), ptr(count), ptr(ws), ptr(dlog), stream())
            if dlogits_ext is not None:  # a caller that also differentiates the logits
                tot = torch.empty((M, V), dtype=torch.float32, device=dev)
                call("mmdx_axpby", M * V, 1.0, ptr(F.cast(dlog, torch.float32)), 1.0,
                     ptr(dlogits_ext.float().contiguous()), ptr(tot), stream())
                dlog = F.cast(tot, T)
        else:
            dlog = F.cast(dlogits_ext.contiguous().reshape(M, V), T)
        # logits = scale * hd @ W^T
        dW = torch.empty((V, D), dtype=torch.float32, device=dev)
        F.gemm(dlog, V, False, hd, D, False, V, D, M, dW, D, alpha=ctx.scale, compute_dtype=T)
        dhd = torch.empty((M, D), dtype=T, device=dev)
        F.gemm(dlog, V, True, wc, D, False, M, D, V, dhd, D, alpha=ctx.scale, compute_dtype=T)
        dhf = _dropout_bwd(dhd, ctx.md, ctx.p)
        dh = torch.zeros((M, D), dtype=T, device=dev)
        dlnf = _rms_bwd(h.reshape(M, D), dhf, lnf, rf, dh)
        return dh.reshape(B, Ls, D), dW, dlnf, None, None, None, None, None


def shift_right(labels, start_id=0, pad_id=0):
    """T5PreTrainedModel._shift_right: [start] + labels[:-1], -100 -> pad."""
    out = torch.empty_like(labels)
    out[:, 1:] = labels[:, :-1]
    out[:, 0] = start_id
    return out.masked_fill(out == -100, pad_id)


class _DecodeState:
    """KV-cached incremental decoder of one generate() call (what transformers' generate does
    with its past_key_values): every decoder weight is cast / concatenated ONCE, the
    cross-attention K/V of the condition tokens are computed once per block, the relative-
    position bias is built once for the longest sequence, and each step runs the decoder on
    ONE new token per running beam, appending its self-attention K/V to per-block caches
    (mmdx_t5_decode_attn).  The beam's ancestry lives in a slot table (key j of row r is in
    cache row slots[r, j]), so reordering beams moves no cache data.  The step ends on the
    device with the logits processors and the candidate top-k (mmdx_beam_topk): only
    2 * num_beams (score, index) pairs per batch row come back to the host."""

    def __init__(self, head, enc_r, T, Lmax):
        m = head.m
        dev = enc_r.device
        D, H = head.D, head.H
        R, Kc = enc_r.shape[0], enc_r.shape[1]
        self.head, self.T, self.dev, self.R, self.Lmax, self.D, self.H = head, T, dev, R, Lmax, D, H
        self.V = head.head_weight().shape[0]
        e2 = enc_r.to(T).contiguous().reshape(R * Kc, D)
        self.Kc = Kc
        self.blocks = []
        for blk in head._blocks():
            sa, ca, ff = blk.layer[0], blk.layer[1], blk.layer[2]
            at, xt = sa.SelfAttention, ca.EncDecAttention
            wkv2 = _cat_cast([xt.k.weight, xt.v.weight], T, dev)
            kv = _mm(e2, wkv2, R * Kc, 2 * D, D, torch.empty((R * Kc, 2 * D), dtype=T, device=dev))
            self.blocks.append(dict(
                ln0=sa.layer_norm.weight.detach(), wqkv=_cat_cast([at.q.weight, at.k.weight,
                                                                   at.v.weight], T, dev),
                wo=F.cast(at.o.weight, T), ln1=ca.layer_norm.weight.detach(),
                wq2=F.cast(xt.q.weight, T), kv=kv, wo2=F.cast(xt.o.weight, T),
                ln2=ff.layer_norm.weight.detach(), wi=F.cast(ff.DenseReluDense.wi.weight, T),
                wo3=F.cast(ff.DenseReluDense.wo.weight, T),
                kc=torch.empty((R, Lmax, D), dtype=T, device=dev),
                vc=torch.empty((R, Lmax, D), dtype=T, device=dev)))
        self.I = self.blocks[0]["wi"].shape[0]
        self.lnf = m.decoder.final_layer_norm.weight.detach()
        self.w_head = F.cast(head.head_weight(), T)
        self.table = m.shared.weight.detach()
        rel = head._blocks()[0].layer[0].SelfAttention.relative_attention_bias.weight.detach()
        self.bias = torch.empty((H, Lmax, Lmax), dtype=torch.float32, device=dev)
        call("mmdx_t5_position_bias", ptr(rel), H, Lmax, head.nb, head.maxd, ptr(self.bias),
             stream())
        # per-step buffers
        e = lambda *shape, dt=T: torch.empty(shape, dtype=dt, device=dev)  # noqa: E731
        self.h, self.n, self.att, self.x2 = e(R, D), e(R, D), e(R, D), e(R, D)
        self.qkv, self.f = e(R, 3 * D), e(R, self.I)
        self.logits = e(R, self.V, dt=torch.float32)
        self.lp = e(R, self.V, dt=torch.float32)
        # one host -> device upload per step: tokens (int64 [R]), run scores (fp32 [R]), the
        # slot table (int32 [R, Lmax]) and the banned (row, token) pairs (int32, <= R*Lmax)
        self.off_sc = 8 * R
        self.off_slot = self.off_sc + 4 * R
        self.off_ban = self.off_slot + 4 * R * Lmax
        self.nbytes = self.off_ban + 8 * R * Lmax
        self.stage_h = torch.empty(self.nbytes, dtype=torch.uint8, pin_memory=True)
        self.stage_d = torch.empty(self.nbytes, dtype=torch.uint8, device=dev)
        self.out_v = e(1, dt=torch.float32)
        self.out_i = e(1, dt=torch.int64)
        self.host_v = self.host_i = None

    def step(self, tokens, pos, slots, run_sc, bans, eos_ban, B, nb, k):
        """Decoder step at position `pos` for every running beam; returns the top-k
        (scores, flat indices i*V + v) per batch row as numpy arrays [B, k]."""
        R, D, H, T, st = self.R, self.D, self.H, self.T, stream()
        hb = self.stage_h.numpy()
        hb[:self.off_sc].view(np.int64)[:] = tokens
        hb[self.off_sc:self.off_slot].view(np.float32)[:] = run_sc
        hb[self.off_slot:self.off_ban].view(np.int32)[:] = slots.reshape(-1)
        nban = len(bans)
        if nban:
            hb[self.off_ban:self.off_ban + 8 * nban].view(np.int32)[:] = bans.reshape(-1)
        nup = self.off_ban + 8 * nban
        self.stage_d[:nup].copy_(self.stage_h[:nup], non_blocking=True)
        toks = self.stage_d[:self.off_sc].view(torch.int64)
        sc = self.stage_d[self.off_sc:self.off_slot].view(torch.float32)
        sl = self.stage_d[self.off_slot:self.off_ban].view(torch.int32)
        ban = self.stage_d[self.off_ban:].view(torch.int32)
        hd = self.head
        h, n, att, qkv = self.h, self.n, self.att, self.qkv
        dc = L.dtype_code(T)
        call("mmdx_embed_gather", dc, ptr(toks), R, D, ptr(self.table), ptr(h), st)
        for b in self.blocks:
            call("mmdx_rmsnorm_fwd", dc, ptr(h), R, D, ptr(b["ln0"]), float(hd.eps), ptr(n),
                 None, st)
            _mm(n, b["wqkv"], R, 3 * D, D, qkv)
            call("mmdx_t5_decode_attn", dc, ptr(qkv), R, H, int(pos), self.Lmax, ptr(b["kc"]),
                 ptr(b["vc"]), ptr(sl), ptr(self.bias), ptr(att), st)
            _mm(att, b["wo"], R, D, D, h, beta=1.0)                    # h += attn out
            call("mmdx_rmsnorm_fwd", dc, ptr(h), R, D, ptr(b["ln1"]), float(hd.eps), ptr(n),
                 None, st)
            _mm(n, b["wq2"], R, D, D, att)
            call("mmdx_xattn_fwd", dc, ptr(att), D, ptr(b["kv"]), R, 1, self.Kc, H, 1.0, 0.0, 0,
                 None, ptr(self.x2), None, st)
            _mm(self.x2, b["wo2"], R, D, D, h, beta=1.0)             # h += cross-attn out
            call("mmdx_rmsnorm_fwd", dc, ptr(h), R, D, ptr(b["ln2"]), float(hd.eps), ptr(n),
                 None, st)
            _mm(n, b["wi"], R, self.I, D, self.f, act=L.ACT_RELU)
            _mm(self.f, b["wo3"], R, D, self.I, h, beta=1.0)          # h += FFN out
        call("mmdx_rmsnorm_fwd", dc, ptr(h), R, D, ptr(self.lnf), float(hd.eps), ptr(n), None,
             st)
        _mm(n, self.w_head, R, self.V, D, self.logits, alpha=hd.scale)
        call("mmdx_log_softmax", ptr(self.logits), R, self.V, ptr(self.lp), st)
        if self.out_v.numel() != B * k:
            self.out_v = torch.empty(B * k, dtype=torch.float32, device=self.dev)
            self.out_i = torch.empty(B * k, dtype=torch.int64, device=self.dev)
            self.host_v = torch.empty(B * k, dtype=torch.float32, pin_memory=True)
            self.host_i = torch.empty(B * k, dtype=torch.int64, pin_memory=True)
        call("mmdx_beam_topk", ptr(self.lp), B, nb, self.V, ptr(sc), ptr(ban), nban,
             int(eos_ban), k, ptr(self.out_v), ptr(self.out_i), st)
        self.host_v.copy_(self.out_v, non_blocking=True)
        self.host_i.copy_(self.out_i, non_blocking=True)
        torch.cuda.current_stream().synchronize()
        return (self.host_v.numpy().reshape(B, k).copy(), self.host_i.numpy().reshape(B, k).copy())


def _ngram_bans(hist, ngram):
    """NoRepeatNGramLogitsProcessor for every row of hist [R, cur]: (row, token) pairs that
    would complete an n-gram already in the row (vectorised; same pairs as the loop)."""
    R, cur = hist.shape
    if ngram <= 0 or cur + 1 < ngram:
        return np.zeros((0, 2), dtype=np.int32)
    w = ngram - 1
    nwin = cur - ngram + 1
    if nwin <= 0:
        return np.zeros((0, 2), dtype=np.int32)
    if w == 0:
        rr = np.repeat(np.arange(R), cur)
        return np.stack([rr, hist.reshape(-1)], 1).astype(np.int32)
    prev = hist[:, cur - w:]
    win = np.lib.stride_tricks.sliding_window_view(hist[:, :cur - 1], w, axis=1)[:, :nwin]
    match = (win == prev[:, None, :]).all(axis=2)
    rr, ss = np.nonzero(match)
    return np.stack([rr, hist[rr, ss + w]], 1).astype(np.int32)


class T5Head:
    """Runs `model` (a transformers T5ForConditionalGeneration) decoder-only on mmdx kernels."""

    def __init__(self, model):
        self.m = model
        c = model.config
        self.D, self.H = c.d_model, c.num_heads
        self.eps = c.layer_norm_epsilon
        self.p = c.dropout_rate
        self.nb = c.relative_attention_num_buckets
        self.maxd = c.relative_attention_max_distance
        self.start = c.decoder_start_token_id if c.decoder_start_token_id is not None else 0
        self.pad = c.pad_token_id if c.pad_token_id is not None else 0
        # tied (t5-small): lm_head IS shared.weight, logits scaled by d_model^-0.5; untied
        # (T5 v1.1 style): the separate lm_head.weight, no scale (modeling_t5.py)
        self.tied = bool(getattr(c, "tie_word_embeddings", True))
        self.scale = c.d_model ** -0.5 if self.tied else 1.0
        if c.feed_forward_proj != "relu" or c.d_kv != 64:
            raise NotImplementedError("mmdx T5 head: t5-small family (ReLU FFN, d_kv 64)")

    def _blocks(self):
        return self.m.decoder.block

    def head_weight(self):
        """The [V, D] output projection: the shared embedding when tied, else lm_head."""
        return self.m.shared.weight if self.tied else self.m.lm_head.weight

    def hidden(self, dec_ids, enc, T):
        """Decoder hidden states before final_layer_norm: [B, L, D] in T."""
        m = self.m
        dev = enc.device
        B, Ls = dec_ids.shape
        training = m.training
        h = _EmbedFn.apply(dec_ids.long().contiguous(), m.shared.weight, T)
        if training and self.p > 0:
            h = F.dropout(h, self.p, True)
        table = self._blocks()[0].layer[0].SelfAttention.relative_attention_bias.weight
        bias = torch.empty((self.H, Ls, Ls), dtype=torch.float32, device=dev)
        call("mmdx_t5_position_bias", ptr(table.detach()), self.H, Ls, self.nb, self.maxd,
             ptr(bias), stream())
        cfg = _BlockCfg(self.H, self.eps, self.p, training, self.nb, self.maxd)
        enc = enc.to(T).contiguous()
        for blk in self._blocks():
            sa, ca, ff = blk.layer[0], blk.layer[1], blk.layer[2]
            h = _T5BlockFn.apply(
                h, enc, table, bias, cfg, sa.layer_norm.weight, sa.SelfAttention.q.weight,
                sa.SelfAttention.k.weight, sa.SelfAttention.v.weight, sa.SelfAttention.o.weight,
                ca.layer_norm.weight, ca.EncDecAttention.q.weight, ca.EncDecAttention.k.weight,
                ca.EncDecAttention.v.weight, ca.EncDecAttention.o.weight, ff.layer_norm.weight,
                ff.DenseReluDense.wi.weight, ff.DenseReluDense.wo.weight)
        return h

    def forward(self, enc, labels=None, decoder_input_ids=None, T=torch.float32):
        """(loss, logits [B, L, V] fp32) as T5ForConditionalGeneration(encoder_outputs=enc,
        labels=labels)."""
        L.require_device(enc)
        if decoder_input_ids is None:
            if labels is None:
                raise ValueError("T5 head needs labels or decoder_input_ids")
            decoder_input_ids = shift_right(labels, self.start, self.pad)
        h = self.hidden(decoder_input_ids, enc, T)
        m = self.m
        lab = labels.long().contiguous() if labels is not None else None
        loss, logits = _HeadFn.apply(h, self.head_weight(), m.decoder.final_layer_norm.weight, lab,
                                     self.eps, self.p, m.training, self.scale)
        return (loss if labels is not None else None), logits

    # -------------------------------------------------------------------------- generate
    @torch.no_grad()
    def _last_log_probs(self, seqs, enc, T):
        """log_softmax of the last position's logits for each running sequence [R, V], by
        re-running the decoder over the whole prefix (no cache): the reference the
        incremental decoder (_DecodeState) is tested against."""
        h = self.hidden(seqs, enc, T)
        R, Ls, D = h.shape
        m = self.m
        last = h[:, -1, :].contiguous()
        hf, _ = _rms(last, m.decoder.final_layer_norm.weight, self.eps)
        wc = F.cast(self.head_weight(), T)
        V = wc.shape[0]
        logits = torch.empty((R, V), dtype=torch.float32, device=h.device)
        _mm(hf, wc, R, V, D, logits, alpha=self.scale)
        lp = torch.empty_like(logits)
        call("mmdx_log_softmax", ptr(logits), R, V, ptr(lp), stream())
        return lp

    @torch.no_grad()
    def generate(self, enc, num_beams=4, max_new_tokens=180, min_new_tokens=0,
                 no_repeat_ngram_size=0, length_penalty=1.0, early_stopping=True,
                 eos_token_id=1, pad_token_id=0, T=torch.float32, _stepper=None, **unused):
        """Beam search as transformers' GenerationMixin._beam_search (vectorised form, the
        logits processors MinNewTokensLength + NoRepeatNGram, stopping on max length / EOS),
        restated on the host in float32 over decoder forwards on the GPU.  Returns the best
        sequence per batch row, [B, 1 + generated] int64 (decoder start token first).

        `_stepper` (tests only) replaces the device step: a callable (hist [R, cur] int64,
        pos, slots, run_scores [R], bans, eos_ban) -> (top-k scores [B, k], flat indices
        [B, k]) with k = 2 * num_beams; the host loop is then checked on its own."""
        was = self.m.training
        self.m.eval()
        try:
            return self._beam(enc, num_beams, max_new_tokens, min_new_tokens,
                              no_repeat_ngram_size, length_penalty, early_stopping,
                              eos_token_id, pad_token_id, T, _stepper)
        finally:
            self.m.train(was)

    def _beam(self, enc, nb, max_new, min_new, ngram, lp_pen, early, eos, pad, T, stepper):
        B = enc.shape[0]
        dev = enc.device
        prompt = 1
        max_len = prompt + max_new
        V = self.m.config.vocab_size
        k_keep = max(2, 1 + 1) * nb
        if k_keep > 16:
            raise NotImplementedError("mmdx beam search: num_beams <= 8")
        fill = pad or eos
        f32 = np.float32
        run_seq = np.full((B, nb, max_len), fill, dtype=np.int64)
        run_seq[:, :, 0] = self.start
        run_len = np.zeros((B, nb), dtype=np.int64)     # generated tokens per running beam
        run_sc = np.zeros((B, nb), dtype=f32)
        run_sc[:, 1:] = f32(-1e9)
        seqs = run_seq.copy()
        seq_len = np.zeros((B, nb), dtype=np.int64)
        beam_sc = np.full((B, nb), f32(-1e9), dtype=f32)
        fin = np.zeros((B, nb), dtype=bool)
        unsat = np.ones((B, 1), dtype=bool)
        top_mask = np.zeros(k_keep, dtype=bool)
        top_mask[:nb] = True
        R = B * nb
        if stepper is None:
            dec = _DecodeState(self, enc.repeat_interleave(nb, dim=0), T, max_len)

            def stepper(hist, pos, slots, sc, bans, eos_ban):
                return dec.step(hist[:, pos], pos, slots, sc, bans, eos_ban, B, nb, k_keep)
        slots = np.zeros((R, max_len), dtype=np.int32)  # cache row of key j for beam r
        rows = np.arange(R, dtype=np.int32)
        base = (np.arange(B) * nb)[:, None]
        cur = prompt
        while True:
            pos = cur - 1
            slots[:, pos] = rows                         # this step's K/V: (row r, pos)
            # logits processors (applied on the device): MinNewTokensLength bans EOS,
            # NoRepeatNGram bans the tokens that would repeat an n-gram
            hist = run_seq[:, :, :cur].reshape(R, cur)
            bans = _ngram_bans(hist, ngram)
            eos_ban = eos if cur - prompt < min_new else -1
            # top-k of the running scores + log-probs (descending; torch.topk order on ties
            # is not pinned — ties are measure-zero on float scores)
            tk_lp, idx = stepper(hist, pos, slots, run_sc.reshape(R), bans, eos_ban)
            tk_beam = idx // V
            tk_tok = idx % V
            tk_seq = np.take_along_axis(run_seq, tk_beam[:, :, None], axis=1).copy()
            tk_seq[:, :, cur] = tk_tok
            tk_len = np.take_along_axis(run_len, tk_beam, axis=1) + 1
            hits = (tk_tok == eos) | (cur + 1 >= max_len)
            # running beams for the next step
            tk_run = (tk_lp + hits.astype(f32) * f32(-1e9)).astype(f32)
            nxt = np.argsort(-tk_run, axis=1, kind="stable")[:, :nb]
            parent = np.take_along_axis(tk_beam, nxt, axis=1) + base   # cache rows
            slots = slots[parent.reshape(R)]
            run_seq = np.take_along_axis(tk_seq, nxt[:, :, None], axis=1)
            run_sc = np.take_along_axis(tk_run, nxt, axis=1)
            run_len = np.take_along_axis(tk_len, nxt, axis=1)
            # finished beams
            did = hits & top_mask[None, :]
            norm = (tk_lp / f32((cur + 1 - prompt) ** lp_pen)).astype(f32)
            full = np.all(fin, axis=1, keepdims=True) & (early is True)
            norm = norm + full.astype(f32) * f32(-1e9)
            norm = norm + (~unsat).astype(f32) * f32(-1e9)
            norm = norm + (~did).astype(f32) * f32(-1e9)
            m_seq = np.concatenate([seqs, tk_seq], axis=1)
            m_sc = np.concatenate([beam_sc, norm], axis=1)
            m_len = np.concatenate([seq_len, tk_len], axis=1)
            m_fin = np.concatenate([fin, did], axis=1)
            sel = np.argsort(-m_sc, axis=1, kind="stable")[:, :nb]
            seqs = np.take_along_axis(m_seq, sel[:, :, None], axis=1)
            beam_sc = np.take_along_axis(m_sc, sel, axis=1)
            seq_len = np.take_along_axis(m_len, sel, axis=1)
            fin = np.take_along_axis(m_fin, sel, axis=1)
            cur += 1
            # early-stop heuristic (early_stopping True / False: best length = cur - prompt)
            if early == "never" and lp_pen > 0.0:
                best_len = max_len - prompt
            else:
                best_len = cur - prompt
            best_run = run_sc[:, :1] / f32(best_len ** lp_pen)
            worst = np.where(fin, np.min(beam_sc, axis=1, keepdims=True), f32(-1e9))
            unsat = unsat & np.any(best_run > worst, axis=1, keepdims=True)
            improvement = np.any(unsat)
            open_beam = not (np.all(fin) and early is True)
            valid = not np.all(hits)
            if not (improvement and open_beam and valid):
                break
        out_len = prompt + int(seq_len[:, 0].max())
        return torch.from_numpy(seqs[:, 0, :out_len].copy())
