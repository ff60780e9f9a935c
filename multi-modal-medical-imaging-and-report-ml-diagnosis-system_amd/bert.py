"""BERT-base encoder on the mmdx kernels, state_dict-identical to transformers' BertModel.

The reference builds it with `AutoModel.from_pretrained("bert-base-uncased")`
(training_pipeline.py:360) and calls it at TP:470/473; its arithmetic is transformers'
BertEmbeddings / BertLayer (modeling_bert.py).  Here each BertLayer is ONE autograd node:
fused QKV GEMM -> attention core (MFMA, in-LDS softmax) -> out-proj GEMM -> Add&LayerNorm ->
FFN up GEMM (+GELU epilogue) -> FFN down GEMM -> Add&LayerNorm, with a hand-sequenced
backward whose residual gradients are summed inside GEMM epilogues (beta = 1).
Hidden-state dropout runs on the mmdx dropout kernel in train mode; attention-probability
dropout (BertSelfAttention's, p = config.attention_probs_dropout_prob) is fused into the
attention kernel (counter-based hash, keep bit carried in the saved probabilities' sign).
RNG streams cannot match torch's, so parity runs use p = 0 on both sides; the dropout
arithmetic itself is checked against an explicit masked reference (tests/test_text_gpu.py).
"""
from __future__ import annotations

import math
from types import SimpleNamespace

import torch
import torch.nn as nn

from . import _lib as L
from . import functional as F
from ._lib import call, ptr, stream
from .layers import Embedding, LayerNorm, Linear


class _Out(SimpleNamespace):
    pass


def _cat_cast(ws, T, device):
    """Concatenate fp32 tensors along dim 0 into one compute-dtype buffer (device casts)."""
    rows = sum(w.shape[0] for w in ws)
    out = torch.empty((rows,) + tuple(ws[0].shape[1:]), dtype=T, device=device)
    o = 0
    for w in ws:
        n = w.shape[0]
        call("mmdx_cast", L.dtype_code(T), L.F32, ptr(w), w.numel(), ptr(out[o:o + n]), stream())
        o += n
    return out


def _ws(n, dev):
    return L.workspace(n, dev)


def _ln_bwd(xs, dy, gamma, mean, rstd):
    D = xs.shape[-1]
    rows = xs.numel() // D
    dx = torch.empty_like(xs)
    dg = torch.empty(D, dtype=torch.float32, device=xs.device)
    db = torch.empty(D, dtype=torch.float32, device=xs.device)
    n = L.lib().mmdx_layernorm_workspace_size(rows, D)
    w = _ws(n, xs.device)
    call("mmdx_layernorm_bwd", L.dtype_code(xs.dtype), ptr(xs), ptr(dy), rows, D, ptr(gamma),
         ptr(mean), ptr(rstd), ptr(dx), ptr(dg), ptr(db), 0.0, ptr(w), n, stream())
    return dx, dg, db


def _ln_fwd(x, res, gamma, beta, eps):
    D = x.shape[-1]
    rows = x.numel() // D
    y = torch.empty_like(x)
    xs = torch.empty_like(x)
    mean = torch.empty(rows, dtype=torch.float32, device=x.device)
    rstd = torch.empty(rows, dtype=torch.float32, device=x.device)
    call("mmdx_layernorm_fwd", L.dtype_code(x.dtype), ptr(x), ptr(res), rows, D, ptr(gamma),
         ptr(beta), float(eps), ptr(y), ptr(xs), ptr(mean), ptr(rstd), stream())
    return y, xs, mean, rstd


def _ln_fwd_drop(x, res, gamma, beta, eps, p, seed):
    """LayerNorm(dropout(x) + res) in one pass; returns (y, xsum, mean, rstd, rng)."""
    D = x.shape[-1]
    rows = x.numel() // D
    y = torch.empty_like(x)
    xs = torch.empty_like(x)
    mean = torch.empty(rows, dtype=torch.float32, device=x.device)
    rstd = torch.empty(rows, dtype=torch.float32, device=x.device)
    rng = torch.empty(1, dtype=torch.int64, device=x.device)
    call("mmdx_layernorm_fwd_dropout", L.dtype_code(x.dtype), ptr(x), ptr(res), rows, D,
         ptr(gamma), ptr(beta), float(eps), float(p), L.dropout_seed(seed),
         ptr(L.rng_counter(x.device)), ptr(y), ptr(xs), ptr(mean), ptr(rstd), ptr(rng), stream())
    return y, xs, mean, rstd, rng


def _ln_bwd_drop(xs, dy, gamma, mean, rstd, p, rng):
    """(d xsum, its dropout backward, dgamma, dbeta)."""
    D = xs.shape[-1]
    rows = xs.numel() // D
    dx = torch.empty_like(xs)
    dxd = torch.empty_like(xs)
    dg = torch.empty(D, dtype=torch.float32, device=xs.device)
    db = torch.empty(D, dtype=torch.float32, device=xs.device)
    n = L.lib().mmdx_layernorm_workspace_size(rows, D)
    w = _ws(n, xs.device)
    call("mmdx_layernorm_bwd_dropout", L.dtype_code(xs.dtype), ptr(xs), ptr(dy), rows, D,
         ptr(gamma), ptr(mean), ptr(rstd), float(p), ptr(rng), ptr(dx), ptr(dxd), ptr(dg),
         ptr(db), 0.0, ptr(w), n, stream())
    return dx, dxd, dg, db


def _dropout_fwd(x, p, seed):
    y = torch.empty_like(x)
    m = torch.empty(x.shape, dtype=torch.uint8, device=x.device)
    call("mmdx_dropout_fwd", L.dtype_code(x.dtype), ptr(x), x.numel(), float(p),
         L.dropout_seed(seed), 0, ptr(L.rng_counter(x.device)), ptr(y), ptr(m), stream())
    return y, m


def _dropout_bwd(dy, m, p):
    dx = torch.empty_like(dy)
    call("mmdx_dropout_bwd", L.dtype_code(dy.dtype), ptr(dy), ptr(m), dy.numel(), float(p),
         ptr(dx), stream())
    return dx


_SEED = [0xB127]


class _BertLayerFn(torch.autograd.Function):
    """One transformers BertLayer (post-LN) forward/backward on mmdx kernels."""

    @staticmethod
    def forward(ctx, h, mask, cfg, wq, bq, wk, bk, wv, bv, wo, bo, g1, b1, wi, bi, wo2, bo2, g2,
                b2):
        B, Ls, D = h.shape
        Hn, eps, p = cfg.num_attention_heads, cfg.layer_norm_eps, cfg.p_hidden
        T = h.dtype
        dev = h.device
        M = B * Ls
        x = h.reshape(M, D)
        wqkv = _cat_cast([wq, wk, wv], T, dev)
        bqkv = torch.empty(3 * D, dtype=torch.float32, device=dev)
        for i, bb in enumerate((bq, bk, bv)):
            call("mmdx_axpby", D, 1.0, ptr(bb), 0.0, None, ptr(bqkv[i * D:(i + 1) * D]),
                 stream())
        qkv = torch.empty((M, 3 * D), dtype=T, device=dev)
        F.gemm(x, D, True, wqkv, D, True, M, 3 * D, D, qkv, 3 * D, bias=bqkv, compute_dtype=T)
        att = torch.empty((M, D), dtype=T, device=dev)
        keep = any(ctx.needs_input_grad)
        scale = 1.0 / math.sqrt(D // Hn)
        # BertSelfAttention's dropout on attention_probs (train mode), fused in the kernel
        pa = float(cfg.p_attn) if (cfg.training and keep) else 0.0
        if pa > 0:
            _SEED[0] += 1
        ctx.attn = F.attention_fwd(qkv, mask, B, Ls, Hn, scale, pa,
                                   L.dropout_seed(_SEED[0]) if pa > 0 else 0,
                                   L.rng_counter(dev), att, keep)
        woc = F.cast(wo, T)
        a = torch.empty((M, D), dtype=T, device=dev)
        F.gemm(att, D, True, woc, D, True, M, D, D, a, D, bias=bo, compute_dtype=T)
        m1 = None
        if p > 0 and cfg.training:   # dropout inside the LayerNorm pass (keep bits in m1)
            _SEED[0] += 1
            h1, xs1, mu1, rs1, m1 = _ln_fwd_drop(a, x, g1, b1, eps, p, _SEED[0])
        else:
            h1, xs1, mu1, rs1 = _ln_fwd(a, x, g1, b1, eps)
        wic = F.cast(wi, T)
        I = wi.shape[0]
        f = torch.empty((M, I), dtype=T, device=dev)
        pre = torch.empty((M, I), dtype=T, device=dev)
        F.gemm(h1, D, True, wic, D, True, M, I, D, f, I, bias=bi, act=L.ACT_GELU, preact=pre,
               compute_dtype=T)
        wo2c = F.cast(wo2, T)
        f2 = torch.empty((M, D), dtype=T, device=dev)
        F.gemm(f, I, True, wo2c, I, True, M, D, I, f2, D, bias=bo2, compute_dtype=T)
        m2 = None
        if p > 0 and cfg.training:
            _SEED[0] += 1
            h2, xs2, mu2, rs2, m2 = _ln_fwd_drop(f2, h1, g2, b2, eps, p, _SEED[0])
        else:
            h2, xs2, mu2, rs2 = _ln_fwd(f2, h1, g2, b2, eps)
        ctx.save_for_backward(x, mask, wqkv, qkv, att, woc, xs1, mu1, rs1, g1, h1, wic,
                              pre, f, wo2c, xs2, mu2, rs2, g2)
        ctx.m1, ctx.m2, ctx.p, ctx.pa = m1, m2, p, pa
        ctx.dims = (B, Ls, D, Hn, I, scale)
        return h2.reshape(B, Ls, D)

    @staticmethod
    def backward(ctx, dh2):
        (x, mask, wqkv, qkv, att, woc, xs1, mu1, rs1, g1, h1, wic, pre, f, wo2c, xs2, mu2,
         rs2, g2) = ctx.saved_tensors
        B, Ls, D, Hn, I, scale = ctx.dims
        T = x.dtype
        dev = x.device
        M = B * Ls
        dh2 = F.cast(dh2.contiguous().reshape(M, D), T)
        # LN2: X = d(f2 + h1)
        if ctx.m2 is not None:
            X, dX2, dg2, db2 = _ln_bwd_drop(xs2, dh2, g2, mu2, rs2, ctx.p, ctx.m2)
        else:
            X, dg2, db2 = _ln_bwd(xs2, dh2, g2, mu2, rs2)
            dX2 = X
        # FFN down: f2 = f Wo2^T + bo2
        # dpre = (dX2 Wo2) * gelu'(pre): the GELU backward in the GEMM epilogue
        dpre = torch.empty((M, I), dtype=T, device=dev)
        F.gemm(dX2, D, True, wo2c, I, False, M, I, D, dpre, I, act=L.ACT_GELU_BWD, preact=pre,
               compute_dtype=T)
        dWo2 = torch.empty((D, I), dtype=torch.float32, device=dev)
        dbo2 = torch.empty(D, dtype=torch.float32, device=dev)
        F.gemm_wgrad_bias(dX2, D, f, I, D, I, M, dWo2, I, dbo2, compute_dtype=T)
        dWi = torch.empty((I, D), dtype=torch.float32, device=dev)
        dbi = torch.empty(I, dtype=torch.float32, device=dev)
        F.gemm_wgrad_bias(dpre, I, h1, D, I, D, M, dWi, D, dbi, compute_dtype=T)
        # X := dpre Wi + X  (residual into h1)
        F.gemm(dpre, I, True, wic, D, False, M, D, I, X, D, beta=1.0, compute_dtype=T)
        # LN1: Y = d(a + x)
        if ctx.m1 is not None:
            Y, dY1, dg1, db1 = _ln_bwd_drop(xs1, X, g1, mu1, rs1, ctx.p, ctx.m1)
        else:
            Y, dg1, db1 = _ln_bwd(xs1, X, g1, mu1, rs1)
            dY1 = Y
        datt = torch.empty((M, D), dtype=T, device=dev)
        F.gemm(dY1, D, True, woc, D, False, M, D, D, datt, D, compute_dtype=T)
        dWo = torch.empty((D, D), dtype=torch.float32, device=dev)
        dbo = torch.empty(D, dtype=torch.float32, device=dev)
        F.gemm_wgrad_bias(dY1, D, att, D, D, D, M, dWo, D, dbo, compute_dtype=T)
        dqkv = torch.empty((M, 3 * D), dtype=T, device=dev)
        F.attention_bwd(qkv, ctx.attn, att, datt, mask, B, Ls, Hn, scale, ctx.pa, dqkv)
        dWqkv = torch.empty((3 * D, D), dtype=torch.float32, device=dev)
        dbqkv = torch.empty(3 * D, dtype=torch.float32, device=dev)
        F.gemm_wgrad_bias(dqkv, 3 * D, x, D, 3 * D, D, M, dWqkv, D, dbqkv, compute_dtype=T)
        # Y := dqkv Wqkv + Y  (residual into x)
        F.gemm(dqkv, 3 * D, True, wqkv, D, False, M, D, 3 * D, Y, D, beta=1.0, compute_dtype=T)
        dx = Y.reshape(B, Ls, D)
        return (dx, None, None,
                dWqkv[:D], dbqkv[:D], dWqkv[D:2 * D], dbqkv[D:2 * D], dWqkv[2 * D:],
                dbqkv[2 * D:], dWo, dbo, dg1, db1, dWi, dbi, dWo2, dbo2, dg2, db2)


class _EmbedFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, ids, tt, word, pos, typ, gamma, beta, eps, T):
        B, Ls = ids.shape
        D = word.shape[1]
        dev = ids.device
        y = torch.empty((B, Ls, D), dtype=T, device=dev)
        xs = torch.empty((B, Ls, D), dtype=T, device=dev)
        mean = torch.empty(B * Ls, dtype=torch.float32, device=dev)
        rstd = torch.empty(B * Ls, dtype=torch.float32, device=dev)
        call("mmdx_embed_ln_fwd", L.dtype_code(T), ptr(ids), ptr(tt), B, Ls, D, ptr(word),
             ptr(pos), ptr(typ), ptr(gamma), ptr(beta), float(eps), ptr(y), ptr(xs), ptr(mean),
             ptr(rstd), stream())
        ctx.save_for_backward(ids, tt, xs, mean, rstd, gamma)
        ctx.shapes = (word.shape, pos.shape, typ.shape)
        return y

    @staticmethod
    def backward(ctx, dy):
        ids, tt, xs, mean, rstd, gamma = ctx.saved_tensors
        B, Ls = ids.shape
        D = xs.shape[-1]
        dy = F.cast(dy.contiguous(), xs.dtype)
        dx, dg, db = _ln_bwd(xs, dy, gamma, mean, rstd)
        dev = ids.device
        ws, ps, ts = ctx.shapes
        dword = torch.zeros(ws, dtype=torch.float32, device=dev)
        dpos = torch.zeros(ps, dtype=torch.float32, device=dev)
        dtyp = torch.zeros(ts, dtype=torch.float32, device=dev)
        call("mmdx_embed_bwd", L.dtype_code(xs.dtype), ptr(ids), ptr(tt), B, Ls, D, ptr(dx),
             ptr(dword), ptr(dpos), ptr(dtyp), 0, stream())
        return None, None, dword, dpos, dtyp, dg, db, None, None


# ----------------------------------------------------------------------------- modules
class BertEmbeddings(nn.Module):
    def __init__(self, cfg):
        super().__init__()
        self.word_embeddings = Embedding(cfg.vocab_size, cfg.hidden_size, padding_idx=0)
        self.position_embeddings = Embedding(cfg.max_position_embeddings, cfg.hidden_size)
        self.token_type_embeddings = Embedding(cfg.type_vocab_size, cfg.hidden_size)
        self.LayerNorm = LayerNorm(cfg.hidden_size, eps=cfg.layer_norm_eps)


class BertSelfAttention(nn.Module):
    def __init__(self, cfg):
        super().__init__()
        self.query = Linear(cfg.hidden_size, cfg.hidden_size)
        self.key = Linear(cfg.hidden_size, cfg.hidden_size)
        self.value = Linear(cfg.hidden_size, cfg.hidden_size)


class _DenseLN(nn.Module):
    def __init__(self, din, dout, eps):
        super().__init__()
        self.dense = Linear(din, dout)
        self.LayerNorm = LayerNorm(dout, eps=eps)


class BertAttention(nn.Module):
    def __init__(self, cfg):
        super().__init__()
        self.self = BertSelfAttention(cfg)
        self.output = _DenseLN(cfg.hidden_size, cfg.hidden_size, cfg.layer_norm_eps)


class _Intermediate(nn.Module):
    def __init__(self, cfg):
        super().__init__()
        self.dense = Linear(cfg.hidden_size, cfg.intermediate_size)


class BertLayer(nn.Module):
    def __init__(self, cfg):
        super().__init__()
        self.attention = BertAttention(cfg)
        self.intermediate = _Intermediate(cfg)
        self.output = _DenseLN(cfg.intermediate_size, cfg.hidden_size, cfg.layer_norm_eps)

    def params(self):
        s, o = self.attention.self, self.attention.output
        return [s.query.weight, s.query.bias, s.key.weight, s.key.bias, s.value.weight,
                s.value.bias, o.dense.weight, o.dense.bias, o.LayerNorm.weight, o.LayerNorm.bias,
                self.intermediate.dense.weight, self.intermediate.dense.bias,
                self.output.dense.weight, self.output.dense.bias, self.output.LayerNorm.weight,
                self.output.LayerNorm.bias]


class _Encoder(nn.Module):
    def __init__(self, cfg):
        super().__init__()
        self.layer = nn.ModuleList([BertLayer(cfg) for _ in range(cfg.num_hidden_layers)])


class _Pooler(nn.Module):
    def __init__(self, cfg):
        super().__init__()
        self.dense = Linear(cfg.hidden_size, cfg.hidden_size)


def bert_base_config(num_hidden_layers=12, dropout=0.1):
    """BertConfig() defaults = bert-base-uncased geometry (transformers configuration_bert)."""
    return SimpleNamespace(vocab_size=30522, hidden_size=768, num_hidden_layers=num_hidden_layers,
                           num_attention_heads=12, intermediate_size=3072,
                           hidden_dropout_prob=dropout, attention_probs_dropout_prob=dropout,
                           max_position_embeddings=512, type_vocab_size=2, layer_norm_eps=1e-12,
                           initializer_range=0.02, pad_token_id=0,
                           _name_or_path="bert-base-uncased")


class BertModel(nn.Module):
    def __init__(self, config=None):
        super().__init__()
        self.config = config or bert_base_config()
        self.embeddings = BertEmbeddings(self.config)
        self.encoder = _Encoder(self.config)
        self.pooler = _Pooler(self.config)
        self.compute_dtype = torch.float32
        self._init_weights()

    @classmethod
    def from_name(cls, name: str):
        """'bert-base-uncased' (12 layers) or 'bert-base-uncased@N' (first N layers) —
        built offline from the BertConfig defaults; a local HF directory's weights can be
        loaded with load_state_dict (keys are identical)."""
        layers = 12
        if "@" in name:
            name, n = name.split("@", 1)
            layers = int(n)
        return cls(bert_base_config(layers))

    def _init_weights(self):  # BertPreTrainedModel._init_weights
        std = self.config.initializer_range
        for m in self.modules():
            if isinstance(m, nn.Linear):
                nn.init.normal_(m.weight, 0.0, std)
                nn.init.zeros_(m.bias)
            elif isinstance(m, nn.Embedding):
                nn.init.normal_(m.weight, 0.0, std)
                if m.padding_idx is not None:
                    with torch.no_grad():
                        m.weight[m.padding_idx].zero_()
            elif isinstance(m, nn.LayerNorm):
                nn.init.ones_(m.weight)
                nn.init.zeros_(m.bias)

    def forward(self, input_ids, attention_mask=None, token_type_ids=None, return_dict=True):
        T = self.compute_dtype
        L.require_device(input_ids)
        ids = input_ids.long().contiguous()
        B, Ls = ids.shape
        mask = (attention_mask.long().contiguous() if attention_mask is not None
                else torch.ones_like(ids))
        tt = (token_type_ids.long().contiguous() if token_type_ids is not None
              else torch.zeros_like(ids))
        e = self.embeddings
        h = _EmbedFn.apply(ids, tt, e.word_embeddings.weight, e.position_embeddings.weight,
                           e.token_type_embeddings.weight, e.LayerNorm.weight, e.LayerNorm.bias,
                           self.config.layer_norm_eps, T)
        cfg = SimpleNamespace(num_attention_heads=self.config.num_attention_heads,
                              layer_norm_eps=self.config.layer_norm_eps,
                              p_hidden=self.config.hidden_dropout_prob,
                              p_attn=self.config.attention_probs_dropout_prob,
                              training=self.training)
        # the whole layer stack as one native launch plan per direction (xplan); the eager
        # per-layer nodes when gradients are off or some encoder parameter is frozen
        from . import xplan
        params = [q for layer in self.encoder.layer for q in layer.params()]
        keep = torch.is_grad_enabled()
        pcfg = SimpleNamespace(heads=self.config.num_attention_heads,
                               eps=self.config.layer_norm_eps,
                               p=float(self.config.hidden_dropout_prob) if self.training else 0.0,
                               pa=(float(self.config.attention_probs_dropout_prob)
                                   if self.training and keep else 0.0))
        out = xplan.run_stack("bert", h, mask, pcfg, self.encoder, params) if params else None
        if out is not None:
            return _Out(last_hidden_state=out)
        for layer in self.encoder.layer:
            h = _BertLayerFn.apply(h, mask, cfg, *layer.params())
        return _Out(last_hidden_state=h)
