"""Structure of the transformer-stack launch plans (mmdx.xplan), recorded on the host with
CPU tensors standing in for device memory (nothing is launched): the parameter-gradient
layout tiles one flat buffer exactly (what the data-parallel reducer relies on), every
weight is cast by the single multi-tensor launch at the head of the forward, the workspace
placeholder is patched everywhere, and the op mix per layer is the eager node's.  The
plans' arithmetic is checked on the GPU against the eager nodes (test_stack_plans_gpu.py).
"""
import math

import pytest
import torch

from mmdx import _lib as L
from mmdx import bert as MB
from mmdx import xplan
from mmdx.vit import VitTrunk

CPU = torch.device("cpu")


def _ops(lst):
    return [lst.arr[i] for i in range(lst.n)]


def _check_layout(pl, params):
    items = sorted(pl.grads.items, key=lambda t: t[2])
    assert sorted(i for i, _, _ in items) == list(range(len(params)))
    off = 0
    for idx, shape, o in items:
        assert o == off, "gaps or overlaps in the gradient buffer"
        assert tuple(params[idx].shape) == shape
        off += math.prod(shape)
    assert off == pl.grads.n == sum(q.numel() for q in params)


def _check_ops(pl, n_weights, n_layers, gemm_fwd, gemm_bwd):
    fwd, bwd = _ops(pl.fwd), _ops(pl.bwd)
    assert fwd[0].op == L.OP_CONV_PACK_MULTI and fwd[0].i[0] == n_weights
    assert not any(o.op == L.OP_CAST and o.dtype != o.i[0] for o in fwd[1:]), \
        "a weight cast outside the multi-tensor launch"
    for o in fwd + bwd:
        for j in range(12):
            assert not (o.ext[j] == -1 and o.p[j] == 1), "unpatched workspace placeholder"
    assert sum(o.op == L.OP_GEMM for o in fwd) == gemm_fwd * n_layers
    # the four weight gradients per layer carry their bias gradients (no column-sum ops)
    assert sum(o.op == L.OP_GEMM_BIAS_GRAD for o in bwd) == 4 * n_layers
    assert sum(o.op == L.OP_GEMM for o in bwd) == (gemm_bwd - 4) * n_layers
    assert not any(o.op == L.OP_BIAS_GRAD for o in bwd)
    assert not any(o.op == L.OP_GELU_BWD for o in bwd), "GELU backward not fused"
    assert sum(o.op == L.OP_EVENT for o in fwd) == 2 * len(pl.fwd.conv_names)


@pytest.mark.parametrize("p", [0.0, 0.1])
def test_bert_stack_plan_structure(p):
    m = MB.BertModel.from_name("bert-base-uncased@2")
    params = [q for lay in m.encoder.layer for q in lay.params()]
    pl = xplan._build_bert(params, 2, 16, 768, 12, 3072, 1e-12, p, p, torch.bfloat16, CPU)
    _check_layout(pl, params)
    # per layer: 3 (q, k, v) + out + FFN up + FFN down weights cast; GEMMs fwd 4, bwd 8
    _check_ops(pl, 6 * 2, 2, 4, 8)
    # hidden dropout inside the two LayerNorm passes per layer (forward and backward), no
    # separate dropout launch or mask; attention-probability dropout inside the attention op
    fwd, bwd = _ops(pl.fwd), _ops(pl.bwd)
    assert not any(o.op in (L.OP_DROPOUT_FWD, L.OP_DROPOUT_BWD) for o in fwd + bwd)
    assert sum(o.op == L.OP_LN_FWD_DROP for o in fwd) == (4 if p > 0 else 0)
    assert sum(o.op == L.OP_LN_BWD_DROP for o in bwd) == (4 if p > 0 else 0)
    seeds = [o.l[1] for o in fwd if o.op == L.OP_LN_FWD_DROP]
    assert len(set(seeds)) == len(seeds), "two dropout ops share a seed"


def test_vit_stack_plan_structure():
    m = VitTrunk(layers=2)
    params = []
    for blk in m.encoder.layers:
        at = blk.self_attention
        params += [blk.ln_1.weight, blk.ln_1.bias, at.in_proj_weight, at.in_proj_bias,
                   at.out_proj.weight, at.out_proj.bias, blk.ln_2.weight, blk.ln_2.bias,
                   blk.mlp[0].weight, blk.mlp[0].bias, blk.mlp[3].weight, blk.mlp[3].bias]
    pl = xplan._build_vit(params, 2, 197, 768, 12, 3072, 1e-6, torch.float16, CPU)
    _check_layout(pl, params)
    _check_ops(pl, 4 * 2, 2, 4, 8)


def test_plan_cache_evicts_idle_stale_keys(monkeypatch):
    """Plans recorded for keys no longer used (other batch shapes, re-allocated parameters)
    are dropped once more than MAX_PLAN_KEYS keys exist and their arenas are idle; a busy
    arena (its backward still pending) is never dropped."""
    from mmdx import resnet as RN

    class _A:
        def __init__(self):
            self.b = False

        def busy(self):
            return self.b

    class _P:
        def __init__(self):
            self.arena = _A()

    monkeypatch.setattr(RN, "MAX_PLAN_KEYS", 2)
    cache = {}
    p0 = RN.plan_cache_get(cache, "k0", _P)
    p0.arena.b = True                       # k0's backward pending
    RN.plan_cache_get(cache, "k1", _P)
    RN.plan_cache_get(cache, "k2", _P)
    RN.plan_cache_get(cache, "k3", _P)
    assert "k0" in cache                    # busy: kept
    p0.arena.b = False
    RN.plan_cache_get(cache, "k4", _P)
    assert len(cache) <= 3 and "k0" not in cache and "k4" in cache
    again = RN.plan_cache_get(cache, "k4", _P)
    assert again is cache["k4"][0]          # an idle plan of the key is reused


def _small_vit_params(nl, D=64, I=128):
    g = torch.Generator().manual_seed(0)
    shapes = ((D,), (D,), (3 * D, D), (3 * D,), (D, D), (D,), (D,), (D,), (I, D), (I,),
              (D, I), (D,))
    return [torch.randn(sh, generator=g) for _ in range(nl) for sh in shapes]


@pytest.mark.parametrize("seg", [3, 1, 0])
def test_stack_backward_segments(monkeypatch, seg):
    """The stack backward is cut every SEG_LAYERS layers; each cut's gradient region is the
    contiguous slice of those layers' parameter gradients (the data-parallel reducer issues
    its in-place all-reduce there, xplan.STACK_SEGMENT_HOOK).  The regions cover the layers
    above layer 0's group exactly once, last layer first."""
    monkeypatch.setattr(xplan, "SEG_LAYERS", seg)
    nl = 12
    params = _small_vit_params(nl)
    pl = xplan._build_vit(params, 2, 17, 64, 1, 128, 1e-6, torch.float16, CPU)
    per_layer = sum(q.numel() for q in params[:12])
    if seg == 0:
        assert pl.grad_regions == [] and len(pl.bwd.bounds) == 2
        return
    want = []
    top = nl
    while top - seg > 0:
        want.append(((top - seg) * per_layer, top * per_layer))
        top -= seg
    assert pl.grad_regions == want
    assert len(pl.bwd.bounds) == len(want) + 2
    # bert: same rule over its layout
    m = MB.BertModel.from_name("bert-base-uncased@2")
    bp = [q for lay in m.encoder.layer for q in lay.params()]
    bpl = xplan._build_bert(bp, 2, 16, 768, 12, 3072, 1e-12, 0.0, 0.0, torch.bfloat16, CPU)
    n1 = sum(q.numel() for q in bp[:16])
    assert bpl.grad_regions == ([(n1, 2 * n1)] if seg == 1 else [])
