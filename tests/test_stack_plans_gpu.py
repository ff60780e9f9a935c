"""GPU: the transformer encoder stacks replayed from native launch plans (mmdx.xplan: the
BERT-base text tower's and the ViT-B/16 image tower's layers as one autograd node, one plan
call per direction) against the eager per-layer nodes they replace (MMDX_STACK_PLANS=0).

Both paths issue the same kernels with the same operands in the same order (the plan shares
one workspace where the eager nodes allocate one per call; every kernel overwrites its
workspace before reading it), so with dropout off the forward output, the input gradient
and EVERY parameter gradient must be bit-identical, in fp32, bf16 and fp16 (C5).  With
dropout on, the plan draws its masks from the device launch counter: two steps differ and
stay finite.  The eager nodes themselves are checked against transformers / the oracle in
test_text_gpu.py and test_vit_gpu.py; the benched C5 step (test_benched_path_gpu.py) runs
the plan path against the CPU oracle.
"""
import pytest
import torch

import mmdx
from mmdx import bert as MB
from mmdx import xplan
from mmdx.vit import VitTrunk

pytestmark = pytest.mark.gpu

DTYPES = [torch.float32, torch.bfloat16, torch.float16]


def _bert_run(dev, dt, plans, monkeypatch, p=0.0, steps=1):
    monkeypatch.setenv("MMDX_STACK_PLANS", "1" if plans else "0")
    torch.manual_seed(3)
    m = MB.BertModel.from_name("bert-base-uncased@2")
    m.config.hidden_dropout_prob = p
    m.config.attention_probs_dropout_prob = p
    m.compute_dtype = dt
    m.to(dev).train()
    g = torch.Generator().manual_seed(4)
    ids = torch.randint(1000, 30522, (3, 37), generator=g).to(dev)
    mask = torch.ones(3, 37, dtype=torch.long)
    mask[1, 20:] = 0
    mask = mask.to(dev)
    w = torch.randn(3, 37, 768, generator=g).to(dev)
    outs = []
    for _ in range(steps):
        for q in m.parameters():
            q.grad = None
        h = m(input_ids=ids, attention_mask=mask).last_hidden_state
        (h.float() * w).sum().backward()
        outs.append((h.detach().clone(),
                     {n: q.grad.detach().clone() for n, q in m.named_parameters()
                      if q.grad is not None}))
    return outs


@pytest.mark.parametrize("dt", DTYPES)
def test_bert_stack_plan_matches_eager(dev, dt, monkeypatch):
    (h0, g0), = _bert_run(dev, dt, False, monkeypatch)
    (h1, g1), = _bert_run(dev, dt, True, monkeypatch)
    assert torch.equal(h0, h1)
    assert set(g0) == set(g1)
    bad = [n for n in g0 if not torch.equal(g0[n], g1[n])]
    assert not bad, bad


def test_bert_stack_plan_dropout_draws_fresh_masks(dev, monkeypatch):
    (ha, ga), (hb, gb) = _bert_run(dev, torch.bfloat16, True, monkeypatch, p=0.1, steps=2)
    assert torch.isfinite(ha.float()).all() and torch.isfinite(hb.float()).all()
    assert not torch.equal(ha, hb), "a replayed plan reused its dropout masks"
    for n in ga:
        assert torch.isfinite(ga[n]).all() and torch.isfinite(gb[n]).all(), n


def test_bert_plan_gradients_tile_one_buffer(dev, monkeypatch):
    """The parameter gradients of a plan backward are views of ONE flat fp32 buffer that
    they cover exactly (the data-parallel reducer all-reduces it in place)."""
    (_, grads), = _bert_run(dev, torch.bfloat16, True, monkeypatch)
    monkeypatch.setenv("MMDX_STACK_PLANS", "1")
    torch.manual_seed(3)
    m = MB.BertModel.from_name("bert-base-uncased@2")
    m.compute_dtype = torch.bfloat16
    m.to(dev).train()
    ids = torch.randint(1000, 30522, (2, 16)).to(dev)
    m(input_ids=ids).last_hidden_state.float().sum().backward()
    enc = [q.grad for lay in m.encoder.layer for q in lay.params()]
    st = {g.untyped_storage().data_ptr() for g in enc}
    assert len(st) == 1
    assert sum(g.numel() for g in enc) * 4 == enc[0].untyped_storage().nbytes()


def _vit_run(dev, dt, plans, monkeypatch):
    monkeypatch.setenv("MMDX_STACK_PLANS", "1" if plans else "0")
    torch.manual_seed(0)
    m = VitTrunk(layers=2)
    m.compute_dtype = dt
    m.to(dev)
    g = torch.Generator().manual_seed(5)
    x = torch.randn(2, 3, 224, 224, generator=g).to(dev)
    f = m(x)
    dy = torch.randn(f.shape, generator=g).to(dev)
    f.float().backward(dy)
    return f.detach().clone(), {n: q.grad.detach().clone() for n, q in m.named_parameters()}


@pytest.mark.parametrize("dt", DTYPES)
def test_vit_stack_plan_matches_eager(dev, dt, monkeypatch):
    f0, g0 = _vit_run(dev, dt, False, monkeypatch)
    f1, g1 = _vit_run(dev, dt, True, monkeypatch)
    assert torch.equal(f0, f1)
    bad = [n for n in g0 if not torch.equal(g0[n], g1[n])]
    assert not bad, bad


def test_stack_plan_not_used_without_grad(dev, monkeypatch):
    monkeypatch.setenv("MMDX_STACK_PLANS", "1")
    m = MB.BertModel.from_name("bert-base-uncased@2").to(dev)
    ids = torch.randint(1000, 30522, (2, 16)).to(dev)
    with torch.no_grad():
        m(input_ids=ids)
    assert not m.encoder.__dict__.get("_mmdx_stack_plans"), "plan built for a no-grad forward"
    assert xplan.enabled()
    mmdx.text_encoders  # noqa: B018 (the package's text towers import cleanly)
