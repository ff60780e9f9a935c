"""Text-tower parity: attention core, BiLSTM recurrence, BERT layers vs PyTorch / transformers.

fp32 tolerances: outputs rel 1e-4 of scale; grads 1 - cosine <= 1e-5 (fp32 vs fp32 ref).
bf16: rel 3e-2.
"""
import math

import pytest
import torch

import mmdx
from mmdx import _lib as L
from oracle import ref_cpu as R
from parity_util import cosine, norm_ratio, rel_err

pytestmark = pytest.mark.gpu


def _ref_attention(q, k, v, mask, scale):
    s = torch.einsum("blhd,bmhd->bhlm", q, k) * scale
    if mask is not None:
        s = s + (1.0 - mask[:, None, None, :].float()) * -1e30
    p = s.softmax(-1)
    return torch.einsum("bhlm,bmhd->blhd", p, v)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16, torch.float16])
@pytest.mark.parametrize("B,Ls,H", [(2, 128, 12), (3, 37, 2), (2, 197, 4), (1, 256, 1),
                                    (1, 1, 3), (2, 16, 8), (4, 129, 6)])
@pytest.mark.parametrize("masked", [True, False])
def test_attention(dev, dt, B, Ls, H, masked):
    """Forward, saved probabilities and backward against torch fp32.  The shapes cover the
    16-bit kernels' cases: L % 4 != 0 (probability tiles transposed through LDS), a second
    128-query block holding one query (L 129), single-key rows (L 1), and B*H not a multiple
    of 8 (plain block order instead of the XCD-grouped one)."""
    g = torch.Generator().manual_seed(B * Ls + H)
    qkv = torch.randn(B, Ls, 3, H, 64, generator=g)
    if dt != torch.float32:
        qkv = qkv.to(dt).float()
    mask = None
    if masked:
        lens = torch.randint(1, Ls + 1, (B,), generator=g)
        mask = (torch.arange(Ls)[None] < lens[:, None]).long()
    scale = 0.125
    qr = qkv.clone().requires_grad_(True)
    o = _ref_attention(qr[:, :, 0], qr[:, :, 1], qr[:, :, 2], mask, scale)
    do = torch.randn(o.shape, generator=g)
    if dt != torch.float32:
        do = do.to(dt).float()
    o.backward(do)
    dc = L.dtype_code(dt)
    qd = qkv.to(dev, dt).contiguous()
    md = mask.to(dev) if mask is not None else None
    out = torch.empty(B, Ls, H, 64, dtype=dt, device=dev)
    probs = torch.empty(B, H, Ls, Ls, device=dev)
    L.call("mmdx_attention_fwd", dc, qd.data_ptr(), md.data_ptr() if md is not None else None,
           B, Ls, H, scale, 0.0, 0, None, out.data_ptr(), probs.data_ptr(), L.stream())
    tol = 1e-4 if dt == torch.float32 else 3e-2
    assert rel_err(out, o) <= tol
    with torch.no_grad():
        q, k = qkv[:, :, 0], qkv[:, :, 1]
        sc = torch.einsum("blhd,bmhd->bhlm", q, k) * scale
        if mask is not None:
            sc = sc + (1.0 - mask[:, None, None, :].float()) * -1e30
        assert rel_err(probs, sc.softmax(-1)) <= 1e-4
    dqkv = torch.empty_like(qd)
    n = L.lib().mmdx_attention_workspace_size(dc, B, Ls, H)
    ws = torch.empty(n, dtype=torch.uint8, device=dev)
    L.call("mmdx_attention_bwd", dc, qd.data_ptr(), probs.data_ptr(),
           do.to(dev, dt).contiguous().data_ptr(), md.data_ptr() if md is not None else None, B,
           Ls, H, scale, 0.0, dqkv.data_ptr(), ws.data_ptr(), n, L.stream())
    for i, name in enumerate("qkv"):
        e = rel_err(dqkv[:, :, i], qr.grad[:, :, i])
        assert e <= (2e-4 if dt == torch.float32 else 5e-2), f"d{name} {e}"


@pytest.mark.parametrize("dt,B,Ls", [(torch.float32, 20, 33), (torch.bfloat16, 20, 33),
                                    (torch.bfloat16, 128, 128), (torch.bfloat16, 256, 128)])
def test_bilstm_tower(dev, dt, B, Ls):
    """BiLSTM tower vs torch's CPU nn.LSTM (the oracle).  bf16 at B = 20 / 128 / 256 runs the
    cooperative forward variants RT = 1 / 2 / 4 (C4 = 128, C3 = 256 per GPU) and the
    recurrent backward at the benched geometry (L = 128)."""
    torch.manual_seed(0)
    torch.set_num_threads(16)
    ref = R.RefBiLSTM()
    enc = mmdx.text_encoders.BiLSTMEncoder()
    enc.load_state_dict(ref.state_dict())
    enc.compute_dtype = dt
    g = torch.Generator().manual_seed(2)
    ids = torch.randint(1000, 30522, (B, Ls), generator=g)
    h_ref = ref(ids).last_hidden_state
    dh = torch.randn(h_ref.shape, generator=g)
    h_ref.backward(dh)
    enc.to(dev)
    h = enc(ids.to(dev)).last_hidden_state
    h.backward(dh.to(dev, dt))
    torch.cuda.synchronize()
    tol = 1e-4 if dt == torch.float32 else 5e-2
    assert rel_err(h, h_ref) <= tol
    mmdx.bilstm.check_recurrence()
    gm = dict(enc.named_parameters())
    bad = []
    for n, p in ref.named_parameters():
        c = cosine(gm[n].grad, p.grad)
        r = abs(norm_ratio(gm[n].grad, p.grad) - 1.0)
        print(f"{n}: 1-cos {1 - c:.3e}  |norm ratio - 1| {r:.3e}")
        if 1 - c > (5e-5 if dt == torch.float32 else 2e-2) or r > (1e-4 if dt == torch.float32
                                                                     else 5e-2):
            bad.append((n, c, r))
    assert not bad, bad


def test_bert_layers_parity_fp32(dev):
    torch.manual_seed(0)
    ref = R.ref_bert(num_hidden_layers=2, dropout=0.0)
    mine = mmdx.text_encoders.BertModel.from_name("bert-base-uncased@2")
    mine.config.hidden_dropout_prob = 0.0
    mine.config.attention_probs_dropout_prob = 0.0
    missing = mine.load_state_dict(ref.state_dict(), strict=False)
    assert not missing.missing_keys and not missing.unexpected_keys, missing
    g = torch.Generator().manual_seed(3)
    B, Ls = 3, 40
    ids = torch.randint(1000, 30522, (B, Ls), generator=g)
    ids[:, 0] = 101
    lens = torch.tensor([40, 17, 9])
    mask = (torch.arange(Ls)[None] < lens[:, None]).long()
    ids[mask == 0] = 0
    ref.train()
    h_ref = ref(input_ids=ids, attention_mask=mask).last_hidden_state
    dh = torch.randn(h_ref.shape, generator=g) * mask[..., None]
    h_ref.backward(dh)
    mine.to(dev).train()
    h = mine(ids.to(dev), mask.to(dev)).last_hidden_state
    h.backward(dh.to(dev))
    torch.cuda.synchronize()
    valid = mask.bool()
    assert rel_err(h.cpu()[valid], h_ref[valid]) <= 1e-4
    gm = dict(mine.named_parameters())
    for n, p in ref.named_parameters():
        if p.grad is None:
            assert gm[n].grad is None or gm[n].grad.abs().max() == 0, n
            continue
        if n.endswith("attention.self.key.bias"):
            # softmax is shift-invariant per query row: dL/db_key == 0 analytically; both
            # sides hold rounding noise only — check it is noise-sized.
            qb = gm[n.replace("key.bias", "query.bias")].grad.abs().max()
            assert gm[n].grad.abs().max() <= 1e-3 * qb, n
            continue
        c = cosine(gm[n].grad, p.grad)
        assert 1 - c <= 1e-5, f"{n}: cos {c}"


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16, torch.float16])
def test_text_encoder_transformer_bert(dev, dt):
    torch.manual_seed(1)
    ref = R.RefTextEncoderTransformer("bert-base-uncased", bert_layers=2, dropout=0.0)
    mine = mmdx.TextEncoderTransformer("bert-base-uncased@2", compute_dtype=dt)
    mine.encoder.config.hidden_dropout_prob = 0.0
    mine.encoder.config.attention_probs_dropout_prob = 0.0
    mine.load_state_dict(ref.state_dict())
    tok = {"input_ids": torch.randint(1000, 30522, (2, 96)),
           "attention_mask": torch.ones(2, 96, dtype=torch.long),
           "token_type_ids": torch.zeros(2, 96, dtype=torch.long)}
    tok["attention_mask"][1, 50:] = 0
    ref.eval()
    with torch.no_grad():
        out_ref = ref(**tok)
    mine.to(dev).eval()
    with torch.no_grad():
        out = mine(**{k: v.to(dev) for k, v in tok.items()})
    # shape contracts of the reference (TP:898-899, TP:921)
    assert tuple(out["embeddings"].shape) == (2, 512)
    assert tuple(out["logits"].shape) == (2, 13)
    tol = 1e-4 if dt == torch.float32 else 5e-2
    assert rel_err(out["embeddings"], out_ref["embeddings"]) <= tol
    assert rel_err(out["logits"], out_ref["logits"]) <= tol


@pytest.mark.parametrize("B", [128, 200, 40])
def test_lstm_coop_forward_matches_partitioned(dev, B):
    """The cooperative bf16 recurrence (8 waves, W_hh in LDS; h exchanged through a counter
    barrier; B = 200 runs as two independent 128-row groups, the second ragged; B = 40 the
    64-row variant) reproduces the batch-partitioned kernel (same MFMA k order; fp32
    contraction order of the cell update may differ, so h may differ by one bf16 ulp): max
    abs difference <= 1e-2 on h (bf16, |h| < 1), c and gates."""
    H, Ls = 256, 24
    g = torch.Generator().manual_seed(B)
    xg = (torch.randn(B * Ls, 2 * 4 * H, generator=g) * 0.5).to(dev)
    whh = (torch.randn(2 * 4 * H, H, generator=g) * 0.05).to(dev, torch.bfloat16)
    outs = []
    for coop in (True, False):
        hout = torch.empty(B, Ls, 2 * H, dtype=torch.bfloat16, device=dev)
        cs = torch.empty(2, Ls, B, H, device=dev)
        gs = torch.empty(2, Ls, B, 4 * H, device=dev)
        n = L.lib().mmdx_lstm_fwd_workspace_size(L.dtype_code(torch.bfloat16), B, Ls, H) if coop else 0
        assert (n > 0) == coop
        ws = torch.empty(max(n, 16), dtype=torch.uint8, device=dev)
        status = torch.zeros(4, dtype=torch.int32, device=dev)
        L.call("mmdx_lstm_fwd", L.dtype_code(torch.bfloat16), xg.data_ptr(), whh.data_ptr(), B,
               Ls, H, hout.data_ptr(), cs.data_ptr(), gs.data_ptr(),
               ws.data_ptr() if coop else None, n, status.data_ptr(), 0, 0, L.stream())
        torch.cuda.synchronize()
        assert int(status[0]) == 0
        outs.append((hout.float(), cs, gs))
    for a, b in zip(outs[0], outs[1]):
        assert (a - b).abs().max().item() <= 1e-2 * max(1.0, b.abs().max().item())
        assert (a - b).abs().mean().item() <= 1e-4


@pytest.mark.parametrize("B", [128, 200, 40])
def test_lstm_coop_backward_matches_partitioned(dev, B):
    """The cooperative bf16 backward (4 workgroups per 16-row block and direction, W_hh^T in
    registers, dG slices exchanged through a counter) against the batch-partitioned kernel on
    the same saved forward: same bf16 dG operand, packed fragments and k order, so dG (dxg)
    and dW_hh agree to the last bit except where the compiler contracted a multiply-add
    differently; B = 200 and 40 leave a ragged last row block."""
    H, Ls = 256, 24
    bf = L.dtype_code(torch.bfloat16)
    g = torch.Generator().manual_seed(B + 1)
    xg = (torch.randn(B * Ls, 2 * 4 * H, generator=g) * 0.5).to(dev)
    whh = (torch.randn(2 * 4 * H, H, generator=g) * 0.05).to(dev, torch.bfloat16)
    dh = (torch.randn(B, Ls, 2 * H, generator=g) * 0.1).to(dev, torch.bfloat16)
    hout = torch.empty(B, Ls, 2 * H, dtype=torch.bfloat16, device=dev)
    cs = torch.empty(2, Ls, B, H, device=dev)
    gs = torch.empty(2, Ls, B, H, 4, device=dev)
    n = L.lib().mmdx_lstm_fwd_workspace_size(bf, B, Ls, H)
    ws = torch.empty(n, dtype=torch.uint8, device=dev)
    status = torch.zeros(4, dtype=torch.int32, device=dev)
    L.call("mmdx_lstm_fwd", bf, xg.data_ptr(), whh.data_ptr(), B, Ls, H, hout.data_ptr(),
           cs.data_ptr(), gs.data_ptr(), ws.data_ptr(), n, status.data_ptr(), 0, 0, L.stream())
    outs = []
    for coop in (True, False):
        dxg = torch.full((B * Ls, 2 * 4 * H), float("nan"), dtype=torch.bfloat16, device=dev)
        dwhh = torch.empty(2 * 4 * H, H, device=dev)
        nb = L.lib().mmdx_lstm_workspace_size(bf, B, Ls, H)
        wsb = torch.empty(nb, dtype=torch.uint8, device=dev)
        L.call("mmdx_lstm_bwd", bf, whh.data_ptr(), hout.data_ptr(), cs.data_ptr(),
               gs.data_ptr(), dh.data_ptr(), B, Ls, H, dxg.data_ptr(), dwhh.data_ptr(),
               wsb.data_ptr(), nb, status.data_ptr() if coop else None, 0, 0, L.stream())
        torch.cuda.synchronize()
        assert int(status[0]) == 0
        outs.append((dxg.float(), dwhh))
    (a_dg, a_dw), (b_dg, b_dw) = outs
    assert torch.isfinite(a_dg).all() and torch.isfinite(a_dw).all()
    # a contraction difference in one step's fp32 cell math can move a dG element by a bf16
    # ulp, and the recurrence carries it on (dc, dh_next): bound the difference by one ulp of
    # the tensor's scale and require most elements to agree exactly
    err = (a_dg - b_dg).abs()
    assert err.max().item() <= 2.0 ** -7 * b_dg.abs().max().item(), err.max().item()
    same = (a_dg == b_dg).float().mean().item()
    assert same >= 0.9, same
    assert (a_dw - b_dw).abs().max().item() <= 1e-2 * b_dw.abs().max().item()


def test_lstm_coop_backward_lost_peer_raises(dev):
    """The cooperative backward's bounded wait: with workgroup 0 of direction 0 never
    signalling (debug flag 1), every peer gives up, the launch completes (the grid drains),
    the sticky status word reads 2 and the host's poll raises RecurrenceError naming
    mmdx_lstm_bwd; a healthy launch afterwards (status reset) leaves it at 0."""
    from mmdx import bilstm as BL
    B, H, Ls = 128, 256, 16
    bf = L.dtype_code(torch.bfloat16)
    g = torch.Generator().manual_seed(3)
    xg = (torch.randn(B * Ls, 2 * 4 * H, generator=g) * 0.5).to(dev)
    whh = (torch.randn(2 * 4 * H, H, generator=g) * 0.05).to(dev, torch.bfloat16)
    dh = (torch.randn(B, Ls, 2 * H, generator=g) * 0.1).to(dev, torch.bfloat16)
    hout = torch.empty(B, Ls, 2 * H, dtype=torch.bfloat16, device=dev)
    cs = torch.empty(2, Ls, B, H, device=dev)
    gs = torch.empty(2, Ls, B, H, 4, device=dev)
    n = L.lib().mmdx_lstm_fwd_workspace_size(bf, B, Ls, H)
    ws = torch.empty(n, dtype=torch.uint8, device=dev)
    st = BL.coop_status(dev)
    st.reset()
    L.call("mmdx_lstm_fwd", bf, xg.data_ptr(), whh.data_ptr(), B, Ls, H, hout.data_ptr(),
           cs.data_ptr(), gs.data_ptr(), ws.data_ptr(), n, st.word.data_ptr(), 0, 0, L.stream())
    nb = L.lib().mmdx_lstm_workspace_size(bf, B, Ls, H)
    wsb = torch.empty(nb, dtype=torch.uint8, device=dev)
    dxg = torch.empty(B * Ls, 2 * 4 * H, dtype=torch.bfloat16, device=dev)
    dwhh = torch.empty(2 * 4 * H, H, device=dev)

    def bwd(flags, spin):
        L.call("mmdx_lstm_bwd", bf, whh.data_ptr(), hout.data_ptr(), cs.data_ptr(),
               gs.data_ptr(), dh.data_ptr(), B, Ls, H, dxg.data_ptr(), dwhh.data_ptr(),
               wsb.data_ptr(), nb, st.word.data_ptr(), spin, flags, L.stream())
        st.after_launch()
        torch.cuda.synchronize()
    try:
        bwd(1, 20000)
        assert int(st.word[0]) == 2
        with pytest.raises(BL.RecurrenceError, match="mmdx_lstm_bwd"):
            BL.check_recurrence()
    finally:
        torch.cuda.synchronize()
        st.reset()
    bwd(0, 0)
    BL.check_recurrence()
    assert int(st.word[0]) == 0
    assert torch.isfinite(dxg.float()).all()


def test_lstm_coop_lost_peer_raises(dev):
    """A peer workgroup that never signals (debug flag: workgroup 0 of direction 0 drops its
    signals) makes the cooperative recurrence time out: every workgroup leaves (the launch
    completes), the sticky status word reads 1 and the host raises RecurrenceError at its
    next poll instead of training on garbage.  A healthy launch afterwards (status reset)
    leaves the word at 0."""
    from mmdx import bilstm as BL
    torch.manual_seed(0)
    enc = mmdx.text_encoders.BiLSTMEncoder().to(dev)
    enc.compute_dtype = torch.bfloat16
    ids = torch.randint(1000, 30522, (128, 16), device=dev)
    st = BL.coop_status(dev)
    st.reset()
    BL.DEBUG.update(spin_limit=20000, flags=1)
    try:
        with torch.no_grad():
            enc(ids)
        torch.cuda.synchronize()
        with pytest.raises(BL.RecurrenceError):
            BL.check_recurrence()
        # the next forward refuses to run on top of a lost peer
        with pytest.raises(BL.RecurrenceError):
            with torch.no_grad():
                enc(ids)
    finally:
        BL.DEBUG.update(spin_limit=0, flags=0)
        torch.cuda.synchronize()
        st.reset()
    with torch.no_grad():
        enc(ids)
    torch.cuda.synchronize()
    BL.check_recurrence()
    assert int(st.word[0]) == 0


@pytest.mark.parametrize("dt,Ls", [(torch.float32, 128), (torch.bfloat16, 128),
                                   (torch.float16, 97)])
def test_attention_prob_dropout(dev, dt, Ls):
    """Attention-probability dropout (BertSelfAttention's, train mode).  The kept set is read
    back from the saved probabilities' sign bit; forward and backward must equal an explicit
    reference that applies exactly that mask: O = (P*keep/(1-p)) V, autograd for the
    gradients.  The drop rate must be p (binomial 6-sigma band) and a second launch (device
    counter advanced) must draw a different mask."""
    B, H, pd = 2, 4, 0.1
    g = torch.Generator().manual_seed(7)
    qkv = torch.randn(B, Ls, 3, H, 64, generator=g)
    if dt != torch.float32:
        qkv = qkv.to(dt).float()
    lens = torch.tensor([Ls, 70])
    mask = (torch.arange(Ls)[None] < lens[:, None]).long()
    scale = 0.125
    dc = L.dtype_code(dt)
    qd = qkv.to(dev, dt).contiguous()
    md = mask.to(dev)
    ctr = torch.zeros(1, dtype=torch.int64, device=dev)
    out = torch.empty(B, Ls, H, 64, dtype=dt, device=dev)
    probs = torch.empty(B, H, Ls, Ls, device=dev)
    L.call("mmdx_attention_fwd", dc, qd.data_ptr(), md.data_ptr(), B, Ls, H, scale, pd, 1234,
           ctr.data_ptr(), out.data_ptr(), probs.data_ptr(), L.stream())
    torch.cuda.synchronize()
    assert int(ctr.item()) == 1
    pr = probs.cpu()
    keep = ~torch.signbit(pr)
    valid = (mask[:, None, None, :].expand(B, H, Ls, Ls) > 0)
    n = valid.sum().item()
    frac = 1.0 - (keep & valid).sum().item() / n
    assert abs(frac - pd) <= 6 * (pd * (1 - pd) / n) ** 0.5, frac
    # the reference with this exact mask
    qr = qkv.clone().requires_grad_(True)
    q, k, v = qr[:, :, 0], qr[:, :, 1], qr[:, :, 2]
    s = torch.einsum("blhd,bmhd->bhlm", q, k) * scale
    s = s + (1.0 - mask[:, None, None, :].float()) * -1e30
    p = s.softmax(-1)
    assert rel_err(pr.abs(), p.detach()) <= (1e-5 if dt == torch.float32 else 3e-2)
    pdrop = p * keep.float() / (1 - pd)
    o = torch.einsum("bhlm,bmhd->blhd", pdrop, v)
    do = torch.randn(o.shape, generator=g)
    if dt != torch.float32:
        do = do.to(dt).float()
    o.backward(do)
    tol = 1e-4 if dt == torch.float32 else 3e-2
    assert rel_err(out, o) <= tol
    dqkv = torch.empty_like(qd)
    nws = L.lib().mmdx_attention_workspace_size(dc, B, Ls, H)
    ws = torch.empty(nws, dtype=torch.uint8, device=dev)
    L.call("mmdx_attention_bwd", dc, qd.data_ptr(), probs.data_ptr(),
           do.to(dev, dt).contiguous().data_ptr(), md.data_ptr(), B, Ls, H, scale, pd,
           dqkv.data_ptr(), ws.data_ptr(), nws, L.stream())
    torch.cuda.synchronize()
    for i, name in enumerate("qkv"):
        e = rel_err(dqkv[:, :, i], qr.grad[:, :, i])
        assert e <= (2e-4 if dt == torch.float32 else 5e-2), f"d{name} {e}"
    # next launch: fresh mask
    probs2 = torch.empty_like(probs)
    L.call("mmdx_attention_fwd", dc, qd.data_ptr(), md.data_ptr(), B, Ls, H, scale, pd, 1234,
           ctr.data_ptr(), out.data_ptr(), probs2.data_ptr(), L.stream())
    torch.cuda.synchronize()
    keep2 = ~torch.signbit(probs2.cpu())
    assert (keep2 != keep)[valid].float().mean().item() > 0.1


def test_bert_train_mode_with_default_dropout(dev):
    """The reference's text phase 2 (TP:926-939) trains BERT with the default config
    (hidden and attention dropout 0.1): forward + backward run, outputs and gradients are
    finite, and train-mode outputs differ from eval-mode ones (dropout active)."""
    torch.manual_seed(0)
    mine = mmdx.TextEncoderTransformer("bert-base-uncased@2", compute_dtype=torch.bfloat16)
    assert mine.encoder.config.attention_probs_dropout_prob == 0.1
    mine.to(dev).unfreeze_encoder()
    ids = torch.randint(1000, 30522, (4, 64), device=dev)
    mask = torch.ones(4, 64, dtype=torch.long, device=dev)
    out = mine(input_ids=ids, attention_mask=mask)
    out["logits"].float().sum().backward()
    torch.cuda.synchronize()
    for n, p in mine.named_parameters():
        if ".pooler." in n:      # unused by the mean-pooled tower (as in the reference)
            continue
        assert p.grad is not None and torch.isfinite(p.grad).all(), n
    mine.eval()
    with torch.no_grad():
        ev = mine(input_ids=ids, attention_mask=mask)["embeddings"]
    assert not torch.allclose(ev.float(), out["embeddings"].detach().float())

