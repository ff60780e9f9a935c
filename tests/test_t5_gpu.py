"""T5 report head on the mmdx kernels vs transformers' T5 on CPU.

The oracle is the reference's own dependency (transformers T5ForConditionalGeneration,
training_pipeline.py:545; installed 5.15.0, reference pin 4.56.1) built from a local
T5Config (t5-small geometry, 2 decoder layers for test time), fp32, dropout 0, the same
weights on both sides.  Tolerances (fp32): kernels rel <= 2e-5 (1e-4 for the 32128-way
softmax paths); teacher-forced loss rel <= 1e-5, logits max-abs <= 1e-4 * max(1, |ref|),
every parameter gradient and the condition-token gradient 1 - cos <= 1e-5 with the norm
ratio within 1e-4; beam search: the device step along the reference's search (see the test).
"""
import pytest
import torch
import torch.nn.functional as tF

import mmdx
from mmdx import _lib as L
from parity_util import cosine, norm_ratio, rel_err

pytestmark = pytest.mark.gpu


def _t5(layers=2, seed=0, dropout=0.0):
    from transformers import T5Config, T5ForConditionalGeneration
    torch.manual_seed(seed)
    cfg = T5Config(d_model=512, d_ff=2048, d_kv=64, num_layers=layers, num_decoder_layers=layers,
                   num_heads=8, vocab_size=32128, relative_attention_num_buckets=32,
                   relative_attention_max_distance=128, dropout_rate=dropout,
                   layer_norm_epsilon=1e-6, feed_forward_proj="relu", decoder_start_token_id=0,
                   eos_token_id=1, pad_token_id=0, tie_word_embeddings=True)
    cfg._attn_implementation = "eager"
    return T5ForConditionalGeneration(cfg)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_rmsnorm(dev, dt):
    g = torch.Generator().manual_seed(3)
    x = torch.randn(37, 512, generator=g)
    w = torch.rand(512, generator=g) + 0.5
    dy = torch.randn(37, 512, generator=g)
    if dt == torch.bfloat16:
        x, dy = x.bfloat16().float(), dy.bfloat16().float()
    xr = x.clone().requires_grad_(True)
    wr = w.clone().requires_grad_(True)
    y = wr * (xr * torch.rsqrt(xr.pow(2).mean(-1, keepdim=True) + 1e-6))
    y.backward(dy)
    from mmdx.t5 import _rms, _rms_bwd
    xd = x.to(dev, dt)
    yd, r = _rms(xd, w.to(dev), 1e-6)
    acc = torch.full_like(xd, 0.5)
    dw = _rms_bwd(xd, dy.to(dev, dt), w.to(dev), r, acc)
    torch.cuda.synchronize()
    tol = 2e-5 if dt == torch.float32 else 2e-2
    assert rel_err(yd, y) <= tol
    assert rel_err(acc.float().cpu() - 0.5, xr.grad) <= (tol if dt == torch.float32 else 3e-2)
    assert rel_err(dw, wr.grad) <= tol


@pytest.mark.parametrize("p_drop", [0.0, 0.1])
def test_cross_attention_small_k(dev, p_drop):
    """Cross-attention over K = 4 condition tokens (T5 EncDecAttention core, no scaling):
    forward/backward vs an explicit reference with the kernel's own dropout mask."""
    B, Lq, Lk, H = 3, 21, 4, 8
    g = torch.Generator().manual_seed(5)
    q = torch.randn(B, Lq, H, 64, generator=g)
    kv = torch.randn(B, Lk, 2, H, 64, generator=g)
    dout = torch.randn(B, Lq, H, 64, generator=g)
    qd, kvd = q.to(dev).contiguous(), kv.to(dev).contiguous()
    out = torch.empty(B, Lq, H, 64, device=dev)
    probs = torch.empty(B, H, Lq, Lk, device=dev)
    ctr = torch.zeros(1, dtype=torch.int64, device=dev)
    L.call("mmdx_xattn_fwd", L.F32, qd.data_ptr(), H * 64, kvd.data_ptr(), B, Lq, Lk, H, 1.0,
           p_drop, 99, ctr.data_ptr(), out.data_ptr(), probs.data_ptr(), L.stream())
    torch.cuda.synchronize()
    keep = (~torch.signbit(probs.cpu())).float()
    qr = q.clone().requires_grad_(True)
    kr = kv.clone().requires_grad_(True)
    s = torch.einsum("blhd,bkhd->bhlk", qr, kr[:, :, 0])
    p = s.softmax(-1)
    assert rel_err(probs.abs(), p.detach()) <= 1e-5
    o = torch.einsum("bhlk,bkhd->blhd", p * keep / (1 - p_drop), kr[:, :, 1])
    o.backward(dout)
    assert rel_err(out, o) <= 2e-5
    dq = torch.empty_like(qd)
    dkv = torch.empty_like(kvd)
    n = L.lib().mmdx_xattn_workspace_size(B, Lq, Lk, H)
    ws = torch.empty(n, dtype=torch.uint8, device=dev)
    L.call("mmdx_xattn_bwd", L.F32, qd.data_ptr(), H * 64, kvd.data_ptr(), probs.data_ptr(),
           dout.to(dev).contiguous().data_ptr(), B, Lq, Lk, H, 1.0, p_drop, dq.data_ptr(),
           H * 64, dkv.data_ptr(), ws.data_ptr(), n, L.stream())
    torch.cuda.synchronize()
    assert rel_err(dq, qr.grad) <= 2e-5
    assert rel_err(dkv, kr.grad) <= 2e-5
    if p_drop > 0:
        frac = 1 - keep.mean().item()
        assert 0.05 < frac < 0.15


def test_cross_entropy_ignore_index(dev):
    g = torch.Generator().manual_seed(8)
    R, V = 50, 32128
    logits = torch.randn(R, V, generator=g) * 3
    tgt = torch.randint(0, V, (R,), generator=g)
    tgt[::7] = -100
    lr = logits.clone().requires_grad_(True)
    loss_ref = tF.cross_entropy(lr, tgt, ignore_index=-100)
    (loss_ref * 2.5).backward()
    ld, td = logits.to(dev), tgt.to(dev)
    loss = torch.empty((), device=dev)
    cnt = torch.empty((), device=dev)
    n = L.lib().mmdx_cross_entropy_workspace_size(R)
    ws = torch.empty(n, dtype=torch.uint8, device=dev)
    L.call("mmdx_cross_entropy_fwd", ld.data_ptr(), td.data_ptr(), R, V, loss.data_ptr(),
           cnt.data_ptr(), ws.data_ptr(), n, L.stream())
    gs = torch.tensor(2.5, device=dev)
    dl = torch.empty(R, V, device=dev)
    L.call("mmdx_cross_entropy_bwd", L.F32, ld.data_ptr(), td.data_ptr(), R, V, gs.data_ptr(),
           cnt.data_ptr(), ws.data_ptr(), dl.data_ptr(), L.stream())
    torch.cuda.synchronize()
    assert int(cnt.item()) == int((tgt != -100).sum())
    assert abs(loss.item() - loss_ref.item()) <= 1e-5 * abs(loss_ref.item())
    assert rel_err(dl, lr.grad) <= 1e-4


def test_position_bias_matches_transformers(dev):
    ref = _t5(1)
    att = ref.decoder.block[0].layer[0].SelfAttention
    Ls = 300   # crosses max_distance (128): every bucket in use
    want = att.compute_bias(Ls, Ls)[0]     # [H, L, L]
    table = att.relative_attention_bias.weight.detach().to(dev)
    got = torch.empty(8, Ls, Ls, device=dev)
    L.call("mmdx_t5_position_bias", table.data_ptr(), 8, Ls, 32, 128, got.data_ptr(), L.stream())
    torch.cuda.synchronize()
    # the causal mask hides k > q; compare the visible cells exactly
    vis = torch.tril(torch.ones(Ls, Ls, dtype=torch.bool))
    assert torch.equal(got.cpu()[:, vis], want.detach()[:, vis])


def _head_case(dev, layers=2, B=3, Lr=20, seed=0):
    ref = _t5(layers, seed)
    mine = _t5(layers, seed)
    mine.load_state_dict(ref.state_dict())
    mine.to(dev).train()
    ref.train()
    g = torch.Generator().manual_seed(seed + 10)
    enc = torch.randn(B, 4, 512, generator=g)
    labels = torch.randint(2, 32128, (B, Lr), generator=g)
    labels[1, 12:] = -100
    labels[2, 5:] = -100
    return ref, mine, enc, labels


def test_t5_teacher_forced_parity(dev):
    """report_model(encoder_outputs=cond, labels=labels) (TP:597-604): loss, logits and every
    gradient (decoder, tied embedding/lm_head, relative-position table, condition tokens)."""
    from transformers.modeling_outputs import BaseModelOutput
    from mmdx.t5 import T5Head
    ref, mine, enc, labels = _head_case(dev)
    er = enc.clone().requires_grad_(True)
    out = ref(encoder_outputs=BaseModelOutput(last_hidden_state=er), labels=labels,
              return_dict=True)
    out.loss.backward()
    ed = enc.to(dev).requires_grad_(True)
    loss, logits = T5Head(mine).forward(ed, labels=labels.to(dev))
    loss.backward()
    torch.cuda.synchronize()
    assert abs(loss.item() - out.loss.item()) <= 1e-5 * abs(out.loss.item())
    assert (logits.cpu() - out.logits.detach()).abs().max() <= 1e-4 * max(
        1.0, out.logits.abs().max().item())
    gm = dict(mine.named_parameters())
    checked = 0
    for n, p in ref.named_parameters():
        if p.grad is None:      # the encoder is bypassed (encoder_outputs given)
            assert gm[n].grad is None, n
            continue
        c, r = 1 - cosine(gm[n].grad, p.grad), abs(norm_ratio(gm[n].grad, p.grad) - 1)
        assert c <= 1e-5 and r <= 1e-4, (n, c, r)
        checked += 1
    assert checked >= 2 * 13 + 2
    c, r = 1 - cosine(ed.grad, er.grad), abs(norm_ratio(ed.grad, er.grad) - 1)
    assert c <= 1e-5 and r <= 1e-4, (c, r)


@pytest.mark.parametrize("eos_x", [1.0, 16.0])
def test_t5_beam_generate_matches_transformers(dev, eos_x):
    """report_model.generate(encoder_outputs=cond, num_beams=4, no_repeat_ngram_size=3,
    min_new_tokens, max_new_tokens, length_penalty=1.1, early_stopping=True) (IP:190-196).
    (1) The device step (KV-cached decoder, device logits processors, top-k) is checked at
    every step of the reference's own search (parity_util.BeamStepCheck: top-8 candidate
    scores to 2e-5 of max(1, |score|), candidate ids wherever the score is separated from its
    neighbours by more than twice that); the host loop driven by the reference step returns
    transformers' ids exactly (its CPU test: test_beam_host_cpu.py).  (2) End to end, mmdx
    generate() returns transformers' ids exactly when no candidate of that search was within
    the tolerance of a neighbour (a near-tie may legitimately break either way in fp32).
    eos_x scales the EOS embedding row (tied head) so hypotheses finish mid-search."""
    from transformers.modeling_outputs import BaseModelOutput
    from mmdx.t5 import T5Head, _DecodeState
    from parity_util import BeamStepCheck, hf_beam_stepper
    ref = _t5(2, seed=4).eval()
    with torch.no_grad():
        ref.shared.weight[1].mul_(eos_x)
    mine = _t5(2, seed=4)
    mine.load_state_dict(ref.state_dict())
    mine.to(dev).eval()
    g = torch.Generator().manual_seed(21)
    enc = torch.randn(2, 4, 512, generator=g)
    nb, max_new = 4, 14
    kw = dict(num_beams=nb, max_new_tokens=max_new, min_new_tokens=3, no_repeat_ngram_size=3,
              length_penalty=1.1, early_stopping=True, eos_token_id=1, pad_token_id=0)
    with torch.no_grad():
        want = ref.generate(encoder_outputs=BaseModelOutput(last_hidden_state=enc), **kw)
    head = T5Head(mine)
    encd = enc.to(dev)
    dec = _DecodeState(head, encd.repeat_interleave(nb, dim=0), torch.float32, 1 + max_new)
    chk = BeamStepCheck(hf_beam_stepper(ref, enc, nb, 2 * nb), dec, 2, nb, 2 * nb, tol=2e-5)
    replay = head.generate(encd, _stepper=chk, **kw)
    print(f"steps {chk.steps}, max err {chk.max_err:.2e}, min gap {chk.min_gap:.2e}, "
          f"near-ties {chk.ambiguous}")
    assert chk.steps >= 4 and torch.equal(replay, want)
    if eos_x != 1.0:
        assert (want[:, 1:] == 1).any()
    got = head.generate(encd, **kw)
    if chk.ambiguous == 0:
        assert torch.equal(got.cpu(), want), (got, want)


def test_fusion_report_head_plumbing(dev):
    """FusionTransformerModel with its T5 head (TP:595-604): forward with report_labels
    returns gen.loss; the total loss (BCE + gen, TP:1049-1053) back-propagates into
    cond_proj, the fusion MLP and the T5 decoder; generate returns token ids."""
    torch.manual_seed(0)
    fus = mmdx.FusionTransformerModel(1024, 512, 1024, 13, dropout=0.0,
                                      init_t5_from_config=True).to(dev).train()
    z_img = torch.randn(2, 1024, device=dev)
    z_txt = torch.randn(2, 512, device=dev)
    labels = torch.randint(2, 32128, (2, 16), device=dev)
    labels[1, 9:] = -100
    out = fus(z_img, z_txt, report_labels=labels)
    assert out["gen"] is not None and out["gen"].logits.shape == (2, 16, 32128)
    y = (torch.rand(2, 13, device=dev) < 0.3).float()
    loss = mmdx.BCEWithLogitsLoss()(out["disease_logits"], y) + 1.0 * out["gen"].loss
    loss.backward()
    torch.cuda.synchronize()
    for n in ("cond_proj.0.weight", "fusion_mlp.0.weight",
              "report_model.decoder.block.0.layer.0.SelfAttention.q.weight",
              "report_model.shared.weight"):
        p = dict(fus.named_parameters())[n]
        assert p.grad is not None and torch.isfinite(p.grad).all() and p.grad.abs().max() > 0, n
    fus.eval()
    ids = fus.generate(z_img, z_txt, num_beams=2, max_new_tokens=5, min_new_tokens=2,
                       no_repeat_ngram_size=3, eos_token_id=1, pad_token_id=0)
    assert ids.shape[0] == 2 and ids[:, 0].eq(0).all() and ids.shape[1] <= 6


def test_incremental_decoder_matches_full_recompute(dev):
    """The KV-cached decoder step (t5._DecodeState: appended self-attention K/V, slot-table
    beam reordering, device logits processors + top-k) against re-running the decoder over
    the whole prefix (T5Head._last_log_probs) at every position, with a beam reorder
    (rows permuted mid-sequence), n-gram bans and the EOS ban: the top-k scores agree to
    1e-4 and the indices are equal."""
    import numpy as np
    from mmdx.t5 import T5Head, _DecodeState, _ngram_bans
    torch.manual_seed(0)
    m = _t5(2, seed=7)
    m.to(dev).eval()
    head = T5Head(m)
    B, nb, L, k = 2, 2, 12, 4
    R = B * nb
    enc = torch.randn(B, 4, 512, device=dev)
    enc_r = enc.repeat_interleave(nb, dim=0)
    g = np.random.default_rng(3)
    seq = g.integers(2, 200, size=(R, L)).astype(np.int64)
    seq[:, 0] = 0
    seq[:, 6:9] = seq[:, 2:5]          # repeated n-grams so the ban fires
    dec = _DecodeState(head, enc_r, torch.float32, L)
    slots = np.zeros((R, L), dtype=np.int32)
    rows = np.arange(R, dtype=np.int32)
    V = m.config.vocab_size
    run_sc = g.standard_normal(R).astype(np.float32)
    for pos in range(L):
        if pos == 5:  # beam reorder: new row r continues old row perm[r]
            perm = np.array([1, 1, 3, 2])
            slots, seq = slots[perm], seq[perm]
        slots[:, pos] = rows
        bans = _ngram_bans(seq[:, :pos + 1], 3)
        eos_ban = 1 if pos < 4 else -1
        val, idx = dec.step(seq[:, pos], pos, slots, run_sc, bans, eos_ban, B, nb, k)
        with torch.no_grad():
            lp = head._last_log_probs(torch.from_numpy(seq[:, :pos + 1]).to(dev), enc_r,
                                      torch.float32).cpu().numpy()
        if eos_ban >= 0:
            lp[:, eos_ban] = -np.inf
        for r, t in bans:
            lp[r, t] = -np.inf
        acc = (lp + run_sc[:, None]).reshape(B, nb * V)
        ref_idx = np.argsort(-acc, axis=1, kind="stable")[:, :k]
        ref_val = np.take_along_axis(acc, ref_idx, axis=1)
        assert np.array_equal(idx, ref_idx), (pos, idx, ref_idx)
        assert np.abs(val - ref_val).max() <= 1e-4, pos
