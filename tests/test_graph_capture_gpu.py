"""hipGraph capture of mmdx launch sequences == eager execution, bit for bit.

include/mmdx.h promises that every entry point is stream-ordered and graph-capturable (no
allocation, no synchronisation, no host readback on the launch path).  These tests capture
real launch sequences with torch.cuda.graph / make_graphed_callables and replay them:
  * a dense GEMM and the 16-bit attention forward + backward (whose LDS attribute is now set
    once per kernel, outside any capture);
  * the cooperative BiLSTM recurrence alone, on an idle device and beside a ResNet-50 trunk
    forward at the C4 batch on another stream (its workgroups spin on each other: a graph
    replay that could not make them co-resident would time out and set the status word);
  * whole text towers (BiLSTM for C3/C4, BERT-base@2 for C5) forward + backward through
    make_graphed_callables, parameters' gradients included.
Outputs and gradients must equal the eager run's bit for bit (the embedding-table gradient,
a scatter-add of repeated token rows, to 1e-6: its atomic add order is free).
"""
import pytest
import torch

import mmdx
from mmdx import _lib as L
from mmdx import bilstm as BL
from parity_util import synth_batch

pytestmark = pytest.mark.gpu


def _capture(fn, warm=2):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(warm):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        out = fn()
    torch.cuda.synchronize()
    return g, out


def test_capture_gemm(dev):
    from mmdx import functional as F
    g = torch.Generator().manual_seed(0)
    A = torch.randn(1000, 768, generator=g).to(dev, torch.bfloat16)
    B = torch.randn(3072, 768, generator=g).to(dev, torch.bfloat16)
    C = torch.empty(1000, 3072, device=dev)

    def run():
        F.gemm(A, 768, 1, B, 768, 1, 1000, 3072, 768, C, 3072, compute_dtype=torch.bfloat16)
        return C

    want = run().clone()
    C.zero_()
    gr, _ = _capture(run)
    C.zero_()
    gr.replay()
    torch.cuda.synchronize()
    assert torch.equal(C, want)


@pytest.mark.parametrize("dt", [torch.float16, torch.bfloat16])
def test_capture_attention(dev, dt):
    B, Ls, H = 8, 197, 12
    g = torch.Generator().manual_seed(1)
    qkv = torch.randn(B, Ls, 3, H, 64, generator=g).to(dev, dt)
    dout = torch.randn(B, Ls, H, 64, generator=g).to(dev, dt)
    out = torch.empty(B, Ls, H, 64, dtype=dt, device=dev)
    probs = torch.empty(B, H, Ls, Ls, device=dev)
    dqkv = torch.empty_like(qkv)
    n = L.lib().mmdx_attention_workspace_size(L.dtype_code(dt), B, Ls, H)
    ws = torch.empty(n, dtype=torch.uint8, device=dev)

    def run():
        L.call("mmdx_attention_fwd", L.dtype_code(dt), qkv.data_ptr(), None, B, Ls, H, 0.125,
               0.0, 0, None, out.data_ptr(), probs.data_ptr(), L.stream())
        L.call("mmdx_attention_bwd", L.dtype_code(dt), qkv.data_ptr(), probs.data_ptr(),
               dout.data_ptr(), None, B, Ls, H, 0.125, 0.0, dqkv.data_ptr(), ws.data_ptr(), n,
               L.stream())
        return out

    run()
    torch.cuda.synchronize()
    want = (out.clone(), dqkv.clone())
    gr, _ = _capture(run)
    out.zero_()
    dqkv.zero_()
    gr.replay()
    torch.cuda.synchronize()
    assert torch.equal(out, want[0]) and torch.equal(dqkv, want[1])


def _lstm_fwd_call(x_g, whh, B, Ls, H, hout, cs, gs, fws, fw, st):
    L.call("mmdx_lstm_fwd", L.BF16, x_g.data_ptr(), whh.data_ptr(), B, Ls, H, hout.data_ptr(),
           cs.data_ptr(), gs.data_ptr(), fws.data_ptr(), fw, st.word.data_ptr(), 0, 0,
           L.stream())


def test_capture_lstm_recurrence_beside_trunk(dev):
    """The cooperative recurrence (C4 shape: B 128, L 128, H 256) replayed from a graph on a
    high-priority stream while the main stream runs the ResNet-50 trunk forward at B 128."""
    B, Ls, H = 128, 128, 256
    g = torch.Generator().manual_seed(2)
    xg = (torch.randn(B * Ls, 8 * H, generator=g) * 0.5).to(dev)
    whh = (torch.randn(8 * H, H, generator=g) * 0.05).to(dev, torch.bfloat16)
    hout = torch.empty(B, Ls, 2 * H, dtype=torch.bfloat16, device=dev)
    cs = torch.empty(2, Ls, B, H, device=dev)
    gs = torch.empty(2, Ls, B, 4 * H, device=dev)
    fw = L.lib().mmdx_lstm_fwd_workspace_size(L.BF16, B, Ls, H)
    assert fw > 0, "expected the cooperative path"
    fws = torch.empty(fw, dtype=torch.uint8, device=dev)
    st = BL.coop_status(dev)
    st.reset()

    def run():
        _lstm_fwd_call(xg, whh, B, Ls, H, hout, cs, gs, fws, fw, st)
        return hout

    run()
    torch.cuda.synchronize()
    want = (hout.clone(), cs.clone(), gs.clone())
    assert int(st.word[0].item()) == 0
    img = mmdx.ImageEncoderCNN("resnet50", 1024, 13, compute_dtype=torch.bfloat16).to(dev)
    img.unfreeze_backbone()
    x, _, _, _ = synth_batch(B, 8, hw=224)
    x = x.to(dev)
    side = torch.cuda.Stream(device=dev, priority=-1)

    def beside_trunk(launch, what):
        with torch.no_grad():
            for k in range(3):
                hout.zero_()
                cs.zero_()
                gs.zero_()
                side.wait_stream(torch.cuda.current_stream())
                img(x)                      # the trunk on the main stream
                with torch.cuda.stream(side):
                    launch()                # the recurrence beside it
                torch.cuda.current_stream().wait_stream(side)
                torch.cuda.synchronize()
                assert int(st.word[0].item()) == 0, f"{what} {k}: recurrence timed out"
                for name, a, b in (("h", hout, want[0]), ("c", cs, want[1]), ("gates", gs, want[2])):
                    assert torch.equal(a, b), (what, k, name, (a.float() - b.float()).abs().max().item())

    beside_trunk(run, "eager")              # eager launches are deterministic
    gr, _ = _capture(run)
    beside_trunk(gr.replay, "graph replay")


class _Tower(torch.nn.Module):
    def __init__(self, txt):
        super().__init__()
        self.txt = txt

    def forward(self, ids, mask):
        return self.txt(input_ids=ids, attention_mask=mask)["embeddings"]


@pytest.mark.parametrize("name,dt", [("bilstm", torch.bfloat16),
                                     ("bert-base-uncased@2", torch.float16)])
def test_capture_text_tower_fwd_bwd(dev, name, dt):
    torch.manual_seed(0)
    # (no warm-up classifier: every captured parameter must reach the output)
    txt = mmdx.TextEncoderTransformer(name, 512, 13, use_warmup_classifier=False,
                                      compute_dtype=dt)
    if hasattr(txt.encoder, "config") and hasattr(txt.encoder.config, "hidden_dropout_prob"):
        txt.encoder.config.hidden_dropout_prob = 0.0
        txt.encoder.config.attention_probs_dropout_prob = 0.0
    txt.to(dev).unfreeze_encoder()
    for n, p in txt.named_parameters():   # BERT's pooler does not reach the mean-pooled output
        if "pooler" in n:
            p.requires_grad_(False)
    tower = _Tower(txt)
    _, ids, mask, _ = synth_batch(32, 128)
    ids, mask = ids.to(dev), mask.to(dev)
    gout = torch.randn(32, 512, generator=torch.Generator().manual_seed(3)).to(dev)
    out = tower(ids, mask)
    out.backward(gout)
    torch.cuda.synchronize()
    want = out.detach().clone()
    wgrads = {n: p.grad.clone() for n, p in tower.named_parameters() if p.grad is not None}
    tower.zero_grad(set_to_none=True)
    # the eager graph must be gone before capture: a live `out` keeps its AccumulateGrad
    # nodes bound to the eager stream, and the captured backward would then synchronise with
    # that stream (torch warns; hipStreamEndCapture crashed on it)
    del out
    gt = torch.cuda.make_graphed_callables(tower, (ids, mask))
    tower.zero_grad(set_to_none=True)
    out = gt(ids, mask)
    out.backward(gout)
    torch.cuda.synchronize()
    assert torch.equal(out.detach(), want)
    got = {n: p.grad for n, p in tower.named_parameters() if p.grad is not None}
    assert set(got) == set(wgrads)
    for n, w in wgrads.items():
        if "embed" in n or "word_embeddings" in n:
            torch.testing.assert_close(got[n], w, rtol=1e-6, atol=1e-9, msg=n)
        else:
            assert torch.equal(got[n], w), n
    if name == "bilstm":
        BL.check_recurrence()
        assert int(BL.coop_status(dev).word[0].item()) == 0
