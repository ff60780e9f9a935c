"""Build-defined C3/C4 report encoder: Embedding(30522, 256) -> 2-layer BiLSTM(256/dir).

Parameters live in a real `nn.LSTM` (names weight_ih_l0, weight_hh_l0_reverse, ...), so the
state_dict is interchangeable with a PyTorch BiLSTM; execution is:
  xg   = x [W_ih_f; W_ih_r]^T + (b_ih + b_hh)   one MFMA GEMM over all B*L tokens (fp32 out)
  h    = recurrence(xg, W_hh)                    mmdx_lstm_fwd, batch-partitioned, no grid sync
backward: mmdx_lstm_bwd (dG + dW_hh), then dW_ih / dX / bias grads as GEMMs + column sums.
"""
from __future__ import annotations

from types import SimpleNamespace

import os

import torch
import torch.nn as nn

from . import _lib as L
from . import functional as F
from ._lib import call, ptr, stream
from .layers import Embedding

VOCAB = 30522


class _Out(SimpleNamespace):
    pass


class RecurrenceError(RuntimeError):
    """The cooperative LSTM recurrence lost a peer workgroup: its outputs are invalid."""


class _CoopStatus:
    """Sticky device status word of the cooperative recurrences (mmdx_lstm_fwd sets 1,
    mmdx_lstm_bwd 2).

    After every cooperative launch the word is copied (async, same stream) into pinned host
    memory behind an event.  `poll()` raises RecurrenceError once a completed copy shows a
    timeout; it never blocks unless asked, so the step keeps its asynchrony and the error
    surfaces at the next forward (or at `check_recurrence()` — the bench calls it after the
    timed region, the training loop at its loss sync)."""

    def __init__(self, dev):
        self.word = torch.zeros(4, dtype=torch.int32, device=dev)
        self.host = torch.zeros(4, dtype=torch.int32, pin_memory=True)
        self.ev = None

    def after_launch(self):
        if torch.cuda.is_current_stream_capturing():
            return
        self.host.copy_(self.word, non_blocking=True)
        self.ev = torch.cuda.Event()
        self.ev.record()

    def poll(self, block=False):
        if block:
            # read the device word itself: a graph-replayed launch (hipGraph capture skips
            # the per-launch copy) sets it too
            code = int(self.word[0].item())
            if code != 0:
                self._raise(code)
            return
        ev = self.ev
        if ev is None or not ev.query():
            return
        code = int(self.host[0])
        if code != 0:
            self._raise(code)

    @staticmethod
    def _raise(code):
        which = "mmdx_lstm_bwd" if code == 2 else "mmdx_lstm_fwd"
        raise RecurrenceError(
                f"mmdx BiLSTM: the cooperative recurrence timed out waiting for a peer "
                f"workgroup ({which} status={code}); the text tower's outputs and gradients "
                f"of this step are invalid")

    def reset(self):
        self.word.zero_()
        self.host.zero_()
        self.ev = None


_STATUS: dict = {}


def coop_status(dev) -> _CoopStatus:
    key = (dev.type, dev.index if dev.index is not None else torch.cuda.current_device())
    st = _STATUS.get(key)
    if st is None:
        st = _STATUS[key] = _CoopStatus(dev)
    return st


def check_recurrence(block=True):
    """Raise RecurrenceError if any cooperative LSTM launch so far lost a peer."""
    for st in list(_STATUS.values()):
        st.poll(block=block)


# debug knobs of the cooperative forward (tests force the timeout path through these)
DEBUG = {"spin_limit": 0, "flags": 0}

# the cooperative recurrent backward (mmdx_lstm_bwd with a status word) is opt-in
# (MMDX_LSTM_BWD_COOP=1): 0.70 vs 1.0 ms per launch in the C4 step, but it holds 64 CUs
# where the batch-partitioned kernel holds 16, and beside the throughput-bound image
# backward CU-time is what counts: C4 8738 vs 8830 samples/s (r05, paired).  Same outputs as
# the partitioned kernel to one bf16 ulp of scale (fp32 contraction differences in the cell
# math propagate through the recurrence; tests/test_text_gpu.py).
BWD_COOP = os.environ.get("MMDX_LSTM_BWD_COOP", "0") == "1"


def _cat_cast(ws, T, dev):
    rows = sum(w.shape[0] for w in ws)
    out = torch.empty((rows,) + tuple(ws[0].shape[1:]), dtype=T, device=dev)
    o = 0
    for w in ws:
        n = w.shape[0]
        call("mmdx_cast", L.dtype_code(T), L.F32, ptr(w), w.numel(), ptr(out[o:o + n]), stream())
        o += n
    return out


class _LSTMLayerFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, H, wih_f, whh_f, bih_f, bhh_f, wih_r, whh_r, bih_r, bhh_r):
        B, Ls, In = x.shape
        T = x.dtype
        dev = x.device
        M = B * Ls
        G4 = 4 * H
        wih = _cat_cast([wih_f, wih_r], T, dev)                 # [8H, In]
        whh = _cat_cast([whh_f, whh_r], T, dev)                 # [2*4H, H]
        bias = torch.empty(2 * G4, dtype=torch.float32, device=dev)
        call("mmdx_axpby", G4, 1.0, ptr(bih_f), 1.0, ptr(bhh_f), ptr(bias[:G4]), stream())
        call("mmdx_axpby", G4, 1.0, ptr(bih_r), 1.0, ptr(bhh_r), ptr(bias[G4:]), stream())
        # the recurrences read xg unit-interleaved ([M][2][H][4]: one 16-B load per (row,
        # unit)), so the projection runs on W_ih / bias rows permuted (dir, g, u) -> (dir, u, g);
        # the backward's GEMMs keep the gate-major W_ih (dG is gate-major)
        wih_p = wih.view(2, 4, H, In).transpose(1, 2).reshape(2 * G4, In)
        bias_p = bias.view(2, 4, H).transpose(1, 2).reshape(2 * G4)
        xg = torch.empty((M, 2 * G4), dtype=torch.float32, device=dev)
        F.gemm(x.reshape(M, In), In, True, wih_p, In, True, M, 2 * G4, In, xg, 2 * G4,
               bias=bias_p, compute_dtype=T)
        hout = torch.empty((B, Ls, 2 * H), dtype=T, device=dev)
        cs = torch.empty((2, Ls, B, H), dtype=torch.float32, device=dev)
        gs = torch.empty((2, Ls, B, H, 4), dtype=torch.float32, device=dev)
        fw = L.lib().mmdx_lstm_fwd_workspace_size(L.dtype_code(T), B, Ls, H)
        fws = L.workspace(fw, dev)
        status = coop_status(dev) if fw else None
        if status is not None and not torch.cuda.is_current_stream_capturing():
            status.poll()  # an earlier launch that lost a peer fails this step loudly
        call("mmdx_lstm_fwd", L.dtype_code(T), ptr(xg), ptr(whh), B, Ls, H, ptr(hout), ptr(cs),
             ptr(gs), ptr(fws), fw, ptr(status.word) if status else None,
             int(DEBUG["spin_limit"]), int(DEBUG["flags"]), stream())
        ctx.save_for_backward(x, wih, whh, hout, cs, gs)
        ctx.H = H
        return hout

    @staticmethod
    def backward(ctx, dh):
        x, wih, whh, hout, cs, gs = ctx.saved_tensors
        H = ctx.H
        B, Ls, In = x.shape
        T = x.dtype
        dev = x.device
        M = B * Ls
        G4 = 4 * H
        dh = F.cast(dh.contiguous(), T)
        dxg = torch.empty((M, 2 * G4), dtype=T, device=dev)
        dwhh = torch.empty((2 * G4, H), dtype=torch.float32, device=dev)
        n = L.lib().mmdx_lstm_workspace_size(L.dtype_code(T), B, Ls, H)
        ws = L.workspace(n, dev)
        # the cooperative backward (bf16, H 256) shares the forward's sticky status word
        fw = L.lib().mmdx_lstm_fwd_workspace_size(L.dtype_code(T), B, Ls, H)
        status = coop_status(dev) if fw and BWD_COOP else None
        call("mmdx_lstm_bwd", L.dtype_code(T), ptr(whh), ptr(hout), ptr(cs), ptr(gs), ptr(dh), B,
             Ls, H, ptr(dxg), ptr(dwhh), ptr(ws), n, ptr(status.word) if status else None,
             int(DEBUG["spin_limit"]), int(DEBUG["flags"]), stream())
        if status is not None:
            status.after_launch()
        dwih = torch.empty((2 * G4, In), dtype=torch.float32, device=dev)
        db = torch.empty(2 * G4, dtype=torch.float32, device=dev)
        # dW_ih and the (shared) bias gradient in one launch sequence
        F.gemm_wgrad_bias(dxg, 2 * G4, x.reshape(M, In), In, 2 * G4, In, M, dwih, In, db,
                          compute_dtype=T)
        db2 = torch.empty_like(db)
        call("mmdx_axpby", 2 * G4, 1.0, ptr(db), 0.0, None, ptr(db2), stream())
        dx = None
        if ctx.needs_input_grad[0]:
            dx = torch.empty((M, In), dtype=T, device=dev)
            F.gemm(dxg, 2 * G4, True, wih, In, False, M, In, 2 * G4, dx, In, compute_dtype=T)
            dx = dx.reshape(B, Ls, In)
        return (dx, None, dwih[:G4], dwhh[:G4], db[:G4], db2[:G4], dwih[G4:], dwhh[G4:], db[G4:],
                db2[G4:])


class _GatherFn(torch.autograd.Function):
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
        dout = dout.contiguous()
        dtab = torch.zeros(ctx.tshape, dtype=torch.float32, device=dout.device)
        call("mmdx_embed_scatter", L.dtype_code(dout.dtype), ptr(ids), B * Ls, ctx.tshape[1],
             ptr(dout), ptr(dtab), stream())
        return None, dtab, None


class LSTMParams(nn.Module):
    """Parameter container with nn.LSTM's names, shapes and init (bidirectional,
    batch_first), without nn.LSTM's cuDNN/MIOpen weight flattening on .to(device)."""

    def __init__(self, input_size, hidden_size, num_layers):
        super().__init__()
        self.input_size, self.hidden_size, self.num_layers = input_size, hidden_size, num_layers
        k = hidden_size ** -0.5
        for l in range(num_layers):
            lin = input_size if l == 0 else 2 * hidden_size
            for sfx in ("", "_reverse"):
                for name, shape in ((f"weight_ih_l{l}", (4 * hidden_size, lin)),
                                    (f"weight_hh_l{l}", (4 * hidden_size, hidden_size)),
                                    (f"bias_ih_l{l}", (4 * hidden_size,)),
                                    (f"bias_hh_l{l}", (4 * hidden_size,))):
                    p = nn.Parameter(torch.empty(shape))
                    nn.init.uniform_(p, -k, k)
                    self.register_parameter(name + sfx, p)


class BiLSTMEncoder(nn.Module):
    def __init__(self, vocab_size=VOCAB, emb=256, hidden=256, layers=2):
        super().__init__()
        self.config = SimpleNamespace(hidden_size=2 * hidden, vocab_size=vocab_size,
                                      _name_or_path="bilstm")
        self.embed = Embedding(vocab_size, emb)
        self.lstm = LSTMParams(emb, hidden, layers)
        self.hidden = hidden
        self.compute_dtype = torch.float32

    def forward(self, input_ids, attention_mask=None, token_type_ids=None, return_dict=True):
        T = self.compute_dtype
        L.require_device(input_ids)
        ids = input_ids.long().contiguous()
        h = _GatherFn.apply(ids, self.embed.weight, T)
        m = self.lstm
        for l in range(m.num_layers):
            sfx = f"_l{l}"
            h = _LSTMLayerFn.apply(
                h, self.hidden,
                getattr(m, "weight_ih" + sfx), getattr(m, "weight_hh" + sfx),
                getattr(m, "bias_ih" + sfx), getattr(m, "bias_hh" + sfx),
                getattr(m, "weight_ih" + sfx + "_reverse"),
                getattr(m, "weight_hh" + sfx + "_reverse"),
                getattr(m, "bias_ih" + sfx + "_reverse"), getattr(m, "bias_hh" + sfx + "_reverse"))
        # the status word is sticky: one device->host copy after the last layer covers every
        # cooperative launch of this forward
        st = _STATUS.get((h.device.type, h.device.index))
        if st is not None:
            st.after_launch()
        return _Out(last_hidden_state=h)
