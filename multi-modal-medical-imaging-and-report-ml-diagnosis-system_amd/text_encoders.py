"""Text-encoder backbones for TextEncoderTransformer (training_pipeline.py:348-508).

* `BertModel`        — bert-base (the reference's `AutoModel.from_pretrained(...)`, TP:360),
                       state_dict-identical to transformers' BertModel; runs on mmdx kernels.
* `EmbedMeanEncoder` — build-defined C2 tower: Embedding(30522, 768) + masked mean.
* `BiLSTMEncoder`    — build-defined C3/C4 tower: Embedding(30522, 256) + 2-layer BiLSTM.

Each backbone exposes `config.hidden_size` and `forward(input_ids, attention_mask,
token_type_ids, return_dict=True)` returning an object with `last_hidden_state`, like the
HF model the reference calls (TP:470/473).  Towers whose pooling can be fused also expose
`pooled_mean(...)`, which TextEncoderTransformer.encode prefers.
"""
from __future__ import annotations

import math
from types import SimpleNamespace

import torch
import torch.nn as nn

from . import _lib as L
from . import functional as F
from .layers import Embedding, LayerNorm, Linear

from .bert import BertModel  # noqa: E402,F401
from .bilstm import BiLSTMEncoder  # noqa: E402,F401

VOCAB = 30522


class _Out(SimpleNamespace):
    pass


def _compute_dtype(mod):
    return getattr(mod, "compute_dtype", torch.float32)


class EmbedMeanEncoder(nn.Module):
    """C2 text tower: out = masked_mean(E[ids]) fused in one gather-reduce kernel."""

    def __init__(self, vocab_size=VOCAB, hidden_size=768):
        super().__init__()
        self.config = SimpleNamespace(hidden_size=hidden_size, vocab_size=vocab_size,
                                      _name_or_path="embed-mean")
        self.embed = Embedding(vocab_size, hidden_size)
        self.compute_dtype = torch.float32

    def pooled_mean(self, input_ids, attention_mask, token_type_ids=None):
        return F.embed_mean(input_ids, attention_mask, self.embed.weight, self.compute_dtype)

    def forward(self, input_ids, attention_mask=None, token_type_ids=None, return_dict=True):
        B, Ls = input_ids.shape
        D = self.config.hidden_size
        out = torch.empty((B, Ls, D), dtype=self.compute_dtype, device=input_ids.device)
        L.call("mmdx_embed_gather", L.dtype_code(self.compute_dtype),
               L.ptr(input_ids.contiguous()), B * Ls, D, L.ptr(self.embed.weight), L.ptr(out),
               L.stream())
        return _Out(last_hidden_state=out)
