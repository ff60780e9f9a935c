"""Parameter-holding modules whose forward runs on the mmdx kernels.

They subclass the torch.nn modules the reference instantiates (nn.Linear, nn.LayerNorm,
nn.Embedding), so parameter names, shapes and default initialisation are PyTorch's and
`state_dict()` is interchangeable with the reference's; only `forward` differs.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from . import _lib as L
from . import functional as F


class Linear(nn.Linear):
    """nn.Linear whose forward is the MFMA GEMM (+bias, +activation epilogue)."""

    def forward(self, x, act: int = L.ACT_NONE, out_dtype=None):
        shp = x.shape
        y = F.linear(x.reshape(-1, shp[-1]), self.weight, self.bias, act, out_dtype)
        return y.reshape(*shp[:-1], self.out_features)


class GELU(nn.GELU):
    """Marker module (exact-erf GELU); fused into the preceding GEMM's epilogue."""


class Dropout(nn.Dropout):
    def forward(self, x):
        return F.dropout(x, self.p, self.training)


class LayerNorm(nn.LayerNorm):
    def forward(self, x, residual=None):
        return F.layer_norm(x.contiguous(), self.weight, self.bias, self.eps, residual)


class Embedding(nn.Embedding):
    """Parameter holder; lookups are fused into the consuming kernels."""
