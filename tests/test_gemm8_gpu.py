"""GPU: the 8-wave dense GEMM tiles — 128 x 128 with 64 x 32 per wave (MMDX_GEMM_8W128, the
default since round 5) and, for the forward orientation, 256 x 256 with 128 x 64 per wave
(MMDX_GEMM256_FWD_MIN), gemm_dense.hip — against the 4-wave 128 x 128 kernel and a torch
fp32 matmul, in the three operand layouts the Linear layers use: forward (A, B k-major),
input gradient (B R-major), weight gradient (A and B R-major), fp16 and bf16, ragged M / N /
K.

Both tilings accumulate every output over the same K tiles in the same MFMA order, so the
results must be BIT-IDENTICAL; the fp32 matmul check bounds the kernel error itself
(rel 1e-2 of the output scale: 16-bit inputs, fp32 accumulation, 16-bit store).
"""
import pytest
import torch

from mmdx import functional as F

pytestmark = pytest.mark.gpu

SHAPES = [  # M, N, K  (>= 256 128x128 tiles, so the plan does not split K)
    (2056, 2048, 776),
    (4000, 1032, 200),
    (2304, 2304, 768),
]


def _gemm(layout, a, b, M, N, K, out_dtype):
    C = torch.empty(M, N, dtype=out_dtype, device=a.device)
    if layout == "fwd":  # C = A[M,K] . B[N,K]^T
        F.gemm(a, K, 1, b, K, 1, M, N, K, C, N)
    elif layout == "dgrad":  # C = A[M,K] . B[K,N]
        F.gemm(a, K, 1, b, N, 0, M, N, K, C, N)
    else:  # "wgrad": C = A[K,M]^T . B[K,N]
        F.gemm(a, M, 0, b, N, 0, M, N, K, C, N)
    return C


def _operands(layout, M, N, K, dt, dev, seed):
    g = torch.Generator().manual_seed(seed)
    ash = (K, M) if layout == "wgrad" else (M, K)
    bsh = (N, K) if layout == "fwd" else (K, N)
    a = torch.randn(*ash, generator=g).to(dt)
    b = torch.randn(*bsh, generator=g).to(dt)
    ad, bd = a.double(), b.double()
    ref = ad @ bd.t() if layout == "fwd" else ad @ bd if layout == "dgrad" else ad.t() @ bd
    return a.to(dev), b.to(dev), ref


@pytest.mark.parametrize("knob", ["MMDX_GEMM256_FWD_MIN", "MMDX_GEMM_8W128"])
@pytest.mark.parametrize("layout", ["fwd", "dgrad", "wgrad"])
@pytest.mark.parametrize("dt", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("shape", SHAPES)
def test_gemm8_matches_4wave(dev, knob, layout, dt, shape, knobs):
    if knob == "MMDX_GEMM256_FWD_MIN" and layout != "fwd":
        pytest.skip("256 x 256 tiles serve the forward orientation only")
    M, N, K = shape
    a, b, ref = _operands(layout, M, N, K, dt, dev, M + N + K)
    knobs("MMDX_GEMM256_FWD_MIN", 0)  # the 4-wave kernel is the baseline
    knobs("MMDX_GEMM_8W128", 0)
    for out_dtype in (dt, torch.float32):
        knobs(knob, 0)
        c4 = _gemm(layout, a, b, M, N, K, out_dtype)
        knobs(knob, 1)
        c8 = _gemm(layout, a, b, M, N, K, out_dtype)
        torch.cuda.synchronize()
        assert torch.isfinite(c8.float()).all()
        knobs(knob, 0)
        assert torch.equal(c4, c8), (layout, dt, shape, out_dtype)
        err = (c8.double().cpu() - ref).abs().max().item() / ref.abs().max().item()
        assert err <= 1e-2, (layout, dt, shape, out_dtype, err)


@pytest.mark.parametrize("dt", [torch.float16, torch.bfloat16])
def test_gemm256_forward_epilogue(dev, dt, knobs):
    """The 256 x 256 tiles under the Linear forward's fused epilogue (bias + GELU + the saved
    pre-activation, the FFN-up GEMM; MMDX_GEMM256_FWD_MIN selects these tiles for the large
    ViT-B forward GEMMs by default) are bit-identical to the 4-wave kernel."""
    from mmdx import _lib as L
    M, N, K = 3152, 3072, 768
    a, b, ref = _operands("fwd", M, N, K, dt, dev, 11)
    bias = torch.randn(N, device=dev)
    outs = []
    # arm 0: the 128 x 128 kernel (the 256 x 256 threshold off); arm 1: 256 x 256
    for knob in ("0", "1"):
        knobs("MMDX_GEMM256_FWD_MIN", knob)
        C = torch.empty(M, N, dtype=dt, device=dev)
        pre = torch.empty(M, N, dtype=dt, device=dev)
        F.gemm(a, K, 1, b, K, 1, M, N, K, C, N, bias=bias, act=L.ACT_GELU, preact=pre)
        outs.append((C, pre))
    torch.cuda.synchronize()
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
    # one rounding of an fp32-accumulated value to the 16-bit type: 2^-8 (bf16) / 2^-11 (fp16)
    # of the output scale, plus the fp32 accumulation of K = 768 products
    tol = (2.0 ** -8 if dt == torch.bfloat16 else 2.0 ** -11) + 1e-5
    pre_ref = ref + bias.double().cpu()
    err = (outs[1][1].double().cpu() - pre_ref).abs().max().item() / pre_ref.abs().max().item()
    assert err <= tol, ("preact", err)
    c_ref = torch.nn.functional.gelu(pre_ref)
    err = (outs[1][0].double().cpu() - c_ref).abs().max().item() / c_ref.abs().max().item()
    assert err <= tol, ("gelu output", err)
