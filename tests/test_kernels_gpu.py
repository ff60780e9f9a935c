"""Kernel-level parity: every HIP op vs a plain PyTorch fp32 reference of the same op.

Tolerances: fp32 path (exact-f32 MFMA, different summation order) rel 1e-5 of the output
scale; bf16 path rel 2e-2 (bf16 inputs, fp32 accumulation).
"""
import math
import pytest
import torch
import torch.nn.functional as tF

import mmdx
from mmdx import _lib as L
from mmdx import functional as F

pytestmark = pytest.mark.gpu

TOL = {torch.float32: 2e-5, torch.bfloat16: 2e-2, torch.float16: 4e-3}


def _close(out, ref, dt, what=""):
    out = out.float().cpu()
    ref = ref.float().cpu()
    scale = ref.abs().max().clamp(min=1e-6)
    err = (out - ref).abs().max() / scale
    assert err <= TOL[dt], f"{what}: rel err {err:.3e} > {TOL[dt]}"


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16, torch.float16])
@pytest.mark.parametrize("M,N,K", [(64, 13, 1024), (200, 1024, 1536), (13, 1024, 64),
                                   (1000, 96, 40), (37, 130, 1000), (8192, 768, 768)])
@pytest.mark.parametrize("ak,bk", [(1, 1), (1, 0), (0, 0), (0, 1)])
def test_gemm(dev, dt, M, N, K, ak, bk):
    g = torch.Generator().manual_seed(M * 7 + N * 3 + K)
    A = torch.randn(M, K, generator=g)
    B = torch.randn(N, K, generator=g)
    bias = torch.randn(N, generator=g)
    ref = A @ B.T + bias
    Ad = (A if ak else A.T.contiguous()).to(dev, dt)
    Bd = (B if bk else B.T.contiguous()).to(dev, dt)
    C = torch.empty(M, N, dtype=torch.float32, device=dev)
    F.gemm(Ad, K if ak else M, ak, Bd, K if bk else N, bk, M, N, K, C, N,
           bias=bias.to(dev), compute_dtype=dt)
    torch.cuda.synchronize()
    if dt != torch.float32:
        ref = A.to(dt).float() @ B.to(dt).float().T + bias
    _close(C, ref, dt, f"gemm {M}x{N}x{K} ak={ak} bk={bk}")


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_gemm_gelu_preact_beta(dev, dt):
    g = torch.Generator().manual_seed(1)
    M, N, K = 96, 256, 128
    A, B = torch.randn(M, K, generator=g), torch.randn(N, K, generator=g)
    C0 = torch.randn(M, N, generator=g)
    Ad, Bd = A.to(dev, dt), B.to(dev, dt)
    if dt == torch.bfloat16:
        A, B = A.bfloat16().float(), B.bfloat16().float()
    pre_ref = A @ B.T
    C = C0.to(dev)
    pre = torch.empty(M, N, device=dev)
    F.gemm(Ad, K, 1, Bd, K, 1, M, N, K, C, N, act=L.ACT_GELU, beta=0.5, preact=pre,
           compute_dtype=dt)
    _close(pre, pre_ref, dt, "preact")
    _close(C, tF.gelu(pre_ref) + 0.5 * C0, dt, "gelu+beta")


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16, torch.float16])
@pytest.mark.parametrize("MNK,beta", [((96, 256, 128), 0.0), ((200, 3072, 768), 0.0),
                                      ((37, 130, 64), 0.5), ((4096, 64, 2048), 0.0)])
@pytest.mark.parametrize("extra", [False, True])
def test_gemm_gelu_bwd_epilogue(dev, dt, MNK, beta, extra):
    """act = MMDX_ACT_GELU_BWD: C = (A B^T) * gelu'(pre) (+ bias + addend) (+ beta C), pre
    read from `preact` (the FFN backward's fused GELU gradient); vector and scalar epilogues
    (N % 8 != 0), split-K (K = 2048 on a small grid) through the reduce kernel.  `extra` adds
    a bias and an addend, which the 16-B vector branch does not carry: the epilogue must take
    the per-element path for them (apply()'s order: gelu' first, then bias, addend)."""
    M, N, K = MNK
    g = torch.Generator().manual_seed(M + N)
    A, B = torch.randn(M, K, generator=g) / 8, torch.randn(N, K, generator=g) / 8
    P = torch.randn(M, N, generator=g)
    C0 = torch.randn(M, N, generator=g)
    bias, add = torch.randn(N, generator=g), torch.randn(M, N, generator=g)
    Ad, Bd, Pd = A.to(dev, dt), B.to(dev, dt), P.to(dev, dt)
    A, B, P = Ad.float().cpu(), Bd.float().cpu(), Pd.float().cpu()
    x = P.double()
    grad = 0.5 * (1 + torch.erf(x / 2 ** 0.5)) + x * torch.exp(-0.5 * x * x) / (2 * math.pi) ** 0.5
    ref = (A.double() @ B.double().T) * grad + beta * C0.to(dt).double()
    if extra:
        ref = ref + bias.double() + add.double()
    C = C0.to(dev, dt)
    bd, addd = bias.to(dev), add.to(dev)
    L.call("mmdx_gemm", L.dtype_code(dt), M, N, K, Ad.data_ptr(), K, 1, Bd.data_ptr(), K, 1,
           C.data_ptr(), N, L.dtype_code(dt), bd.data_ptr() if extra else None,
           addd.data_ptr() if extra else None, L.ACT_GELU_BWD, 1.0, beta,
           Pd.data_ptr(), *_ws(dt, M, N, K, dev), L.stream())
    torch.cuda.synchronize()
    err = ((C.double().cpu() - ref).abs().max() / ref.abs().max()).item()
    assert err <= (2e-5 if dt == torch.float32 else 1e-2), err
    assert torch.equal(Pd.float().cpu(), P), "the pre-activation input was written"


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16, torch.float16])
@pytest.mark.parametrize("act", ["none", "relu", "gelu"])
@pytest.mark.parametrize("ldc_pad", [0, 1])
def test_gemm_epilogue_bias_addend_preact(dev, dt, act, ldc_pad):
    """C = act(A B^T + bias + addend) + beta C with the pre-activation copied out — the
    16-B-per-8-columns epilogue (ldc % 8 == 0) and the per-element one (ldc odd) against a
    float64 reference of the same rounded operands; 16-bit outputs."""
    M, N, K = 300, 256, 192
    ldc = N + ldc_pad
    g = torch.Generator().manual_seed(11 + ldc_pad)
    A, B = torch.randn(M, K, generator=g) / 8, torch.randn(N, K, generator=g) / 8
    bias, add = torch.randn(N, generator=g), torch.randn(M, ldc, generator=g)
    C0 = torch.randn(M, ldc, generator=g)
    Ad, Bd = A.to(dev, dt), B.to(dev, dt)
    C = C0.to(dev, dt)
    pre = torch.full((M, ldc), 7.0, device=dev).to(dt)
    code = {"none": L.ACT_NONE, "relu": L.ACT_RELU, "gelu": L.ACT_GELU}[act]
    L.call("mmdx_gemm", L.dtype_code(dt), M, N, K, Ad.data_ptr(), K, 1, Bd.data_ptr(), K, 1,
           C.data_ptr(), ldc, L.dtype_code(dt), bias.to(dev).data_ptr(),
           add.to(dev).data_ptr(), code, 1.0, 0.5, pre.data_ptr(),
           *_ws(dt, M, N, K, dev), L.stream())
    torch.cuda.synchronize()
    Ar, Br = Ad.double().cpu(), Bd.double().cpu()
    z = Ar @ Br.T + bias.double() + add[:, :N].double()
    y = {"none": z, "relu": z.clamp(min=0), "gelu": tF.gelu(z)}[act]
    ref = y + 0.5 * C0.to(dt).double()[:, :N]
    tol = 2e-5 if dt == torch.float32 else 1e-2
    for what, got, want in (("C", C, ref), ("preact", pre, z)):
        got = got.double().cpu()
        err = ((got[:, :N] - want).abs().max() / want.abs().max()).item()
        assert err <= tol, (what, err)
    if ldc_pad:   # the padding column is never written
        assert torch.equal(C.cpu()[:, N:], C0.to(dt)[:, N:])
        assert torch.all(pre.float().cpu()[:, N:] == 7.0)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16, torch.float16])
@pytest.mark.parametrize("M,N", [(8192, 768), (12608, 3072), (300, 130), (64, 2304), (1000, 13),
                                 (8, 8)])
@pytest.mark.parametrize("beta", [0.0, 1.0])
def test_bias_grad(dev, dt, M, N, beta):
    """Bias gradients = column sums of dY [M, N] (the two-pass column-sum kernels; with
    MMDX_BIAS_GRAD_GEMM=1 and 16-bit M, N % 8 == 0 the 1 x N x M GEMM against a ones row),
    accumulated onto db when beta = 1, against float64 sums of the same rounded values."""
    g = torch.Generator().manual_seed(M + N)
    dy = torch.randn(M, N, generator=g).to(dev, dt)
    db0 = torch.randn(N, generator=g).to(dev)
    db = db0.clone()
    n = L.lib().mmdx_bias_grad_workspace_size(M, N)
    w = torch.empty(max(n, 1), dtype=torch.uint8, device=dev)
    L.call("mmdx_bias_grad", L.dtype_code(dt), dy.data_ptr(), M, N, db.data_ptr(), beta,
           w.data_ptr(), n, L.stream())
    torch.cuda.synchronize()
    ref = dy.double().cpu().sum(0) + beta * db0.double().cpu()
    bound = 2e-6 * dy.double().abs().cpu().sum(0) + 1e-6 * db0.double().abs().cpu() + 1e-12
    err = (db.double().cpu() - ref).abs()
    assert (err <= bound).all(), (err / bound).max().item()


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16, torch.float32])
@pytest.mark.parametrize("M,N,K", [(768, 3072, 8192), (2304, 768, 12608), (768, 768, 1000),
                                   (520, 130, 64), (3072, 768, 256)])
def test_gemm_wgrad_bias(dev, dt, M, N, K):
    """dW = dY^T X and db = column sums of dY (mmdx_gemm_bias_grad; 16-bit split-K grids fuse
    the sums into the GEMM's column-tile-0 blocks, the rest runs GEMM + column sums)."""
    g = torch.Generator().manual_seed(M + N + K)
    dY = (torch.randn(K, M, generator=g) / 4).to(dev, dt)
    X = (torch.randn(K, N, generator=g) / 4).to(dev, dt)
    dW = torch.full((M, N), float("nan"), device=dev)
    db = torch.full((M,), float("nan"), device=dev)
    n = L.lib().mmdx_gemm_bias_grad_workspace_size(L.dtype_code(dt), M, N, K)
    w = torch.empty(max(n, 1), dtype=torch.uint8, device=dev)
    L.call("mmdx_gemm_bias_grad", L.dtype_code(dt), M, N, K, dY.data_ptr(), M, X.data_ptr(), N,
           dW.data_ptr(), N, L.F32, db.data_ptr(), w.data_ptr(), n, L.stream())
    torch.cuda.synchronize()
    a, b = dY.double().cpu(), X.double().cpu()
    _close(dW, a.T @ b, dt if dt != torch.float32 else torch.float32, "dW")
    ref = a.sum(0)
    bound = 2e-6 * a.abs().sum(0) + 1e-12
    assert ((db.double().cpu() - ref).abs() <= bound).all(), \
        ((db.double().cpu() - ref).abs() / bound).max().item()


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16, torch.float32])
@pytest.mark.parametrize("M,N,K,ldc", [(300, 256, 192, 256), (300, 256, 192, 257),
                                       (37, 768, 3072, 768), (12608, 768, 64, 768),
                                       (12608, 768, 3072, 768)])
def test_gemm_residual(dev, dt, M, N, K, ldc):
    """mmdx_gemm_res: C = A B^T + bias + residual equals the copy-then-beta-1 form bit for bit
    (vector and per-element epilogues, split-K through the reduce: K 3072 on a small grid;
    12608 x 768 x 3072 is the ViT-B FFN-down shape, 150 256 x 256 tiles: the 8-wave forward
    kernel's residual epilogue under the default MMDX_GEMM256_FWD_MIN)."""
    g = torch.Generator().manual_seed(M + N + K + ldc)
    A = (torch.randn(M, K, generator=g) / 8).to(dev, dt)
    B = (torch.randn(N, K, generator=g) / 8).to(dev, dt)
    bias = torch.randn(N, generator=g).to(dev)
    res = torch.randn(M, ldc, generator=g).to(dev, dt)
    n = L.lib().mmdx_gemm_workspace_size(L.dtype_code(dt), M, N, K)
    w = torch.empty(max(n, 1), dtype=torch.uint8, device=dev)
    C1 = torch.full((M, ldc), 3.0, device=dev).to(dt)
    L.call("mmdx_gemm_res", L.dtype_code(dt), M, N, K, A.data_ptr(), K, 1, B.data_ptr(), K, 1,
           C1.data_ptr(), ldc, L.dtype_code(dt), bias.data_ptr(), None, L.ACT_NONE, 1.0, 0.0,
           None, res.data_ptr(), w.data_ptr(), n, L.stream())
    C0 = res.clone()
    L.call("mmdx_gemm", L.dtype_code(dt), M, N, K, A.data_ptr(), K, 1, B.data_ptr(), K, 1,
           C0.data_ptr(), ldc, L.dtype_code(dt), bias.data_ptr(), None, L.ACT_NONE, 1.0, 1.0,
           None, w.data_ptr(), n, L.stream())
    torch.cuda.synchronize()
    assert torch.equal(C1[:, :N], C0[:, :N])
    if ldc > N:
        assert torch.all(C1.float()[:, N:] == 3.0)
    ref = A.double().cpu() @ B.double().cpu().T + bias.double().cpu() + res.double().cpu()[:, :N]
    _close(C1[:, :N], ref, dt, "gemm residual")


def _ws(dt, M, N, K, dev):
    n = L.lib().mmdx_gemm_workspace_size(L.dtype_code(dt), M, N, K)
    w = torch.empty(max(n, 1), dtype=torch.uint8, device=dev)
    _WS_KEEP.append(w)
    return w.data_ptr(), n


_WS_KEEP = []


CONVS = [  # N, C, H, W, K, k, s, p
    (2, 64, 14, 14, 64, 3, 1, 1),
    (2, 64, 15, 15, 128, 3, 2, 1),
    (3, 256, 7, 7, 64, 1, 1, 0),
    (2, 64, 14, 14, 256, 1, 2, 0),
    (2, 3, 32, 32, 64, 7, 2, 3),
    (1, 128, 9, 9, 512, 3, 2, 1),
    # small grids with C, K multiples of 128: 128-deep K tiles (fwd and stride-1 dgrad)
    (2, 256, 14, 14, 256, 3, 1, 1),
    (3, 128, 7, 7, 128, 3, 1, 1),
    (2, 512, 7, 7, 1024, 1, 1, 0),
]


def _nhwc(x, cp, dt):
    N, C, H, W = x.shape
    y = torch.zeros(N, H, W, cp)
    y[..., :C] = x.permute(0, 2, 3, 1)
    return y.to(dt)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("cfg", CONVS)
def test_conv_fwd_dgrad_wgrad(dev, dt, cfg):
    _conv_case(dev, dt, cfg)


# production M: the C4 batch (N = 128) at layer1's 56x56 (M = 401,408 rows), the 3x3 and
# the 1x1 expansion, layer2's strided 1x1 downsample (M = 100,352) and the layer3 / layer4
# 3x3s (128-deep K tiles) — the exact launch geometry of the benched step (grid sizes,
# split-K depth of the wgrad, BN stat blocks)
@pytest.mark.parametrize("cfg", [(128, 64, 56, 56, 64, 3, 1, 1), (128, 64, 56, 56, 256, 1, 1, 0),
                                 (128, 256, 56, 56, 512, 1, 2, 0),
                                 (128, 512, 7, 7, 512, 3, 1, 1), (128, 256, 14, 14, 256, 3, 1, 1)])
def test_conv_production_m(dev, cfg):
    torch.set_num_threads(16)
    _conv_case(dev, torch.bfloat16, cfg)


def _conv_case(dev, dt, cfg):
    N, C, H, W, K, k, s, p = cfg
    vec = 4 if dt == torch.float32 else 8
    cp = (C + vec - 1) // vec * vec
    g = torch.Generator().manual_seed(sum(cfg))
    x = torch.randn(N, C, H, W, generator=g)
    w = torch.randn(K, C, k, k, generator=g) * 0.1
    if dt == torch.bfloat16:
        x, w = x.bfloat16().float(), w.bfloat16().float()
    xr = x.clone().requires_grad_(True)
    wr = w.clone().requires_grad_(True)
    yr = tF.conv2d(xr, wr, stride=s, padding=p)
    dy = torch.randn(yr.shape, generator=g)
    if dt == torch.bfloat16:
        dy = dy.bfloat16().float()
    yr.backward(dy)
    P, Q = yr.shape[2], yr.shape[3]
    d = L.ConvDesc(N, H, W, cp, K, k, k, s, s, p, p, P, Q)
    dc = L.dtype_code(dt)
    wd = w.to(dev)
    wk = torch.empty(K, k, k, cp, dtype=dt, device=dev)
    wc = torch.empty(cp, k, k, K, dtype=dt, device=dev)
    L.call("mmdx_conv_pack_weight", dc, d, C, wd.data_ptr(), wk.data_ptr(), wc.data_ptr(),
           L.stream())
    xd = _nhwc(x, cp, dt).to(dev)
    y = torch.empty(N, P, Q, K, dtype=dt, device=dev)
    nst = L.lib().mmdx_conv_fwd_stat_blocks(d)
    part = torch.empty(K, nst, 2, device=dev)  # channel-major [K][blocks] (mean, M2)
    L.call("mmdx_conv_fwd", dc, d, xd.data_ptr(), wk.data_ptr(), y.data_ptr(), part.data_ptr(),
           L.stream())
    _close(y.permute(0, 3, 1, 2), yr.detach(), dt, f"fwd {cfg}")
    # epilogue BatchNorm statistics: merge the per-128-row (mean, M2) blocks on the host
    M = N * P * Q
    cnt = torch.tensor([min(128, M - 128 * b) for b in range(nst)], dtype=torch.float64)
    pm, p2 = part[..., 0].t().double().cpu(), part[..., 1].t().double().cpu()
    mean = (pm * cnt[:, None]).sum(0) / M
    m2 = (p2 + cnt[:, None] * (pm - mean) ** 2).sum(0)
    yref = yr.detach().double()
    _close(mean, yref.mean((0, 2, 3)), torch.float32 if dt == torch.float32 else dt, "stat mean")
    _close(m2 / M, yref.var((0, 2, 3), unbiased=False), dt, "stat var")
    dyd = dy.permute(0, 2, 3, 1).contiguous().to(dev, dt)
    dx = torch.empty(N, H, W, cp, dtype=dt, device=dev)
    L.call("mmdx_conv_dgrad", dc, d, dyd.data_ptr(), wc.data_ptr(), dx.data_ptr(), 0.0,
           L.stream())
    if C == cp:
        _close(dx.permute(0, 3, 1, 2), xr.grad, dt, f"dgrad {cfg}")
    dw = torch.empty(K, C, k, k, device=dev)
    ws_n = L.lib().mmdx_conv_wgrad_workspace_size(dc, d)
    ws = torch.empty(ws_n, dtype=torch.uint8, device=dev)
    L.call("mmdx_conv_wgrad", dc, d, C, xd.data_ptr(), dyd.data_ptr(), dw.data_ptr(), 0.0,
           ws.data_ptr(), ws_n, L.stream())
    _close(dw, wr.grad, dt, f"wgrad {cfg}")


@pytest.mark.parametrize("cfg", [(21, 64, 56, 56, 256, 3, 1, 1), (11, 256, 56, 56, 512, 1, 1, 0)])
def test_conv_fwd_large_ragged(dev, cfg):
    """bf16 forward on large grids (>= 512 256-row tiles), M ragged (M mod 256 = 64 / 128:
    the last 128-row slabs are partial), with the per-128-row BN statistics slabs."""
    N, C, H, W, K, k, s, p = cfg
    g = torch.Generator().manual_seed(7)
    x = torch.randn(N, C, H, W, generator=g).bfloat16().float()
    w = (torch.randn(K, C, k, k, generator=g) * 0.05).bfloat16().float()
    yr = tF.conv2d(x, w, stride=s, padding=p)
    P, Q = yr.shape[2], yr.shape[3]
    M = N * P * Q
    assert ((M + 255) // 256) * (K // 128) >= 512
    d = L.ConvDesc(N, H, W, C, K, k, k, s, s, p, p, P, Q)
    wk = torch.empty(K, k, k, C, dtype=torch.bfloat16, device=dev)
    wc = torch.empty(C, k, k, K, dtype=torch.bfloat16, device=dev)
    L.call("mmdx_conv_pack_weight", 1, d, C, w.to(dev).data_ptr(), wk.data_ptr(),
           wc.data_ptr(), L.stream())
    xd = x.permute(0, 2, 3, 1).contiguous().to(dev, torch.bfloat16)
    y = torch.empty(N, P, Q, K, dtype=torch.bfloat16, device=dev)
    nst = L.lib().mmdx_conv_fwd_stat_blocks(d)
    assert nst == (M + 127) // 128
    part = torch.full((K, nst, 2), float("nan"), device=dev)
    L.call("mmdx_conv_fwd", 1, d, xd.data_ptr(), wk.data_ptr(), y.data_ptr(), part.data_ptr(),
           L.stream())
    _close(y.permute(0, 3, 1, 2), yr, torch.bfloat16, f"fwd {cfg}")
    assert torch.isfinite(part).all(), "a 128-row statistics slab was not written"
    cnt = torch.tensor([min(128, M - 128 * b) for b in range(nst)], dtype=torch.float64)
    pm, p2 = part[..., 0].t().double().cpu(), part[..., 1].t().double().cpu()
    mean = (pm * cnt[:, None]).sum(0) / M
    m2 = (p2 + cnt[:, None] * (pm - mean) ** 2).sum(0)
    yref = yr.double()
    _close(mean, yref.mean((0, 2, 3)), torch.bfloat16, "stat mean")
    _close(m2 / M, yref.var((0, 2, 3), unbiased=False), torch.bfloat16, "stat var")
    # per-slab check of the last two slabs (the ragged tile)
    yt = yr.permute(0, 2, 3, 1).reshape(M, K).double()
    for b in (nst - 2, nst - 1):
        rows = yt[128 * b:min(M, 128 * b + 128)]
        _close(pm[b], rows.mean(0), torch.bfloat16, f"slab {b} mean")
    _wgrad_check(dev, x, w, yr, g, d, cfg)


@pytest.mark.parametrize("cfg", [(48, 64, 56, 56, 64, 1, 1, 0), (48, 64, 56, 56, 128, 1, 1, 0)])
def test_conv_wgrad_deep_split(dev, cfg):
    """Weight gradients split >= 128 ways over K = N*P*Q (the stem / layer1 regime): the
    partials go through the split-group reduction (wgrad_reduce_z_kernel, Z = 16)."""
    N, C, H, W, K, k, s, p = cfg
    g = torch.Generator().manual_seed(11)
    x = torch.randn(N, C, H, W, generator=g).bfloat16().float()
    w = (torch.randn(K, C, k, k, generator=g) * 0.05).bfloat16().float()
    yr = tF.conv2d(x, w, stride=s, padding=p)
    d = L.ConvDesc(N, H, W, C, K, k, k, s, s, p, p, yr.shape[2], yr.shape[3])
    ws_n = L.lib().mmdx_conv_wgrad_workspace_size(1, d)
    assert ws_n >= 128 * K * C * k * k * 4, "expected >= 128 splits"
    _wgrad_check(dev, x, w, yr, g, d, cfg)


def _wgrad_check(dev, x, w, yr, g, d, cfg):
    """bf16 weight gradient vs torch fp32 on the bf16-rounded operands, beta 1 then 0."""
    N, C, H, W, K, k, s, p = cfg
    xd = x.permute(0, 2, 3, 1).contiguous().to(dev, torch.bfloat16)
    dy = torch.randn(yr.shape, generator=g).bfloat16().float()
    dwr = torch.nn.grad.conv2d_weight(x, w.shape, dy, stride=s, padding=p)
    dyd = dy.permute(0, 2, 3, 1).contiguous().to(dev, torch.bfloat16)
    ws_n = L.lib().mmdx_conv_wgrad_workspace_size(1, d)
    ws = torch.empty(ws_n, dtype=torch.uint8, device=dev)
    dw = torch.full((K, C, k, k), 0.5, device=dev)
    L.call("mmdx_conv_wgrad", 1, d, C, xd.data_ptr(), dyd.data_ptr(), dw.data_ptr(), 1.0,
           ws.data_ptr(), ws_n, L.stream())
    _close(dw - 0.5, dwr, torch.bfloat16, "wgrad beta 1")
    L.call("mmdx_conv_wgrad", 1, d, C, xd.data_ptr(), dyd.data_ptr(), dw.data_ptr(), 0.0,
           ws.data_ptr(), ws_n, L.stream())
    _close(dw, dwr, torch.bfloat16, "wgrad")


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("train", [1, 0])
@pytest.mark.parametrize("res,relu", [(False, True), (True, True), (False, False)])
def test_batchnorm(dev, dt, train, res, relu):
    g = torch.Generator().manual_seed(3)
    N, H, W, C = 4, 9, 7, 64
    x = torch.randn(N, C, H, W, generator=g) * 2 + 0.5
    r = torch.randn(N, C, H, W, generator=g)
    if dt == torch.bfloat16:
        x, r = x.bfloat16().float(), r.bfloat16().float()
    bn = torch.nn.BatchNorm2d(C)
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5, generator=g)
        bn.bias.uniform_(-0.5, 0.5, generator=g)
        bn.running_mean.uniform_(-0.2, 0.2, generator=g)
        bn.running_var.uniform_(0.5, 2, generator=g)
    rm0, rv0 = bn.running_mean.clone(), bn.running_var.clone()
    bn.train(bool(train))
    xr = x.clone().requires_grad_(True)
    rr = r.clone().requires_grad_(True)
    yr = bn(xr)
    if res:
        yr = yr + rr
    if relu:
        yr = torch.relu(yr)
    dy = torch.randn(yr.shape, generator=g)
    yr.backward(dy)
    to = lambda t: t.permute(0, 2, 3, 1).contiguous().to(dev, dt)
    xd, rd, dyd = to(x), to(r), to(dy)
    rows = N * H * W
    gam, bet = bn.weight.detach().to(dev), bn.bias.detach().to(dev)
    rm, rv = rm0.to(dev), rv0.to(dev)
    mean = torch.empty(C, device=dev)
    rstd = torch.empty(C, device=dev)
    y = torch.empty_like(xd)
    ws_n = L.lib().mmdx_bn_workspace_size(rows, C)
    ws = torch.empty(ws_n, dtype=torch.uint8, device=dev)
    dc = L.dtype_code(dt)
    L.call("mmdx_bn_fwd", dc, train, xd.data_ptr(), rows, C, None, 0, 0, gam.data_ptr(),
           bet.data_ptr(),
           rm.data_ptr(), rv.data_ptr(), 0.1, 1e-5, mean.data_ptr(), rstd.data_ptr(),
           rd.data_ptr() if res else None, int(relu), y.data_ptr(), ws.data_ptr(), ws_n,
           L.stream())
    _close(y.permute(0, 3, 1, 2), yr.detach(), dt, "bn fwd")
    if train:
        _close(rm, bn.running_mean, torch.float32, "running_mean")
        _close(rv, bn.running_var, torch.float32, "running_var")
    dx = torch.empty_like(xd)
    dres = torch.empty_like(xd)
    dg = torch.empty(C, device=dev)
    db = torch.empty(C, device=dev)
    L.call("mmdx_bn_bwd", dc, train, xd.data_ptr(), y.data_ptr(), dyd.data_ptr(), rows, C,
           gam.data_ptr(), bet.data_ptr(), mean.data_ptr(), rstd.data_ptr(), int(relu), None, 0,
           dx.data_ptr(), dres.data_ptr() if res else None, dg.data_ptr(), db.data_ptr(), 0.0,
           ws.data_ptr(), ws_n, L.stream())
    if relu and not res:  # mask recomputed from x instead of read from y: identical result
        dx2 = torch.empty_like(xd)
        L.call("mmdx_bn_bwd", dc, train, xd.data_ptr(), None, dyd.data_ptr(), rows, C,
               gam.data_ptr(), bet.data_ptr(), mean.data_ptr(), rstd.data_ptr(), 1, None, 0,
               dx2.data_ptr(), None, None, None, 0.0, ws.data_ptr(), ws_n, L.stream())
        assert torch.equal(dx2, dx)
    tol_dt = dt
    _close(dx.permute(0, 3, 1, 2), xr.grad, tol_dt, "bn dx")
    _close(dg, bn.weight.grad, tol_dt, "dgamma")
    _close(db, bn.bias.grad, tol_dt, "dbeta")
    if res:
        _close(dres.permute(0, 3, 1, 2), rr.grad, tol_dt, "dres")


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("hwp", [(12, 11, 1), (16, 16, 1), (13, 14, 0), (112, 112, 1)])
def test_pools(dev, dt, hwp):
    """3x3 / stride-2 max pool (the stem's, specialised kernels) fwd + bwd, ties included."""
    g = torch.Generator().manual_seed(4)
    H, W, pad = hwp
    N, C = (2, 64) if H < 100 else (4, 64)
    x = torch.randn(N, C, H, W, generator=g)
    x[:, :, :4, :4] = 0.0  # ties, as after ReLU
    if dt == torch.bfloat16:
        x = x.bfloat16().float()
    xr = x.clone().requires_grad_(True)
    yr = tF.max_pool2d(xr, 3, 2, pad)
    dy = torch.randn(yr.shape, generator=g)
    if dt == torch.bfloat16:
        dy = dy.bfloat16().float()
    yr.backward(dy)
    P, Q = yr.shape[2:]
    xd = x.permute(0, 2, 3, 1).contiguous().to(dev, dt)
    y = torch.empty(N, P, Q, C, dtype=dt, device=dev)
    am = torch.empty(N, P, Q, C, dtype=torch.uint8, device=dev)
    dc = L.dtype_code(dt)
    L.call("mmdx_maxpool_fwd", dc, xd.data_ptr(), N, H, W, C, 3, 2, pad, y.data_ptr(),
           am.data_ptr(), P, Q, L.stream())
    _close(y.permute(0, 3, 1, 2), yr.detach(), dt, "maxpool fwd")
    dyd = dy.permute(0, 2, 3, 1).contiguous().to(dev, dt)
    dx = torch.empty_like(xd)
    L.call("mmdx_maxpool_bwd", dc, am.data_ptr(), dyd.data_ptr(), N, H, W, C, 3, 2, pad, P, Q,
           dx.data_ptr(), L.stream())
    _close(dx.permute(0, 3, 1, 2), xr.grad, dt, "maxpool bwd")
    f = torch.empty(N, C, dtype=dt, device=dev)
    L.call("mmdx_avgpool_fwd", dc, xd.data_ptr(), N, H * W, C, f.data_ptr(), L.stream())
    _close(f, x.mean((2, 3)), dt, "avgpool")


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("hwp", [(12, 11, 1), (112, 112, 1), (13, 14, 0)])
def test_maxpool_bn_fused(dev, dt, hwp):
    """The stem's train-mode BN + ReLU fused into the 3x3/2 pool (mmdx_maxpool_bn_fwd) equals
    mmdx_bn_fwd's apply followed by mmdx_maxpool_fwd BIT FOR BIT (pooled values and argmax
    bytes; about half of every window is ReLU zeros, so the tie rule is exercised), and the
    statistics-only BN call (y == NULL) saves the same mean / rstd / running stats."""
    g = torch.Generator().manual_seed(11)
    H, W, pad = hwp
    N, C = (2, 64) if H < 100 else (8, 64)
    rows = N * H * W
    x = (torch.randn(rows, C, generator=g) * 2 + 0.3).to(dev, dt)
    gam = (torch.rand(C, generator=g) + 0.5).to(dev)
    gam[::7] *= -1.0  # negative scales: the max is taken after the affine map
    bet = (torch.randn(C, generator=g) * 0.2).to(dev)
    dc = L.dtype_code(dt)
    ws_n = L.lib().mmdx_bn_workspace_size(rows, C)
    ws = torch.empty(ws_n, dtype=torch.uint8, device=dev)
    outs = []
    for apply in (True, False):
        rm, rv = torch.zeros(C, device=dev), torch.ones(C, device=dev)
        mean, rstd = torch.empty(C, device=dev), torch.empty(C, device=dev)
        a = torch.empty_like(x) if apply else None
        L.call("mmdx_bn_fwd", dc, 1, x.data_ptr(), rows, C, None, 0, 0, gam.data_ptr(),
               bet.data_ptr(), rm.data_ptr(), rv.data_ptr(), 0.1, 1e-5, mean.data_ptr(),
               rstd.data_ptr(), None, 1, a.data_ptr() if apply else None, ws.data_ptr(), ws_n,
               L.stream())
        P, Q = (H + 2 * pad - 3) // 2 + 1, (W + 2 * pad - 3) // 2 + 1
        y = torch.empty(N, P, Q, C, dtype=dt, device=dev)
        am = torch.empty(N, P, Q, C, dtype=torch.uint8, device=dev)
        if apply:
            L.call("mmdx_maxpool_fwd", dc, a.data_ptr(), N, H, W, C, 3, 2, pad, y.data_ptr(),
                   am.data_ptr(), P, Q, L.stream())
        else:
            L.call("mmdx_maxpool_bn_fwd", dc, x.data_ptr(), N, H, W, C, 3, 2, pad,
                   gam.data_ptr(), bet.data_ptr(), mean.data_ptr(), rstd.data_ptr(), 1,
                   y.data_ptr(), am.data_ptr(), P, Q, L.stream())
        outs.append((y, am, mean, rstd, rm, rv))
    torch.cuda.synchronize()
    for u, v, name in zip(outs[0], outs[1], ("pooled", "argmax", "mean", "rstd", "rm", "rv")):
        assert torch.equal(u, v), name
    assert (outs[0][0] == 0).any()  # all-zero windows: a nine-way tie after the ReLU

    # backward: mmdx_bn_bwd_pool (pool gradient gathered inside the BN backward) equals
    # mmdx_maxpool_bwd + mmdx_bn_bwd (ReLU mask from x) bit for bit
    y, am, mean, rstd = outs[1][:4]
    dyp = torch.randn(y.shape, generator=g).to(dev, dt)
    da = torch.empty_like(x)
    L.call("mmdx_maxpool_bwd", dc, am.data_ptr(), dyp.data_ptr(), N, H, W, C, 3, 2, pad, P, Q,
           da.data_ptr(), L.stream())
    res = []
    for fused in (False, True):
        dx = torch.empty_like(x)
        dg, db = torch.empty(C, device=dev), torch.empty(C, device=dev)
        if fused:
            L.call("mmdx_bn_bwd_pool", dc, 1, x.data_ptr(), am.data_ptr(), dyp.data_ptr(), N, H,
                   W, C, 3, 2, pad, P, Q, gam.data_ptr(), bet.data_ptr(), mean.data_ptr(),
                   rstd.data_ptr(), 1, dx.data_ptr(), dg.data_ptr(), db.data_ptr(), 0.0,
                   ws.data_ptr(), ws_n, L.stream())
        else:
            L.call("mmdx_bn_bwd", dc, 1, x.data_ptr(), None, da.data_ptr(), rows, C,
                   gam.data_ptr(), bet.data_ptr(), mean.data_ptr(), rstd.data_ptr(), 1, None, 0,
                   dx.data_ptr(), None, dg.data_ptr(), db.data_ptr(), 0.0, ws.data_ptr(), ws_n,
                   L.stream())
        res.append((dx, dg, db))
    torch.cuda.synchronize()
    for u, v, name in zip(res[0], res[1], ("dx", "dgamma", "dbeta")):
        assert torch.equal(u, v), name
    assert res[0][0].abs().sum() > 0


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_layernorm_bce_gelu(dev, dt):
    g = torch.Generator().manual_seed(5)
    rows, D = 70, 1024
    x = torch.randn(rows, D, generator=g) + 3.0
    res = torch.randn(rows, D, generator=g)
    ln = torch.nn.LayerNorm(D)
    with torch.no_grad():
        ln.weight.uniform_(0.5, 1.5, generator=g)
        ln.bias.uniform_(-1, 1, generator=g)
    if dt == torch.bfloat16:
        x, res = x.bfloat16().float(), res.bfloat16().float()
    xr = x.clone().requires_grad_(True)
    yr = ln(xr + res)
    dy = torch.randn(yr.shape, generator=g)
    yr.backward(dy)
    xd = x.to(dev, dt).requires_grad_(True)
    y = F.layer_norm(xd, ln.weight.detach().to(dev), ln.bias.detach().to(dev), 1e-5,
                     residual=res.to(dev, dt))
    _close(y, yr.detach(), dt, "ln fwd")
    y.backward(dy.to(dev, dt))
    _close(xd.grad, xr.grad, dt, "ln dx")
    # BCE
    z = torch.randn(16, 13, generator=g) * 4
    t = (torch.rand(16, 13, generator=g) < 0.15).float()
    zr = z.clone().requires_grad_(True)
    lr_ = tF.binary_cross_entropy_with_logits(zr, t)
    lr_.backward()
    zd = z.to(dev).requires_grad_(True)
    loss = F.bce_with_logits(zd, t.to(dev))
    loss.backward()
    assert abs(loss.item() - lr_.item()) <= 1e-6 * max(1, abs(lr_.item()))
    _close(zd.grad, zr.grad, torch.float32, "bce grad")


def test_adamw_matches_torch(dev):
    g = torch.Generator().manual_seed(6)
    shapes = [(1024, 1536), (1024,), (13, 1024), (13,), (7, 3, 5)]
    ps = [torch.randn(s, generator=g) for s in shapes]
    ref = [p.clone().requires_grad_(True) for p in ps]
    mine = [torch.nn.Parameter(p.to(dev)) for p in ps]
    o_ref = torch.optim.AdamW([{"params": ref[:2], "lr": 5e-4},
                               {"params": ref[2:], "lr": 1e-3}], weight_decay=1e-2)
    o_mine = mmdx.AdamW([{"params": mine[:2], "lr": 5e-4}, {"params": mine[2:], "lr": 1e-3}],
                        weight_decay=1e-2)
    for step in range(3):
        grads = [torch.randn(s, generator=g) for s in shapes]
        for p, gr in zip(ref, grads):
            p.grad = gr.clone()
        for p, gr in zip(mine, grads):
            p.grad = gr.to(dev)
        torch.nn.utils.clip_grad_norm_(ref, 1.0)
        mmdx.clip_grad_norm_(mine, 1.0)
        o_ref.step()
        o_mine.step()
    for a, b in zip(mine, ref):
        assert torch.allclose(a.detach().cpu(), b.detach(), rtol=1e-5, atol=1e-6)


def test_adamw_moving_grads_many_tensors(dev):
    """The per-step gradient column refresh (mmdx_adamw_patch_grads, 256 pointers per
    launch): 300 tensors whose gradient buffers move on some steps and stay on others, with
    an lr change in between (whole-table re-upload) — every step equals torch.optim.AdamW."""
    g = torch.Generator().manual_seed(11)
    shapes = [(int(n),) for n in torch.randint(1, 3000, (300,), generator=g)] + [(70000,)]
    ps = [torch.randn(s, generator=g) for s in shapes]
    ref = [p.clone().requires_grad_(True) for p in ps]
    mine = [torch.nn.Parameter(p.to(dev)) for p in ps]
    o_ref = torch.optim.AdamW([{"params": ref[:150], "lr": 5e-4},
                               {"params": ref[150:], "lr": 1e-3}], weight_decay=1e-2)
    o_mine = mmdx.AdamW([{"params": mine[:150], "lr": 5e-4}, {"params": mine[150:], "lr": 1e-3}],
                        weight_decay=1e-2)
    for step in range(5):
        grads = [torch.randn(s, generator=g) for s in shapes]
        for p, gr in zip(ref, grads):
            p.grad = gr.clone()
        if step == 2:   # same device buffers as the previous step: no refresh needed
            for p, gr in zip(mine, grads):
                p.grad.copy_(gr)
        else:
            for p, gr in zip(mine, grads):
                p.grad = gr.to(dev)
        if step == 3:
            for o in (o_ref, o_mine):
                o.param_groups[1]["lr"] = 2e-4
        norm_ref = torch.nn.utils.clip_grad_norm_(ref, 1.0)
        norm = mmdx.clip_grad_norm_(mine, 1.0)
        assert abs(float(norm) - float(norm_ref)) <= 1e-5 * float(norm_ref)
        o_ref.step()
        o_mine.step()
        for a, b in zip(mine, ref):
            assert torch.allclose(a.detach().cpu(), b.detach(), rtol=1e-5, atol=1e-6), step


def test_adamw_state_roundtrip_and_lr_change(dev):
    """the fused AdamW must follow torch.optim.AdamW across (i) a
    state_dict() -> load_state_dict() into a NEW optimizer (new exp_avg / exp_avg_sq storage,
    step restored) and (ii) an lr / weight-decay change through param_groups mid-run."""
    g = torch.Generator().manual_seed(9)
    shapes = [(300, 70), (70,), (5, 3)]
    ps = [torch.randn(s, generator=g) for s in shapes]
    ref = [p.clone().requires_grad_(True) for p in ps]
    mine = [torch.nn.Parameter(p.to(dev)) for p in ps]
    o_ref = torch.optim.AdamW([{"params": ref[:2], "lr": 5e-4}, {"params": ref[2:], "lr": 1e-3}],
                              weight_decay=1e-2)
    o_mine = mmdx.AdamW([{"params": mine[:2], "lr": 5e-4}, {"params": mine[2:], "lr": 1e-3}],
                        weight_decay=1e-2)

    def step(o_r, o_m):
        grads = [torch.randn(s, generator=g) for s in shapes]
        for p, gr in zip(ref, grads):
            p.grad = gr.clone()
        for p, gr in zip(mine, grads):
            p.grad = gr.to(dev)
        o_r.step()
        o_m.step()

    for _ in range(2):
        step(o_ref, o_mine)
    import io
    buf = io.BytesIO()
    torch.save(o_mine.state_dict(), buf)   # a checkpoint: fresh storage on load
    buf.seek(0)
    sd = torch.load(buf, weights_only=True)
    o_mine2 = mmdx.AdamW([{"params": mine[:2], "lr": 5e-4}, {"params": mine[2:], "lr": 1e-3}],
                         weight_decay=1e-2)
    o_mine2.load_state_dict(sd)
    for st in o_mine2.state.values():   # the loaded moments are new storage
        assert all(st[k].data_ptr() != o_mine.state[p][k].data_ptr()
                   for p in mine if p in o_mine.state for k in ("exp_avg",))
    step(o_ref, o_mine2)
    for gr_r, gr_m in zip(o_ref.param_groups, o_mine2.param_groups):
        gr_r["lr"] *= 0.5
        gr_m["lr"] *= 0.5
        gr_r["weight_decay"] = gr_m["weight_decay"] = 0.05
    for _ in range(2):
        step(o_ref, o_mine2)
    for a, b in zip(mine, ref):
        assert torch.allclose(a.detach().cpu(), b.detach(), rtol=1e-5, atol=1e-6)
    assert float(o_mine2.state[mine[0]]["step"].item()) == 5.0


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_dropout_counter_rng_and_graph_replay(dev, dt):
    """nn.Dropout semantics (TP:538): keep rate 1-p, kept values scaled by 1/(1-p), backward
    = dy * mask / (1-p); the device counter gives a fresh mask on every call, also when the
    launch is replayed from a captured graph."""
    from mmdx import functional as F
    n, p = 1 << 18, 0.1
    x = torch.ones(n, dtype=dt, device=dev)
    y1 = F.dropout(x, p, True)
    y2 = F.dropout(x, p, True)
    keep = (y1 != 0).float().mean().item()
    assert abs(keep - (1 - p)) < 0.005
    kept = y1[y1 != 0].float()
    assert torch.allclose(kept, torch.full_like(kept, 1 / (1 - p)), rtol=1e-2 if dt != torch.float32 else 1e-6)
    assert not torch.equal(y1 != 0, y2 != 0)
    xr = torch.randn(n, dtype=torch.float32, device=dev).to(dt).requires_grad_(True)
    yr = F.dropout(xr, p, True)
    dy = torch.randn(n, dtype=torch.float32, device=dev).to(dt)
    yr.backward(dy)
    m = (yr != 0) | (xr == 0)
    ref = torch.where(m, dy.float() / (1 - p), torch.zeros_like(dy.float()))
    assert torch.allclose(xr.grad.float(), ref, rtol=1e-2 if dt != torch.float32 else 1e-6, atol=1e-6)
    # graph capture: two replays, two different masks
    static_x = torch.ones(n, dtype=dt, device=dev)
    F.dropout(static_x, p, True)  # warm up allocations
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        static_y = F.dropout(static_x, p, True)
    g.replay()
    m1 = (static_y != 0).clone()
    g.replay()
    m2 = (static_y != 0).clone()
    assert not torch.equal(m1, m2)
    assert abs(m2.float().mean().item() - (1 - p)) < 0.005


@pytest.mark.parametrize("cfg,mode", [
    ((2, 14, 14, 64, 64, 3, 1), "plain"), ((2, 9, 7, 64, 128, 1, 1), "plain"),
    ((3, 15, 13, 64, 128, 3, 2), "plain"), ((2, 28, 28, 128, 64, 3, 2), "plain"),
    ((2, 9, 7, 64, 128, 1, 1), "residual"), ((3, 15, 13, 256, 64, 1, 1), "residual"),
    ((2, 14, 14, 64, 64, 3, 1), "residual")])
def test_dgrad_fused_bn_stats(dev, cfg, mode):
    """dgrad with the consumer BN's backward statistics in its epilogue, then mmdx_bn_bwd on
    those partials == dgrad, then mmdx_bn_bwd with its own reduce pass (bf16; ragged row
    counts; stride 2 runs as output phases).  "residual": the dgrad accumulates onto the
    identity-path gradient (beta = 1) and the consumer is a residual unit whose ReLU mask is
    its output `out` (the bottleneck conv1 -> previous block's conv3 case).  Only the
    summation order differs."""
    N, H, W, C, K, k, s = cfg
    p = k // 2
    dt = torch.bfloat16
    dc = L.dtype_code(dt)
    g = torch.Generator().manual_seed(11)
    P, Q = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
    d = L.ConvDesc(N, H, W, C, K, k, k, s, s, p, p, P, Q)
    tiles = L.lib().mmdx_conv_dgrad_stat_blocks(dc, d)
    assert tiles > 0
    w = (torch.randn(K, C, k, k, generator=g) * 0.1).to(dev)
    wk = torch.empty(K, k, k, C, dtype=dt, device=dev)
    wc = torch.empty(C, k, k, K, dtype=dt, device=dev)
    L.call("mmdx_conv_pack_weight", dc, d, C, w.data_ptr(), wk.data_ptr(), wc.data_ptr(),
           L.stream())
    dy = torch.randn(N, P, Q, K, generator=g).to(dev, dt)
    y = torch.randn(N, H, W, C, generator=g).to(dev, dt)       # BN input of the consumer
    gam = (torch.rand(C, generator=g) + 0.5).to(dev)
    bet = (torch.randn(C, generator=g) * 0.1).to(dev)
    mean = (torch.randn(C, generator=g) * 0.1).to(dev)
    rstd = (torch.rand(C, generator=g) + 0.5).to(dev)
    rows = N * H * W
    residual = mode == "residual"
    beta = 1.0 if residual else 0.0
    out = torch.randn(N, H, W, C, generator=g).clamp(min=0).to(dev, dt) if residual else None
    dx0 = torch.randn(N, H, W, C, generator=g).to(dev, dt)     # identity-path gradient
    dx_a = dx0.clone()
    part = torch.empty(C, tiles, 2, device=dev)
    L.call("mmdx_conv_dgrad_bnstat", dc, d, dy.data_ptr(), wc.data_ptr(), dx_a.data_ptr(), beta,
           y.data_ptr(), L.ptr(out), gam.data_ptr(), bet.data_ptr(), mean.data_ptr(),
           rstd.data_ptr(), 1, part.data_ptr(), L.stream())
    dx_b = dx0.clone()
    L.call("mmdx_conv_dgrad", dc, d, dy.data_ptr(), wc.data_ptr(), dx_b.data_ptr(), beta,
           L.stream())
    torch.cuda.synchronize()
    assert torch.equal(dx_a, dx_b)
    ws_n = L.lib().mmdx_bn_workspace_size(rows, C)
    ws = torch.empty(ws_n, dtype=torch.uint8, device=dev)
    outs = []
    for sp, nb in ((part, tiles), (None, 0)):
        dcv = torch.empty_like(y)
        dg = torch.empty(C, device=dev)
        db = torch.empty(C, device=dev)
        L.call("mmdx_bn_bwd", dc, 1, y.data_ptr(), L.ptr(out), dx_a.data_ptr(), rows, C,
               gam.data_ptr(), bet.data_ptr(), mean.data_ptr(), rstd.data_ptr(), 1,
               L.ptr(sp), nb, dcv.data_ptr(), None, dg.data_ptr(), db.data_ptr(), 0.0,
               ws.data_ptr(), ws_n, L.stream())
        outs.append((dcv.float(), dg, db))
    torch.cuda.synchronize()
    (ca, ga, ba), (cb, gb, bb) = outs
    assert (ga - gb).abs().max().item() <= 1e-4 * max(1.0, gb.abs().max().item())
    assert (ba - bb).abs().max().item() <= 1e-4 * max(1.0, bb.abs().max().item())
    assert (ca - cb).abs().max().item() <= 2e-2 * max(1.0, cb.abs().max().item())


def test_dgrad_bnstat_rejects_strided_accumulation(dev):
    d = L.ConvDesc(2, 16, 16, 64, 64, 3, 3, 2, 2, 1, 1, 8, 8)
    z = torch.zeros(1 << 20, dtype=torch.bfloat16, device=dev)
    f = torch.zeros(1 << 16, device=dev)
    with pytest.raises(RuntimeError, match="stride-1"):
        L.call("mmdx_conv_dgrad_bnstat", 1, d, z.data_ptr(), z.data_ptr(), z.data_ptr(), 1.0,
               z.data_ptr(), None, f.data_ptr(), f.data_ptr(), f.data_ptr(), f.data_ptr(), 1,
               f.data_ptr(), L.stream())

STEMS = [  # N, C, H, W, K, k, s, p  (C = image channels, NCHW fp32 input)
    (2, 3, 32, 32, 64, 7, 2, 3),
    (3, 3, 37, 30, 64, 7, 2, 3),   # ragged: odd H, M not a multiple of 128
    (1, 1, 20, 20, 32, 7, 2, 3),   # grayscale
    (2, 3, 16, 18, 64, 3, 2, 1),   # even kernel half-width: S2 = 2
    (1, 3, 224, 224, 64, 7, 2, 3),  # the ResNet stem at full resolution
]


@pytest.mark.parametrize("cfg", STEMS)
@pytest.mark.parametrize("beta", [0.0, 1.0])
def test_stem_pixel_pair_conv(dev, cfg, beta):
    """backbone.0 (TP:183) as a conv over pixel pairs (mmdx_stem_pair_*: zero-bordered
    [N][H+2p][(W+2p)/2][8] image, stride (2,1) R x ceil(S/2) conv on the generic kernels) vs
    torch conv2d fp32 on the bf16-rounded operands: fwd, BN epilogue stats, wgrad."""
    dt = torch.bfloat16
    N, C, H, W, K, k, s, p = cfg
    g = torch.Generator().manual_seed(7 + sum(cfg))
    x = torch.randn(N, C, H, W, generator=g)
    w = torch.randn(K, C, k, k, generator=g) * 0.1
    xb, wb = x.bfloat16().float(), w.bfloat16().float()
    wr = wb.clone().requires_grad_(True)
    yr = tF.conv2d(xb, wr, stride=s, padding=p)
    dy = torch.randn(yr.shape, generator=g).bfloat16().float()
    yr.backward(dy)
    d = L.ConvDesc()
    L.call("mmdx_stem_pair_desc", N, C, H, W, K, k, k, s, p, d)
    assert (d.P, d.Q, d.C, d.S) == (yr.shape[2], yr.shape[3], 8, (k + 1) // 2)
    xd = x.to(dev).contiguous()
    xp = torch.empty(N, d.H, d.W, 8, dtype=dt, device=dev)
    L.call("mmdx_stem_pair_input", xd.data_ptr(), N, C, H, W, p, xp.data_ptr(), L.stream())
    ref_pad = tF.pad(xb, (p, p, p, p))  # [N,C,H+2p,W+2p] -> pairs of pixels x 4 channels
    ref_pair = torch.zeros(N, d.H, 2 * d.W, 4)
    ref_pair[..., :C] = ref_pad.permute(0, 2, 3, 1)
    assert torch.equal(xp.float().cpu(), ref_pair.reshape(N, d.H, d.W, 8))
    wp = torch.empty(K, d.R, d.S, 8, dtype=dt, device=dev)
    L.call("mmdx_stem_pair_pack_weight", w.to(dev).data_ptr(), K, C, k, k, wp.data_ptr(),
           L.stream())
    y = torch.empty(N, d.P, d.Q, K, dtype=dt, device=dev)
    nst = L.lib().mmdx_conv_fwd_stat_blocks(d)
    part = torch.empty(K, nst, 2, device=dev)
    L.call("mmdx_conv_fwd", 1, d, xp.data_ptr(), wp.data_ptr(), y.data_ptr(), part.data_ptr(),
           L.stream())
    _close(y.permute(0, 3, 1, 2), yr.detach(), dt, f"stem fwd {cfg}")
    M = N * d.P * d.Q
    rpb = L.lib().mmdx_conv_fwd_stat_rows(d)  # 128, or a direct-stem block's rows
    assert nst == (M + rpb - 1) // rpb
    cnt = torch.tensor([min(rpb, M - rpb * b) for b in range(nst)], dtype=torch.float64)
    pm, p2 = part[..., 0].t().double().cpu(), part[..., 1].t().double().cpu()
    mean = (pm * cnt[:, None]).sum(0) / M
    m2 = (p2 + cnt[:, None] * (pm - mean) ** 2).sum(0)
    yref = yr.detach().double()
    _close(mean, yref.mean((0, 2, 3)), dt, "stem stat mean")
    _close(m2 / M, yref.var((0, 2, 3), unbiased=False), dt, "stem stat var")
    dyd = dy.permute(0, 2, 3, 1).contiguous().to(dev, dt)
    dwp = torch.empty(K, 8, d.R, d.S, device=dev)
    ws_n = L.lib().mmdx_conv_wgrad_workspace_size(1, d)
    ws = torch.empty(max(1, ws_n), dtype=torch.uint8, device=dev)
    L.call("mmdx_conv_wgrad", 1, d, 8, xp.data_ptr(), dyd.data_ptr(), dwp.data_ptr(), 0.0,
           ws.data_ptr(), ws_n, L.stream())
    dw0 = torch.randn(K, C, k, k, generator=g)
    dw = dw0.to(dev)
    L.call("mmdx_stem_pair_grad", dwp.data_ptr(), K, C, k, k, dw.data_ptr(), beta, L.stream())
    _close(dw, wr.grad + beta * dw0, dt, f"stem wgrad {cfg}")


@pytest.mark.parametrize("cfg", [(2, 3, 32, 32, 64, 7, 2, 3), (3, 3, 64, 96, 64, 7, 2, 3),
                                 (4, 3, 224, 224, 64, 7, 2, 3)])
def test_stem_direct_matches_implicit_gemm(dev, cfg, knobs):
    """The direct stem forward and weight gradient (input rows staged in LDS once, operand
    fragments read from them; MMDX_STEM_DIRECT) against the implicit-GEMM kernels on the same
    pixel-pair operands: the
    same MFMA sequence per output, so y is BIT-IDENTICAL; its BatchNorm partials are per
    block of 2 output rows (mmdx_conv_fwd_stat_rows) and merge to the same per-channel mean
    and variance (fp64 host merge, rel 1e-5)."""
    dt = torch.bfloat16
    N, C, H, W, K, k, s, p = cfg
    g = torch.Generator().manual_seed(11 + sum(cfg))
    x = torch.randn(N, C, H, W, generator=g).to(dev)
    w = (torch.randn(K, C, k, k, generator=g) * 0.1).to(dev)
    d = L.ConvDesc()
    L.call("mmdx_stem_pair_desc", N, C, H, W, K, k, k, s, p, d)
    xp = torch.empty(N, d.H, d.W, 8, dtype=dt, device=dev)
    L.call("mmdx_stem_pair_input", x.data_ptr(), N, C, H, W, p, xp.data_ptr(), L.stream())
    wp = torch.empty(K, d.R, d.S, 8, dtype=dt, device=dev)
    L.call("mmdx_stem_pair_pack_weight", w.data_ptr(), K, C, k, k, wp.data_ptr(), L.stream())
    M = N * d.P * d.Q
    res = {}
    for mode in ("0", "1"):
        knobs("MMDX_STEM_DIRECT", mode)
        rpb = L.lib().mmdx_conv_fwd_stat_rows(d)
        nst = L.lib().mmdx_conv_fwd_stat_blocks(d)
        assert rpb == (128 if mode == "0" else 2 * d.Q)
        y = torch.empty(N, d.P, d.Q, K, dtype=dt, device=dev)
        part = torch.full((K, nst, 2), float("nan"), device=dev)
        L.call("mmdx_conv_fwd", 1, d, xp.data_ptr(), wp.data_ptr(), y.data_ptr(),
               part.data_ptr(), L.stream())
        torch.cuda.synchronize()
        assert torch.isfinite(part).all()
        cnt = torch.tensor([min(rpb, M - rpb * b) for b in range(nst)], dtype=torch.float64)
        pm, p2 = part[..., 0].t().double().cpu(), part[..., 1].t().double().cpu()
        mean = (pm * cnt[:, None]).sum(0) / M
        var = (p2 + cnt[:, None] * (pm - mean) ** 2).sum(0) / M
        res[mode] = (y, mean, var)
    assert torch.equal(res["0"][0], res["1"][0])
    for j in (1, 2):
        a, b = res["0"][j], res["1"][j]
        assert ((a - b).abs() / b.abs().clamp(min=1e-3)).max().item() <= 1e-5, j
    # weight gradient: the direct kernel (whole 2-row pixel tiles per K split, operands read
    # k-major from the staged dy / input rows) sums the same 32-pixel groups in the same order
    # into the same split-K slabs: bit-identical
    dy = torch.randn(N, d.P, d.Q, K, generator=g).to(dev, dt)
    ws_n = L.lib().mmdx_conv_wgrad_workspace_size(1, d)
    ws = torch.empty(max(1, ws_n), dtype=torch.uint8, device=dev)
    dws = {}
    for mode in ("0", "1"):
        knobs("MMDX_STEM_DIRECT", mode)
        dwp = torch.full((K, 8, d.R, d.S), float("nan"), device=dev)
        L.call("mmdx_conv_wgrad", 1, d, 8, xp.data_ptr(), dy.data_ptr(), dwp.data_ptr(), 0.0,
               ws.data_ptr(), ws_n, L.stream())
        torch.cuda.synchronize()
        dws[mode] = dwp
    assert torch.isfinite(dws["1"]).all()
    assert torch.equal(dws["0"], dws["1"])


def test_stem_pixel_pair_rejects_odd_width(dev):
    d = L.ConvDesc()
    with pytest.raises(RuntimeError, match="even padded width"):
        L.call("mmdx_stem_pair_desc", 1, 3, 29, 29, 64, 7, 7, 2, 3, d)


def test_conv_pack_multi_matches_single(dev):
    """mmdx_conv_pack_multi (all trunk weights in one launch) == one mmdx_conv_pack_weight per
    weight, bit for bit, including ragged tiles and a NULL CRSK output."""
    shapes = [(64, 24, 24, 7), (256, 64, 64, 1), (128, 128, 128, 3), (24, 40, 40, 3),
              (2048, 512, 512, 1)]
    g = torch.Generator().manual_seed(3)
    items = (L.PackItem * len(shapes))()
    outs, refs, nb = [], [], 0
    for j, (K, cm, C, k) in enumerate(shapes):
        w = (torch.randn(K, cm, k, k, generator=g)).to(dev)
        wk = torch.empty(K, k, k, C, dtype=torch.bfloat16, device=dev)
        wc = torch.empty(C, k, k, K, dtype=torch.bfloat16, device=dev) if j != 1 else None
        items[j] = L.PackItem(w.data_ptr(), wk.data_ptr(),
                              wc.data_ptr() if wc is not None else None, K, C, cm, k * k, nb)
        nb += L.lib().mmdx_conv_pack_blocks(K, C, k * k)
        d = L.ConvDesc(1, 8, 8, C, K, k, k, 1, 1, k // 2, k // 2, 8, 8)
        rk = torch.empty_like(wk)
        rc = torch.empty_like(wc) if wc is not None else None
        L.call("mmdx_conv_pack_weight", 1, d, cm, w.data_ptr(), rk.data_ptr(),
               rc.data_ptr() if rc is not None else None, L.stream())
        outs.append((w, wk, wc))
        refs.append((rk, rc))
    raw = torch.frombuffer(bytearray(bytes(items)), dtype=torch.uint8).to(dev)
    L.call("mmdx_conv_pack_multi", 1, raw.data_ptr(), len(shapes), nb, L.stream())
    torch.cuda.synchronize()
    for (w, wk, wc), (rk, rc) in zip(outs, refs):
        assert torch.equal(wk, rk)
        if wc is not None:
            assert torch.equal(wc, rc)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("cfg,res,relu", [((2, 64, 14, 14, 256, 1, 1, 0), True, True),
                                          ((3, 64, 15, 15, 64, 3, 2, 1), False, True),
                                          ((2, 128, 9, 9, 512, 3, 1, 1), True, False)])
def test_conv_fwd_bn_eval(dev, dt, cfg, res, relu):
    """Eval-mode conv + BatchNorm (running stats) (+residual) (+ReLU) in one launch
    (mmdx_conv_fwd_bn_eval) vs torch: relu(bn_eval(conv(x, w)) + res)."""
    N, C, H, W, K, k, s, p = cfg
    g = torch.Generator().manual_seed(sum(cfg) + res)
    x = torch.randn(N, C, H, W, generator=g)
    w = torch.randn(K, C, k, k, generator=g) * 0.1
    gamma, beta = torch.randn(K, generator=g), torch.randn(K, generator=g)
    rm, rv = torch.randn(K, generator=g) * 0.3, torch.rand(K, generator=g) + 0.5
    if dt == torch.bfloat16:
        x, w = x.bfloat16().float(), w.bfloat16().float()
    y = tF.conv2d(x, w, stride=s, padding=p)
    y = tF.batch_norm(y, rm, rv, gamma, beta, training=False, eps=1e-5)
    P, Q = y.shape[2], y.shape[3]
    r = torch.randn(N, K, P, Q, generator=g)
    if dt == torch.bfloat16:
        r = r.bfloat16().float()
    if res:
        y = y + r
    if relu:
        y = y.clamp(min=0)
    d = L.ConvDesc(N, H, W, C, K, k, k, s, s, p, p, P, Q)
    dc = L.dtype_code(dt)
    wk = torch.empty(K, k, k, C, dtype=dt, device=dev)
    wc = torch.empty(C, k, k, K, dtype=dt, device=dev)
    L.call("mmdx_conv_pack_weight", dc, d, C, w.to(dev).data_ptr(), wk.data_ptr(),
           wc.data_ptr(), L.stream())
    xd = x.permute(0, 2, 3, 1).contiguous().to(dev, dt)
    rd = r.permute(0, 2, 3, 1).contiguous().to(dev, dt)
    out = torch.empty(N, P, Q, K, dtype=dt, device=dev)
    bn = [t.to(dev) for t in (gamma, beta, rm, rv)]
    L.call("mmdx_conv_fwd_bn_eval", dc, d, xd.data_ptr(), wk.data_ptr(), out.data_ptr(),
           *[t.data_ptr() for t in bn], 1e-5, rd.data_ptr() if res else None, int(relu),
           L.stream())
    _close(out.permute(0, 3, 1, 2), y, dt, f"bn-eval {cfg}")


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_bn_relu_bitmask(dev, dt):
    """A residual unit's BN backward reading the forward's 1-bit ReLU mask
    (mmdx_bn_fwd_ex / mmdx_bn_bwd_ex) equals the one reading the unit's output, bit for bit,
    including elements that are exactly zero after the residual add."""
    g = torch.Generator().manual_seed(5)
    rows, C = 3000, 64
    x = torch.randn(rows, C, generator=g).to(dev, dt)
    r = torch.randn(rows, C, generator=g)
    r[:100] = 0.0
    r = r.to(dev, dt)
    dy = torch.randn(rows, C, generator=g).to(dev, dt)
    gam = (torch.rand(C, generator=g) + 0.5).to(dev)
    bet = (torch.randn(C, generator=g) * 0.1).to(dev)
    dc = L.dtype_code(dt)
    vec = 4 if dt == torch.float32 else 8
    ws_n = L.lib().mmdx_bn_workspace_size(rows, C)
    ws = torch.empty(ws_n, dtype=torch.uint8, device=dev)
    mean, rstd = torch.empty(C, device=dev), torch.empty(C, device=dev)
    rm, rv = torch.zeros(C, device=dev), torch.ones(C, device=dev)
    y = torch.empty_like(x)
    mask = torch.empty(rows, C // vec, dtype=torch.uint8, device=dev)
    L.call("mmdx_bn_fwd_ex", dc, 1, x.data_ptr(), rows, C, None, 0, 0, gam.data_ptr(),
           bet.data_ptr(), rm.data_ptr(), rv.data_ptr(), 0.1, 1e-5, mean.data_ptr(),
           rstd.data_ptr(), r.data_ptr(), 1, y.data_ptr(), mask.data_ptr(), ws.data_ptr(), ws_n,
           L.stream())
    bits = ((y.view(rows, C // vec, vec).float() > 0).to(torch.int32)
            << torch.arange(vec, device=dev, dtype=torch.int32)).sum(-1)
    assert torch.equal(mask.to(torch.int32), bits)
    outs = []
    for use_mask in (False, True):
        dx, dres = torch.empty_like(x), torch.empty_like(x)
        dgm, dbt = torch.empty(C, device=dev), torch.empty(C, device=dev)
        L.call("mmdx_bn_bwd_ex", dc, 1, x.data_ptr(), None if use_mask else y.data_ptr(),
               dy.data_ptr(), rows, C, gam.data_ptr(), bet.data_ptr(), mean.data_ptr(),
               rstd.data_ptr(), 1, None, 0, dx.data_ptr(), dres.data_ptr(), dgm.data_ptr(),
               dbt.data_ptr(), 0.0, mask.data_ptr() if use_mask else None, ws.data_ptr(), ws_n,
               L.stream())
        outs.append((dx, dres, dgm, dbt))
    torch.cuda.synchronize()
    for u, v, name in zip(outs[0], outs[1], ("dx", "dres", "dgamma", "dbeta")):
        assert torch.equal(u, v), name


@pytest.mark.parametrize("cfg", [(2, 256, 14, 14, 64, 1, 1, 0), (4, 64, 56, 56, 64, 1, 1, 0),
                                 (2, 128, 9, 9, 128, 3, 1, 1)])
def test_conv_dgrad_accmask(dev, cfg):
    """dgrad + (ReLU bit ? acc_src : 0) in the epilogue (mmdx_conv_dgrad_accmask) equals a
    beta-1 dgrad onto the masked source, bit for bit (the identity block's conv1 dgrad)."""
    dt = torch.bfloat16
    N, C, H, W, K, k, s, p = cfg
    g = torch.Generator().manual_seed(sum(cfg))
    d = L.ConvDesc(N, H, W, C, K, k, k, s, s, p, p, H, W)
    dc = L.dtype_code(dt)
    wm = (torch.randn(K, C, k, k, generator=g) * 0.1).to(dev)
    wk = torch.empty(K, k, k, C, dtype=dt, device=dev)
    wc = torch.empty(C, k, k, K, dtype=dt, device=dev)
    L.call("mmdx_conv_pack_weight", dc, d, C, wm.data_ptr(), wk.data_ptr(), wc.data_ptr(),
           L.stream())
    dy = torch.randn(N, H, W, K, generator=g).to(dev, dt)
    src = torch.randn(N, H, W, C, generator=g).to(dev, dt)
    pos = torch.rand(N, H, W, C, generator=g) > 0.5
    bits = (pos.view(-1, C // 8, 8).to(torch.int32) << torch.arange(8, dtype=torch.int32)).sum(-1)
    mask = bits.to(torch.uint8).to(dev)
    ref = torch.where(pos.to(dev), src, torch.zeros_like(src))
    L.call("mmdx_conv_dgrad", dc, d, dy.data_ptr(), wc.data_ptr(), ref.data_ptr(), 1.0,
           L.stream())
    got = torch.empty_like(src)
    L.call("mmdx_conv_dgrad_accmask", dc, d, dy.data_ptr(), wc.data_ptr(), got.data_ptr(),
           src.data_ptr(), mask.data_ptr(), L.stream())
    torch.cuda.synchronize()
    assert torch.equal(got, ref)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_bn_bwd_masked_dy(dev, dt):
    """A downsample BN's backward reading its upstream gradient as dy + 1-bit ReLU mask
    (mmdx_bn_bwd_masked_dy) equals mmdx_bn_bwd on the materialised masked dy, bit for bit."""
    g = torch.Generator().manual_seed(9)
    rows, C = 2500, 128
    vec = 4 if dt == torch.float32 else 8
    x = torch.randn(rows, C, generator=g).to(dev, dt)
    dy = torch.randn(rows, C, generator=g).to(dev, dt)
    pos = torch.rand(rows, C, generator=g) > 0.4
    bits = (pos.view(rows, C // vec, vec).to(torch.int32)
            << torch.arange(vec, dtype=torch.int32)).sum(-1)
    mask = bits.to(torch.uint8).to(dev)
    dym = torch.where(pos.to(dev), dy, torch.zeros_like(dy))
    gam = (torch.rand(C, generator=g) + 0.5).to(dev)
    bet = (torch.randn(C, generator=g) * 0.1).to(dev)
    dc = L.dtype_code(dt)
    ws_n = L.lib().mmdx_bn_workspace_size(rows, C)
    ws = torch.empty(ws_n, dtype=torch.uint8, device=dev)
    mean, rstd = torch.empty(C, device=dev), torch.empty(C, device=dev)
    y = torch.empty_like(x)
    L.call("mmdx_bn_fwd", dc, 1, x.data_ptr(), rows, C, None, 0, 0, gam.data_ptr(),
           bet.data_ptr(), None, None, 0.1, 1e-5, mean.data_ptr(), rstd.data_ptr(), None, 0,
           y.data_ptr(), ws.data_ptr(), ws_n, L.stream())
    outs = []
    for masked in (False, True):
        dx = torch.empty_like(x)
        dgm, dbt = torch.empty(C, device=dev), torch.empty(C, device=dev)
        if masked:
            L.call("mmdx_bn_bwd_masked_dy", dc, 1, x.data_ptr(), dy.data_ptr(), mask.data_ptr(),
                   rows, C, gam.data_ptr(), bet.data_ptr(), mean.data_ptr(), rstd.data_ptr(),
                   dx.data_ptr(), dgm.data_ptr(), dbt.data_ptr(), 0.0, ws.data_ptr(), ws_n,
                   L.stream())
        else:
            L.call("mmdx_bn_bwd", dc, 1, x.data_ptr(), None, dym.data_ptr(), rows, C,
                   gam.data_ptr(), bet.data_ptr(), mean.data_ptr(), rstd.data_ptr(), 0, None, 0,
                   dx.data_ptr(), None, dgm.data_ptr(), dbt.data_ptr(), 0.0, ws.data_ptr(), ws_n,
                   L.stream())
        outs.append((dx, dgm, dbt))
    torch.cuda.synchronize()
    for u, v, name in zip(outs[0], outs[1], ("dx", "dgamma", "dbeta")):
        assert torch.equal(u, v), name
