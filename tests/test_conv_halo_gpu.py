"""GPU: the halo-band A operand (DmaHalo) of the same-size stride-1 convs over 64 channels
(ResNet layer1's 3x3 forward, C = 64, and its stride-1 dgrad, K = 64), switched by
MMDX_CONV_HALO on the 256 x 64 8-wave tiles (MMDX_CONV_N64_WIDE=5) and the 128 x 64 4-wave
tiles (MMDX_CONV_N64_WIDE=0, C2's layer1).

The band holds exactly the input pixels the per-tap DmaK gather would DMA (same values, zeros
where a tap leaves the image, same k order and MFMA sequence per output), so every output —
forward, BN statistics slabs, eval-mode fused BN, dgrad with beta 0 / 1, the masked
accumulation and the fused consumer-BN partials — must be BIT-IDENTICAL to the gather kernel.
Shapes cover ragged M (not a multiple of 256), blocks spanning several small images (W 20),
a 5x5 filter, and a geometry whose band does not fit (W 90: the gather path runs).
The forward and dgrad are also checked against fp64 torch on the same bf16 operands.
(reference: the trunk's conv2 of every layer1 Bottleneck, TP:183 via torchvision resnet50)
"""
import pytest
import torch

from test_conv8_gpu import _run_all

pytestmark = pytest.mark.gpu

SHAPES = [  # N, C, H, W, K, k, s, p
    (8, 64, 56, 56, 64, 3, 1, 1),
    (3, 64, 56, 56, 64, 3, 1, 1),
    (5, 64, 20, 20, 64, 3, 1, 1),
    (4, 64, 20, 20, 64, 5, 1, 2),
    (2, 64, 90, 90, 64, 3, 1, 1),
]


@pytest.mark.parametrize("halo", ["1", "3", "4"])
@pytest.mark.parametrize("wide", ["5", "0"])
@pytest.mark.parametrize("cfg", SHAPES)
def test_halo_band_matches_gather(dev, cfg, wide, halo, monkeypatch):
    """MMDX_CONV_HALO = 1 / 3 / 4: 2 / 3 / 4 weight-operand stages (256-row tiles)."""
    if wide == "0" and halo != "1":
        pytest.skip("the 128 x 64 halo tiles take the stage count of the gather kernel")
    monkeypatch.setenv("MMDX_CONV_N64_WIDE", wide)
    monkeypatch.setenv("MMDX_CONV_HALO", "0")
    a = _run_all(dev, cfg, "0", monkeypatch)
    monkeypatch.setenv("MMDX_CONV_HALO", halo)
    b = _run_all(dev, cfg, "0", monkeypatch)
    for key in a:
        assert torch.isfinite(b[key].float()).all(), key
        assert torch.equal(a[key], b[key]), key


@pytest.mark.parametrize("wide", ["5", "0"])
@pytest.mark.parametrize("cfg", SHAPES[:4])
def test_halo_band_vs_fp64(dev, cfg, wide, monkeypatch):
    from mmdx import _lib as L
    monkeypatch.setenv("MMDX_CONV_N64_WIDE", wide)
    monkeypatch.setenv("MMDX_CONV_HALO", "1")
    N, C, H, W, K, k, s, p = cfg
    dt = torch.bfloat16
    P, Q = H, W
    d = L.ConvDesc(N, H, W, C, K, k, k, s, s, p, p, P, Q)
    g = torch.Generator().manual_seed(7 + sum(cfg))
    w = (torch.randn(K, C, k, k, generator=g) * 0.05).to(dt).float()
    wd = w.to(dev)
    wk = torch.empty(K, k, k, C, dtype=dt, device=dev)
    wc = torch.empty(C, k, k, K, dtype=dt, device=dev)
    L.call("mmdx_conv_pack_weight", 1, d, C, wd.data_ptr(), wk.data_ptr(), wc.data_ptr(),
           L.stream())
    x = torch.randn(N, H, W, C, generator=g).to(dt)
    dy = torch.randn(N, P, Q, K, generator=g).to(dt)
    xd, dyd = x.to(dev), dy.to(dev)
    y = torch.empty(N, P, Q, K, dtype=dt, device=dev)
    nst = L.lib().mmdx_conv_fwd_stat_blocks(d)
    part = torch.empty((K, nst, 2), device=dev)
    L.call("mmdx_conv_fwd", 1, d, xd.data_ptr(), wk.data_ptr(), y.data_ptr(), part.data_ptr(),
           L.stream())
    dx = torch.empty(N, H, W, C, dtype=dt, device=dev)
    L.call("mmdx_conv_dgrad", 1, d, dyd.data_ptr(), wc.data_ptr(), dx.data_ptr(), 0.0,
           L.stream())
    torch.cuda.synchronize()
    x64, w64, dy64 = x.double().permute(0, 3, 1, 2), w.double(), dy.double().permute(0, 3, 1, 2)
    y_ref = torch.nn.functional.conv2d(x64, w64, padding=p).permute(0, 2, 3, 1)
    dx_ref = torch.nn.grad.conv2d_input(x64.shape, w64, dy64, padding=p).permute(0, 2, 3, 1)
    # fp32 accumulation of bf16 products, one bf16 rounding of the result: 2^-8 of the value
    # plus the fp32 sum's error (K*C*k*k terms)
    for got, ref in ((y, y_ref), (dx, dx_ref)):
        err = (got.double().cpu() - ref).abs()
        bound = ref.abs() * 2.0 ** -8 + 1e-5 * ref.abs().max()
        assert (err <= bound).all(), (err - bound).max().item()
