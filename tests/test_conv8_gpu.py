"""GPU: the 8-wave 256 x 128 conv kernel (igemm_dma_kernel<256, 128, ..., 512 threads>,
three operand stages) against the 4-wave 128-row kernels, switched by MMDX_CONV8_MIN
(0 = off, 1 = every eligible launch), and the 8-wave weight gradient (MMDX_WGRAD8).

Both kernels accumulate every output over the same K tiles in the same MFMA order, and the
BatchNorm statistics of a 128-row slab merge the same two 64-row wave slices, so the forward
output, the stride-1 and phase-decomposed dgrads, the masked accumulation (accmask) and the
eval-mode fused BN forward must be BIT-IDENTICAL; the per-128-row (mean, M2) slabs agree to
rtol 2e-6 (a tile full in one kernel and ragged in the other merges on another code path).  The fused
consumer-BN partial sums (dgrad_bnstat) are additive: a 256-row tile puts its sums in its
first 128-row slot and zeros in the second, so the per-channel totals must agree to 1e-5
(summation order only).  The weight gradients split K differently (one block per CU vs
two): rel 1e-4.  Ragged M (not a multiple of 256) and strided convs included.
"""
import pytest
import torch

from mmdx import _lib as L

pytestmark = pytest.mark.gpu

SHAPES = [  # N, C, H, W, K, k, s, p
    (4, 128, 28, 28, 128, 3, 1, 1),
    (3, 256, 14, 14, 512, 1, 1, 0),
    (2, 128, 15, 15, 256, 3, 2, 1),
    (2, 256, 14, 14, 1024, 1, 2, 0),
    (8, 64, 28, 28, 128, 3, 1, 1),
]


def _run_all(dev, cfg, mode, monkeypatch):
    monkeypatch.setenv("MMDX_CONV8_MIN", mode)
    monkeypatch.setenv("MMDX_WGRAD8", "0" if mode == "0" else "1")
    N, C, H, W, K, k, s, p = cfg
    dt = torch.bfloat16
    dc = 1
    P, Q = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
    d = L.ConvDesc(N, H, W, C, K, k, k, s, s, p, p, P, Q)
    g = torch.Generator().manual_seed(sum(cfg))
    w = (torch.randn(K, C, k, k, generator=g) * 0.05).to(dev)
    wk = torch.empty(K, k, k, C, dtype=dt, device=dev)
    wc = torch.empty(C, k, k, K, dtype=dt, device=dev)
    L.call("mmdx_conv_pack_weight", dc, d, C, w.data_ptr(), wk.data_ptr(), wc.data_ptr(),
           L.stream())
    x = torch.randn(N, H, W, C, generator=g).to(dev, dt)
    dy = torch.randn(N, P, Q, K, generator=g).to(dev, dt)
    out = {}
    y = torch.empty(N, P, Q, K, dtype=dt, device=dev)
    nst = L.lib().mmdx_conv_fwd_stat_blocks(d)
    part = torch.full((K, nst, 2), float("nan"), device=dev)
    L.call("mmdx_conv_fwd", dc, d, x.data_ptr(), wk.data_ptr(), y.data_ptr(), part.data_ptr(),
           L.stream())
    out["y"], out["stats"] = y, part
    gam = (torch.rand(K, generator=g) + 0.5).to(dev)
    bet = (torch.randn(K, generator=g) * 0.1).to(dev)
    rm = (torch.randn(K, generator=g) * 0.1).to(dev)
    rv = (torch.rand(K, generator=g) + 0.5).to(dev)
    res = torch.randn(N, P, Q, K, generator=g).to(dev, dt)
    ye = torch.empty_like(y)
    L.call("mmdx_conv_fwd_bn_eval", dc, d, x.data_ptr(), wk.data_ptr(), ye.data_ptr(),
           gam.data_ptr(), bet.data_ptr(), rm.data_ptr(), rv.data_ptr(), 1e-5, res.data_ptr(), 1,
           L.stream())
    out["eval"] = ye
    dx0 = torch.randn(N, H, W, C, generator=g).to(dev, dt)
    dx = dx0.clone()
    L.call("mmdx_conv_dgrad", dc, d, dy.data_ptr(), wc.data_ptr(), dx.data_ptr(), 0.0,
           L.stream())
    out["dgrad"] = dx
    if s == 1:
        dxb = dx0.clone()
        L.call("mmdx_conv_dgrad", dc, d, dy.data_ptr(), wc.data_ptr(), dxb.data_ptr(), 1.0,
               L.stream())
        out["dgrad_beta"] = dxb
        pos = torch.rand(N, H, W, C, generator=g) > 0.5
        bits = (pos.view(-1, C // 8, 8).to(torch.int32)
                << torch.arange(8, dtype=torch.int32)).sum(-1)
        mask = bits.to(torch.uint8).to(dev)
        got = torch.empty_like(dx0)
        L.call("mmdx_conv_dgrad_accmask", dc, d, dy.data_ptr(), wc.data_ptr(), got.data_ptr(),
               dx0.data_ptr(), mask.data_ptr(), L.stream())
        out["accmask"] = got
    dw = torch.full((K, C, k, k), 0.25, device=dev)
    ws_n = L.lib().mmdx_conv_wgrad_workspace_size(dc, d)
    ws = torch.empty(ws_n, dtype=torch.uint8, device=dev)
    L.call("mmdx_conv_wgrad", dc, d, C, x.data_ptr(), dy.data_ptr(), dw.data_ptr(), 1.0,
           ws.data_ptr(), ws_n, L.stream())
    out["wgrad"] = dw
    tiles = L.lib().mmdx_conv_dgrad_stat_blocks(dc, d)
    if tiles > 0:
        yb = torch.randn(N, H, W, C, generator=g).to(dev, dt)
        gm = (torch.rand(C, generator=g) + 0.5).to(dev)
        bt = (torch.randn(C, generator=g) * 0.1).to(dev)
        mu = (torch.randn(C, generator=g) * 0.1).to(dev)
        rs = (torch.rand(C, generator=g) + 0.5).to(dev)
        sp = torch.full((C, tiles, 2), float("nan"), device=dev)
        dxs = torch.empty_like(dx0)
        L.call("mmdx_conv_dgrad_bnstat", dc, d, dy.data_ptr(), wc.data_ptr(), dxs.data_ptr(),
               0.0, yb.data_ptr(), None, gm.data_ptr(), bt.data_ptr(), mu.data_ptr(),
               rs.data_ptr(), 1, sp.data_ptr(), L.stream())
        out["bnstat_dx"], out["bnstat_part"] = dxs, sp
    torch.cuda.synchronize()
    return out


@pytest.mark.parametrize("cfg", SHAPES)
def test_conv8_matches_4wave_kernel(dev, cfg, monkeypatch):
    a = _run_all(dev, cfg, "0", monkeypatch)
    b = _run_all(dev, cfg, "1", monkeypatch)
    for key in a:
        if key == "wgrad":  # split boundaries differ (one block per CU vs two): fp32 order
            err = ((a[key] - b[key]).abs().max() / (a[key] - 0.25).abs().max()).item()
            assert err <= 1e-4, (key, err)
            continue
        if key == "stats":
            # the same merges, but a tile that is full in one kernel and ragged in the other
            # (M mod 256 != M mod 128) takes the general-count path there, where the
            # compiler may contract a multiply-add differently: last-bit differences
            assert torch.isfinite(b[key]).all(), "an unwritten statistics slab"
            torch.testing.assert_close(b[key], a[key], rtol=2e-6, atol=1e-6, msg=key)
            continue
        if key == "bnstat_part":
            pa, pb = a[key], b[key]
            assert torch.isfinite(pb).all(), "an unwritten partial slot"
            ta, tb = pa.double().sum(1), pb.double().sum(1)
            err = ((ta - tb).abs().max() / ta.abs().max().clamp(min=1e-12)).item()
            assert err <= 1e-5, (key, err)
            continue
        assert torch.isfinite(b[key].float()).all(), key
        assert torch.equal(a[key], b[key]), key


@pytest.mark.parametrize("ns", ["3", "4", "5"])
@pytest.mark.parametrize("cfg", SHAPES)
def test_bk32_stages_match_bk64(dev, cfg, ns, monkeypatch):
    """MMDX_CONV_BK32 = NS: the forward / stride-1 dgrad tiles with 32-deep K tiles in NS
    stages run the same MFMA sequence per output (k-steps of 32 in the same order, same
    128-row tiles): every output and statistics slab is bit-identical to the 64-deep kernel."""
    monkeypatch.delenv("MMDX_CONV_BK32", raising=False)
    a = _run_all(dev, cfg, "0", monkeypatch)
    monkeypatch.setenv("MMDX_CONV_BK32", ns)
    b = _run_all(dev, cfg, "0", monkeypatch)
    for key in a:
        assert torch.isfinite(b[key].float()).all(), key
        assert torch.equal(a[key], b[key]), key


KNOBS_8W = ["MMDX_CONV_8W128", "MMDX_DGRAD_PHASE_8W", "MMDX_CONV_8W64", "MMDX_WGRAD_8W"]


@pytest.mark.parametrize("knob", KNOBS_8W)
@pytest.mark.parametrize("cfg", SHAPES)
def test_8wave_128row_tiles_match_4wave(dev, cfg, knob, monkeypatch):
    """The 128-row tiles in 8 waves (MMDX_CONV_8W128: 128 x 128 as 2 x 4 waves of 64 x 32, the
    default since round 5; MMDX_DGRAD_PHASE_8W: the same for the phase-decomposed strided
    dgrad; MMDX_CONV_8W64: 128 x 64
    as 4 x 2 waves of 32 x 32; MMDX_WGRAD_8W: the R-major 128 x 128 weight-gradient tiles) run
    the same K tiles in the same MFMA order per output, and the same K splits: every output
    and partial is bit-identical to the 4-wave kernels, and so are the statistics slabs where
    a wave still covers 64 rows (MMDX_CONV_8W64's 32-row wave slices merge a 128-row slab in
    four Chan steps instead of two: last-bit differences, rtol 2e-6; its consumer-BN partial sums
    add 32-row slices: per-channel totals to 1e-5)."""
    for k in KNOBS_8W:
        monkeypatch.setenv(k, "0")
    a = _run_all(dev, cfg, "0", monkeypatch)
    monkeypatch.setenv(knob, "1")
    b = _run_all(dev, cfg, "0", monkeypatch)
    for key in a:
        assert torch.isfinite(b[key].float()).all(), key
        if key == "stats" and knob == "MMDX_CONV_8W64":
            torch.testing.assert_close(b[key], a[key], rtol=2e-6, atol=1e-6, msg=key)
            continue
        if key == "bnstat_part" and knob == "MMDX_CONV_8W64":  # 32-row partial sums: order
            ta, tb = a[key].double().sum(1), b[key].double().sum(1)
            err = ((ta - tb).abs().max() / ta.abs().max().clamp(min=1e-12)).item()
            assert err <= 1e-5, (key, err)
            continue
        assert torch.equal(a[key], b[key]), (knob, key)
