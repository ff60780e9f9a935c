"""GPU: the conv tile variants the dispatcher chooses between, each against the 4-wave
128-row kernels on the same operands:

* MMDX_CONV_8W128 (default on since round 5): the 128 x 128 k-major tiles as 2 x 4 waves of
  64 x 32 instead of 2 x 2 waves of 64 x 64;
* MMDX_CONV_N64_WIDE (auto: on at >= 1024 blocks): 256 x 64 tiles in 8 waves of 64 x 32 for
  the N <= 64 GEMMs (layer1's C = K = 64 convs and 256 -> 64 dgrads) instead of 128 x 64.

Every variant accumulates each output over the same K tiles in the same MFMA order, so the
forward output, the stride-1 and phase-decomposed dgrads, the masked accumulation (accmask)
and the eval-mode fused BN forward must be BIT-IDENTICAL.  The per-128-row (mean, M2) slabs
merge the same 64-row wave slices (rtol 2e-6: a tile full in one kernel and ragged in the
other takes the general-count path there).  The fused consumer-BN partial sums
(dgrad_bnstat) are additive: a 256-row tile puts its sums in its first 128-row slot and zeros
in the second, so the per-channel totals must agree to 1e-5 (summation order only).  Ragged M
and strided convs included.  (The round-3..5 opt-in variants these tests used to cover were
retired in round 6: tools/lab/RETIRED.md.)
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
# GEMMs with >= 384 tiles of 128 x 128 (conv.hip kNarrowBelow), so the 128 x 128 kernels run
# at all (the small SHAPES above take the 128 x 64 tiles): forward and stride-1 dgrad both
# with N = 256, ragged M (25704 rows) in the third
SHAPES128 = [
    (32, 128, 28, 28, 256, 3, 1, 1),
    (32, 256, 28, 28, 256, 1, 1, 0),
    (34, 256, 27, 28, 256, 3, 1, 1),
]
# N <= 64 GEMMs (forward K = 64, dgrad C = 64), ragged 256-row tiles
SHAPES64 = [
    (5, 64, 28, 28, 64, 3, 1, 1),
    (3, 256, 28, 29, 64, 1, 1, 0),
    (4, 64, 27, 28, 256, 1, 1, 0),
]


def _run_all(dev, cfg):
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


def _compare(a, b, tag):
    for key in a:
        assert torch.isfinite(b[key].float()).all(), (tag, key)
        if key == "stats":
            torch.testing.assert_close(b[key], a[key], rtol=2e-6, atol=1e-6, msg=key)
            continue
        if key == "bnstat_part":
            ta, tb = a[key].double().sum(1), b[key].double().sum(1)
            err = ((ta - tb).abs().max() / ta.abs().max().clamp(min=1e-12)).item()
            assert err <= 1e-5, (tag, key, err)
            continue
        assert torch.equal(a[key], b[key]), (tag, key)


@pytest.mark.parametrize("cfg", SHAPES + SHAPES128)
def test_8wave_128row_tiles_match_4wave(dev, cfg, knobs):
    """MMDX_CONV_8W128: the default 8-wave 128 x 128 tiles against the 4-wave ones."""
    knobs("MMDX_CONV_N64_WIDE", 0)
    knobs("MMDX_CONV_8W128", 0)
    a = _run_all(dev, cfg)
    knobs("MMDX_CONV_8W128", 1)
    b = _run_all(dev, cfg)
    _compare(a, b, "8w128")


@pytest.mark.parametrize("cfg", SHAPES64)
def test_256row_n64_tiles_match_128row(dev, cfg, knobs):
    """MMDX_CONV_N64_WIDE: the 256 x 64 8-wave tiles (forced on) against 128 x 64."""
    knobs("MMDX_CONV_N64_WIDE", 0)
    a = _run_all(dev, cfg)
    knobs("MMDX_CONV_N64_WIDE", 1)
    b = _run_all(dev, cfg)
    _compare(a, b, "n64wide")

