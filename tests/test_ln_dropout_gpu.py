"""LayerNorm(dropout(x) + residual) in one pass (mmdx_layernorm_fwd_dropout / _bwd_dropout,
BertSelfOutput / BertOutput in train mode) == mmdx_dropout_fwd followed by mmdx_layernorm_fwd
(and mmdx_layernorm_bwd followed by mmdx_dropout_bwd), bit for bit: the same keep bits from
the same seed and device counter, the dropped value rounded to the compute dtype before the
residual add exactly as the dropout kernel stores it."""
import pytest
import torch

from mmdx import _lib as L

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16, torch.float32])
@pytest.mark.parametrize("rows,D,p", [(301, 768, 0.1), (64, 512, 0.5), (7, 64, 0.1)])
def test_layernorm_dropout_fused_equals_unfused(dev, dt, rows, D, p):
    g = torch.Generator().manual_seed(rows + D)
    x = torch.randn(rows, D, generator=g).to(dev, dt)
    res = torch.randn(rows, D, generator=g).to(dev, dt)
    dy = torch.randn(rows, D, generator=g).to(dev, dt)
    gam = (1 + 0.1 * torch.randn(D, generator=g)).to(dev)
    bet = (0.1 * torch.randn(D, generator=g)).to(dev)
    dc = L.dtype_code(dt)
    seed = L.dropout_seed(4242)
    st = L.stream()
    n = L.lib().mmdx_layernorm_workspace_size(rows, D)
    ws = torch.empty(max(n, 1), dtype=torch.uint8, device=dev)

    def outs():
        return [torch.empty(rows, D, dtype=dt, device=dev) for _ in range(2)] + \
               [torch.empty(rows, device=dev) for _ in range(2)]

    # unfused
    ctr = torch.zeros(1, dtype=torch.int64, device=dev)
    xd = torch.empty_like(x)
    mask = torch.empty(rows, D, dtype=torch.uint8, device=dev)
    L.call("mmdx_dropout_fwd", dc, x.data_ptr(), x.numel(), p, seed, 0, ctr.data_ptr(),
           xd.data_ptr(), mask.data_ptr(), st)
    y0, xs0, m0, r0 = outs()
    L.call("mmdx_layernorm_fwd", dc, xd.data_ptr(), res.data_ptr(), rows, D, gam.data_ptr(),
           bet.data_ptr(), 1e-12, y0.data_ptr(), xs0.data_ptr(), m0.data_ptr(), r0.data_ptr(), st)
    dx0, dxd0 = torch.empty_like(x), torch.empty_like(x)
    dg0, db0 = torch.empty(D, device=dev), torch.empty(D, device=dev)
    L.call("mmdx_layernorm_bwd", dc, xs0.data_ptr(), dy.data_ptr(), rows, D, gam.data_ptr(),
           m0.data_ptr(), r0.data_ptr(), dx0.data_ptr(), dg0.data_ptr(), db0.data_ptr(), 0.0,
           ws.data_ptr(), n, st)
    L.call("mmdx_dropout_bwd", dc, dx0.data_ptr(), mask.data_ptr(), x.numel(), p,
           dxd0.data_ptr(), st)
    torch.cuda.synchronize()
    assert int(ctr.item()) == 1
    # fused, from the same counter value
    ctr.zero_()
    y1, xs1, m1, r1 = outs()
    rng = torch.empty(1, dtype=torch.int64, device=dev)
    L.call("mmdx_layernorm_fwd_dropout", dc, x.data_ptr(), res.data_ptr(), rows, D,
           gam.data_ptr(), bet.data_ptr(), 1e-12, p, seed, ctr.data_ptr(), y1.data_ptr(),
           xs1.data_ptr(), m1.data_ptr(), r1.data_ptr(), rng.data_ptr(), st)
    dx1, dxd1 = torch.empty_like(x), torch.empty_like(x)
    dg1, db1 = torch.empty(D, device=dev), torch.empty(D, device=dev)
    L.call("mmdx_layernorm_bwd_dropout", dc, xs1.data_ptr(), dy.data_ptr(), rows, D,
           gam.data_ptr(), m1.data_ptr(), r1.data_ptr(), p, rng.data_ptr(), dx1.data_ptr(),
           dxd1.data_ptr(), dg1.data_ptr(), db1.data_ptr(), 0.0, ws.data_ptr(), n, st)
    torch.cuda.synchronize()
    assert int(ctr.item()) == 1
    for name, a, b in (("y", y1, y0), ("xsum", xs1, xs0), ("mean", m1, m0), ("rstd", r1, r0),
                       ("dx", dx1, dx0), ("dx_drop", dxd1, dxd0), ("dgamma", dg1, dg0),
                       ("dbeta", db1, db0)):
        assert torch.equal(a, b), name
    # the drop rate is p (binomial 6-sigma band)
    frac = 1.0 - mask.float().mean().item()
    assert abs(frac - p) <= 6 * (p * (1 - p) / mask.numel()) ** 0.5


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16, torch.float32])
def test_layernorm_bwd_residual(dev, dt):
    """mmdx_layernorm_bwd_residual: dx = LN'(dy) + residual_grad in one rounding, gamma / beta
    gradients unchanged (equal to mmdx_layernorm_bwd's bit for bit)."""
    rows, D = 197, 768
    g = torch.Generator().manual_seed(5)
    x = torch.randn(rows, D, generator=g).to(dev, dt)
    dy = torch.randn(rows, D, generator=g).to(dev, dt)
    r = torch.randn(rows, D, generator=g).to(dev, dt)
    gam = (1 + 0.1 * torch.randn(D, generator=g)).to(dev)
    bet = torch.zeros(D, device=dev)
    dc = L.dtype_code(dt)
    st = L.stream()
    y = torch.empty_like(x)
    mean, rstd = torch.empty(rows, device=dev), torch.empty(rows, device=dev)
    L.call("mmdx_layernorm_fwd", dc, x.data_ptr(), None, rows, D, gam.data_ptr(), bet.data_ptr(),
           1e-6, y.data_ptr(), None, mean.data_ptr(), rstd.data_ptr(), st)
    n = L.lib().mmdx_layernorm_workspace_size(rows, D)
    ws = torch.empty(max(n, 1), dtype=torch.uint8, device=dev)
    dx0, dx1 = torch.empty_like(x), torch.empty_like(x)
    dg0, db0, dg1, db1 = (torch.empty(D, device=dev) for _ in range(4))
    L.call("mmdx_layernorm_bwd", dc, x.data_ptr(), dy.data_ptr(), rows, D, gam.data_ptr(),
           mean.data_ptr(), rstd.data_ptr(), dx0.data_ptr(), dg0.data_ptr(), db0.data_ptr(), 0.0,
           ws.data_ptr(), n, st)
    L.call("mmdx_layernorm_bwd_residual", dc, x.data_ptr(), dy.data_ptr(), rows, D,
           gam.data_ptr(), mean.data_ptr(), rstd.data_ptr(), r.data_ptr(), dx1.data_ptr(),
           dg1.data_ptr(), db1.data_ptr(), 0.0, ws.data_ptr(), n, st)
    torch.cuda.synchronize()
    assert torch.equal(dg0, dg1) and torch.equal(db0, db1)
    want = dx0.double() + r.double()   # dx0 is rounded once already: allow two roundings
    u = {torch.bfloat16: 2.0 ** -8, torch.float16: 2.0 ** -11, torch.float32: 2.0 ** -24}[dt]
    bound = 2 * u * (dx0.double().abs() + r.double().abs() + want.abs()) + 1e-30
    assert ((dx1.double() - want).abs() <= bound).all()
