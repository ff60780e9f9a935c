"""GPU: mmdx.GradScaler against torch.amp.GradScaler driving torch.optim.AdamW, in the
reference's order (TP:1056-1061: scale(loss).backward(), clip_grad_norm_(1.0) on the SCALED
gradients, scaler.step, scaler.update) and in torch's documented order (unscale_ first).

* A forced overflow (one inf gradient) skips the step — parameters, moments and the step
  count untouched — and halves the scale; growth_interval clean steps double it.
* Over a sequence of steps with an overflow in the middle, parameters match torch's to
  rtol 1e-5 / atol 1e-7 (fp32 AdamW arithmetic, different summation orders in the norm).
* The fused `clip_and_step` equals the unfused clip_grad_norm_ + scaler.step sequence.
* scaler.scale(loss) and its backward multiply by the scale (mmdx_mul_dev_scalar).
"""
import math

import pytest
import torch

import mmdx

pytestmark = pytest.mark.gpu


def _params(dev, seed=0):
    g = torch.Generator().manual_seed(seed)
    shapes = [(64, 33), (33,), (1000,), (7, 5, 3)]
    return [torch.randn(s, generator=g).to(dev) for s in shapes]


def _grads(step, dev, inf_at=None):
    g = torch.Generator().manual_seed(100 + step)
    gs = [torch.randn(s, generator=g).to(dev) * 0.3 for s in [(64, 33), (33,), (1000,),
                                                                (7, 5, 3)]]
    if inf_at == step:
        gs[2][17] = float("inf")
    return gs


def _run(dev, mine, order, n_steps=6, inf_at=3, interval=2):
    ps = [torch.nn.Parameter(t.clone()) for t in _params(dev)]
    groups = [{"params": ps[:2], "lr": 5e-4}, {"params": ps[2:], "lr": 2e-5}]
    if mine:
        opt = mmdx.AdamW(groups, weight_decay=1e-2)
        sc = mmdx.GradScaler(init_scale=1024.0, growth_interval=interval)
        clip = mmdx.clip_grad_norm_
    else:
        opt = torch.optim.AdamW(groups, weight_decay=1e-2)
        sc = torch.amp.GradScaler("cuda", init_scale=1024.0, growth_interval=interval)
        clip = torch.nn.utils.clip_grad_norm_
    scales = []
    for step in range(n_steps):
        # scale a unit "loss" to create the scaler's state, then plant scaled gradients
        s = sc.scale(torch.ones((), device=dev)).item()
        for p, g in zip(ps, _grads(step, dev, inf_at)):
            p.grad = (g * s).contiguous()
        if order == "reference":
            clip(ps, 1.0)
            sc.step(opt)
        elif order == "unscale_first":
            sc.unscale_(opt)
            clip(ps, 1.0)
            sc.step(opt)
        elif order == "fused":
            sc.clip_and_step(opt, 1.0)
        sc.update()
        scales.append(sc.get_scale())
    torch.cuda.synchronize()
    return [p.detach().cpu() for p in ps], scales, opt


@pytest.mark.parametrize("order", ["reference", "unscale_first"])
def test_gradscaler_matches_torch(dev, order):
    mine, s_mine, _ = _run(dev, True, order)
    ref, s_ref, _ = _run(dev, False, order)
    assert s_mine == s_ref, (s_mine, s_ref)
    assert s_mine[3] == s_mine[2] / 2           # the overflow step backed off
    for a, b in zip(mine, ref):
        torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-7)


def test_fused_clip_and_step_equals_reference_order(dev):
    a, sa, _ = _run(dev, True, "reference")
    b, sb, _ = _run(dev, True, "fused")
    assert sa == sb
    for x, y in zip(a, b):
        torch.testing.assert_close(x, y, rtol=1e-6, atol=1e-8)


def test_overflow_skips_the_step(dev):
    ps = [torch.nn.Parameter(t.clone()) for t in _params(dev)]
    opt = mmdx.AdamW(ps, lr=1e-3)
    sc = mmdx.GradScaler(init_scale=4096.0, growth_interval=2)
    s = sc.scale(torch.ones((), device=dev)).item()
    for p, g in zip(ps, _grads(0, dev)):
        p.grad = g * s
    sc.step(opt)
    sc.update()
    torch.cuda.synchronize()
    after1 = [p.detach().clone() for p in ps]
    st = opt.state[ps[0]]
    m1 = st["exp_avg"].clone()
    assert float(st["step"].item()) == 1.0
    for p, g in zip(ps, _grads(1, dev, inf_at=1)):
        p.grad = g * s
    sc.step(opt)
    sc.update()
    torch.cuda.synchronize()
    assert sc.get_scale() == 2048.0
    assert float(sc.found_inf.item()) == 1.0
    assert float(st["step"].item()) == 1.0     # no step counted
    assert torch.equal(st["exp_avg"], m1)
    for p, a in zip(ps, after1):
        assert torch.equal(p.detach(), a)        # no update
    for k in (2, 3):
        for p, g in zip(ps, _grads(k, dev)):
            p.grad = g * sc.get_scale()
        sc.step(opt)
        sc.update()
    torch.cuda.synchronize()
    assert sc.get_scale() == 4096.0             # grew back after growth_interval clean steps
    assert float(st["step"].item()) == 3.0


def test_scale_forward_backward(dev):
    sc = mmdx.GradScaler(init_scale=256.0)
    x = torch.tensor(0.75, device=dev, requires_grad=True)
    y = sc.scale(x)
    y.backward()
    torch.cuda.synchronize()
    assert y.item() == 192.0 and x.grad.item() == 256.0
    off = mmdx.GradScaler(enabled=False)
    assert off.scale(x) is x


def test_two_optimizers_any_overflow_backs_off(dev):
    """With two optimizers the scale backs off when EITHER overflowed (torch.amp keeps one
    found_inf per optimizer and update() takes them all): here the first overflows and the
    second, stepped last, is clean."""
    pa = [torch.nn.Parameter(t.clone()) for t in _params(dev)[:2]]
    pb = [torch.nn.Parameter(t.clone()) for t in _params(dev, 1)[2:]]
    oa, ob = mmdx.AdamW(pa, lr=1e-3), mmdx.AdamW(pb, lr=1e-3)
    sc = mmdx.GradScaler(init_scale=1024.0)
    sc.scale(torch.ones((), device=dev))
    ga = _grads(0, dev)
    ga[0][3, 4] = float("nan")
    for p, g in zip(pa, ga[:2]):
        p.grad = g * 1024.0
    for p, g in zip(pb, _grads(0, dev)[2:]):
        p.grad = g * 1024.0
    before_b = [p.detach().clone() for p in pb]
    sc.step(oa)
    sc.step(ob)
    sc.update()
    torch.cuda.synchronize()
    assert sc.get_scale() == 512.0
    assert all(not torch.equal(p.detach(), b) for p, b in zip(pb, before_b))  # b stepped
    with pytest.raises(AssertionError):
        sc.update()          # nothing checked since the last update (torch's assertion)


def test_finite_gradients_whose_squares_overflow_are_not_an_overflow(dev):
    """found_inf comes from a per-element inf/NaN check, not from the sum of squares: finite
    gradients of ~1e30 (their squares overflow fp32) do not skip the step."""
    ps = [torch.nn.Parameter(torch.zeros(64, device=dev))]
    opt = mmdx.AdamW(ps, lr=1e-3)
    sc = mmdx.GradScaler(init_scale=1.0)
    sc.scale(torch.ones((), device=dev))
    ps[0].grad = torch.full((64,), 1e30, device=dev)
    sc.step(opt)
    sc.update()
    torch.cuda.synchronize()
    assert float(sc.found_inf.item()) == 0.0
    assert sc.get_scale() == 1.0
    assert float(opt.state[ps[0]]["step"].item()) == 1.0


def test_state_dict_before_first_use_keeps_the_growth_tracker(dev):
    """load_state_dict on a scaler that has not created its device state yet keeps the saved
    growth tracker (two clean steps recorded): the next clean step grows the scale."""
    dst = mmdx.GradScaler(init_scale=1.0, growth_interval=3)
    dst.load_state_dict({"scale": 64.0, "growth_factor": 2.0, "backoff_factor": 0.5,
                         "growth_interval": 3, "_growth_tracker": 2})
    ps = [torch.nn.Parameter(torch.zeros(8, device=dev))]
    opt = mmdx.AdamW(ps, lr=1e-3)
    dst.scale(torch.ones((), device=dev))
    ps[0].grad = torch.ones(8, device=dev)
    dst.step(opt)
    dst.update()               # the 3rd clean step since the saved tracker: grows now
    torch.cuda.synchronize()
    assert dst.get_scale() == 128.0


def test_clip_and_step_without_gradients(dev):
    ps = [torch.nn.Parameter(torch.zeros(8, device=dev))]
    opt = mmdx.AdamW(ps, lr=1e-3)
    sc = mmdx.GradScaler()
    with pytest.warns(RuntimeWarning, match="no parameter has a gradient"):
        norm = sc.clip_and_step(opt, 1.0)
    assert float(norm) == 0.0
    sc.scale(torch.ones((), device=dev))
    sc.clip_and_step(opt, 1.0)   # (warned once per scaler)
    sc.update()                # a no-gradient step records no inf check: update() keeps state
    torch.cuda.synchronize()
    assert sc.get_scale() == 2.0 ** 16
    # GradScaler.step without gradients is an error, as torch.amp.GradScaler's is (gradients
    # that never reached the optimizer must not turn into silently skipped steps)
    sc.scale(torch.ones((), device=dev))
    with pytest.raises(AssertionError, match="No inf checks were recorded"):
        sc.step(opt)


@pytest.mark.parametrize("bad", [float("inf"), float("nan")])
def test_clip_norm_nonfinite_matches_torch(dev, bad):
    """Without AMP, an inf (NaN) gradient makes clip_grad_norm_ return an inf (NaN) norm and a
    clip coefficient of 0 (NaN), as torch.nn.utils.clip_grad_norm_ does; the non-finite flag
    rides beside the sum of squares, not in it."""
    g = torch.Generator().manual_seed(3)
    vals = [torch.randn(300, generator=g), torch.randn(17, 5, generator=g)]
    vals[1][2, 3] = bad
    mine = [torch.nn.Parameter(v.clone().to(dev)) for v in vals]
    ref = [torch.nn.Parameter(v.clone().to(dev)) for v in vals]
    for p, v in zip(mine + ref, vals + vals):
        p.grad = v.clone().to(dev) * 0.5
    n_mine = mmdx.clip_grad_norm_(mine, 1.0)
    n_ref = torch.nn.utils.clip_grad_norm_(ref, 1.0)
    torch.cuda.synchronize()
    nm, nr = float(n_mine), float(n_ref)
    assert (math.isinf(nm) and math.isinf(nr)) if bad == float("inf") else \
        (math.isnan(nm) and math.isnan(nr)), (nm, nr)
    for a, b in zip(mine, ref):   # the clipped gradients: same finite / inf / NaN pattern
        ga, gb = a.grad.cpu(), b.grad.cpu()
        assert torch.equal(torch.isnan(ga), torch.isnan(gb))
        fin = torch.isfinite(gb)
        assert torch.equal(ga[fin], gb[fin])
