"""Every conv and BatchNorm launch of the benched bf16 trunk step, at the benched geometry.

The C4 step's image trunk (ResNet-50 at 128 x 224 x 224, bf16, train mode; TP:866-880 is the
image phase-2 step it is) and C2's ResNet-18 at 64 are run once through the production
launch plan (`resnet._TrunkFn`: pixel-pair direct stem, LDS-DMA implicit-GEMM convs, stride-2
phase dgrads, the downsample dgrad accumulating onto conv1's, `accmask` identity dgrads,
dgrad-epilogue BN partials, BN + ReLU fused into the stem pool, 1-bit ReLU masks, split-K
weight gradients).  Afterwards the plan's arena still holds every tensor each launch read and
wrote, so every launch is checked against a float64 reference of the same operation ON THE
SAME bf16 INPUTS it read — not a model-level statistic, so a wrong tap, tile, phase, mask
bit or slab fails however chaotic the random-init network is (test_benched_path_gpu.py's
model-level bars are loose for that reason).

Bars, element by element (written in `_Report.check`):
  * a bf16 output rounded once: |got - ref| <= 2^-8 |ref|  (round to nearest)
    + 2e-5 x the same sum over |terms| (fp32 accumulation in any order: the conv references
    recompute it as the conv of |x| and |w|);
  * two roundings (the downsample dgrad added onto conv1's bf16 dgrad): 2^-8 of both;
  * fp32 outputs (weight gradients, BN gamma / beta gradients, batch statistics): only the
    accumulation term;
  * ReLU masks recomputed from the pre-activation: elements within 1e-5 of the threshold are
    excluded (at most 1e-4 of a tensor); 1-bit masks must equal out > 0 bit for bit.
"""
import pytest
import torch
import torch.nn.functional as tF

import mmdx
from parity_util import synth_batch

pytestmark = pytest.mark.gpu

U = 2.0 ** -8     # bf16 round to nearest: |round(v) - v| <= 2^-8 |v|
ACC = 2e-5        # fp32 accumulation error bound, relative to the sum of |terms|
TINY = 1e-30


def _nchw(t):
    return t.permute(0, 3, 1, 2).double()


def _bits(mask_u8, shape_nhwc):
    """1-bit ReLU mask [rows][C/8] bytes (bit e = channel 8j+e) -> bool NCHW."""
    N, H, W, C = shape_nhwc
    b = mask_u8.view(N * H * W, C // 8).long()
    bits = (b.unsqueeze(-1) >> torch.arange(8, device=b.device)) & 1
    return bits.view(N, H, W, C).permute(0, 3, 1, 2).bool()


class _Report:
    def __init__(self):
        self.worst = {}
        self.n = 0

    def check(self, what, got, ref, bound, skip=None):
        err = (got.double() - ref).abs()
        r = err / (bound + TINY)
        if skip is not None:
            r = r.masked_fill(skip, 0.0)
        w = r.max().item()
        self.n += 1
        k = what.split(" ")[0]
        if w > self.worst.get(k, (0.0, ""))[0]:
            self.worst[k] = (w, what)
        assert w <= 1.0, f"{what}: error {w:.3f}x its bound (max |err| {err.max().item():.3e})"


def _conv_refs(x, w, dy, stride, pad):
    """fwd / dgrad / wgrad of one conv in float64 and their |term| sums."""
    y = tF.conv2d(x, w, stride=stride, padding=pad)
    ya = tF.conv2d(x.abs(), w.abs(), stride=stride, padding=pad)
    out = {"y": y, "y_acc": ya}
    if dy is not None:
        out["dx"] = torch.nn.grad.conv2d_input(x.shape, w, dy, stride=stride, padding=pad)
        out["dx_acc"] = torch.nn.grad.conv2d_input(x.shape, w.abs(), dy.abs(), stride=stride,
                                                   padding=pad)
        out["dw"] = torch.nn.grad.conv2d_weight(x, w.shape, dy, stride=stride, padding=pad)
        out["dw_acc"] = torch.nn.grad.conv2d_weight(x.abs(), w.shape, dy.abs(), stride=stride,
                                                    padding=pad)
    return out


def _bn_fwd_checks(rep, tag, u, ref, res_ref=None):
    """Batch statistics (from the conv epilogue's fp32 slabs) against the float64 conv
    output; the apply pass (+residual)(+ReLU) and its 1-bit mask against the stored y."""
    bn = u["bn"]
    y_ref = ref["y"]
    mean_ref = y_ref.mean((0, 2, 3))
    var_ref = y_ref.var((0, 2, 3), unbiased=False)
    acc_mean = ACC * ref["y_acc"].mean((0, 2, 3)) + 1e-6 * y_ref.abs().mean((0, 2, 3))
    rep.check(f"bnstat-mean {tag}", u["mean"], mean_ref, acc_mean)
    rstd_ref = (var_ref + bn.eps).rsqrt()
    rep.check(f"bnstat-rstd {tag}", u["rstd"], rstd_ref, 1e-4 * rstd_ref)
    if u["out"] is None:
        return
    y = _nchw(u["y"])
    g = bn.weight.detach().double().view(1, -1, 1, 1)
    b = bn.bias.detach().double().view(1, -1, 1, 1)
    m = u["mean"].double().view(1, -1, 1, 1)
    rs = u["rstd"].double().view(1, -1, 1, 1)
    pre = (y - m) * rs * g + b
    mag = (y.abs() + m.abs()) * (rs * g).abs() + b.abs()   # fp32 y*scale + shift magnitudes
    if u["res"] is not None:
        r = _nchw(u["res"])
        pre = pre + r
        mag = mag + r.abs()
    out_ref = pre.clamp(min=0) if u["relu"] else pre
    got = _nchw(u["out"])
    rep.check(f"bn-apply {tag}", got, out_ref, U * out_ref.abs() + 1e-6 * mag)
    if u.get("rmask") is not None:
        N, P, Q, K = u["out"].shape
        assert torch.equal(_bits(u["rmask"], (N, P, Q, K)), got > 0), f"relu bit mask {tag}"


def _bn_bwd_checks(rep, tag, u, plan, grads):
    """dconv (the BN backward's output, which the wgrad / dgrad launches read) and the BN
    gamma / beta gradients, from the unit's upstream gradient and its ReLU-mask source."""
    bn = u["bn"]
    y = _nchw(u["y"])
    N, C = y.shape[0], y.shape[1]
    M = y.numel() // C
    gam = bn.weight.detach().double().view(1, -1, 1, 1)
    bet = bn.bias.detach().double().view(1, -1, 1, 1)
    m = u["mean"].double().view(1, -1, 1, 1)
    rs = u["rstd"].double().view(1, -1, 1, 1)
    xh = (y - m) * rs
    pre = xh * gam + bet
    kind = u["bwd_kind"]
    skip = None
    extra = 0.0
    if kind == "res":
        g = _nchw(u["dout"]) * (_nchw(u["out"]) > 0)
    elif kind == "masked":
        g = _nchw(u["dout"]) * _bits(u["dout_mask"], tuple(u["dout"].shape))
    elif kind in ("relu", "pool"):
        if kind == "pool":
            sp = plan.stem_pool
            n0, h0, w0, c0, p0, q0 = sp["geom"]
            dp = _nchw(u["dout"])
            am = sp["argmax"].permute(0, 3, 1, 2).long()
            G = torch.zeros(n0, c0, h0 + 2, w0 + 2, dtype=torch.float64, device=y.device)
            for k in range(9):
                r_, s_ = divmod(k, 3)
                G[:, :, r_:r_ + 2 * p0:2, s_:s_ + 2 * q0:2] += dp * (am == k)
            gp = G[:, :, 1:h0 + 1, 1:w0 + 1]
            dout = gp.to(torch.bfloat16).double()   # the kernel rounds the gathered sum
            extra = U * gp.abs()
        else:
            dout = _nchw(u["dout"])
        g = dout * (pre > 0)
        # mask elements whose pre-activation sits at the threshold within rounding
        skip = pre.abs() <= 1e-5 * ((y.abs() + m.abs()) * (rs * gam).abs() + bet.abs()) + TINY
        assert skip.sum().item() <= max(4, 1e-4 * skip.numel()), f"{tag}: threshold band"
    else:
        g = _nchw(u["dout"])
    sg = g.sum((0, 2, 3))
    sgx = (g * xh).sum((0, 2, 3))
    s1 = g.abs().sum((0, 2, 3))
    s2 = (g * xh).abs().sum((0, 2, 3))
    a = gam * rs
    ref = a * (g - sg.view(1, -1, 1, 1) / M - xh * sgx.view(1, -1, 1, 1) / M)
    bound = (U * ref.abs()
             + ACC * a.abs() * (g.abs() + s1.view(1, -1, 1, 1) / M
                                + xh.abs() * s2.view(1, -1, 1, 1) / M)
             + 1e-6 * a.abs() * (sgx.abs().view(1, -1, 1, 1) / M) * rs * (y.abs() + m.abs()))
    if not isinstance(extra, float):
        bound = bound + a.abs() * extra
    rep.check(f"bn-bwd {tag}", _nchw(u["dconv"]), ref, bound, skip=skip)
    band = 0.0
    if skip is not None:
        band = ((_nchw(u["dout"]) if kind == "relu" else dout).abs() * (1 + xh.abs())
                * skip).sum((0, 2, 3))
    gw, gb = grads[id(bn.weight)], grads[id(bn.bias)]
    rep.check(f"bn-dgamma {tag}", gw, sgx, ACC * s2 + band + TINY)
    rep.check(f"bn-dbeta {tag}", gb, sg, ACC * s1 + band + TINY)


# C4's per-GPU batch, C2's, and C3's 256 on one GPU: at 256 the dispatcher picks other tiles,
# stage counts and split-K depths for some launches (tools/dispatch_diff.py lists them;
# profiles/r06_dispatch_b128_vs_b256.txt), so C3's geometry is checked launch by launch too
@pytest.mark.parametrize("arch,B", [("resnet50", 128), ("resnet18", 64), ("resnet50", 256)])
def test_every_trunk_launch_bf16(dev, arch, B):
    torch.manual_seed(0)
    img = mmdx.ImageEncoderCNN(arch, 1024, 13, compute_dtype=torch.bfloat16).to(dev)
    img.unfreeze_backbone()
    trunk = img.backbone
    x, _, _, _ = synth_batch(B, 8, hw=224)
    x = x.to(dev)
    feats = trunk(x)
    g = torch.Generator().manual_seed(3)
    dfeat = torch.randn(feats.shape, generator=g).to(dev)
    feats.backward(dfeat)
    torch.cuda.synchronize()
    plans = [pl for lst in trunk.__dict__["_mmdx_plans"].values() for pl in lst]
    assert len(plans) == 1
    plan = plans[0]
    grads = {id(p): p.grad.double() for p in trunk.parameters()}
    rep = _Report()

    # ---- stem: pair-conv forward, statistics, BN + ReLU inside the max pool
    su = plan.stem_pool["u"]
    assert su["pair"] and plan.stem_pool["fused"], "bf16 stem: pixel pairs, pool-fused BN"
    conv = su["conv"]
    xb = x.to(torch.bfloat16).double()
    wb = conv.weight.detach().to(torch.bfloat16).double()
    ref = _conv_refs(xb, wb, _nchw(su["dconv"]), conv.stride, conv.padding)
    rep.check("fwd stem", _nchw(su["y"]), ref["y"], U * ref["y"].abs() + ACC * ref["y_acc"])
    _bn_fwd_checks(rep, "stem", su, ref)
    n0, h0, w0, c0, p0, q0 = plan.stem_pool["geom"]
    bn = su["bn"]
    sc = (bn.weight.detach().double() * su["rstd"].double()).view(1, -1, 1, 1)
    sh = bn.bias.detach().double().view(1, -1, 1, 1) - su["mean"].double().view(1, -1, 1, 1) * sc
    ys = _nchw(su["y"])
    t = (ys * sc + sh).clamp(min=0)
    tmag = tF.max_pool2d(ys.abs() * sc.abs() + sh.abs(), 3, 2, 1)  # fp32 y*scale + shift
    pooled = tF.max_pool2d(t, 3, 2, 1)
    rep.check("pool stem", _nchw(plan.stem_pool["pooled"]), pooled,
              U * pooled.abs() + 1e-6 * tmag + TINY)
    win = tF.pad(t, (1, 1, 1, 1), value=-1.0).unfold(2, 3, 2).unfold(3, 3, 2)
    win = win.reshape(n0, c0, p0, q0, 9)
    am = plan.stem_pool["argmax"].permute(0, 3, 1, 2).long().unsqueeze(-1)
    at = win.gather(-1, am).squeeze(-1)
    rep.check("pool-argmax stem", at, pooled, 2 * U * pooled.abs() + 2e-6 * tmag + TINY)
    rep.check("wgrad stem", grads[id(conv.weight)], ref["dw"], ACC * ref["dw_acc"] + TINY)
    _bn_bwd_checks(rep, "stem", su, plan, grads)
    del ref, t, win

    # ---- head of the backward: avgpool
    xl = plan.blocks[-1][0][-1]["out"]
    fr = _nchw(xl).mean((2, 3))
    rep.check("avgpool-fwd", plan.feats.double(), fr, U * fr.abs() + 1e-6 * _nchw(xl).abs().mean((2, 3)))
    hw = xl.shape[1] * xl.shape[2]
    dt_ref = (dfeat.view(B, -1).to(torch.bfloat16).double() / hw)[:, :, None, None].expand(
        -1, -1, xl.shape[1], xl.shape[2])
    rep.check("avgpool-bwd", _nchw(plan.dtop), dt_ref, U * dt_ref.abs() + TINY)

    # ---- every block: conv + BN units, downsample, block-input gradient
    n_units = 1
    for bi, (bu, ds_u, _shape) in enumerate(plan.blocks):
        tagb = f"b{bi}"
        assert bu[-1].get("rmask") is not None, "bf16 residual units keep 1-bit masks"
        refs = []
        for k, u in enumerate(bu + ([ds_u] if ds_u is not None else [])):
            n_units += 1
            conv = u["conv"]
            tag = f"{tagb}.{'ds' if u is ds_u else k} {tuple(conv.weight.shape)} s{conv.stride}"
            xin = _nchw(u["x"])
            wb = conv.weight.detach().to(torch.bfloat16).double()
            ref = _conv_refs(xin, wb, _nchw(u["dconv"]), conv.stride, conv.padding)
            rep.check(f"fwd {tag}", _nchw(u["y"]), ref["y"],
                      U * ref["y"].abs() + ACC * ref["y_acc"])
            _bn_fwd_checks(rep, tag, u, ref)
            _bn_bwd_checks(rep, tag, u, plan, grads)
            rep.check(f"wgrad {tag}", grads[id(conv.weight)], ref["dw"],
                      ACC * ref["dw_acc"] + TINY)
            if u is not ds_u and k > 0:
                rep.check(f"dgrad {tag}", _nchw(u["dx"]), ref["dx"],
                          U * ref["dx"].abs() + ACC * ref["dx_acc"])
            refs.append(ref)
            del ref["y"], ref["y_acc"], ref["dw"], ref["dw_acc"]
        # block-input gradient: conv1's dgrad + the downsample's dgrad (two roundings), or
        # + the identity path's masked gradient (accmask: one rounding)
        r1 = refs[0]
        got = _nchw(bu[0]["dx"])
        if ds_u is not None:
            rd = refs[-1]
            want = r1["dx"] + rd["dx"]
            bound = (U * (want.abs() + r1["dx"].abs() + rd["dx"].abs())
                     + ACC * (r1["dx_acc"] + rd["dx_acc"]))
            kind = "dgrad-ds"
        else:
            last = bu[-1]
            mk = _bits(last["rmask"], tuple(last["out"].shape))
            idn = _nchw(last["dout"]) * mk
            want = r1["dx"] + idn
            bound = U * want.abs() + ACC * r1["dx_acc"]
            kind = "dgrad-accmask"
        rep.check(f"{kind} {tagb} s{bu[0]['conv'].stride if ds_u is None else ds_u['conv'].stride}",
                  got, want, bound + TINY)
        del refs
    n_conv = sum(1 for m in trunk.modules() if isinstance(m, mmdx.resnet.Conv2d))
    assert n_units == n_conv, (n_units, n_conv)
    print(f"\n{arch} B={B}: {rep.n} launch checks over {n_units} conv units; worst error / bound:")
    for k, (w, what) in sorted(rep.worst.items()):
        print(f"  {k:18s} {w:.3f}  ({what})")
