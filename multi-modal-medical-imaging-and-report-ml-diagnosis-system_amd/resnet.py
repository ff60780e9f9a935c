"""ResNet-18/50 image trunk on the mmdx HIP kernels (NHWC, implicit-GEMM MFMA convs).

Module tree and parameter names mirror torchvision's resnet (v1.5: stride on the 3x3
conv) exactly as ImageEncoderCNN wraps it — `nn.Sequential(*list(m.children())[:-1])`
(training_pipeline.py:183) — so `backbone.0.weight`, `backbone.4.0.conv1.weight`,
`backbone.4.0.downsample.1.running_mean`, ... round-trip with the reference's state_dict.

Execution does NOT walk the module tree: the whole trunk is one autograd node whose
forward and backward are hand-sequenced C-ABI calls (conv -> BN(+res)(+ReLU) per unit),
with the residual-path gradient summed inside the dgrad epilogue (beta = 1).
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn

from . import _lib as L
from ._lib import call, ptr, stream

_VEC = {torch.float32: 4, torch.bfloat16: 8}


class _NoTimer:
    def __call__(self, name):
        return self

    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


# bench.py installs a HIP-event timer here to measure the implicit-GEMM conv launches.
CONV_TIMER = _NoTimer()


# ----------------------------------------------------------------------------- modules
class Conv2d(nn.Module):
    def __init__(self, cin, cout, k, stride=1, padding=0):
        super().__init__()
        self.in_channels, self.out_channels = cin, cout
        self.kernel_size, self.stride, self.padding = k, stride, padding
        self.weight = nn.Parameter(torch.empty(cout, cin, k, k))
        # torchvision resnet init: kaiming_normal_(mode="fan_out", nonlinearity="relu")
        nn.init.kaiming_normal_(self.weight, mode="fan_out", nonlinearity="relu")

    def extra_repr(self):
        return (f"{self.in_channels}, {self.out_channels}, kernel_size={self.kernel_size}, "
                f"stride={self.stride}, padding={self.padding}")


class BatchNorm2d(nn.Module):
    def __init__(self, c, eps=1e-5, momentum=0.1):
        super().__init__()
        self.num_features, self.eps, self.momentum = c, eps, momentum
        self.weight = nn.Parameter(torch.ones(c))
        self.bias = nn.Parameter(torch.zeros(c))
        self.register_buffer("running_mean", torch.zeros(c))
        self.register_buffer("running_var", torch.ones(c))
        self.register_buffer("num_batches_tracked", torch.tensor(0, dtype=torch.long))


class ReLU(nn.Module):
    pass


class MaxPool2d(nn.Module):
    def __init__(self, k=3, stride=2, padding=1):
        super().__init__()
        self.kernel_size, self.stride, self.padding = k, stride, padding


class AdaptiveAvgPool2d(nn.Module):
    def __init__(self, out=1):
        super().__init__()
        self.output_size = out


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, inplanes, planes, stride=1, downsample=None):
        super().__init__()
        self.conv1 = Conv2d(inplanes, planes, 1)
        self.bn1 = BatchNorm2d(planes)
        self.conv2 = Conv2d(planes, planes, 3, stride, 1)
        self.bn2 = BatchNorm2d(planes)
        self.conv3 = Conv2d(planes, planes * 4, 1)
        self.bn3 = BatchNorm2d(planes * 4)
        self.relu = ReLU()
        self.downsample = downsample
        self.stride = stride

    def units(self):
        return [(self.conv1, self.bn1, True), (self.conv2, self.bn2, True),
                (self.conv3, self.bn3, True)]


class BasicBlock(nn.Module):
    expansion = 1

    def __init__(self, inplanes, planes, stride=1, downsample=None):
        super().__init__()
        self.conv1 = Conv2d(inplanes, planes, 3, stride, 1)
        self.bn1 = BatchNorm2d(planes)
        self.relu = ReLU()
        self.conv2 = Conv2d(planes, planes, 3, 1, 1)
        self.bn2 = BatchNorm2d(planes)
        self.downsample = downsample
        self.stride = stride

    def units(self):
        return [(self.conv1, self.bn1, True), (self.conv2, self.bn2, True)]


ARCHS = {
    "resnet18": (BasicBlock, [2, 2, 2, 2]),
    "resnet34": (BasicBlock, [3, 4, 6, 3]),
    "resnet50": (Bottleneck, [3, 4, 6, 3]),
    "resnet101": (Bottleneck, [3, 4, 23, 3]),
}


def _make_layer(block, inplanes, planes, blocks, stride):
    downsample = None
    if stride != 1 or inplanes != planes * block.expansion:
        downsample = nn.Sequential(Conv2d(inplanes, planes * block.expansion, 1, stride),
                                   BatchNorm2d(planes * block.expansion))
    layers = [block(inplanes, planes, stride, downsample)]
    inplanes = planes * block.expansion
    for _ in range(1, blocks):
        layers.append(block(inplanes, planes))
    return nn.Sequential(*layers), inplanes


class ResNetTrunk(nn.Sequential):
    """`Sequential(conv1, bn1, relu, maxpool, layer1..4, avgpool)`; forward = fused engine.

    Input: fp32 NCHW images [B,3,H,W] (the tensor image_transfom_into_tensor makes,
    TP:112-119), or an already-converted NHWC compute-dtype tensor.  Output: [B, feat, 1, 1]
    like torchvision's trunk (flatten(1) is applied by the caller, TP:281/288).
    """

    def __init__(self, arch="resnet50"):
        block, counts = ARCHS[arch]
        conv1 = Conv2d(3, 64, 7, 2, 3)
        bn1 = BatchNorm2d(64)
        inplanes = 64
        l1, inplanes = _make_layer(block, inplanes, 64, counts[0], 1)
        l2, inplanes = _make_layer(block, inplanes, 128, counts[1], 2)
        l3, inplanes = _make_layer(block, inplanes, 256, counts[2], 2)
        l4, inplanes = _make_layer(block, inplanes, 512, counts[3], 2)
        super().__init__(conv1, bn1, ReLU(), MaxPool2d(), l1, l2, l3, l4, AdaptiveAvgPool2d(1))
        self.arch = arch
        self.feat_dim = inplanes
        self.compute_dtype = torch.float32
        # torchvision zero-inits no residual BN by default; bn weights 1, biases 0 (above).

    # parameters in engine order (conv.weight, bn.weight, bn.bias per unit)
    def engine_params(self):
        ps = [self[0].weight, self[1].weight, self[1].bias]
        for layer in list(self)[4:8]:
            for blk in layer:
                for conv, bn, _ in blk.units():
                    ps += [conv.weight, bn.weight, bn.bias]
                if blk.downsample is not None:
                    ps += [blk.downsample[0].weight, blk.downsample[1].weight,
                           blk.downsample[1].bias]
        return ps

    def forward(self, x):
        params = self.engine_params()
        need_grad = torch.is_grad_enabled() and any(p.requires_grad for p in params)
        # torch convs accept any strides (e.g. a channels-last view from a PIL transform)
        feats = _TrunkFn.apply(x.contiguous(), self, need_grad, *params)
        return feats.view(feats.shape[0], feats.shape[1], 1, 1)


# ----------------------------------------------------------------------------- engine
class _Unit:
    """One conv + BN (+residual)(+ReLU) step; holds its forward state for the backward."""
    __slots__ = ("conv", "bn", "relu", "desc", "cm", "x", "y", "out", "mean", "rstd", "wc",
                 "shape_in", "train")


def _desc(N, H, W, C, conv):
    k, s, p = conv.kernel_size, conv.stride, conv.padding
    P = (H + 2 * p - k) // s + 1
    Q = (W + 2 * p - k) // s + 1
    return L.ConvDesc(N, H, W, C, conv.out_channels, k, k, s, s, p, p, P, Q)


def _conv_bn(conv, bn, relu, x, N, H, W, C, cm, res, train, keep):
    T = x.dtype
    dt = L.dtype_code(T)
    d = _desc(N, H, W, C, conv)
    K, k = conv.out_channels, conv.kernel_size
    dev = x.device
    wk = torch.empty((K, k, k, C), dtype=T, device=dev)
    wc = torch.empty((C, k, k, K), dtype=T, device=dev) if keep else None
    st = stream()
    call("mmdx_conv_pack_weight", dt, d, cm, ptr(conv.weight), ptr(wk), ptr(wc), st)
    y = torch.empty((N, d.P, d.Q, K), dtype=T, device=dev)
    nstat = L.lib().mmdx_conv_fwd_stat_blocks(d) if train else 0
    # BN batch statistics come out of the conv epilogue (per 128-row block, fp32 accums)
    part = torch.empty((nstat, K, 2), dtype=torch.float32, device=dev) if train else None
    with CONV_TIMER("fwd"):
        call("mmdx_conv_fwd", dt, d, ptr(x), ptr(wk), ptr(y), ptr(part), st)
    out = torch.empty_like(y)
    rows = N * d.P * d.Q
    mean = torch.empty(K, dtype=torch.float32, device=dev)
    rstd = torch.empty(K, dtype=torch.float32, device=dev)
    ws_n = L.lib().mmdx_bn_workspace_size(rows, K)
    ws = L.workspace(ws_n, dev)
    call("mmdx_bn_fwd", dt, int(train), ptr(y), rows, K, ptr(part), nstat, 128, ptr(bn.weight),
         ptr(bn.bias), ptr(bn.running_mean), ptr(bn.running_var), float(bn.momentum),
         float(bn.eps), ptr(mean), ptr(rstd), ptr(res), int(relu), ptr(out), ptr(ws), ws_n, st)
    u = None
    if keep:
        u = _Unit()
        u.conv, u.bn, u.relu, u.desc, u.cm = conv, bn, relu, d, cm
        u.x, u.y, u.out, u.mean, u.rstd, u.wc, u.train = x, y, out, mean, rstd, wc, train
    return out, d, u


def _unit_bwd(u, dout, want_dx, dx_acc=None, want_res=False):
    """BN(+res)(+ReLU) backward then conv wgrad/dgrad. Returns (dx, dres, dw, dgamma, dbeta).
    If dx_acc is given, dgrad accumulates into it (beta = 1) and it is returned as dx."""
    d = u.desc
    T = u.y.dtype
    dt = L.dtype_code(T)
    dev = u.y.device
    st = stream()
    rows = d.N * d.P * d.Q
    K = d.K
    dconv = torch.empty_like(u.y)
    dres = torch.empty_like(u.y) if want_res else None
    dg = torch.empty(K, dtype=torch.float32, device=dev)
    db = torch.empty(K, dtype=torch.float32, device=dev)
    ws_n = L.lib().mmdx_bn_workspace_size(rows, K)
    ws = L.workspace(ws_n, dev)
    # units without a residual recompute their ReLU mask from y (out is not read)
    out = u.out if want_res else None
    call("mmdx_bn_bwd", dt, int(u.train), ptr(u.y), ptr(out), ptr(dout), rows, K,
         ptr(u.bn.weight), ptr(u.bn.bias), ptr(u.mean), ptr(u.rstd), int(u.relu), ptr(dconv),
         ptr(dres),
         ptr(dg), ptr(db), 0.0, ptr(ws), ws_n, st)
    dw = torch.empty_like(u.conv.weight)
    ws_n = L.lib().mmdx_conv_wgrad_workspace_size(dt, d)
    ws = L.workspace(ws_n, dev)
    with CONV_TIMER("wgrad"):
        call("mmdx_conv_wgrad", dt, d, u.cm, ptr(u.x), ptr(dconv), ptr(dw), 0.0, ptr(ws), ws_n,
             st)
    dx = None
    if want_dx:
        if dx_acc is not None:
            dx = dx_acc
            beta = 1.0
        else:
            dx = torch.empty((d.N, d.H, d.W, d.C), dtype=T, device=dev)
            beta = 0.0
        with CONV_TIMER("dgrad"):
            call("mmdx_conv_dgrad", dt, d, ptr(dconv), ptr(u.wc), ptr(dx), beta, st)
    return dx, dres, dw, dg, db


class _TrunkFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, trunk, need_grad, *params):
        L.require_device(x)
        T = trunk.compute_dtype
        dt = L.dtype_code(T)
        train = trunk.training
        keep = bool(need_grad)
        st = stream()
        dev = x.device
        vec = _VEC[T]
        if x.dim() != 4:
            raise ValueError("expected images [B,3,H,W]")
        if x.dtype == torch.float32 and x.shape[1] == 3:
            N, Cin, H, W = x.shape
            cp = vec
            x0 = torch.empty((N, H, W, cp), dtype=T, device=dev)
            call("mmdx_nchw_to_nhwc", dt, ptr(x.contiguous()), N, Cin, H, W, cp, ptr(x0), st)
        else:  # pre-converted NHWC, channel-padded
            N, H, W, cp = x.shape
            if x.dtype != T:
                raise TypeError("NHWC trunk input must already be in the compute dtype")
            x0 = x
        units = []          # forward order, for the backward
        plan = []           # structure: ("stem"), ("block", [u...], ds_unit, has_ds)
        stem = trunk[0]
        a, d, u = _conv_bn(stem, trunk[1], True, x0, N, H, W, cp, 3, None, train, keep)
        H, W, C = d.P, d.Q, d.K
        # maxpool 3x3/2 pad 1
        mp = trunk[3]
        P = (H + 2 * mp.padding - mp.kernel_size) // mp.stride + 1
        Q = (W + 2 * mp.padding - mp.kernel_size) // mp.stride + 1
        pooled = torch.empty((N, P, Q, C), dtype=T, device=dev)
        am = torch.empty((N, P, Q, C), dtype=torch.uint8, device=dev)
        call("mmdx_maxpool_fwd", dt, ptr(a), N, H, W, C, mp.kernel_size, mp.stride, mp.padding,
             ptr(pooled), ptr(am), P, Q, st)
        stem_state = (u, am, (N, H, W, C, P, Q))
        x_cur, H, W = pooled, P, Q
        blocks = []
        for layer in list(trunk)[4:8]:
            for blk in layer:
                x_in = x_cur
                Hin, Win, Cin_b = H, W, C
                bu = []
                h = x_in
                hH, hW, hC = H, W, C
                specs = blk.units()
                ds_u = None
                if blk.downsample is not None:
                    idn, dd, ds_u = _conv_bn(blk.downsample[0], blk.downsample[1], False, x_in,
                                             N, H, W, C, C, None, train, keep)
                else:
                    idn = x_in
                for i, (conv, bn, relu) in enumerate(specs):
                    res = idn if i == len(specs) - 1 else None
                    h, dd, uu = _conv_bn(conv, bn, relu, h, N, hH, hW, hC, hC, res, train, keep)
                    hH, hW, hC = dd.P, dd.Q, dd.K
                    bu.append(uu)
                blocks.append((bu, ds_u, (Hin, Win, Cin_b)))
                x_cur, H, W, C = h, hH, hW, hC
        feats = torch.empty((N, C), dtype=T, device=dev)
        call("mmdx_avgpool_fwd", dt, ptr(x_cur), N, H * W, C, ptr(feats), st)
        if train:  # every BN's num_batches_tracked += 1, in one multi-tensor launch
            torch._foreach_add_([m.num_batches_tracked for m in trunk.modules()
                                 if isinstance(m, BatchNorm2d)], 1)
        if keep:
            ctx.state = (stem_state, blocks, (N, H, W, C), x.dtype == torch.float32)
            ctx.trunk = trunk
        return feats

    @staticmethod
    def backward(ctx, dfeats):
        stem_state, blocks, (N, H, W, C), _ = ctx.state
        trunk = ctx.trunk
        T = trunk.compute_dtype
        dt = L.dtype_code(T)
        st = stream()
        dev = dfeats.device
        from .functional import cast
        dfeats = cast(dfeats.contiguous(), T)
        grads = {}
        dx = torch.empty((N, H, W, C), dtype=T, device=dev)
        call("mmdx_avgpool_bwd", dt, ptr(dfeats), N, H * W, C, ptr(dx), st)
        for bu, ds_u, _shape in reversed(blocks):
            dout = dx
            # last unit carries the residual
            n = len(bu)
            last = bu[-1]
            dh, dres, dw, dg, db = _unit_bwd(last, dout, True, want_res=True)
            grads[id(last.conv.weight)] = dw
            grads[id(last.bn.weight)] = dg
            grads[id(last.bn.bias)] = db
            for uu in reversed(bu[:-1]):
                is_first = uu is bu[0]
                if is_first:
                    # d(block input) = dgrad(conv1) + identity-path grad
                    if ds_u is not None:
                        dxi, _, dw2, dg2, db2 = _unit_bwd(ds_u, dres, True)
                        grads[id(ds_u.conv.weight)] = dw2
                        grads[id(ds_u.bn.weight)] = dg2
                        grads[id(ds_u.bn.bias)] = db2
                    else:
                        dxi = dres
                    dh, _, dw, dg, db = _unit_bwd(uu, dh, True, dx_acc=dxi)
                else:
                    dh, _, dw, dg, db = _unit_bwd(uu, dh, True)
                grads[id(uu.conv.weight)] = dw
                grads[id(uu.bn.weight)] = dg
                grads[id(uu.bn.bias)] = db
            dx = dh
        # stem: maxpool backward then conv/BN (no dgrad into the image)
        u, am, (N0, H0, W0, C0, P0, Q0) = stem_state
        da = torch.empty((N0, H0, W0, C0), dtype=T, device=dev)
        mp = trunk[3]
        call("mmdx_maxpool_bwd", dt, ptr(am), ptr(dx), N0, H0, W0, C0, mp.kernel_size, mp.stride,
             mp.padding, P0, Q0, ptr(da), st)
        _, _, dw, dg, db = _unit_bwd(u, da, False)
        grads[id(u.conv.weight)] = dw
        grads[id(u.bn.weight)] = dg
        grads[id(u.bn.bias)] = db
        params = trunk.engine_params()
        out = [None, None, None]
        for p in params:
            out.append(grads.get(id(p)) if p.requires_grad else None)
        ctx.state = None
        return tuple(out)
