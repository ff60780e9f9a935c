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

import ctypes
import os
import math
import weakref

import torch
import torch.nn as nn

from . import _lib as L
from ._lib import call, ptr, stream

_VEC = {torch.float32: 4, torch.bfloat16: 8, torch.float16: 8}


class _NoTimer:
    active = False

    def __call__(self, name):
        return self

    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


# bench.py installs a HIP-event timer here to measure the implicit-GEMM conv launches: when
# `active`, `take(names)` hands out a (start, end) event pair per conv op of a plan run.
CONV_TIMER = _NoTimer()


class LaunchCost(tuple):
    """Tag of a timed launch: (kind, algorithmic FLOPs, algorithmic HBM bytes — every tensor
    it must read or write touched once).  bench.py prices each launch against its own roof,
    max(FLOPs / MFMA peak, bytes / HBM bandwidth)."""
    __slots__ = ()

    def __new__(cls, kind, flops, nbytes, label=""):
        return tuple.__new__(cls, (kind, int(flops), int(nbytes), label))

    kind = property(lambda s: s[0])
    flops = property(lambda s: s[1])
    nbytes = property(lambda s: s[2])


def conv_cost(kind, conv, N, H, W, P, Q, elt, extra_read=0):
    """LaunchCost of one conv launch over an N x H x W input (true channels, unpadded):
    fwd x + w + y; dgrad dy + w + dx (+ extra_read: a tensor the epilogue adds); wgrad
    x + dy + dw (fp32)."""
    k = conv.kernel_size
    macs = N * P * Q * conv.out_channels * conv.in_channels * k * k
    x = N * H * W * conv.in_channels * elt
    y = N * P * Q * conv.out_channels * elt
    w = conv.out_channels * conv.in_channels * k * k
    b = {"fwd": x + w * elt + y, "dgrad": y + w * elt + x + extra_read,
         "wgrad": x + y + w * 4}[kind]
    return LaunchCost(kind, 2 * macs, b,
                      f"C{conv.in_channels}->K{conv.out_channels} {k}x{k}/{conv.stride} "
                      f"in{N}x{H}x{W}")


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
# The trunk is executed from launch plans (include/mmdx.h, csrc/plan.cpp): the forward and
# the backward of one (batch shape, dtype, mode, parameter set) are recorded once as op
# lists over a buffer arena, then every step replays each with ONE C call.  Per-call
# buffers (the image batch, the upstream gradient, the gradient arena) enter as external
# bases.  An arena holds one forward's saved activations until its backward has run, so a
# second forward while a backward is pending records a second arena instead of clobbering.

def _desc(N, H, W, C, conv):
    k, s, p = conv.kernel_size, conv.stride, conv.padding
    P = (H + 2 * p - k) // s + 1
    Q = (W + 2 * p - k) // s + 1
    return L.ConvDesc(N, H, W, C, conv.out_channels, k, k, s, s, p, p, P, Q)


class _Ext:
    """An operand taken from the per-call external base `k` (+ byte offset)."""
    __slots__ = ("k", "off")

    def __init__(self, k, off=0):
        self.k, self.off = k, off


class _OpList:
    def __init__(self):
        self.ops = []
        self.conv_names = []   # per timed conv op, its tag (fwd / dgrad / wgrad)

    def add(self, code, dtype=0, i=(), l=(), f=(), p=(), d=None, stream=0):
        o = L.PlanOp()
        o.op, o.dtype, o.stream = code, dtype, stream
        for j, v in enumerate(i):
            o.i[j] = int(v)
        for j, v in enumerate(l):
            o.l[j] = int(v)
        for j, v in enumerate(f):
            o.f[j] = float(v)
        for j in range(12):
            o.ext[j] = -1
        for j, v in enumerate(p):
            if isinstance(v, _Ext):
                o.ext[j] = v.k
                o.p[j] = v.off
            elif isinstance(v, torch.Tensor):
                o.p[j] = v.data_ptr()
            else:
                o.p[j] = v  # None or int
        if d is not None:
            o.d = d
        self.ops.append(o)

    def timed(self, name, code, stream=0, **kw):
        k = len(self.conv_names)
        self.add(L.OP_EVENT, i=(2 * k,), stream=stream)
        self.add(code, stream=stream, **kw)
        self.add(L.OP_EVENT, i=(2 * k + 1,), stream=stream)
        self.conv_names.append(name)

    def cut(self):
        """Segment boundary at the current end of the list: run(between=...) returns to the
        caller here (the data-parallel hook issues a layer's all-reduce from the host
        between two segments, with nothing but the plan's own streams)."""
        self.cuts = getattr(self, "cuts", []) + [len(self.ops)]

    def freeze(self):
        arr = (L.PlanOp * len(self.ops))(*self.ops)
        self.arr, self.n = arr, len(self.ops)
        self.bounds = [0] + [c for c in getattr(self, "cuts", []) if 0 < c < self.n] + [self.n]
        self.ops = None
        return self

    def run(self, ext, streams, between=None, timer=None):
        """Replay the list.  between(k): called after segment k (k = 0 .. cuts-1) is
        enqueued and before segment k+1 is; None = one native call for the whole list.
        timer: the launch timer of the timed ops (default CONV_TIMER)."""
        exts = (ctypes.c_void_p * max(1, len(ext)))(*ext)
        sts = (ctypes.c_void_p * len(streams))(*streams)
        evs = None
        timer = CONV_TIMER if timer is None else timer
        if getattr(timer, "active", False) and self.conv_names:
            evs = timer.take(self.conv_names)
            evs = (ctypes.c_void_p * len(evs))(*[e.cuda_event for e in evs])
        if between is None or len(self.bounds) == 2:
            call("mmdx_plan_run", self.arr, self.n, exts, evs, sts, len(streams))
            return
        sz = ctypes.sizeof(L.PlanOp)
        base = ctypes.addressof(self.arr)
        for k, (a, z) in enumerate(zip(self.bounds[:-1], self.bounds[1:])):
            seg = ctypes.cast(base + a * sz, ctypes.POINTER(L.PlanOp))
            call("mmdx_plan_run", seg, z - a, exts, evs, sts, len(streams))
            if k < len(self.bounds) - 2:
                between(k)


class _Arena:
    """Buffers of one recorded forward (+ backward) of the trunk."""

    def __init__(self):
        self.bufs = []
        self.owner = None  # weakref to the autograd ctx token holding the saved activations

    def new(self, shape, dtype, dev):
        t = torch.empty(shape, dtype=dtype, device=dev)
        self.bufs.append(t)
        return t

    def event(self):
        """A synchronisation event owned by the arena (recorded once so it exists)."""
        e = torch.cuda.Event()
        e.record(torch.cuda.current_stream())
        self.bufs.append(e)
        return e.cuda_event

    def busy(self):
        return self.owner is not None and self.owner() is not None


class _Plan:
    """Recorded forward / backward op lists of one trunk configuration (one arena)."""

    def __init__(self, trunk, N, H, W, in_nchw, cin, T, train, keep, dev):
        dt = L.dtype_code(T)
        vec = _VEC[T]
        A = self.arena = _Arena()
        fw = _OpList()
        ws_need = [0, 0]  # per stream: 0 = main, 1 = weight-gradient side stream

        def ws_for(n, st=0):
            ws_need[st] = max(ws_need[st], int(n))

        # ---- forward
        stem_conv = trunk[0]
        # bf16: the stem runs as a conv over pixel pairs of the zero-bordered image
        # (mmdx_stem_pair_*: K = 224, no border taps) instead of a channel-padded NHWC copy
        ks, ss, ps = stem_conv.kernel_size, stem_conv.stride, stem_conv.padding
        stem_pair = (in_nchw and T == torch.bfloat16 and ss == 2 and cin <= 4
                     and stem_conv.in_channels == cin and (W + 2 * ps) % 2 == 0)
        d_pair = None
        if stem_pair:
            d_pair = L.ConvDesc()
            call("mmdx_stem_pair_desc", N, cin, H, W, stem_conv.out_channels, ks, ks, ss, ps,
                 ctypes.byref(d_pair))
            cp = 8
            x0 = A.new((N, d_pair.H, d_pair.W, 8), T, dev)
            fw.add(L.OP_STEM_PAIR_INPUT, i=(N, cin, H, W, ps), p=(_Ext(0), x0))
        elif in_nchw:
            cp = vec
            x0 = A.new((N, H, W, cp), T, dev)
            fw.add(L.OP_NCHW2NHWC, dt, i=(N, cin, H, W, cp), p=(_Ext(0), x0))
        else:
            cp = cin
            x0 = _Ext(0)
        self.x0 = x0
        units = []
        packs = []
        fold = not train and not keep   # eval-mode BN folded into the conv epilogue

        def unit(conv, bn, relu, x, N, H, W, C, cm, res, pair=None, st=0, join=None,
                 stats_only=False):
            """conv + BN(+res)(+ReLU) on stream `st`; `join`: an event the main stream
            waits for before the first op that reads `res` (the downsample branch);
            `stats_only`: the BN's statistics only — its consumer normalises on the fly and
            the post-activation tensor is never written (u["out"] is None)."""
            d = pair if pair is not None else _desc(N, H, W, C, conv)
            K, k = conv.out_channels, conv.kernel_size
            pq = (d.P, d.Q)
            cost = lambda kind, extra=0: conv_cost(kind, conv, N, H, W, pq[0], pq[1],  # noqa
                                                   T.itemsize, extra)
            y = A.new((N, d.P, d.Q, K), T, dev)
            nstat = L.lib().mmdx_conv_fwd_stat_blocks(d) if train else 0
            part = A.new((K, nstat, 2), torch.float32, dev) if train else None
            wk = A.new((K, d.R, d.S, d.C), T, dev)
            if pair is not None:  # stem over pixel pairs: its own weight map, no dgrad copy
                wc = None
                fw.add(L.OP_STEM_PAIR_PACK, i=(K, conv.in_channels, k, k),
                       p=(conv.weight, wk))
            else:
                wc = A.new((C, k, k, K), T, dev) if keep else None
                if C == cm:  # packed by the plan's single multi-tensor pack launch (below)
                    packs.append((conv.weight, wk, wc, K, C, cm, k * k))
                else:  # channel-padded input (fp32 stem): its own pack
                    fw.add(L.OP_CONV_PACK, dt, i=(cm,), p=(conv.weight, wk, wc), d=d)
            if fold:
                # eval forward without a backward (inference, frozen phase 1): BN on running
                # statistics (+residual)(+ReLU) applied in the conv epilogue; y is never
                # materialised and no bn_apply pass runs
                if join is not None:
                    fw.add(L.OP_WAIT, p=(join,), stream=st)
                fw.timed(cost("fwd"), L.OP_CONV_FWD_BNEVAL, stream=st, dtype=dt, i=(int(relu),),
                         f=(bn.eps,),
                         p=(x, wk, y, bn.weight, bn.bias, bn.running_mean, bn.running_var, res),
                         d=d)
                u = dict(conv=conv, bn=bn, relu=relu, d=d, cm=cm, x=x, y=None, out=y,
                         mean=None, rstd=None, wc=wc, pair=pair is not None, res=res)
                units.append(u)
                return y, d, u
            rpb = L.lib().mmdx_conv_fwd_stat_rows(d)  # rows per statistics slab (part)
            out = None if stats_only else A.new((N, d.P, d.Q, K), T, dev)
            rows = N * d.P * d.Q
            mean = A.new((K,), torch.float32, dev)
            rstd = A.new((K,), torch.float32, dev)
            # a residual unit's backward needs its ReLU mask: kept as 1 bit per element
            # (one byte per 16-B channel vector) instead of re-reading its output
            rmask = (A.new((rows, K // vec), torch.uint8, dev)
                     if keep and relu and res is not None and out is not None else None)
            fw.timed(cost("fwd"), L.OP_CONV_FWD, stream=st, dtype=dt,
                     i=(rpb if train else 0,), p=(x, wk, y, part), d=d)
            wsn = L.lib().mmdx_bn_workspace_size(rows, K)
            ws_for(wsn, st)
            if join is not None:
                fw.add(L.OP_WAIT, p=(join,), stream=st)
            fw.add(L.OP_BN_FWD, dt, i=(int(train), K, nstat, int(relu)), l=(rows, rpb, wsn),
                   f=(bn.momentum, bn.eps), stream=st,
                   p=(y, part, bn.weight, bn.bias, bn.running_mean, bn.running_var, mean,
                      rstd, res, out, _WS2 if st else _WS, rmask))
            u = dict(conv=conv, bn=bn, relu=relu, d=d, cm=cm, x=x, y=y, out=out, mean=mean,
                     rstd=rstd, wc=wc, pair=pair is not None, rmask=rmask, res=res, cost=cost)
            units.append(u)
            return out, d, u

        mp = trunk[3]
        # train forward: the stem's BN + ReLU run inside the 3x3/2 pool (mmdx_maxpool_bn_fwd,
        # bit-identical to apply-then-pool) — the 112x112x64 post-activation tensor is never
        # written or re-read; the stem's backward recomputes its ReLU mask from the raw output
        pool_bn = train and not fold and mp.kernel_size == 3 and mp.stride == 2
        a, d, stem_u = unit(stem_conv, trunk[1], True, x0, N, H, W, cp, 3, None,
                            pair=d_pair, stats_only=pool_bn)
        H, W, C = d.P, d.Q, d.K
        P = (H + 2 * mp.padding - mp.kernel_size) // mp.stride + 1
        Q = (W + 2 * mp.padding - mp.kernel_size) // mp.stride + 1
        pooled = A.new((N, P, Q, C), T, dev)
        am = A.new((N, P, Q, C), torch.uint8, dev)
        if pool_bn:
            bn0 = trunk[1]
            fw.add(L.OP_MAXPOOL_BN_FWD, dt,
                   i=(N, H, W, C, mp.kernel_size, mp.stride, mp.padding, P), l=(Q, 1),
                   p=(stem_u["y"], pooled, am, bn0.weight, bn0.bias, stem_u["mean"],
                      stem_u["rstd"]))
        else:
            fw.add(L.OP_MAXPOOL_FWD, dt,
                   i=(N, H, W, C, mp.kernel_size, mp.stride, mp.padding, P),
                   l=(Q,), p=(a, pooled, am))
        stem_geom = (N, H, W, C, P, Q)
        x_cur, H, W = pooled, P, Q
        blocks = []
        # the multi-tensor weight pack (below) runs on the side stream beside the stem (whose
        # weights have their own pack on the main stream); the main stream joins it here,
        # before the first conv that reads a packed weight (70 us off the critical path)
        pack_side = len(packs) == 0
        ev_pack_t = None
        wait_pos = len(fw.ops)
        if pack_side:
            ev_pack_t = A.event()
            fw.add(L.OP_WAIT, p=(ev_pack_t,), stream=0)
        for layer in list(trunk)[4:8]:
            for blk in layer:
                x_in = x_cur
                bu = []
                h, hH, hW, hC = x_in, H, W, C
                ds_u = None
                ds_done = None
                if blk.downsample is not None and not DS_SIDE_STREAM:
                    idn, _, ds_u = unit(blk.downsample[0], blk.downsample[1], False, x_in, N, H,
                                        W, C, C, None)
                elif blk.downsample is not None:
                    # the downsample branch (conv + BN) runs on the side stream beside the
                    # block's conv1 / conv2 / conv3; the main stream joins it right before
                    # the residual BN apply that reads it (the side stream is idle in the
                    # forward: it carries the weight gradients in the backward)
                    ev_in = A.event()
                    fw.add(L.OP_SIGNAL, p=(ev_in,), stream=0)
                    fw.add(L.OP_WAIT, p=(ev_in,), stream=1)
                    idn, _, ds_u = unit(blk.downsample[0], blk.downsample[1], False, x_in, N, H,
                                        W, C, C, None, st=1)
                    ds_done = A.event()
                    fw.add(L.OP_SIGNAL, p=(ds_done,), stream=1)
                else:
                    idn = x_in
                specs = blk.units()
                for i, (conv, bn, relu) in enumerate(specs):
                    last = i == len(specs) - 1
                    res = idn if last else None
                    h, dd, uu = unit(conv, bn, relu, h, N, hH, hW, hC, hC, res,
                                     join=ds_done if last else None)
                    hH, hW, hC = dd.P, dd.Q, dd.K
                    bu.append(uu)
                blocks.append((bu, ds_u, (H, W, C)))
                x_cur, H, W, C = h, hH, hW, hC
        # every conv weight packed (KRSC fwd + CRSK dgrad copies) in ONE launch, first op
        if packs:
            items = (L.PackItem * len(packs))()
            nb = 0
            for j, (wm, wk, wc, K_, C_, cm_, rs) in enumerate(packs):
                items[j] = L.PackItem(wm.data_ptr(), wk.data_ptr(),
                                      wc.data_ptr() if wc is not None else None, K_, C_, cm_,
                                      rs, nb)
                nb += L.lib().mmdx_conv_pack_blocks(K_, C_, rs)
            raw = torch.frombuffer(bytearray(bytes(items)), dtype=torch.uint8)
            tbl = A.new((raw.numel(),), torch.uint8, dev)
            tbl.copy_(raw)
            if pack_side:  # side stream: after whatever the main stream ran before the plan
                ev_start_t = A.event()
                fw.add(L.OP_SIGNAL, p=(ev_start_t,), stream=0)
                fw.add(L.OP_WAIT, p=(ev_start_t,), stream=1)
                fw.add(L.OP_CONV_PACK_MULTI, dt, i=(len(packs),), l=(nb,), p=(tbl,), stream=1)
                fw.add(L.OP_SIGNAL, p=(ev_pack_t,), stream=1)
                head = fw.ops[-4:]
                del fw.ops[-4:]
                fw.ops[0:0] = head
            else:
                fw.add(L.OP_CONV_PACK_MULTI, dt, i=(len(packs),), l=(nb,), p=(tbl,))
                fw.ops.insert(0, fw.ops.pop())
        elif pack_side:
            del fw.ops[wait_pos]
        self.feats = A.new((N, C), T, dev)
        fw.add(L.OP_AVGPOOL_FWD, dt, i=(N, H * W, C), p=(x_cur, self.feats))
        self.out_geom = (N, H, W, C)

        # ---- backward (ext: 0 = dfeats in T, 1 = gradient arena base, 2 = trunk input x0)
        # The weight gradients (wgrad) run on a side stream: they depend on the BN backward
        # of their unit but nothing on the critical dgrad chain depends on them, so they fill
        # the CUs the chain's smaller launches leave idle.  The main stream joins the side
        # stream once at the end, before the optimizer reads the gradients.
        self.bwd = None
        self.tail_event = None
        self.grad_regions = []
        if keep:
            bw = _OpList()
            params = trunk.engine_params()
            self.grad_off = {}
            off = 0
            for prm in params:
                self.grad_off[id(prm)] = off
                off += (prm.numel() * 4 + 15) // 16 * 16  # 16-B aligned, dense for ResNets
            self.grad_bytes = off
            self.params = params

            def g(prm):
                return _Ext(1, self.grad_off[id(prm)])

            def xref(x):
                return _Ext(2) if isinstance(x, _Ext) else x

            def unit_bwd(u, dout, want_dx, dx_acc=None, want_res=False, stats=None,
                         feed=None, pool=None, no_dres=False, acc=None, dout_mask=None):
                """BN(+res)(+ReLU) backward, wgrad (side stream), dgrad.  `stats`: this
                unit's BN-backward partials, already made by the dgrad that produced `dout`;
                `feed`: the unit whose dout this unit's dgrad produces (no residual) — its
                partials are then made in the dgrad epilogue and returned."""
                d = u["d"]
                K = d.K
                rows = d.N * d.P * d.Q
                dconv = A.new(tuple(u["y"].shape), T, dev)
                u["dconv"] = dconv
                # kept for the per-launch parity test (tests/test_trunk_launches_gpu.py):
                # the BN backward's upstream gradient and where its ReLU mask comes from
                u["dout"], u["dout_mask"] = dout, dout_mask
                u["bwd_kind"] = ("masked" if dout_mask is not None else
                                 "pool" if pool is not None else
                                 "res" if want_res else "relu" if u["relu"] else "plain")
                # no_dres: the identity path's gradient is added by conv1's dgrad epilogue
                # from (dout, ReLU bit mask) instead (mmdx_conv_dgrad_accmask)
                dres = (A.new(tuple(u["y"].shape), T, dev) if want_res and not no_dres
                        else None)
                wsn = L.lib().mmdx_bn_workspace_size(rows, K)
                ws_for(wsn)
                # ReLU mask: a residual unit's bit mask from the forward (else its output);
                # no residual: recomputed from y
                rmask = u.get("rmask") if want_res else None
                out = u["out"] if want_res and rmask is None else None
                sp, sb = stats if stats is not None else (None, 0)
                if dout_mask is not None:
                    # a downsample BN: its upstream gradient is the residual unit's dout with
                    # that unit's ReLU bit mask applied on the fly (mmdx_bn_bwd_masked_dy)
                    bw.add(L.OP_BN_BWD_MASKED_DY, dt, i=(int(train), K), l=(rows, wsn),
                           f=(0.0,),
                           p=(u["y"], dout, dout_mask, u["bn"].weight, u["bn"].bias, u["mean"],
                              u["rstd"], dconv, g(u["bn"].weight), g(u["bn"].bias), _WS))
                elif pool is not None:
                    # `dout` is the stem pool's OUTPUT gradient: the BN backward gathers
                    # dL/d(pool input) through the pool's argmax itself (mmdx_bn_bwd_pool)
                    am_, (pN, pH, pW, pC, pk, ps_, pp, pP, pQ) = pool
                    bw.add(L.OP_BN_BWD_POOL, dt,
                           i=(int(train), pN, pH, pW, pC, int(u["relu"]), pP, pQ),
                           l=(wsn, pk, ps_, pp), f=(0.0,),
                           p=(u["y"], am_, dout, u["bn"].weight, u["bn"].bias, u["mean"],
                              u["rstd"], dconv, g(u["bn"].weight), g(u["bn"].bias), _WS))
                else:
                    bw.add(L.OP_BN_BWD, dt, i=(int(train), K, int(u["relu"]), sb),
                           l=(rows, wsn, sp.data_ptr() if sp is not None else 0,
                              rmask.data_ptr() if rmask is not None else 0), f=(0.0,),
                           p=(u["y"], out, dout, u["bn"].weight, u["bn"].bias, u["mean"],
                              u["rstd"], dconv, dres, g(u["bn"].weight), g(u["bn"].bias),
                              _WS))
                wsn = L.lib().mmdx_conv_wgrad_workspace_size(dt, d)
                ws_for(wsn, 1)
                ev = A.event()
                bw.add(L.OP_SIGNAL, p=(ev,), stream=0)
                bw.add(L.OP_WAIT, p=(ev,), stream=1)
                cv = u["conv"]
                if u["pair"]:  # pair-conv gradient [K][8][R][S2], mapped to the master layout
                    dwp = A.new((d.K, d.C, d.R, d.S), torch.float32, dev)
                    bw.timed(u["cost"]("wgrad"), L.OP_CONV_WGRAD, stream=1, dtype=dt, i=(d.C,),
                             l=(wsn,),
                             f=(0.0,), p=(xref(u["x"]), dconv, dwp, _WS2), d=d)
                    bw.add(L.OP_STEM_PAIR_GRAD, stream=1,
                           i=(d.K, cv.in_channels, cv.kernel_size, cv.kernel_size), f=(0.0,),
                           p=(dwp, g(cv.weight)))
                else:
                    bw.timed(u["cost"]("wgrad"), L.OP_CONV_WGRAD, stream=1, dtype=dt,
                             i=(u["cm"],),
                             l=(wsn,), f=(0.0,), p=(xref(u["x"]), dconv, g(cv.weight), _WS2),
                             d=d)
                dx, fed = None, None
                if want_dx:
                    if dx_acc is not None:
                        dx, beta = dx_acc, 1.0
                    else:
                        dx, beta = A.new((d.N, d.H, d.W, d.C), T, dev), 0.0
                    # (units with a residual are not fed: their producer is conv1's dgrad
                    # accumulating onto the identity-path gradient; the ABI supports it
                    # (beta 1, mask from the unit's output) but its heavier epilogue measured
                    # 0.8 ms/step slower than the separate reduce at C4)
                    tiles = (L.lib().mmdx_conv_dgrad_stat_blocks(dt, d)
                             if feed is not None and beta == 0.0 and feed["relu"] else 0)
                    if acc is not None:  # dx = dgrad + (ReLU bit ? acc_src : 0)
                        xb = d.N * d.H * d.W * d.C * T.itemsize
                        bw.timed(u["cost"]("dgrad", xb + xb // 16), L.OP_CONV_DGRAD_ACCMASK,
                                 dtype=dt,
                                 p=(dconv, u["wc"], dx, acc[0], acc[1]), d=d)
                    elif tiles > 0:
                        fed = (A.new((d.C, tiles, 2), torch.float32, dev), tiles)
                        fb = feed["bn"]
                        bw.timed(u["cost"]("dgrad", d.N * d.H * d.W * d.C * T.itemsize),
                                 L.OP_CONV_DGRAD_BNSTAT, dtype=dt, i=(1,), f=(0.0,),
                                 p=(dconv, u["wc"], dx, feed["y"], fb.weight, fb.bias,
                                    feed["mean"], feed["rstd"], fed[0], None), d=d)
                    else:
                        xb = d.N * d.H * d.W * d.C * T.itemsize if beta else 0
                        bw.timed(u["cost"]("dgrad", xb), L.OP_CONV_DGRAD, dtype=dt,
                                 f=(beta,), p=(dconv, u["wc"], dx), d=d)
                u["dx"] = dx
                return dx, dres, fed

            N_, H_, W_, C_ = self.out_geom
            dx = A.new((N_, H_, W_, C_), T, dev)
            self.dtop = dx
            bw.add(L.OP_AVGPOOL_BWD, dt, i=(N_, H_ * W_, C_), p=(_Ext(0), dx))
            # Per-layer gradient regions for data parallelism.  engine_params is in forward
            # order, so layer k's gradients are one contiguous slice of the arena and layers
            # 4, 3, 2 are its tail.  A layer's gradients are final once the side stream has
            # run that layer's weight gradients (each waits for its unit's BN backward, which
            # also writes the BN parameter gradients on the main stream): the plan signals
            # one event on the side stream right after each layer's last wgrad, so the
            # all-reduce of layer 4 runs beside layers 3..1's backward, layer 3's beside
            # layers 2..1's, and so on.  The stem + layer 1 (the arena's head) are reduced
            # after the backward.  self.grad_regions: [(lo, hi, event)] in backward order.
            layer_lo = []
            for li in range(4, 8):
                ids_ = {id(q) for q in trunk[li].parameters()}
                layer_lo.append(min(o for i, o in self.grad_off.items() if i in ids_) // 4)
            layer_hi = layer_lo[1:] + [self.grad_bytes // 4]
            n_blocks = [len(list(trunk[li])) for li in range(4, 8)]
            # block index (reversed order) at which layer li's backward is fully enqueued
            done_at = {}
            acc = 0
            for li in (3, 2, 1):           # layer4, layer3, layer2 (indices into layer_lo)
                acc += n_blocks[li]
                done_at[acc] = li
            self.grad_regions = []
            self.grad_tail = layer_lo[3]
            self.tail_event = None
            for bi, (bu, ds_u, _shape) in enumerate(reversed(blocks)):
                if bi in done_at:
                    li = done_at[bi]
                    bw.add(L.OP_SIGNAL, p=(A.event(),), stream=1)
                    bw.cut()  # TRUNK_SEGMENT_HOOK runs here (region k = segment k)
                    self.grad_regions.append((layer_lo[li], layer_hi[li], A.bufs[-1]))
                    if li == 3:
                        self.tail_event = A.bufs[-1]
                # unit i's dgrad produces the gradient of unit i-1's output (no residual
                # inside a block): it also makes unit i-1's BN-backward partials
                # identity block (bf16, 1-bit ReLU mask kept): conv1's dgrad adds the masked
                # block-output gradient itself, the residual unit writes no d_residual
                # (blocks with a downsample: its BN backward reads the same masked gradient)
                mask_id = (T == torch.bfloat16 and len(bu) > 1
                           and bu[-1].get("rmask") is not None)
                acc_id = mask_id and ds_u is None
                dh, dres, fed = unit_bwd(bu[-1], dx, True, want_res=True,
                                         feed=bu[-2] if len(bu) > 1 else None,
                                         no_dres=mask_id)
                blk_dout = dx
                ds_in = dict(dout_mask=bu[-1]["rmask"]) if mask_id else {}
                ds_dout = blk_dout if mask_id else dres
                for k in range(len(bu) - 2, -1, -1):
                    uu = bu[k]
                    if k == 0 and ds_u is not None and ds_u["d"].stride_h > 1:
                        # d(block input) = dgrad(conv1) + dgrad(strided downsample): conv1's
                        # dgrad writes it (beta 0), then the 1x1/2 downsample's dgrad adds
                        # its one output phase (beta 1; the phases no tap reaches are left
                        # alone) — instead of the downsample writing 3/4 zeros first and
                        # conv1 re-reading the whole tensor to accumulate onto it
                        unit_bwd(ds_u, ds_dout, False, **ds_in)
                        dh, _, _ = unit_bwd(uu, dh, True, stats=fed)
                        dd_ = ds_u["d"]
                        bw.timed(ds_u["cost"]("dgrad", dd_.N * dd_.H * dd_.W * dd_.C
                                              * T.itemsize), L.OP_CONV_DGRAD, dtype=dt,
                                 f=(1.0,), p=(ds_u["dconv"], ds_u["wc"], dh), d=dd_)
                    elif k == 0 and acc_id:
                        dh, _, _ = unit_bwd(uu, dh, True, stats=fed,
                                            acc=(blk_dout, bu[-1]["rmask"]))
                    elif k == 0:
                        # d(block input) = dgrad(conv1) + identity-path grad (beta = 1)
                        if ds_u is not None:
                            dxi, _, _ = unit_bwd(ds_u, ds_dout, True, **ds_in)
                        else:
                            dxi = dres
                        dh, _, _ = unit_bwd(uu, dh, True, dx_acc=dxi, stats=fed)
                    else:
                        dh, _, fed = unit_bwd(uu, dh, True, stats=fed, feed=bu[k - 1])
                dx = dh
            n0, h0, w0, c0, p0, q0 = stem_geom
            if mp.kernel_size == 3 and mp.stride == 2 and mp.padding <= 1 and stem_u["relu"]:
                # the pool's backward runs inside the stem BN backward: the 112x112x64
                # gradient of the pool input is never materialised
                unit_bwd(stem_u, dx, False, pool=(am, (n0, h0, w0, c0, mp.kernel_size,
                                                       mp.stride, mp.padding, p0, q0)))
            else:
                da = A.new((n0, h0, w0, c0), T, dev)
                bw.add(L.OP_MAXPOOL_BWD, dt, i=(n0, h0, w0, c0, mp.kernel_size, mp.stride,
                                                mp.padding, p0), l=(q0,), p=(am, dx, da))
                unit_bwd(stem_u, da, False)  # (no dgrad into the image)
            ev = A.event()
            bw.add(L.OP_SIGNAL, p=(ev,), stream=1)
            bw.add(L.OP_WAIT, p=(ev,), stream=0)
            self.bwd = bw
        # one workspace per stream for the ops of this plan (each stream runs in order)
        ws = [A.new((max(1, n),), torch.uint8, dev) for n in ws_need]
        for lst in (fw,) + ((self.bwd,) if self.bwd is not None else ()):
            for o in lst.ops:
                for j in range(12):
                    if o.ext[j] == -1 and o.p[j] in (_WS_TOKEN, _WS2_TOKEN):
                        o.p[j] = ws[0 if o.p[j] == _WS_TOKEN else 1].data_ptr()
        # the recorded units, blocks and stem pool buffers (read by the per-launch parity test)
        self.units, self.blocks = units, blocks
        self.stem_pool = dict(u=stem_u, argmax=am, pooled=pooled, geom=stem_geom, fused=pool_bn)
        self.fwd = fw.freeze()
        if self.bwd is not None:
            self.bwd.freeze()


# TRUNK_GRAD_HOOK(grads, regions): called right after the trunk backward is enqueued with the
# flat fp32 gradient arena and [(lo, hi, event)] for layers 4, 3, 2 (backward order): after
# `event` fires, grads[lo:hi] is final (data parallelism: start that slice's all-reduce
# early from a comm stream waiting on the event, dist.GradAllReducer.launch_region).
# None = no hook.
TRUNK_GRAD_HOOK = None

# TRUNK_SEGMENT_HOOK(grads, lo, hi): the backward plan is replayed in segments, one per layer
# 4, 3, 2, and the hook is called between them with the weight-gradient stream current:
# everything that writes grads[lo:hi] is already enqueued on that stream (its wgrads wait for
# the layer's BN backward), so a collective issued from it (RCCL: its stream waits on the
# current one) starts when the slice is final, with no stream or event of its own
# (dist.GradAllReducer.trunk_segment).  Takes precedence over TRUNK_GRAD_HOOK.  None = off.
TRUNK_SEGMENT_HOOK = None

# Downsample branch of the forward on the side stream (False: in order on the main stream;
# read when a plan is built — for A/B runs, tools/step_probe.py --ds-main).
DS_SIDE_STREAM = True

# placeholder operands for the plan's per-stream workspaces, patched once sizes are known
_WS_TOKEN, _WS2_TOKEN = 0x1, 0x2
_WS, _WS2 = _WS_TOKEN, _WS2_TOKEN


# MMDX_WGRAD_CUS=n: the weight-gradient stream confined to n evenly spread compute units
# (mmdx_stream_create, a CU-masked HIP stream), leaving the rest to the dgrad / BN chain on
# the main stream; unset or 0 = all CUs (an ordinary stream).
WGRAD_CUS = int(os.environ.get("MMDX_WGRAD_CUS", "0") or 0)


class _NativeStream:
    """Owns a stream made by mmdx_stream_create; `.stream` is its torch.cuda.ExternalStream."""

    def __init__(self, dev, cus):
        h = ctypes.c_void_p()
        with torch.cuda.device(dev):
            L.call("mmdx_stream_create", 0, cus, ctypes.byref(h))
        self.handle = h.value
        self.stream = torch.cuda.ExternalStream(self.handle, device=dev)

    def __del__(self):
        if self.handle:
            try:
                L.lib().mmdx_stream_destroy(self.handle)
            except Exception:  # interpreter shutdown
                pass
            self.handle = None


def _side_stream(trunk, dev):
    key = "_mmdx_wgrad_stream_%d" % dev.index
    st = trunk.__dict__.get(key)
    if st is None:
        if WGRAD_CUS > 0:
            ns = trunk.__dict__[key + "_owner"] = _NativeStream(dev, WGRAD_CUS)
            st = ns.stream
        else:
            st = torch.cuda.Stream(device=dev)
        trunk.__dict__[key] = st
    return st


# recorded configurations kept per module; older keys (another batch shape, re-allocated
# parameters) whose arenas are all idle are dropped, so their buffers can be freed
MAX_PLAN_KEYS = 4


def _plans_for(trunk, key, build):
    """A free arena for `key` (recording a new one if every recorded arena is held)."""
    cache = trunk.__dict__.setdefault("_mmdx_plans", {})
    return plan_cache_get(cache, key, build)


def plan_cache_get(cache, key, build):
    """Shared by the trunk and the encoder-stack plans: an idle plan recorded for `key`, or a
    new one; least recently used keys beyond MAX_PLAN_KEYS are evicted when idle."""
    lst = cache.pop(key, [])
    cache[key] = lst   # most recently used last
    for old in [k for k in cache if k != key][:max(0, len(cache) - MAX_PLAN_KEYS)]:
        if not any(pl.arena.busy() for pl in cache[old]):
            del cache[old]
    for pl in lst:
        if not pl.arena.busy():
            return pl
    pl = build()
    lst.append(pl)
    return pl


class _Token:
    pass


class _TrunkFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, trunk, need_grad, *params):
        L.require_device(x)
        T = trunk.compute_dtype
        train = trunk.training
        keep = bool(need_grad)
        dev = x.device
        if x.dim() != 4:
            raise ValueError("expected images [B,3,H,W]")
        if x.dtype == torch.float32 and x.shape[1] == 3:
            N, cin, H, W = x.shape
            in_nchw = True
        else:  # pre-converted NHWC, channel-padded
            N, H, W, cin = x.shape
            in_nchw = False
            if x.dtype != T:
                raise TypeError("NHWC trunk input must already be in the compute dtype")
        key = (N, H, W, cin, in_nchw, T, train, keep, dev.index,
               tuple(p.data_ptr() for p in params))
        plan = _plans_for(trunk, key,
                          lambda: _Plan(trunk, N, H, W, in_nchw, cin, T, train, keep, dev))
        # the downsample branches run on the side stream (joined inside the plan)
        plan.fwd.run([x.data_ptr()], [stream(), _side_stream(trunk, dev).cuda_stream])
        if train:  # every BN's num_batches_tracked += 1, in one multi-tensor launch
            torch._foreach_add_([m.num_batches_tracked for m in trunk.modules()
                                 if isinstance(m, BatchNorm2d)], 1)
        if keep:
            tok = _Token()
            plan.arena.owner = weakref.ref(tok)
            ctx.tok = tok
            ctx.plan = plan
            ctx.trunk_ref = trunk
            # the stem's wgrad reads the trunk input itself unless the plan converted it
            ctx.x = x if isinstance(plan.x0, _Ext) else None
        return plan.feats.clone()

    @staticmethod
    def backward(ctx, dfeats):
        plan = ctx.plan
        trunk_params = plan.params
        from .functional import cast
        dfeats = cast(dfeats.contiguous(), plan.feats.dtype)
        dev = dfeats.device
        grads = torch.empty(plan.grad_bytes // 4, dtype=torch.float32, device=dev)
        x0 = ctx.x.data_ptr() if isinstance(plan.x0, _Ext) else plan.x0.data_ptr()
        # weight gradients on a side stream (in order on the main stream measured 9.5 %
        # slower at C4: 7128 vs 7876 samples/s)
        side = _side_stream(ctx.trunk_ref, dev)
        seg_hook = TRUNK_SEGMENT_HOOK
        between = None
        if seg_hook is not None and plan.grad_regions:
            regions = plan.grad_regions

            def between(k):
                lo, hi, _ev = regions[k]
                with torch.cuda.stream(side):
                    seg_hook(grads, lo, hi)
        plan.bwd.run([dfeats.data_ptr(), grads.data_ptr(), x0], [stream(), side.cuda_stream],
                     between=between)
        hook = TRUNK_GRAD_HOOK
        if between is None and hook is not None and plan.grad_regions:
            hook(grads, plan.grad_regions)
        plan.arena.owner = None
        ctx.plan = ctx.x = ctx.tok = ctx.trunk_ref = None
        out = [None, None, None]
        for prm in trunk_params:
            if prm.requires_grad:
                o = plan.grad_off[id(prm)] // 4
                out.append(grads[o:o + prm.numel()].view(prm.shape))
            else:
                out.append(None)
        return tuple(out)
