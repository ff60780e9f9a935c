#!/usr/bin/env python3
"""Per-shape conv roofline table: every distinct ResNet-50 conv at batch B (default 128),
fwd / dgrad / wgrad through the C ABI, timed with HIP events on the launching stream.

For each launch: algorithmic FLOPs (2*MAC) and bytes (bf16 operands read once, output
written once; wgrad output fp32), the roofline time max(F/2.5 PF, bytes/8 TB/s), and the
measured time.  `frac` = roofline time / measured time (1.0 = at the bound).
    python tools/conv_bench.py [--batch 128] [--reps 20] [--json out.json]
"""
import argparse
import collections
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

PEAK_F = 2.5e15
PEAK_B = 8.0e12


def shapes(arch="resnet50", hw=224):
    import mmdx
    img = mmdx.ImageEncoderCNN(arch, 1024, 13)
    tr = img.backbone
    out = collections.OrderedDict()

    def conv(c, H, W, dgrad, tag):
        k, s, p = c.kernel_size, c.stride, c.padding
        P = (H + 2 * p - k) // s + 1
        Q = (W + 2 * p - k) // s + 1
        key = (H, W, c.in_channels, c.out_channels, k, s, p)
        if key in out:
            out[key]["count"] += 1
        else:
            out[key] = dict(count=1, dgrad=dgrad, tag=tag)
        return P, Q

    H, W = conv(tr[0], hw, hw, False, "stem")
    H, W = (H + 2 - 3) // 2 + 1, (W + 2 - 3) // 2 + 1
    for li, layer in enumerate(list(tr)[4:8]):
        for blk in layer:
            Hb, Wb = H, W
            for c, _, _ in blk.units():
                H, W = conv(c, H, W, True, f"layer{li + 1}")
            if blk.downsample is not None:
                conv(blk.downsample[0], Hb, Wb, True, f"layer{li + 1}.ds")
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--json", default="")
    ap.add_argument("--filter", default="", help="substring of the shape string to run")
    ap.add_argument("--ops", default="fwd,dgrad,wgrad")
    ap.add_argument("--lib", default="", help="alternative libmmdx_hip.so (A/B builds)")
    ap.add_argument("--ref-gemm", action="store_true",
                    help="also time torch.matmul (hipBLASLt) on the same M x N x K in bf16: "
                         "what a tuned explicit GEMM of that size reaches (no im2col)")
    a = ap.parse_args()
    import mmdx
    from mmdx import _lib as L
    if a.lib:
        L.LIB_PATH = os.path.abspath(a.lib)
    dev = torch.device("cuda", 0)
    dt = torch.bfloat16
    dc = L.dtype_code(dt)
    B = a.batch
    rows = []
    tot = collections.Counter()
    for (H, W, C, K, k, s, p), info in shapes().items():
        if a.filter and a.filter not in f"{H}x{W} C{C} K{K} {k}x{k}/{s}":
            continue
        Cp = (C + 7) // 8 * 8
        P = (H + 2 * p - k) // s + 1
        Q = (W + 2 * p - k) // s + 1
        wm = torch.randn(K, C, k, k, device=dev) * 0.05
        # the bf16 stem runs as the pixel-pair conv the train step uses (resnet.py,
        # mmdx_stem_pair_*): [B][H+2p][(W+2p)/2][8] pairs, R x ceil(k/2) taps, stride (2, 1)
        pair = info["tag"] == "stem" and s == 2 and C <= 4 and (W + 2 * p) % 2 == 0
        if pair:
            d = L.ConvDesc()
            L.call("mmdx_stem_pair_desc", B, C, H, W, K, k, k, s, p, d)
            x = torch.randn(B, d.H, d.W, 8, device=dev).to(dt)
            wk = torch.empty(K, d.R, d.S, 8, dtype=dt, device=dev)
            L.call("mmdx_stem_pair_pack_weight", L.ptr(wm), K, C, k, k, L.ptr(wk), L.stream())
            wc = None
            dw = torch.empty(K, 8, d.R, d.S, device=dev)
        else:
            d = L.ConvDesc(B, H, W, Cp, K, k, k, s, s, p, p, P, Q)
            x = torch.randn(B, H, W, Cp, device=dev).to(dt)
            wk = torch.empty(K, k, k, Cp, dtype=dt, device=dev)
            wc = torch.empty(Cp, k, k, K, dtype=dt, device=dev)
            L.call("mmdx_conv_pack_weight", dc, d, C, L.ptr(wm), L.ptr(wk), L.ptr(wc),
                   L.stream())
            dw = torch.empty_like(wm)
        y = torch.empty(B, P, Q, K, dtype=dt, device=dev)
        dy = torch.randn(B, P, Q, K, device=dev).to(dt)
        dx = torch.empty_like(x)
        cw = 8 if pair else C
        nst = L.lib().mmdx_conv_fwd_stat_blocks(d)
        part = torch.empty(K, nst, 2, device=dev)
        wsn = L.lib().mmdx_conv_wgrad_workspace_size(dc, d)
        ws = torch.empty(max(wsn, 16), dtype=torch.uint8, device=dev)
        ops = {
            "fwd": lambda: L.call("mmdx_conv_fwd", dc, d, L.ptr(x), L.ptr(wk), L.ptr(y),
                                  L.ptr(part), L.stream()),
            "wgrad": lambda: L.call("mmdx_conv_wgrad", dc, d, cw, L.ptr(x), L.ptr(dy), L.ptr(dw),
                                    0.0, L.ptr(ws), wsn, L.stream()),
        }
        if info["dgrad"] and not pair:
            ops["dgrad"] = lambda: L.call("mmdx_conv_dgrad", dc, d, L.ptr(dy), L.ptr(wc),
                                          L.ptr(dx), 0.0, L.stream())
        macs = B * P * Q * K * C * k * k
        xb, yb, wb = x.numel() * 2, B * P * Q * K * 2, wk.numel() * 2
        nbytes = {"fwd": xb + wb + yb, "dgrad": yb + wb + xb, "wgrad": xb + yb + 2 * wb}
        for name, fn in ops.items():
            if name not in a.ops.split(","):
                continue
            for _ in range(3):
                fn()
            torch.cuda.synchronize()
            s0 = torch.cuda.Event(enable_timing=True)
            s1 = torch.cuda.Event(enable_timing=True)
            s0.record()
            for _ in range(a.reps):
                fn()
            s1.record()
            torch.cuda.synchronize()
            ms = s0.elapsed_time(s1) / a.reps
            F = 2 * macs
            bound = max(F / PEAK_F, nbytes[name] / PEAK_B) * 1e3
            r = dict(tag=info["tag"], shape=f"{H}x{W} C{C} K{K} {k}x{k}/{s}", op=name,
                     count=info["count"], M_N_K=_mnk(name, B, H, W, P, Q, C, K, k),
                     us=round(ms * 1e3, 1), tflops=round(F / ms / 1e9, 1),
                     gbs=round(nbytes[name] / ms / 1e6, 1),
                     bound="mfma" if F / PEAK_F > nbytes[name] / PEAK_B else "hbm",
                     frac=round(bound / ms, 3))
            if a.ref_gemm:
                M_, N_, K_ = (int(v) for v in r["M_N_K"].split("x"))
                ga = torch.randn(M_, K_, device=dev).to(dt)
                gb = torch.randn(N_, K_, device=dev).to(dt)
                for _ in range(3):
                    torch.matmul(ga, gb.t())
                torch.cuda.synchronize()
                s0.record()
                for _ in range(a.reps):
                    torch.matmul(ga, gb.t())
                s1.record()
                torch.cuda.synchronize()
                r["ref_gemm_us"] = round(s0.elapsed_time(s1) / a.reps * 1e3, 1)
                tot["ref_" + name] += r["ref_gemm_us"] * 1e-3 * info["count"]
                del ga, gb
            rows.append(r)
            tot[name] += ms * info["count"]
            tot["bound_" + name] += bound * info["count"]
            print(f"{r['tag']:10s} {r['shape']:26s} {name:5s} x{r['count']} {r['M_N_K']:22s} "
                  f"{r['us']:8.1f}us {r['tflops']:7.1f}TF {r['gbs']:7.1f}GB/s {r['bound']} "
                  f"frac {r['frac']:.3f}" + (f"  hipblaslt {r['ref_gemm_us']:7.1f}us"
                                             if a.ref_gemm else ""), flush=True)
    for name in ("fwd", "dgrad", "wgrad"):
        print(f"TOTAL {name}: {tot[name]:.3f} ms/step, roofline {tot['bound_' + name]:.3f} ms "
              f"(frac {tot['bound_' + name] / max(tot[name], 1e-9):.3f})"
              + (f", hipBLASLt same-size GEMMs {tot['ref_' + name]:.3f} ms" if a.ref_gemm else ""))
    if a.json:
        with open(a.json, "w") as f:
            json.dump({"batch": B, "rows": rows, "totals_ms": dict(tot)}, f, indent=1)


def _mnk(op, B, H, W, P, Q, C, K, k):
    if op == "fwd":
        return f"{B * P * Q}x{K}x{C * k * k}"
    if op == "dgrad":
        return f"{B * H * W}x{C}x{K * k * k}"
    return f"{K}x{C * k * k}x{B * P * Q}"


if __name__ == "__main__":
    main()
