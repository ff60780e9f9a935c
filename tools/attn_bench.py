#!/usr/bin/env python3
"""Isolated timing of the attention kernels (mmdx_attention_fwd / _bwd) at the C5 shapes:
ViT-B/16 (B 64, L 197, H 12) and BERT-base (B 64, L 128, H 12), fp16, probabilities saved.
    python tools/attn_bench.py [--reps 20]
"""
import argparse
import math
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402


def timeit(fn, reps):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s = torch.cuda.Event(enable_timing=True)
    e = torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    import mmdx  # noqa: F401
    from mmdx import _lib as L
    dev = torch.device("cuda", 0)
    dt = torch.float16
    for name, B, Ls, H, masked in (("vit", 64, 197, 12, False), ("bert", 64, 128, 12, True)):
        D = 64 * H
        qkv = (torch.randn(B * Ls, 3 * D, device=dev) * 0.5).to(dt)
        mask = torch.ones(B, Ls, dtype=torch.long, device=dev) if masked else None
        out = torch.empty(B * Ls, D, dtype=dt, device=dev)
        probs = torch.empty(B, H, Ls, Ls, device=dev)
        dout = (torch.randn(B * Ls, D, device=dev) * 0.5).to(dt)
        dqkv = torch.empty_like(qkv)
        n = L.lib().mmdx_attention_workspace_size(L.dtype_code(dt), B, Ls, H)
        ws = torch.empty(max(1, n), dtype=torch.uint8, device=dev)
        scale = 1.0 / math.sqrt(64)
        mp = mask.data_ptr() if mask is not None else None

        def fwd():
            L.call("mmdx_attention_fwd", L.dtype_code(dt), qkv.data_ptr(), mp, B, Ls, H, scale,
                   0.0, 0, None, out.data_ptr(), probs.data_ptr(), L.stream())

        def bwd():
            L.call("mmdx_attention_bwd", L.dtype_code(dt), qkv.data_ptr(), probs.data_ptr(),
                   dout.data_ptr(), mp, B, Ls, H, scale, 0.0, dqkv.data_ptr(), ws.data_ptr(), n,
                   L.stream())
        def fwd_np():  # inference form: probabilities not saved
            L.call("mmdx_attention_fwd", L.dtype_code(dt), qkv.data_ptr(), mp, B, Ls, H, scale,
                   0.0, 0, None, out.data_ptr(), None, L.stream())
        tf, tb, tn = timeit(fwd, a.reps), timeit(bwd, a.reps), timeit(fwd_np, a.reps)
        fl = 4.0 * B * H * Ls * Ls * 64
        pbytes = B * H * Ls * Ls * 4
        print(f"{name:5s} B{B} L{Ls} H{H}: fwd {tf:7.1f} us ({fl / tf / 1e6:6.1f} TF, P "
              f"{pbytes / tf / 1e3:6.1f} GB/s)  bwd {tb:7.1f} us ({2 * fl / tb / 1e6:6.1f} TF)  "
              f"fwd w/o P {tn:7.1f} us",
              flush=True)


if __name__ == "__main__":
    main()
