#!/usr/bin/env python3
"""Isolated timing of the LayerNorm kernels (mmdx_layernorm_fwd / _bwd) at the C5 shapes
(ViT-B/16 tokens 64 x 197, BERT-base tokens 64 x 128; D 768; fp16), against the HBM bytes
each call must move: fwd reads x (+ residual) and writes y (+ the sum), bwd reads the sum and
dy and writes dx (+ the small dgamma / dbeta partials).
    python tools/ln_bench.py [--reps 50]
"""
import argparse
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
    ap.add_argument("--reps", type=int, default=50)
    a = ap.parse_args()
    import mmdx  # noqa: F401
    from mmdx import _lib as L
    dev = torch.device("cuda", 0)
    dt = torch.float16
    dc = L.dtype_code(dt)
    D = 768
    for name, rows in (("vit", 64 * 197), ("bert", 64 * 128)):
        x = torch.randn(rows, D, device=dev).to(dt)
        r = torch.randn(rows, D, device=dev).to(dt)
        y = torch.empty_like(x)
        xs = torch.empty_like(x)
        g = torch.randn(D, device=dev)
        b = torch.randn(D, device=dev)
        mean = torch.empty(rows, device=dev)
        rstd = torch.empty(rows, device=dev)
        dy = torch.randn(rows, D, device=dev).to(dt)
        dx = torch.empty_like(x)
        dg = torch.empty(D, device=dev)
        db = torch.empty(D, device=dev)
        n = L.lib().mmdx_layernorm_workspace_size(rows, D)
        ws = torch.empty(n, dtype=torch.uint8, device=dev)

        def fwd():
            L.call("mmdx_layernorm_fwd", dc, x.data_ptr(), r.data_ptr(), rows, D, g.data_ptr(),
                   b.data_ptr(), 1e-6, y.data_ptr(), xs.data_ptr(), mean.data_ptr(),
                   rstd.data_ptr(), L.stream())

        def bwd():
            L.call("mmdx_layernorm_bwd", dc, xs.data_ptr(), dy.data_ptr(), rows, D, g.data_ptr(),
                   mean.data_ptr(), rstd.data_ptr(), dx.data_ptr(), dg.data_ptr(),
                   db.data_ptr(), 0.0, ws.data_ptr(), n, L.stream())
        tf, tb = timeit(fwd, a.reps), timeit(bwd, a.reps)
        el = rows * D * 2
        bf, bb = 4 * el, 3 * el + n
        print(f"{name:5s} rows {rows} D {D}: fwd {tf:6.1f} us ({bf / tf / 1e3:6.0f} GB/s)  "
              f"bwd {tb:6.1f} us ({bb / tb / 1e3:6.0f} GB/s)", flush=True)


if __name__ == "__main__":
    main()
