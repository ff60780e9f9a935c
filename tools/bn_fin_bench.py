#!/usr/bin/env python3
"""Isolated BatchNorm finalize timing (mmdx_bn_finalize) on the C4 trunk's slab geometries:
per-128-row (mean, M2) slabs of every train-mode BN input at batch 128, HIP events around
200 back-to-back launches on the library's stream.
    python tools/bn_fin_bench.py [--batch 128]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--reps", type=int, default=200)
    a = ap.parse_args()
    from mmdx import _lib as L
    dev = torch.device("cuda:0")
    B = a.batch
    geoms = [(B * 56 * 56, 64), (B * 56 * 56, 256), (B * 56 * 56, 128), (B * 28 * 28, 128),
             (B * 28 * 28, 512), (B * 28 * 28, 256), (B * 14 * 14, 256), (B * 14 * 14, 1024),
             (B * 14 * 14, 512), (B * 7 * 7, 512), (B * 7 * 7, 2048)]
    tot = 0.0
    for rows, C in geoms:
        nblk = (rows + 127) // 128
        g = torch.Generator().manual_seed(rows + C)
        part = torch.stack([torch.randn(C, nblk, generator=g),
                            torch.rand(C, nblk, generator=g) * 100], -1).to(dev)
        vec = [torch.rand(C, device=dev) + 0.5 for _ in range(8)]
        args = (part.data_ptr(), nblk, 128, rows, C, vec[0].data_ptr(), vec[1].data_ptr(),
                vec[2].data_ptr(), vec[3].data_ptr(), 0.1, 1e-5, vec[4].data_ptr(),
                vec[5].data_ptr(), vec[6].data_ptr(), vec[7].data_ptr(), L.stream())
        for _ in range(10):
            L.call("mmdx_bn_finalize", *args)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()  # the library launches on torch's current stream (L.stream())
        for _ in range(a.reps):
            L.call("mmdx_bn_finalize", *args)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / a.reps
        tot += us
        print(f"rows {rows:7d} C {C:5d} slabs {nblk:5d}: {us:7.2f} us per launch "
              f"({part.numel() * 4 / us / 1e3:6.1f} GB/s)", flush=True)
    print(f"sum over geometries: {tot:.1f} us")


if __name__ == "__main__":
    main()
