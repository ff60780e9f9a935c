#!/usr/bin/env python3
"""Dense bf16 GEMM throughput of the mmdx MFMA core (mmdx_gemm, both operands k-major),
next to torch.matmul (hipBLASLt) on the same shapes — a calibration point for the conv core.
    python tools/gemm_bench.py [--reps 20]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

SHAPES = [(4096, 4096, 4096), (8192, 8192, 8192), (25088, 256, 2304), (100352, 128, 1152),
          (6272, 512, 4608), (401408, 64, 576), (25088, 1024, 256)]


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
    return s.elapsed_time(e) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    import mmdx
    from mmdx import functional as F
    dev = torch.device("cuda", 0)
    for M, N, K in SHAPES:
        A = (torch.rand(M, K, device=dev) * 2 - 1).bfloat16()
        B = (torch.rand(N, K, device=dev) * 2 - 1).bfloat16()
        C = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
        ms = timeit(lambda: F.gemm(A, K, 1, B, K, 1, M, N, K, C, N), a.reps)
        ms_t = timeit(lambda: torch.matmul(A, B.t()), a.reps)
        fl = 2.0 * M * N * K
        print(f"{M:7d}x{N:5d}x{K:5d}  mmdx {ms * 1e3:8.1f}us {fl / ms / 1e9:7.1f}TF   "
              f"hipBLASLt {ms_t * 1e3:8.1f}us {fl / ms_t / 1e9:7.1f}TF", flush=True)


if __name__ == "__main__":
    main()
