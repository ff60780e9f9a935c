#!/usr/bin/env python3
"""One GEMM case of tools/gemm8ph_lab.py, repeated (for rocprofv3 --pmc passes):
    python tools/gemm8ph_one.py fwd|dgrad|wgrad M N K [--sched 1] [--reps 10] [--mmdx]"""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("case")
    ap.add_argument("M", type=int)
    ap.add_argument("N", type=int)
    ap.add_argument("K", type=int)
    ap.add_argument("--sched", type=int, default=1)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--mmdx", action="store_true")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    dt = torch.float16
    M, N, K = a.M, a.N, a.K
    ak, bk = {"fwd": (1, 1), "dgrad": (1, 0), "wgrad": (0, 0)}[a.case]
    A = (torch.rand(M * K, device=dev) * 2 - 1).to(dt)
    B = (torch.rand(N * K, device=dev) * 2 - 1).to(dt)
    C = torch.empty(M, N, dtype=dt, device=dev)
    lda, ldb = (K if ak else M), (K if bk else N)
    if a.mmdx:
        import mmdx  # noqa: F401
        from mmdx import functional as F
        for _ in range(a.reps):
            F.gemm(A, lda, ak, B, ldb, bk, M, N, K, C, N)
    else:
        lab = ctypes.CDLL(os.path.join(ROOT, "tools", "lab", "libgemm8ph_lab.so"))
        lab.lab_gemm8ph.argtypes = [ctypes.c_int] * 7 + [ctypes.c_void_p, ctypes.c_long,
                                                         ctypes.c_void_p, ctypes.c_long,
                                                         ctypes.c_void_p, ctypes.c_long,
                                                         ctypes.c_int, ctypes.c_void_p,
                                                         ctypes.c_void_p]
        lab.lab_gemm8ph_sched(a.sched)
        st = torch.cuda.current_stream().cuda_stream
        for _ in range(a.reps):
            assert lab.lab_gemm8ph(2, 0, ak, bk, M, N, K, A.data_ptr(), lda, B.data_ptr(), ldb,
                                   C.data_ptr(), N, 1, None, st) == 0
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
