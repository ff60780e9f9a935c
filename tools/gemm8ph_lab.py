#!/usr/bin/env python3
"""Check and time the 8-wave ping-pong GEMM (csrc/gemm8ph.h, lab build tools/lab/libgemm8ph_lab.so)
against mmdx_gemm (the dispatch in the library) and torch.matmul (hipBLASLt) on the C5 Linear
shapes and square calibration points.  fwd = X W^T (both k-major), dgrad = dY W (W R-major),
wgrad = dY^T X (both R-major, fp32 out).
    python tools/gemm8ph_lab.py [--reps 20] [--dtype f16|bf16] [--shapes c5|all] [--splits N]
"""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

LINEARS = [(12608, 2304, 768), (12608, 768, 768), (12608, 3072, 768), (12608, 768, 3072),
           (8192, 2304, 768), (8192, 768, 768), (8192, 3072, 768), (8192, 768, 3072)]
SQUARE = [(4096, 4096, 4096), (8192, 8192, 8192)]


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
    ap.add_argument("--dtype", default="f16", choices=["f16", "bf16"])
    ap.add_argument("--shapes", default="all", choices=["c5", "all"])
    ap.add_argument("--splits", type=int, default=1)
    ap.add_argument("--sched", default="0,1", help="K-loop schedules to time (gemm8ph.h SCHED)")
    a = ap.parse_args()
    import mmdx  # noqa: F401
    from mmdx import functional as F
    lab = ctypes.CDLL(os.path.join(ROOT, "tools", "lab", "libgemm8ph_lab.so"))
    lab.lab_gemm8ph.restype = ctypes.c_int
    lab.lab_gemm8ph.argtypes = [ctypes.c_int] * 7 + [ctypes.c_void_p, ctypes.c_long,
                                                     ctypes.c_void_p, ctypes.c_long,
                                                     ctypes.c_void_p, ctypes.c_long, ctypes.c_int,
                                                     ctypes.c_void_p, ctypes.c_void_p]
    dt = torch.float16 if a.dtype == "f16" else torch.bfloat16
    code = 2 if a.dtype == "f16" else 1
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream().cuda_stream
    scheds = [int(x) for x in a.sched.split(",")]
    tot = {"mmdx": 0.0, **{f"8ph{x}": 0.0 for x in scheds}, "blas": 0.0}
    shapes = LINEARS + ([] if a.shapes == "c5" else SQUARE)
    bad = 0
    for T, O, I in shapes:
        g = torch.Generator(device=dev).manual_seed(T + O + I)
        X = (torch.rand(T, I, device=dev, generator=g) * 2 - 1).to(dt)
        W = (torch.rand(O, I, device=dev, generator=g) * 2 - 1).to(dt)
        dY = (torch.rand(T, O, device=dev, generator=g) * 2 - 1).to(dt)
        cases = {  # name: (M, N, K, A, lda, ak, B, ldb, bk, torch call)
            "fwd": (T, O, I, X, I, 1, W, I, 1, lambda: torch.matmul(X, W.t())),
            "dgrad": (T, I, O, dY, O, 1, W, I, 0, lambda: torch.matmul(dY, W)),
            "wgrad": (O, I, T, dY, O, 0, X, I, 0, lambda: torch.matmul(dY.t(), X)),
        }
        for name, (M, N, K, A, lda, ak, B, ldb, bk, tfn) in cases.items():
            f32 = name == "wgrad"
            C = torch.empty(M, N, dtype=torch.float32 if f32 else dt, device=dev)
            C2 = torch.empty_like(C)
            ws = torch.empty(max(1, a.splits) * M * N if a.splits > 1 else 1, device=dev)

            def run8(sc=scheds[-1]):
                lab.lab_gemm8ph_sched(sc)
                rc = lab.lab_gemm8ph(code, int(f32), ak, bk, M, N, K, A.data_ptr(), lda,
                                     B.data_ptr(), ldb, C2.data_ptr(), N, a.splits,
                                     ws.data_ptr(), stream)
                assert rc == 0, rc
                if a.splits > 1:
                    C2.copy_(ws.view(a.splits, M, N).sum(0))

            res = {"mmdx": timeit(lambda: F.gemm(A, lda, ak, B, ldb, bk, M, N, K, C, N), a.reps)}
            for x in scheds:
                res[f"8ph{x}"] = timeit(lambda: run8(x), a.reps)
            res["blas"] = timeit(tfn, a.reps)
            F.gemm(A, lda, ak, B, ldb, bk, M, N, K, C, N)
            ref = tfn().float()
            e1 = ((C.float() - ref).abs().max() / ref.abs().max()).item()
            ok, e2 = True, 0.0
            for x in scheds:
                C2.fill_(float("nan"))
                run8(x)
                torch.cuda.synchronize()
                ex = ((C2.float() - ref).abs().max() / ref.abs().max()).item()
                e2 = max(e2, ex)
                ok = ok and ex <= max(2 * e1, 1e-2) and torch.isfinite(C2).all().item()
            bad += not ok
            for k in tot:
                tot[k] += res[k]
            fl = 2.0 * M * N * K
            print(f"{name:5s} {M:6d}x{N:5d}x{K:5d}  " + "  ".join(
                f"{k} {v * 1e3:7.1f}us {fl / v / 1e9:6.1f}TF" for k, v in res.items()) +
                f"  err mmdx {e1:.1e} 8ph {e2:.1e}{'' if ok else '  MISMATCH'}", flush=True)
    print("total ms: " + "  ".join(f"{k} {v:.3f}" for k, v in tot.items()), flush=True)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
