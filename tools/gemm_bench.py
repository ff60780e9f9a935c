#!/usr/bin/env python3
"""Dense GEMM throughput of the mmdx MFMA core (mmdx_gemm) with the 4-wave 128 x 128, the
8-wave 128 x 128 (MMDX_GEMM_8W128) and, forward orientation, the 8-wave 256 x 256
(MMDX_GEMM256_FWD_MIN, 128 x 64 per wave) tiles, next to torch.matmul (hipBLASLt) on the same
shapes: the C5 Linear layers (ViT-B/16 12608 tokens, BERT-base 8192 tokens; forward, input
gradient, weight gradient) plus square calibration points.
    python tools/gemm_bench.py [--reps 20] [--dtype f16|bf16]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

# (M tokens, out features, in features)
LINEARS = [(12608, 2304, 768), (12608, 768, 768), (12608, 3072, 768), (12608, 768, 3072),
           (8192, 2304, 768), (8192, 3072, 768), (8192, 768, 3072), (4096, 4096, 4096)]


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
    a = ap.parse_args()
    import mmdx  # noqa: F401
    from mmdx import functional as F
    dt = torch.float16 if a.dtype == "f16" else torch.bfloat16
    dev = torch.device("cuda", 0)
    from mmdx import _lib as L
    tot = {"4w": 0.0, "8w": 0.0, "256": 0.0, "blas": 0.0}
    off = {"MMDX_GEMM_8W128": "0", "MMDX_GEMM256_FWD_MIN": "0"}
    arms = (("4w", dict(off)),
            ("8w", dict(off, MMDX_GEMM_8W128="1")),
            ("256", dict(off, MMDX_GEMM256_FWD_MIN="1")))
    for T, O, I in LINEARS:
        X = (torch.rand(T, I, device=dev) * 2 - 1).to(dt)
        W = (torch.rand(O, I, device=dev) * 2 - 1).to(dt)
        dY = (torch.rand(T, O, device=dev) * 2 - 1).to(dt)
        cases = {  # name: (M, N, K, mmdx call, torch call)
            "fwd": (T, O, I, lambda C: F.gemm(X, I, 1, W, I, 1, T, O, I, C, O),
                    lambda: torch.matmul(X, W.t())),
            "dgrad": (T, I, O, lambda C: F.gemm(dY, O, 1, W, I, 0, T, I, O, C, I),
                      lambda: torch.matmul(dY, W)),
            "wgrad": (O, I, T, lambda C: F.gemm(dY, O, 0, X, I, 0, O, I, T, C, I),
                      lambda: torch.matmul(dY.t(), X)),
        }
        for name, (M, N, K, fn, tfn) in cases.items():
            C = torch.empty(M, N, dtype=dt if name != "wgrad" else torch.float32, device=dev)
            res = {}
            ref = None
            for mode, env in arms:
                os.environ.update(env)
                L.reload_config()
                res[mode] = timeit(lambda: fn(C), a.reps)
                fn(C)
                torch.cuda.synchronize()
                if ref is None:
                    ref = C.clone()
                elif not torch.equal(C, ref):  # every tile variant keeps the K order
                    err = ((C.float() - ref.float()).abs().max() /
                           ref.float().abs().max()).item()
                    print(f"  {mode}: output differs from 4w (max rel {err:.2e})", flush=True)
            res["blas"] = timeit(tfn, a.reps)
            for k in tot:
                tot[k] += res[k]
            fl = 2.0 * M * N * K
            print(f"{name:5s} {M:6d}x{N:5d}x{K:5d}  " + "  ".join(
                f"{k} {v * 1e3:7.1f}us {fl / v / 1e9:6.1f}TF" for k, v in res.items()),
                flush=True)
    print("total ms: " + "  ".join(f"{k} {v:.3f}" for k, v in tot.items()), flush=True)
    for k in off:
        os.environ.pop(k, None)
    L.reload_config()


if __name__ == "__main__":
    main()
