"""Lab: does a CU-masked stream (mmdx_stream_create) confine its kernels?  One large conv
forward timed on the default stream and on streams restricted to n CUs.

    python tools/lab/cu_mask_probe.py
"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
import mmdx  # noqa: E402,F401
from mmdx import _lib as L  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    dt = torch.bfloat16
    N, H, W, C, K = 128, 56, 56, 64, 256
    d = L.ConvDesc(N, H, W, C, K, 1, 1, 1, 1, 0, 0, H, W)
    x = torch.randn(N, H, W, C, device=dev).to(dt)
    w = torch.randn(K, C, 1, 1, device=dev) * 0.05
    wk = torch.empty(K, 1, 1, C, dtype=dt, device=dev)
    wc = torch.empty(C, 1, 1, K, dtype=dt, device=dev)
    L.call("mmdx_conv_pack_weight", 1, d, C, w.data_ptr(), wk.data_ptr(), wc.data_ptr(),
           L.stream())
    y = torch.empty(N, H, W, K, dtype=dt, device=dev)
    part = torch.empty(K, L.lib().mmdx_conv_fwd_stat_blocks(d), 2, device=dev)
    torch.cuda.synchronize()
    for cus in (0, 128, 64, 32, 8):
        h = ctypes.c_void_p()
        L.call("mmdx_stream_create", 0, cus, ctypes.byref(h))
        st = torch.cuda.ExternalStream(h.value, device=dev)
        with torch.cuda.stream(st):
            for _ in range(3):
                L.call("mmdx_conv_fwd", 1, d, x.data_ptr(), wk.data_ptr(), y.data_ptr(),
                       part.data_ptr(), L.stream())
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                L.call("mmdx_conv_fwd", 1, d, x.data_ptr(), wk.data_ptr(), y.data_ptr(),
                       part.data_ptr(), L.stream())
            e1.record()
        torch.cuda.synchronize()
        print(f"cus {cus:4d}: {e0.elapsed_time(e1) / 20 * 1e3:8.1f} us per conv", flush=True)
        L.lib().mmdx_stream_destroy(h.value)


if __name__ == "__main__":
    main()
