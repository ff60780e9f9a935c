#!/usr/bin/env python3
"""Lab probe: where a step of the cooperative BiLSTM forward recurrence (lstm_fwd_coop_kernel)
spends its time.  C4's shape (B 128, L 128, H 256, bf16); the kernel stamps the 100 MHz
realtime clock at its phase boundaries (debug flag COOP_DEBUG_TIMING = 2):
  0 step start  1 peers' h_{t-1} published (poll + barrier)  2 h_{t-1} in LDS
  3 step s-1's backward saves and step s+1's operand loads issued  4 gates + cell update done
  5 h_t slice published (stores drained, counter added)
Also times the forward and backward launches with HIP events, alone and beside a
streaming GEMM load on another stream (the image tower's role in the C4 step).
  python tools/lab/lstm_probe.py [--load]"""
import argparse
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import mmdx  # noqa: E402,F401
from mmdx import _lib as L  # noqa: E402

PH = 8
COOP4 = os.environ.get("MMDX_LSTM_FWD_COOP4", "1") != "0"
# coop4 (default): 0 start 1 wait done 2 h in LDS 3 gates done 4 wave 0 published
NAMES = (["wait", "h->LDS", "gates+cell", "publish"] if COOP4 else
         ["wait", "h->LDS", "issue", "gates+cell", "publish"])
NST = len(NAMES) + 1


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=128)
    ap.add_argument("--L", type=int, default=128)
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    B, Ls, H = a.B, a.L, 256
    G4 = 4 * H
    g = torch.Generator(device=dev).manual_seed(0)
    xg = torch.randn((B * Ls, 2 * G4), generator=g, device=dev) * 0.5
    whh = (torch.randn((2 * G4, H), generator=g, device=dev) * 0.05).to(torch.bfloat16)
    hout = torch.empty((B, Ls, 2 * H), dtype=torch.bfloat16, device=dev)
    cs = torch.empty((2, Ls, B, H), dtype=torch.float32, device=dev)
    gs = torch.empty((2, Ls, B, H, 4), dtype=torch.float32, device=dev)
    need = L.lib().mmdx_lstm_fwd_workspace_size(L.dtype_code(torch.bfloat16), B, Ls, H)
    groups = 1 if B <= 128 else (B + 127) // 128
    tbytes = groups * 2 * 8 * Ls * PH * 8
    ws = torch.zeros(need + tbytes, dtype=torch.uint8, device=dev)
    status = torch.zeros(4, dtype=torch.int32, device=dev)
    bf = L.dtype_code(torch.bfloat16)

    def fwd(debug=0):
        L.call("mmdx_lstm_fwd", bf, L.ptr(xg), L.ptr(whh), B, Ls, H, L.ptr(hout), L.ptr(cs),
               L.ptr(gs), L.ptr(ws), need + tbytes, L.ptr(status), 0, debug, L.stream())

    dh = (torch.randn((B, Ls, 2 * H), generator=g, device=dev) * 0.1).to(torch.bfloat16)
    dxg = torch.empty((B * Ls, 2 * G4), dtype=torch.bfloat16, device=dev)
    dwhh = torch.empty((2 * G4, H), dtype=torch.float32, device=dev)
    nb = L.lib().mmdx_lstm_workspace_size(bf, B, Ls, H)
    nrb = (B + 15) // 16
    tb2 = nrb * 2 * 4 * Ls * PH * 8
    wsb = torch.zeros(nb + tb2, dtype=torch.uint8, device=dev)

    def bwd(coop=True):
        L.call("mmdx_lstm_bwd", bf, L.ptr(whh), L.ptr(hout), L.ptr(cs), L.ptr(gs), L.ptr(dh), B,
               Ls, H, L.ptr(dxg), L.ptr(dwhh), L.ptr(wsb), nb + tb2, L.ptr(status) if coop else None,
               0, 0, L.stream())

    def timed(fn, reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        fn()
        torch.cuda.synchronize()
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / reps

    load_stream = torch.cuda.Stream(device=dev)
    A = torch.randn((8192, 8192), device=dev, dtype=torch.bfloat16)
    Bm = torch.randn((8192, 8192), device=dev, dtype=torch.bfloat16)

    for load in (False, True):
        tag = "beside a GEMM load" if load else "alone"
        if load:
            with torch.cuda.stream(load_stream):
                for _ in range(40):
                    torch.mm(A, Bm)
        f_ms = timed(fwd, a.reps)
        b_ms = timed(bwd, a.reps)
        bp_ms = timed(lambda: bwd(False), a.reps)
        fwd(debug=2)
        torch.cuda.synchronize()
        assert int(status[0].item()) == 0, "recurrence timed out"
        ts = ws[need:].view(torch.int64).cpu().numpy().astype(np.float64)
        ts = ts.reshape(groups, 2, 8, Ls, PH)[..., :NST] * 10.0   # ns (100 MHz clock)
        d = np.diff(ts, axis=-1)                                # [.., step, 5 phases]
        step = ts[..., 1:, 0] - ts[..., :-1, 0]                 # start-to-start
        print(f"== {tag}: fwd {f_ms:.3f} ms/launch ({f_ms * 1e3 / Ls:.2f} us/step), "
              f"bwd {b_ms:.3f} ms/launch ({b_ms * 1e3 / Ls:.2f} us/step; batch-partitioned "
              f"{bp_ms:.3f})")
        print(f"   step start-to-start: mean {step[..., 1:].mean() / 1e3:.2f} us, "
              f"p50 {np.median(step[..., 1:]) / 1e3:.2f}, p90 {np.percentile(step[..., 1:], 90) / 1e3:.2f}")
        for k, n in enumerate(NAMES):
            v = d[..., 1:, k]
            print(f"   {n:11s} mean {v.mean() / 1e3:6.2f} us  p50 {np.median(v) / 1e3:6.2f}  "
                  f"p90 {np.percentile(v, 90) / 1e3:6.2f}  max {v.max() / 1e3:6.2f}")
        # the chain: how long after the LAST peer's publish (phase 5 stamp of step s-1) does
        # each workgroup leave its wait at step s
        pub = ts[..., NST - 1]      # [g, dir, blk, step]
        last = pub.max(axis=2)      # [g, dir, step]
        leave = ts[..., 1]
        lag = leave[..., 1:] - last[:, :, None, :-1]
        print(f"   last peer publish -> wait done: mean {lag.mean() / 1e3:.2f} us, "
              f"p90 {np.percentile(lag, 90) / 1e3:.2f}")
        for dr in range(2):
            for blk in range(8):
                row = " ".join(f"{d[0, dr, blk, 1:, k].mean() / 1e3:5.2f}" for k in range(len(NAMES)))
                lg = lag[0, dr, blk]
                rk = (pub[0, dr, :, :] < pub[0, dr, blk, :][None, :]).sum(axis=0)  # publish rank
                print(f"   dir{dr} wg{blk}: {row}   (phase means, us)  lag mean "
                      f"{lg.mean() / 1e3:5.2f} >2us {np.mean(lg > 2000):4.2f}  last-publisher "
                      f"{np.mean(rk == 7):4.2f}")
        skew = pub.max(axis=2) - pub.min(axis=2)
        print(f"   publish skew across the 8 workgroups: mean {skew.mean() / 1e3:.2f} us")
        os.environ["MMDX_LSTM_BWD_PROBE"] = "1"
        bwd()
        torch.cuda.synchronize()
        del os.environ["MMDX_LSTM_BWD_PROBE"]
        tb = wsb[nb:].view(torch.int64).cpu().numpy().astype(np.float64)
        tb = tb.reshape(nrb, 2, 4, Ls, PH)[..., :6] * 10.0
        db = np.diff(tb, axis=-1)[..., :-1, :]               # the last step has no exchange
        stepb = tb[..., 1:, 0] - tb[..., :-1, 0]
        print(f"   backward step start-to-start: mean {stepb.mean() / 1e3:.2f} us")
        for k, n in enumerate(["dG->LDS", "copy-out+publish", "wait", "peer loads", "MFMA"]):
            v = db[..., k]
            print(f"   bwd {n:17s} mean {v.mean() / 1e3:6.2f} us  p50 {np.median(v) / 1e3:6.2f}  "
                  f"p90 {np.percentile(v, 90) / 1e3:6.2f}")
        torch.cuda.synchronize()


if __name__ == "__main__":
    main()
