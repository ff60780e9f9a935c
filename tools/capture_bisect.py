#!/usr/bin/env python3
"""Which piece of a text tower's launch sequence breaks hipGraph capture?

Each case captures one piece (forward and/or backward) with torch.cuda.graph in a child
process of its own (a host-side crash in hipStreamEndCapture ends only that child), replays
it and compares the result with the eager run.  One line per case: PASS / FAIL / CRASH rc.
  python tools/capture_bisect.py [case ...]
"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CASES = ["gemm_splitk", "bias_grad", "cast", "masked_mean", "embed_gather_scatter",
         "lstm_bwd", "linear_bwd_engine", "bilstm_fwd", "bilstm_fwd_bwd", "bert2_fwd",
         "bert2_fwd_bwd"]


def _capture(torch, fn, warm=2):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(warm):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        out = fn()
    torch.cuda.synchronize()
    return g, out


def run_case(name):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import torch
    import mmdx
    from mmdx import _lib as L
    from mmdx import functional as F
    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(0)
    bf = torch.bfloat16

    def check(fn, outs):
        want = [o.clone() for o in fn()]
        gr, _ = _capture(torch, fn)
        for o in outs:
            o.zero_()
        gr.replay()
        torch.cuda.synchronize()
        got = outs
        return all(torch.equal(a, b) for a, b in zip(got, want))

    if name == "gemm_splitk":   # the BiLSTM dW_ih GEMM: A, B not k-major, K = B*L
        M, N, K = 2048, 256, 16384
        A = torch.randn(K, M, generator=g).to(dev, bf)
        B = torch.randn(K, N, generator=g).to(dev, bf)
        C = torch.empty(M, N, device=dev)
        return check(lambda: [F.gemm(A, M, False, B, N, False, M, N, K, C, N,
                                     compute_dtype=bf)], [C])
    if name == "bias_grad":
        dy = torch.randn(16384, 2048, generator=g).to(dev, bf)
        out = torch.empty(2048, device=dev)
        return check(lambda: [F._bias_grad(dy, 16384, 2048, out)], [out])
    if name == "cast":
        x = torch.randn(4096, 512, generator=g).to(dev)
        y = torch.empty(4096, 512, dtype=bf, device=dev)

        def f():
            L.call("mmdx_cast", L.BF16, L.F32, x.data_ptr(), x.numel(), y.data_ptr(),
                   L.stream())
            return [y]
        return check(f, [y])
    if name == "masked_mean":
        h = torch.randn(32, 128, 512, generator=g).to(dev, bf)
        mask = torch.ones(32, 128, dtype=torch.long, device=dev)
        out = torch.empty(32, 512, dtype=bf, device=dev)
        dh = torch.empty_like(h)

        def f():
            L.call("mmdx_masked_mean_fwd", L.BF16, h.data_ptr(), mask.data_ptr(), 32, 128, 512,
                   out.data_ptr(), L.stream())
            L.call("mmdx_masked_mean_bwd", L.BF16, out.data_ptr(), mask.data_ptr(), 32, 128,
                   512, dh.data_ptr(), L.stream())
            return [out, dh]
        return check(f, [out, dh])
    if name == "embed_gather_scatter":
        ids = torch.randint(1000, 30522, (32 * 128,), generator=g).to(dev)
        tab = torch.randn(30522, 256, generator=g).to(dev)
        out = torch.empty(32 * 128, 256, dtype=bf, device=dev)
        dtab = torch.zeros(30522, 256, device=dev)

        def f():
            L.call("mmdx_embed_gather", L.BF16, ids.data_ptr(), ids.numel(), 256,
                   tab.data_ptr(), out.data_ptr(), L.stream())
            dtab.zero_()
            L.call("mmdx_embed_scatter", L.BF16, ids.data_ptr(), ids.numel(), 256,
                   out.data_ptr(), dtab.data_ptr(), L.stream())
            return [out]
        return check(f, [out])
    if name == "lstm_bwd":
        B, Ls, H = 32, 128, 256
        whh = (torch.randn(8 * H, H, generator=g) * 0.05).to(dev, bf)
        hout = torch.randn(B, Ls, 2 * H, generator=g).to(dev, bf)
        cs = torch.randn(2, Ls, B, H, generator=g).to(dev)
        gs = torch.rand(2, Ls, B, 4 * H, generator=g).to(dev)
        dh = torch.randn(B, Ls, 2 * H, generator=g).to(dev, bf)
        dxg = torch.empty(B * Ls, 8 * H, dtype=bf, device=dev)
        dwhh = torch.empty(8 * H, H, device=dev)
        n = L.lib().mmdx_lstm_workspace_size(L.BF16, B, Ls, H)
        ws = torch.empty(n, dtype=torch.uint8, device=dev)

        def f():
            L.call("mmdx_lstm_bwd", L.BF16, whh.data_ptr(), hout.data_ptr(), cs.data_ptr(),
                   gs.data_ptr(), dh.data_ptr(), B, Ls, H, dxg.data_ptr(), dwhh.data_ptr(),
                   ws.data_ptr(), n, None, 0, 0, L.stream())
            return [dxg, dwhh]
        return check(f, [dxg, dwhh])
    if name == "linear_bwd_engine":   # an mmdx autograd node's backward on the engine thread
        lin = mmdx.layers.Linear(512, 512).to(dev)
        x = torch.randn(32, 512, generator=g).to(dev, bf).requires_grad_(True)
        gl = torch.cuda.make_graphed_callables(lin, (x,))
        y = gl(x)
        y.float().sum().backward()
        torch.cuda.synchronize()
        return True
    if name.endswith("_parity") or name == "lstm_beside_then_bilstm":
        # tests/test_graph_capture_gpu.py's tower test in a fresh process (eager fwd + bwd,
        # then make_graphed_callables, bitwise compare); the last case runs the recurrence
        # test first in the same process, as the pytest session did
        import test_graph_capture_gpu as T
        if name == "lstm_beside_then_bilstm":
            T.test_capture_lstm_recurrence_beside_trunk(dev)
        tname = "bert-base-uncased@2" if name.startswith("bert2") else "bilstm"
        T.test_capture_text_tower_fwd_bwd(dev, tname, bf if tname == "bilstm" else torch.float16)
        return True
    if name.startswith("bilstm") or name.startswith("bert2"):
        from parity_util import synth_batch
        from test_graph_capture_gpu import _Tower
        tname = "bilstm" if name.startswith("bilstm") else "bert-base-uncased@2"
        dt = bf if tname == "bilstm" else torch.float16
        torch.manual_seed(0)
        txt = mmdx.TextEncoderTransformer(tname, 512, 13, use_warmup_classifier=False,
                                          compute_dtype=dt)
        if hasattr(txt.encoder, "config") and hasattr(txt.encoder.config, "hidden_dropout_prob"):
            txt.encoder.config.hidden_dropout_prob = 0.0
            txt.encoder.config.attention_probs_dropout_prob = 0.0
        txt.to(dev).unfreeze_encoder()
        for n_, p in txt.named_parameters():
            if "pooler" in n_:
                p.requires_grad_(False)
        tower = _Tower(txt)
        _, ids, mask, _ = synth_batch(32, 128)
        ids, mask = ids.to(dev), mask.to(dev)
        if name.endswith("_fwd"):
            with torch.no_grad():
                out = tower(ids, mask)
                want = out.clone()
                gr, o = _capture(torch, lambda: tower(ids, mask))
                gr.replay()
                torch.cuda.synchronize()
                return torch.equal(o, want)
        gt = torch.cuda.make_graphed_callables(tower, (ids, mask))
        out = gt(ids, mask)
        out.float().sum().backward()
        torch.cuda.synchronize()
        return True
    raise SystemExit(f"unknown case {name}")


def main():
    if len(sys.argv) > 2 and sys.argv[1] == "--child":
        ok = run_case(sys.argv[2])
        print("RESULT", "PASS" if ok else "FAIL", flush=True)
        sys.exit(0 if ok else 1)
    cases = sys.argv[1:] or CASES
    for c in cases:
        p = subprocess.run([sys.executable, os.path.abspath(__file__), "--child", c],
                           capture_output=True, text=True, timeout=300)
        res = "PASS" if p.returncode == 0 else ("FAIL" if p.returncode == 1 else
                                               f"CRASH rc={p.returncode}")
        print(f"{c:24s} {res}", flush=True)
        if p.returncode not in (0, 1):
            print("  " + "\n  ".join((p.stdout + p.stderr).strip().splitlines()[-12:]), flush=True)


if __name__ == "__main__":
    main()
