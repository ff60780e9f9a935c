#!/usr/bin/env python3
"""Debug: the KV-cached beam step (t5._DecodeState.step) against the full-prefix recompute
(T5Head._last_log_probs + host logits processors + host top-k) along ONE beam search
(the reference path's decisions drive both), printing the first step whose top-k differs.
    python tools/lab/t5_beam_debug.py"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from test_t5_gpu import _t5  # noqa: E402

import mmdx  # noqa: E402,F401
from mmdx.t5 import T5Head, _DecodeState, _ngram_bans  # noqa: E402


def main():
    dev = torch.device("cuda")
    ref = _t5(2, seed=4)
    with torch.no_grad():
        ref.shared.weight.mul_(4.0)
    ref.to(dev).eval()
    head = T5Head(ref)
    g = torch.Generator().manual_seed(21)
    enc = torch.randn(2, 4, 512, generator=g).to(dev)
    B, nb, max_new, min_new, ngram, eos = 2, 4, 14, 6, 3, 1
    R, V, k = B * nb, ref.config.vocab_size, 2 * nb
    L = 1 + max_new
    enc_r = enc.repeat_interleave(nb, dim=0)
    dec = _DecodeState(head, enc_r, torch.float32, L)
    run_seq = np.zeros((B, nb, L), dtype=np.int64)
    run_sc = np.zeros((B, nb), dtype=np.float32)
    run_sc[:, 1:] = -1e9
    slots = np.zeros((R, L), dtype=np.int32)
    base = (np.arange(B) * nb)[:, None]
    for cur in range(1, L):
        pos = cur - 1
        slots[:, pos] = np.arange(R)
        hist = run_seq[:, :, :cur].reshape(R, cur)
        bans = _ngram_bans(hist, ngram)
        eos_ban = eos if cur - 1 < min_new else -1
        val, idx = dec.step(hist[:, pos], pos, slots, run_sc.reshape(R), bans, eos_ban, B, nb, k)
        with torch.no_grad():
            lp = head._last_log_probs(torch.from_numpy(hist).to(dev), enc_r,
                                      torch.float32).cpu().numpy()
        if eos_ban >= 0:
            lp[:, eos] = -np.inf
        for r, t in bans:
            lp[r, t] = -np.inf
        acc = (lp.reshape(B, nb, V) + run_sc[:, :, None]).reshape(B, nb * V)
        ridx = np.argsort(-acc, axis=1, kind="stable")[:, :k]
        rval = np.take_along_axis(acc, ridx, axis=1)
        same = np.array_equal(idx, ridx)
        print(f"cur {cur}: idx equal {same}, max |val diff| {np.abs(val - rval).max():.3e}")
        if not same:
            print(" mine", idx, val, "\n ref ", ridx, rval, "\n bans", bans)
        # follow the reference's decisions (greedy top-nb of the candidates)
        tk_beam, tk_tok = ridx // V, ridx % V
        nxt = np.argsort(-rval, axis=1, kind="stable")[:, :nb]
        parent = np.take_along_axis(tk_beam, nxt, axis=1)
        slots = slots[(parent + base).reshape(R)]
        run_seq = np.take_along_axis(run_seq, parent[:, :, None], axis=1).copy()
        run_seq[:, :, cur] = np.take_along_axis(tk_tok, nxt, axis=1)
        run_sc = np.take_along_axis(rval, nxt, axis=1).astype(np.float32)


if __name__ == "__main__":
    main()
