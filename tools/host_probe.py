#!/usr/bin/env python3
"""Host-side cost of one C4 train step: wall time of enqueueing K steps without
synchronising (the host runs ahead of the GPU until it blocks), vs the synchronised time.
If host enqueue time ~ GPU time, the step is launch-bound.
    python tools/host_probe.py [--steps 10]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=10)
    a = ap.parse_args()
    cfg = dict(bench.CONFIGS["c4"])
    dev = torch.device("cuda", 0)
    img, txt, fus, opt = bench.build(cfg, dev, torch.bfloat16)
    params = [p for g in opt.param_groups for p in g["params"]]
    x, ids, mask, y = bench.synth(cfg, cfg["batch"], dev, 1234)
    side = torch.cuda.Stream(device=dev)
    step = bench.make_step(img, txt, fus, opt, params, None, x, ids, mask, y, side)
    for _ in range(3):
        step()
    torch.cuda.synchronize()
    import cProfile
    import pstats
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"host enqueue {1e3 * (t1 - t0) / a.steps:.3f} ms/step, "
          f"wall {1e3 * (t2 - t0) / a.steps:.3f} ms/step")
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(3):
        step()
    pr.disable()
    torch.cuda.synchronize()
    st = pstats.Stats(pr)
    st.sort_stats("tottime").print_stats(18)


if __name__ == "__main__":
    main()
