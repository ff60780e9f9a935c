#!/usr/bin/env python3
"""cProfile of the host side of bench.py's train step (C4 by default): where the ~16 ms of
Python enqueue time per step goes.   python tools/host_profile.py [--config c4] [--steps 5]"""
import argparse
import cProfile
import os
import time
import pstats
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c4")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--idle", action="store_true",
                    help="profile each step issued onto an idle device (sync between steps)")
    a = ap.parse_args()
    cfg = dict(bench.CONFIGS[a.config])
    dev = torch.device("cuda", 0)
    img, txt, fus, opt = bench.build(cfg, dev, torch.bfloat16)
    params = [p for g in opt.param_groups for p in g["params"]]
    x, ids, mask, y = bench.synth(cfg, cfg["batch"], dev, 1234)
    side = torch.cuda.Stream(device=dev)
    step = bench.make_step(img, txt, fus, opt, params, None, x, ids, mask, y, side)
    for _ in range(3):
        step()
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    pt = cProfile.Profile()   # the text tower's worker thread (TwoTowerForward)
    pool = step.towers._pool
    pool.submit(pt.enable).result()
    host = 0.0
    if a.idle:
        for _ in range(a.steps):
            torch.cuda.synchronize()
            pr.enable()
            t0 = time.perf_counter()
            step()
            host += (time.perf_counter() - t0) / a.steps
            pr.disable()
    else:
        pr.enable()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            step()
        host = (time.perf_counter() - t0) / a.steps
        pr.disable()
    pool.submit(pt.disable).result()
    torch.cuda.synchronize()
    print(f"host time per step (main thread, wall, device busy): {host * 1e3:.2f} ms")
    st = pstats.Stats(pr)
    st.sort_stats("tottime").print_stats(35)
    st.sort_stats("cumulative").print_stats(25)
    print("=== text tower thread ===")
    st2 = pstats.Stats(pt)
    st2.sort_stats("cumulative").print_stats(25)


if __name__ == "__main__":
    main()
