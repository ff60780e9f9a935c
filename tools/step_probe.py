#!/usr/bin/env python3
"""Phase timeline of one C4 train step, GPU side (events on the stream each phase runs on)
next to the host time at which each phase was issued — shows whether a stream waits for
the host (issue-bound) or for the other stream (dependency-bound).
    python tools/step_probe.py [--config c4] [--steps 5] [--no-events]
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
    ap.add_argument("--config", default="c4")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--text-first", action="store_true")
    ap.add_argument("--text-only", action="store_true")
    ap.add_argument("--image-only", action="store_true")
    ap.add_argument("--ds-main", action="store_true",
                    help="downsample branch in order on the main stream (A/B)")
    ap.add_argument("--threads", action="store_true", help="issue the towers from two threads")
    ap.add_argument("--bwd-thread", action="store_true",
                    help="issue the text backward from a worker thread, concurrently with "
                         "the image trunk's backward")
    args = ap.parse_args()
    cfg = dict(bench.CONFIGS[args.config])
    dev = torch.device("cuda", 0)
    import mmdx
    from mmdx import optim as MO
    if args.ds_main:
        mmdx.resnet.DS_SIDE_STREAM = False
    from mmdx.schedule import two_tower_backward
    img, txt, fus, opt = bench.build(cfg, dev, torch.bfloat16)
    params = [p for grp in opt.param_groups for p in grp["params"]]
    x, ids, mask, y = bench.synth(cfg, cfg["batch"], dev, 1234)
    # the bench's stream priorities (MMDX_PRIO, default main+text)
    prio = os.environ.get("MMDX_PRIO", "main+text")
    if prio in ("main", "main+text"):
        torch.cuda.set_stream(torch.cuda.Stream(device=dev, priority=-1))
    side = torch.cuda.Stream(device=dev, priority=-1 if prio in ("text", "main+text") else 0)
    from mmdx.schedule import TwoTowerForward
    towers = TwoTowerForward(text_stream=side)
    marks = []

    def mark(name, st=None):
        st = st or torch.cuda.current_stream()
        e = torch.cuda.Event(enable_timing=True)
        e.record(st)
        marks.append((name, e, time.perf_counter()))

    def step():
        opt.zero_grad(set_to_none=True)
        main = torch.cuda.current_stream()
        mark("start", main)
        side.wait_stream(main)
        if args.threads:
            def text_fn():
                z = txt(input_ids=ids, attention_mask=mask)["embeddings"]
                mark("txt_fwd_done", side)
                return z
            z_img, z_txt = towers(lambda: img(x)["embeddings"], text_fn)
            mark("img_fwd_issued", main)
        elif args.text_first:
            with torch.cuda.stream(side):
                z_txt = txt(input_ids=ids, attention_mask=mask)["embeddings"]
                mark("txt_fwd_done", side)
        if not args.threads:
            z_img = img(x)["embeddings"]
            mark("img_fwd_issued", main)
        if not args.text_first and not args.threads:
            with torch.cuda.stream(side):
                z_txt = txt(input_ids=ids, attention_mask=mask)["embeddings"]
                mark("txt_fwd_done", side)
        main.wait_stream(side)
        logits = fus(z_img, z_txt)["disease_logits"]
        loss = mmdx.BCEWithLogitsLoss()(logits, y)
        mark("head_fwd", main)
        head = [p for p in fus.parameters() if p.requires_grad]
        loss.backward(inputs=[z_img, z_txt] + head, retain_graph=True)
        mark("head_bwd", main)
        side.wait_stream(main)

        def text_bwd():
            torch.cuda.set_device(dev)
            with torch.cuda.stream(side):
                g = z_txt.grad
                z_txt.backward(g)
                z_txt.grad = None
                mark("txt_bwd_done", side)
        fut = towers._pool.submit(text_bwd) if args.bwd_thread else None
        g = z_img.grad
        z_img.backward(g)
        z_img.grad = None
        mark("img_bwd_issued", main)
        if fut is None:
            text_bwd()
        else:
            fut.result()
        main.wait_stream(side)
        mark("joined", main)
        _, scale = MO.grad_norm(params, 1.0)
        opt.step(grad_scale=scale)
        mark("end", main)
        return loss

    if args.image_only:  # the image tower alone (its wgrad stream still concurrent)
        for it in range(6):
            torch.cuda.synchronize()
            e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
            e[0].record()
            z = img(x)["embeddings"]
            e[1].record()
            z.float().sum().backward()
            e[2].record()
            torch.cuda.synchronize()
            print(f"image only: fwd {e[0].elapsed_time(e[1]):.3f} ms  bwd "
                  f"{e[1].elapsed_time(e[2]):.3f} ms")
        return
    if args.text_only:  # the text tower alone: its uncontended forward / backward time
        for it in range(4):
            torch.cuda.synchronize()
            e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
            e[0].record()
            z = txt(input_ids=ids, attention_mask=mask)["embeddings"]
            e[1].record()
            z.float().sum().backward()
            e[2].record()
            torch.cuda.synchronize()
            print(f"text only: fwd {e[0].elapsed_time(e[1]):.3f} ms  bwd "
                  f"{e[1].elapsed_time(e[2]):.3f} ms")
        return
    for _ in range(5):
        step()
    torch.cuda.synchronize()
    for s in range(args.steps):
        marks.clear()
        torch.cuda.synchronize()
        step()
        torch.cuda.synchronize()
        e0, h0 = marks[0][1], marks[0][2]
        print(f"step {s}")
        for name, e, h in marks:
            print(f"  {name:16s} gpu {e0.elapsed_time(e):8.3f} ms   host {1e3 * (h - h0):8.3f} ms")
    # steady state (back-to-back, no sync): total
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(10):
        step()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"back-to-back: {1e3 * (t2 - t0) / 10:.3f} ms/step, host enqueue "
          f"{1e3 * (t1 - t0) / 10:.3f} ms/step")


if __name__ == "__main__":
    main()
