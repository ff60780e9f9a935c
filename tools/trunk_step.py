#!/usr/bin/env python3
"""One bf16 ResNet trunk train step (forward + backward through the production launch plan)
at a given batch, run `--reps` times: the workload tools/dispatch_diff.py profiles to list
which kernels the dispatcher picks at each batch.
    python tools/trunk_step.py --arch resnet50 --batch 256
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--arch", default="resnet50")
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--reps", type=int, default=2)
    a = ap.parse_args()
    import mmdx
    from parity_util import synth_batch
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    img = mmdx.ImageEncoderCNN(a.arch, 1024, 13, compute_dtype=torch.bfloat16).to(dev)
    img.unfreeze_backbone()
    x, _, _, _ = synth_batch(a.batch, 8, hw=224)
    x = x.to(dev)
    for _ in range(a.reps):
        f = img.backbone(x)
        f.backward(torch.ones_like(f))
    torch.cuda.synchronize()
    print(f"trunk step ok: {a.arch} B={a.batch} x{a.reps}", flush=True)


if __name__ == "__main__":
    main()
