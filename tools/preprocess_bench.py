#!/usr/bin/env python3
"""GPU image preprocessing throughput (mmdx_image_preprocess) vs the
reference's per-image CPU transform, on B decoded 512x512 RGB images (the size of the
reference's backend/sample_images).  Reports images/s, the kernels' HBM roofline fraction
(algorithmic bytes = source pixels read once + fp32 output written once) and the CPU rate.
    python tools/preprocess_bench.py [--batch 128] [--reps 20]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402
from PIL import Image  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    from mmdx import _lib as L
    from mmdx import preprocess as PP
    from oracle import ref_cpu as R
    dev = torch.device("cuda", 0)
    g = np.random.default_rng(0)
    ims = [Image.fromarray(g.integers(0, 256, (512, 512, 3), dtype=np.uint8), "RGB")
           for _ in range(a.batch)]
    arrays = [PP._as_array(im) for im in ims]
    descs, coef, temp_bytes, max_trows, total = PP.plan_batch(arrays)
    px = torch.from_numpy(np.concatenate([x.reshape(-1) for x in arrays])).to(dev)
    d_desc = torch.from_numpy(descs.view(np.uint8).copy()).to(dev)
    d_coef = torch.from_numpy(coef).to(dev)
    temp = torch.empty(temp_bytes, dtype=torch.uint8, device=dev)
    out = torch.empty((a.batch, 3, 224, 224), dtype=torch.float32, device=dev)

    def run():
        L.call("mmdx_image_preprocess", px.data_ptr(), d_desc.data_ptr(), a.batch,
               d_coef.data_ptr(), max_trows, 224, 224, temp.data_ptr(), out.data_ptr(),
               L.stream())
    for _ in range(3):
        run()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(a.reps):
        run()
    e.record()
    torch.cuda.synchronize()
    ms = s.elapsed_time(e) / a.reps
    nbytes = total + out.numel() * 4
    ok = torch.equal(out[:4].cpu(), torch.stack([R.reference_transform(im) for im in ims[:4]]))
    t0 = time.perf_counter()
    n = 0
    while time.perf_counter() - t0 < 5.0:
        R.reference_transform(ims[n % len(ims)])
        n += 1
    cpu = n / (time.perf_counter() - t0)
    print(json.dumps({"metric": "images/s (Resize256+CenterCrop224+ToTensor+Normalize)",
                      "batch": a.batch, "gpu_ms_per_batch": round(ms, 4),
                      "gpu_images_per_s": round(a.batch / ms * 1e3, 1),
                      "roofline": {"bound": "hbm", "achieved_GBs": round(nbytes / ms / 1e6, 1),
                                   "peak_GBs": 8000.0,
                                   "frac": round(nbytes / ms / 1e6 / 8000.0, 4),
                                   "algorithmic_bytes_per_batch": int(nbytes)},
                      "bitwise_equal_to_reference": bool(ok),
                      "cpu_baseline": {"images_per_s": round(cpu, 1), "cores": 1,
                                       "kind": "reference (PIL resize + torch normalise)"}}))


if __name__ == "__main__":
    main()
