#!/usr/bin/env python3
"""Stage-by-stage error of the mmdx train forward vs the CPU oracle at a benched geometry.

For R50 + BiLSTM at 224x224, L = 128 and batch B: z_img, z_txt, logits and loss of
  * mmdx bf16 (the benched compute dtype), * mmdx fp32, * the oracle itself under CPU bf16
  autocast (the error bf16 arithmetic alone produces on this model),
each against the fp32 oracle.  Prints one JSON line per variant.
  python tools/parity_probe.py --batch 128
"""
import argparse
import copy
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--hw", type=int, default=224)
    ap.add_argument("--seq", type=int, default=128)
    ap.add_argument("--text", default="bilstm")
    ap.add_argument("--image", default="resnet50")
    ap.add_argument("--grads", action="store_true", help="also compare parameter gradients")
    args = ap.parse_args()
    torch.set_num_threads(16)
    import mmdx
    from parity_util import build_pair, synth_batch
    x, ids, mask, y = synth_batch(args.batch, args.seq, hw=args.hw)
    ref, _, _, _ = build_pair(args.image, args.text)
    ref.train()
    ref.image.unfreeze_backbone()
    ref_bf = copy.deepcopy(ref)

    def stages(img, txt, fus, xx, ii, mm):
        z_img = img(xx)["embeddings"]
        z_txt = txt(input_ids=ii, attention_mask=mm)["embeddings"]
        logits = fus(z_img, z_txt)["disease_logits"]
        return {"z_img": z_img, "z_txt": z_txt, "logits": logits}

    import time
    from parity_util import grad_report
    bce = torch.nn.BCEWithLogitsLoss()
    t0 = time.time()
    with torch.set_grad_enabled(args.grads):
        want = stages(ref.image, ref.text, ref.fusion, x, ids, mask)
        if args.grads:
            bce(want["logits"], y).backward()
        t1 = time.time()
        with torch.autocast("cpu", dtype=torch.bfloat16):
            got_bf = stages(ref_bf.image, ref_bf.text, ref_bf.fusion, x, ids, mask)
        if args.grads:
            bce(got_bf["logits"].float(), y).backward()
        t2 = time.time()
    print(json.dumps({"oracle_fp32_s": round(t1 - t0, 1), "oracle_bf16_s": round(t2 - t1, 1)}))
    gref = {n: p.grad for n, p in ref.named_parameters() if p.grad is not None}

    def grad_summary(name, model):
        if not args.grads:
            return
        gm = {n: p.grad for n, p in model.named_parameters() if p.grad is not None}
        rep = grad_report(gm, gref)
        cs = sorted(rep.items(), key=lambda kv: -kv[1][0])
        rs = sorted(rep.items(), key=lambda kv: -kv[1][1])
        import numpy as np
        print(json.dumps({"variant": name, "grads": len(rep),
                          "median_1mcos": float(np.median([c for c, _ in rep.values()])),
                          "worst_1mcos": [(n, round(c, 6)) for n, (c, _) in cs[:5]],
                          "median_normerr": float(np.median([r for _, r in rep.values()])),
                          "worst_normerr": [(n, round(r, 6)) for n, (_, r) in rs[:5]]}),
              flush=True)

    def report(name, got):
        out = {"variant": name, "batch": args.batch}
        for k, w in want.items():
            g = got[k].detach().float().cpu()
            out[k] = {"max_abs": round((g - w).abs().max().item(), 5),
                      "rel_max": round(((g - w).abs().max() / w.abs().max()).item(), 5),
                      "rel_rms": round(((g - w).norm() / w.norm()).item(), 5),
                      "ref_absmax": round(w.abs().max().item(), 4)}
        print(json.dumps(out), flush=True)

    report("oracle_cpu_bf16_autocast", got_bf)
    grad_summary("oracle_cpu_bf16_autocast", ref_bf)
    dev = torch.device("cuda", 0)
    for dt in (torch.bfloat16, torch.float32):
        _, img, txt, fus = build_pair(args.image, args.text, dtype=dt)
        img.to(dev).unfreeze_backbone()
        txt.to(dev).unfreeze_encoder()
        fus.to(dev).train()
        with torch.set_grad_enabled(args.grads):
            got = stages(img, txt, fus, x.to(dev), ids.to(dev), mask.to(dev))
            if args.grads:
                mmdx.BCEWithLogitsLoss()(got["logits"], y.to(dev)).backward()
        torch.cuda.synchronize()
        name = f"mmdx_{str(dt).split('.')[-1]}"
        report(name, got)
        wrap = torch.nn.ModuleDict({"image": img, "text": txt, "fusion": fus})
        grad_summary(name, wrap)


if __name__ == "__main__":
    main()
