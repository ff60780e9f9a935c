#!/usr/bin/env python3
"""Regenerate the golden vectors in tests/golden/ from the CPU oracle (oracle/ref_cpu.py).

The reference publishes no numeric fixtures (its tests only print shapes), and
cannot be imported offline, so these vectors pin the ORACLE: inputs are seeded, weights
come from a seeded construction (torch.manual_seed before building the module), outputs
are the oracle's fp32 CPU results.  tests/test_oracle_golden.py rebuilds the same modules
from the same seeds and checks them against these files; the GPU parity tests load the
oracle weights into the mmdx modules and compare with the same numbers.

  python tests/golden/make_golden.py          # writes tests/golden/*.npz
"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(HERE))

from oracle import ref_cpu as R  # noqa: E402


def fusion_case():
    torch.manual_seed(0)
    fus = R.RefFusion(dropout=0.0)
    g = torch.Generator().manual_seed(11)
    z_img = torch.randn(4, 1024, generator=g)
    z_txt = torch.randn(4, 512, generator=g)
    y = (torch.rand(4, 13, generator=g) < 0.3).float()
    zi = z_img.clone().requires_grad_(True)
    zt = z_txt.clone().requires_grad_(True)
    logits = fus(zi, zt)["disease_logits"]
    loss = torch.nn.BCEWithLogitsLoss()(logits, y)
    loss.backward()
    return dict(z_img=z_img, z_txt=z_txt, y=y, logits=logits.detach(), loss=loss.detach(),
                d_z_img=zi.grad, d_z_txt=zt.grad,
                d_w0_rows=fus.fusion_mlp[0].weight.grad[:8],
                d_w0_norm=fus.fusion_mlp[0].weight.grad.norm(), d_head=fus.disease_head.weight.grad)


def resnet_case(arch):
    torch.manual_seed(0)
    enc = R.RefImageEncoderCNN(arch, 1024, 13)
    enc.unfreeze_backbone()
    g = torch.Generator().manual_seed(12)
    x = torch.randn(2, 3, 64, 64, generator=g)
    y = (torch.rand(2, 13, generator=g) < 0.3).float()
    out = enc(x)
    loss = torch.nn.BCEWithLogitsLoss()(out["logits"], y)
    loss.backward()
    return dict(x=x, y=y, embeddings=out["embeddings"].detach(), logits=out["logits"].detach(),
                loss=loss.detach(), d_proj_rows=enc.proj.weight.grad[:4],
                d_proj_norm=enc.proj.weight.grad.norm(), d_conv1=enc.backbone[0].weight.grad)


def bert_case():
    torch.manual_seed(0)
    txt = R.RefTextEncoderTransformer("bert-base-uncased", 512, 13, bert_layers=2, dropout=0.0)
    txt.eval()
    g = torch.Generator().manual_seed(13)
    ids = torch.randint(1000, 30522, (3, 16), generator=g)
    ids[:, 0] = 101
    lens = torch.tensor([16, 9, 5])
    mask = (torch.arange(16)[None] < lens[:, None]).long()
    ids[mask == 0] = 0
    with torch.no_grad():
        out = txt(input_ids=ids, attention_mask=mask)
    return dict(ids=ids, mask=mask, embeddings=out["embeddings"], logits=out["logits"])


def c1_case(name="e1.jpg", seed=14):
    """BASELINE config 1: a reference sample image (backend/sample_images/e1.jpg, e2.jpg)
    through image_transfom_into_tensor (TP:112-119) + a 64-token synthetic report, single
    forward, R50 + BERT-base."""
    from PIL import Image
    from oracle.ref_cpu import reference_transform
    img = Image.open(os.path.join(HERE, name)).convert("RGB")
    x = reference_transform(img)[None]
    torch.manual_seed(0)
    model = R.RefMultimodal("resnet50", "bert-base-uncased", dropout=0.0)
    model.eval()
    g = torch.Generator().manual_seed(seed)
    ids = torch.randint(1000, 30522, (1, 64), generator=g)
    ids[0, 0], ids[0, -1] = 101, 102
    mask = torch.ones(1, 64, dtype=torch.long)
    with torch.no_grad():
        logits = model(x, ids, mask)
    return dict(x=x, ids=ids, mask=mask, logits=logits)


def main():
    import sys
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    cases = {"fusion": fusion_case, "resnet18": lambda: resnet_case("resnet18"),
             "resnet50": lambda: resnet_case("resnet50"), "bert2": bert_case, "c1": c1_case,
             "c1_e2": lambda: c1_case("e2.jpg", 15)}
    only = sys.argv[1:]   # e.g. `python make_golden.py c1_e2`: regenerate only those cases
    cases = {k: f() for k, f in cases.items() if not only or k in only}
    for name, d in cases.items():
        path = os.path.join(HERE, f"{name}.npz")
        np.savez_compressed(path, **{k: v.numpy() for k, v in d.items()})
        print(path, os.path.getsize(path))


if __name__ == "__main__":
    main()
