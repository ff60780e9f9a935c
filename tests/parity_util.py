"""Helpers shared by the model-level parity tests (oracle <-> mmdx weight transfer)."""
import torch

import mmdx
from oracle import ref_cpu as R


def build_pair(image_backbone="resnet18", text_model="embed-mean", bert_layers=2, seed=0,
               dtype=torch.float32, dropout=0.0):
    """Oracle model (CPU, seeded) and the mmdx model with identical weights."""
    torch.manual_seed(seed)
    ref = R.RefMultimodal(image_backbone, text_model, bert_layers=bert_layers, dropout=dropout)
    img = mmdx.ImageEncoderCNN(image_backbone, 1024, 13, compute_dtype=dtype)
    txt = mmdx.TextEncoderTransformer(_text_name(text_model, bert_layers), 512, 13,
                                      compute_dtype=dtype)
    fus = mmdx.FusionTransformerModel(1024, 512, 1024, 13, dropout=dropout)
    img.load_state_dict(ref.image.state_dict())
    txt.load_state_dict(ref.text.state_dict(), strict=True)
    fus.load_state_dict(ref.fusion.state_dict())
    return ref, img, txt, fus


def _text_name(text_model, bert_layers):
    if text_model.startswith("bert"):
        return f"bert-base-uncased@{bert_layers}" if bert_layers != 12 else "bert-base-uncased"
    return text_model


def synth_batch(B, L, hw=64, seed=1234, pad=False):
    """SURVEY §8(d) synthetic inputs: U[0,1) images, ImageNet-normalised; [CLS] ids [SEP]."""
    g = torch.Generator().manual_seed(seed)
    x = torch.rand(B, 3, hw, hw, generator=g)
    mean = torch.tensor([0.485, 0.456, 0.406]).view(1, 3, 1, 1)
    std = torch.tensor([0.229, 0.224, 0.225]).view(1, 3, 1, 1)
    x = (x - mean) / std
    ids = torch.randint(1000, 30522, (B, L), generator=g)
    ids[:, 0] = 101
    mask = torch.ones(B, L, dtype=torch.long)
    if pad:
        lens = torch.randint(8, L + 1, (B,), generator=g)
        for b in range(B):
            ids[b, lens[b] - 1] = 102
            ids[b, lens[b]:] = 0
            mask[b, lens[b]:] = 0
    else:
        ids[:, -1] = 102
    labels = (torch.rand(B, 13, generator=torch.Generator().manual_seed(seed + 1)) < 0.15)
    return x, ids, mask, labels.float()


def mmdx_forward(img, txt, fus, x, ids, mask):
    z_img = img(x)["embeddings"]
    z_txt = txt(input_ids=ids, attention_mask=mask)["embeddings"]
    return fus(z_img, z_txt)["disease_logits"]


def rel_err(a, b):
    a = a.detach().float().cpu()
    b = b.detach().float().cpu()
    return ((a - b).abs().max() / b.abs().max().clamp(min=1e-12)).item()


def cosine(a, b):
    a = a.detach().double().cpu().flatten()
    b = b.detach().double().cpu().flatten()
    return (a @ b / (a.norm() * b.norm()).clamp(min=1e-30)).item()


def norm_ratio(a, b):
    """|a| / |b| (fp64): cosine ignores magnitude, so the grad checks pair it with this."""
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    return (a.norm() / b.norm().clamp(min=1e-300)).item()


def grad_report(mine: dict, ref: dict):
    """{name: (1 - cos, |norm ratio - 1|)} over the tensors both sides have."""
    return {n: (1.0 - cosine(mine[n], ref[n]), abs(norm_ratio(mine[n], ref[n]) - 1.0))
            for n in ref}
