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


def beam_score(t5, enc, seq, length_penalty=1.0, eos=1, pad=0):
    """Length-normalised beam score of one generated sequence under transformers' T5 (the
    reference's report head, fp64 teacher forcing): sum of log_softmax log-probs of the
    generated tokens (the logits processors only mask tokens, they do not renormalise)
    divided by (generated length) ** length_penalty, as GenerationMixin._beam_search scores a
    finished hypothesis.  seq: 1-D ids starting with the decoder start token; trailing pads
    after EOS (or after the end of a shorter hypothesis) are ignored."""
    import copy
    from transformers.modeling_outputs import BaseModelOutput
    m = copy.deepcopy(t5).double().eval()
    ids = [int(t) for t in seq]
    n = len(ids)
    if eos in ids[1:]:
        n = ids.index(eos, 1) + 1
    else:
        while n > 1 and ids[n - 1] == pad:
            n -= 1
    x = torch.tensor([ids[:n]])
    with torch.no_grad():
        out = m(encoder_outputs=BaseModelOutput(last_hidden_state=enc.double()[None]),
                decoder_input_ids=x[:, :-1])
        lp = torch.log_softmax(out.logits[0], -1)
    tot = sum(lp[i, ids[i + 1]].item() for i in range(n - 1))
    return tot / float(n - 1) ** length_penalty


def assert_beams_equivalent(t5, enc, got, want, length_penalty=1.0, rtol=1e-4):
    """Beam-search outputs agree: identical ids, or — where duplicate beams tie to within an
    ulp (a random-init T5 repeats tokens, so equal-score hypotheses are common and the
    tie-break order follows the last bit of fp32 sums) — hypotheses with the same
    length-normalised score under the reference model."""
    for b in range(want.shape[0]):
        g = [int(t) for t in got[b]]
        w = [int(t) for t in want[b]]
        if g == w[:len(g)] and all(t == 0 for t in w[len(g):]):
            continue
        sg = beam_score(t5, enc[b], g, length_penalty)
        sw = beam_score(t5, enc[b], w, length_penalty)
        assert abs(sg - sw) <= rtol * abs(sw), (b, sg, sw, g, w)
