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


def hf_beam_stepper(t5, enc, nb, k):
    """The reference's beam step as a stepper for T5Head.generate(_stepper=...): transformers'
    T5 (the reference's report head, IP:190-196) re-run over every running prefix in fp32,
    log_softmax of the last position, the MinNewTokens / NoRepeatNGram bans the host
    loop hands over set to -inf, the running beam scores added, torch.topk over the
    num_beams x vocab candidates of each batch row — GenerationMixin._beam_search's order of
    operations.  enc: [B, Lc, D] condition tokens; the step runs where `t5` lives (a long
    search re-runs every prefix: the GPU copy of transformers' model keeps that fast)."""
    from transformers.modeling_outputs import BaseModelOutput
    B = enc.shape[0]
    mdev = next(t5.parameters()).device
    enc_r = enc.float().to(mdev).repeat_interleave(nb, dim=0)
    V = t5.config.vocab_size

    def step(hist, pos, slots, sc, bans, eos_ban):
        with torch.no_grad():
            out = t5(encoder_outputs=BaseModelOutput(last_hidden_state=enc_r),
                     decoder_input_ids=torch.from_numpy(hist).to(mdev))
            lp = torch.log_softmax(out.logits[:, -1].float(), -1)
        if eos_ban >= 0:
            lp[:, eos_ban] = -float("inf")
        if len(bans):
            b = torch.from_numpy(bans).long().to(mdev)
            lp[b[:, 0], b[:, 1]] = -float("inf")
        s = (lp + torch.from_numpy(sc).float().to(mdev)[:, None]).reshape(B, nb * V)
        v, i = torch.topk(s, k + 1, dim=1)
        step.last = v.cpu().numpy()  # k + 1 values: the gap below the k-th candidate
        return v[:, :k].cpu().numpy().copy(), i[:, :k].cpu().numpy().copy()

    step.vocab = V
    return step


class BeamStepCheck:
    """Stepper that follows the reference's decisions (hf_beam_stepper) and checks the mmdx
    device step (t5._DecodeState: KV-cached decoder, device logits processors, top-k) on the
    same state at every step: the k top candidate scores agree to atol = tol * max(1, max |lp|)
    over the batch row's candidates (lp: a candidate's log-prob, its score minus its parent
    beam's running score; the rounding of a log-softmax scales with the row's logits),
    and the candidate index agrees wherever its score is separated from its neighbours (and
    from the (k+1)-th score) by more than twice that tolerance.  `min_gap` records the smallest
    separation seen: if it stays above the tolerance, the search has no near-tie and the
    end-to-end mmdx output must equal the reference's bit for bit."""

    def __init__(self, ref_step, dec, B, nb, k, tol=1e-4):
        self.ref, self.dec = ref_step, dec
        self.B, self.nb, self.k, self.tol = B, nb, k, tol
        self.min_gap = float("inf")
        self.ambiguous = 0   # candidates within 2 x tolerance of a neighbour (not compared)
        self.max_err = 0.0   # largest |mmdx - reference| / the row's log-prob scale
        self.steps = 0

    def __call__(self, hist, pos, slots, sc, bans, eos_ban):
        import numpy as np
        rv, ri = self.ref(hist, pos, slots, sc, bans, eos_ban)
        full = self.ref.last
        mv, mi = self.dec.step(hist[:, pos], pos, slots, sc, bans, eos_ban, self.B, self.nb,
                               self.k)
        fin = np.isfinite(rv)
        assert np.array_equal(fin, np.isfinite(mv)), (self.steps, rv, mv)
        # the running score is added identically on both sides: the error scales with the
        # candidate's own log-prob, not with the accumulated score
        V = self.ref.vocab
        par = np.take_along_axis(sc.reshape(self.B, self.nb), ri // V, axis=1)
        lp = np.where(fin, rv - par, 0.0)
        scale = np.maximum(1.0, np.abs(lp).max(axis=1, keepdims=True))
        atol = self.tol * np.broadcast_to(scale, lp.shape)
        diff = np.abs(np.where(fin, mv - rv, 0.0))
        self.max_err = max(self.max_err, float((diff / atol).max()) * self.tol)
        assert (diff <= atol).all(), (self.steps, float(diff.max()))
        for b in range(self.B):
            for j in range(self.k):
                if not fin[b, j]:
                    continue
                up = full[b, j - 1] - full[b, j] if j > 0 else np.inf
                dn = full[b, j] - full[b, j + 1]
                gap = min(up, dn)
                self.min_gap = min(self.min_gap, float(gap))
                if gap > 2 * atol[b, j]:
                    assert mi[b, j] == ri[b, j], (self.steps, b, j, mi[b], ri[b])
                else:
                    self.ambiguous += 1
        self.steps += 1
        return rv, ri
