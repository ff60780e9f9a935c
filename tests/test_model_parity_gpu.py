"""Model-level parity: the mmdx multimodal train step vs the CPU oracle.

Stated tolerances: fp32 logits max-abs <= 1e-4*max(1,|ref|), loss rel <= 1e-5.
Gradients are judged against the oracle run in fp64 (the fp32 oracle itself is only
~0.9992-cosine-accurate on deep BatchNorm grads of ResNet-50 at 2x2 final spatial size):
1 - cos(mmdx, oracle64) <= max(5e-4, 8 * (1 - cos(oracle32, oracle64))) for every tensor,
and | |g|/|g64| - 1 | <= max(1e-3, 8x the fp32 oracle's own norm error) (cosine is blind to
a uniformly scaled gradient)
(both fp32 paths accumulate K up to 4608 in different orders; a wrong kernel gives 1-cos >> 1e-2).
bf16 path: logits max-abs <= 5e-2*max(1,|ref|).
"""
import copy
import pytest
import torch

import mmdx
from oracle import ref_cpu as R
from parity_util import build_pair, cosine, mmdx_forward, norm_ratio, rel_err, synth_batch

pytestmark = pytest.mark.gpu


def _grads_by_name(module):
    return {n: p.grad for n, p in module.named_parameters() if p.grad is not None}


@pytest.mark.parametrize("arch,text", [("resnet18", "embed-mean"), ("resnet50", "embed-mean")])
def test_train_step_parity_fp32(dev, arch, text):
    ref, img, txt, fus = build_pair(arch, text)
    ref64 = copy.deepcopy(ref).double()
    x, ids, mask, y = synth_batch(4, 16, hw=64, pad=True)
    ref.train()
    ref.image.unfreeze_backbone()
    logits_ref = ref(x, ids, mask)
    loss_ref = torch.nn.BCEWithLogitsLoss()(logits_ref, y)
    loss_ref.backward()
    ref64.train()
    torch.nn.BCEWithLogitsLoss()(ref64(x.double(), ids, mask), y.double()).backward()

    img.to(dev).unfreeze_backbone()
    txt.to(dev).train()
    fus.to(dev).train()
    logits = mmdx_forward(img, txt, fus, x.to(dev), ids.to(dev), mask.to(dev))
    loss = mmdx.BCEWithLogitsLoss()(logits, y.to(dev))
    loss.backward()
    torch.cuda.synchronize()
    assert (logits.cpu() - logits_ref.detach()).abs().max() <= 1e-4 * max(
        1.0, logits_ref.abs().max().item())
    assert abs(loss.item() - loss_ref.item()) <= 1e-5 * abs(loss_ref.item())
    for mod_ref, mod64, mod in ((ref.image, ref64.image, img), (ref.text, ref64.text, txt),
                                (ref.fusion, ref64.fusion, fus)):
        gr = _grads_by_name(mod_ref)
        g64 = _grads_by_name(mod64)
        gm = _grads_by_name(mod)
        assert set(gr) == set(gm), set(gr) ^ set(gm)
        for n in gr:
            own = 1.0 - cosine(gr[n], g64[n])
            c = 1.0 - cosine(gm[n], g64[n])
            assert c <= max(5e-4, 8 * own), f"grad {n}: 1-cos {c:.2e} (oracle32 {own:.2e})"
            own_r = abs(norm_ratio(gr[n], g64[n]) - 1.0)
            r = abs(norm_ratio(gm[n], g64[n]) - 1.0)
            assert r <= max(1e-3, 8 * own_r), f"grad {n}: |norm ratio-1| {r:.2e} ({own_r:.2e})"
    # BN running statistics follow the train-mode update
    rm = dict(img.named_buffers())
    for n, b in ref.image.named_buffers():
        if "running" in n:
            assert rel_err(rm[n], b) < 1e-4, n


def test_bf16_forward_close(dev):
    ref, img, txt, fus = build_pair("resnet18", "embed-mean", dtype=torch.bfloat16)
    x, ids, mask, y = synth_batch(4, 16, hw=64)
    ref.eval()
    with torch.no_grad():
        logits_ref = ref(x, ids, mask)
    img.to(dev).eval()
    txt.to(dev).eval()
    fus.to(dev).eval()
    with torch.no_grad():
        logits = mmdx_forward(img, txt, fus, x.to(dev), ids.to(dev), mask.to(dev))
    assert (logits.float().cpu() - logits_ref).abs().max() <= 5e-2 * max(
        1.0, logits_ref.abs().max().item())
