"""inference() (IP:151-206 minus T5) on the HIP path vs the oracle's IP:174-186 restatement,
on the reference's own sample image and patient details (tests/golden/e1.jpg,
patient_details.json).  fp32, eval mode.  Tolerance: disease probabilities max-abs <= 1e-5;
the thresholded vector must agree wherever |p - 0.5| > 1e-4."""
import json
import os

import pytest
import torch
from PIL import Image

from oracle import ref_cpu as R
from parity_util import build_pair

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def test_inference_matches_oracle(dev):
    from mmdx.inference_pipeline import inference
    import mmdx
    ref, img, txt, fus = build_pair("resnet18", "embed-mean")
    ref.eval()
    pil = Image.open(os.path.join(GOLD, "e1.jpg")).convert("RGB")
    with open(os.path.join(GOLD, "patient_details.json")) as f:
        text = json.load(f)["e1.jpg"]
    bundle = {"fusion_model": fus, "image_encoder": img, "text_encoder": txt,
              "class_names": mmdx.DISEASES, "thresholds": [0.5] * 13, "version": 999,
              "t5_tok": None}
    out = inference(bundle, pil, text, device="cuda")
    assert set(out) >= {"report_text", "disease_probs", "disease_vector", "model_version"}
    assert out["model_version"] == 999 and out["report_text"] == ""
    x = R.reference_transform(pil).unsqueeze(0)
    tok = dict(mmdx.tokenize_patient_details([text], max_len=96))
    probs, vec = R.inference_probs(ref.image, ref.text, ref.fusion, x,
                                   {k: tok[k] for k in ("input_ids", "attention_mask")})
    mine = torch.tensor([out["disease_probs"][c] for c in mmdx.DISEASES])
    assert (mine - probs).abs().max().item() <= 1e-5
    for j in range(13):
        if abs(probs[j].item() - 0.5) > 1e-4:
            assert out["disease_vector"][j] == int(vec[j])
