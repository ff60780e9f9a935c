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


def test_inference_with_t5_report_head(dev):
    """IP:190-196 on the mmdx T5 decoder: a bundle whose fusion model carries the report head
    beam-generates report token ids (no T5 tokenizer ships offline, so report_text stays ""
    and the ids come back as report_ids); the disease branch is unchanged by the head."""
    from mmdx.inference_pipeline import inference
    import mmdx
    _, img, txt, fus0 = build_pair("resnet18", "embed-mean")
    torch.manual_seed(3)
    fus = mmdx.FusionTransformerModel(1024, 512, 1024, 13, dropout=0.0, init_t5_from_config=True)
    sd = {k: v for k, v in fus0.state_dict().items()}
    fus.load_state_dict(sd, strict=False)
    pil = Image.open(os.path.join(GOLD, "e1.jpg")).convert("RGB")
    with open(os.path.join(GOLD, "patient_details.json")) as f:
        text = json.load(f)["e1.jpg"]
    base = {"image_encoder": img, "text_encoder": txt, "class_names": mmdx.DISEASES,
            "thresholds": [0.5] * 13, "version": 1, "t5_tok": None}
    out0 = inference(dict(base, fusion_model=fus0), pil, text, device="cuda")
    out = inference(dict(base, fusion_model=fus), pil, text, device="cuda",
                    gen_kwargs={"max_new_tokens": 10, "min_new_tokens": 4})
    assert out["report_generated"] and out["report_text"] == ""
    ids = out["report_ids"]
    assert ids[0] == 0 and 5 <= len(ids) <= 11
    assert 1 not in ids[1:5]            # min_new_tokens: no EOS among the first 4 new tokens
    for c in mmdx.DISEASES:
        assert abs(out["disease_probs"][c] - out0["disease_probs"][c]) <= 1e-6
