"""GPU: the reference's daily training driver and its Django predict path, end to end on the
drop-in, checked against the CPU oracle.

1. `training_tests()` (TP:808-1127) runs every phase on a small local feature group (parquet
   + an S3 mirror of JPEGs): the shapes the reference prints (TP:823-824, 861-862, 898-899,
   921, 1006-1009, 1088-1090), finite losses, a fp16 fusion loop under mmdx.GradScaler, the
   registry entry and the local model_bundle.pt.
2. The Django loader's rebuild sequence (backend/api/views.py:188-258, replayed call for
   call on the mmdx classes: key validation, FusionTransformerModel(...,
   init_t5_from_config=True) + strict load_state_dict, ImageEncoderCNN() default,
   TextEncoderTransformer(cfg's model name)), then `inference()` with the reference's
   generate settings (IP:190: 4 beams, 150-180 new tokens, length_penalty 1.1) on the
   reference's own sample image:
   - disease probabilities vs the oracle (oracle/ref_cpu.py on the same state dicts):
     max-abs <= 1e-5, the thresholded vector equal wherever |p - 0.5| > 1e-4;
   - report token ids identical to transformers' T5ForConditionalGeneration.generate on the
     same weights and condition tokens, or of equal length-normalised score where duplicate
     beams tie to within an ulp (the T5 embedding scaled x4 in the bundle so next-token
     margins exceed fp32 reordering noise, as in test_t5_gpu.py).
3. `load_model_from_hopsworks_model_registry` (IP:53-139) on the registry entry + inference.
"""
import copy
import io
import json
import os

import numpy as np
import pytest
import torch
from PIL import Image

import mmdx
from oracle import ref_cpu as R

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
BUCKET = "medical-ml-proj-bucket"


@pytest.fixture(scope="module")
def feature_group(tmp_path_factory):
    import pandas as pd
    root = tmp_path_factory.mktemp("dropin")
    mirror = root / "s3"
    (mirror / BUCKET / "chest-x-ray-images").mkdir(parents=True)
    rng = np.random.default_rng(7)
    rows = []
    for i in range(12):
        key = f"chest-x-ray-images/img{i:02d}.jpg"
        if i == 0:
            data = open(os.path.join(GOLD, "e1.jpg"), "rb").read()
        else:
            h, w = int(rng.integers(240, 520)), int(rng.integers(240, 520))
            mode = "L" if i % 3 == 0 else "RGB"
            arr = rng.integers(0, 256, (h, w) if mode == "L" else (h, w, 3), dtype=np.uint8)
            buf = io.BytesIO()
            Image.fromarray(arr, mode).save(buf, format="JPEG", quality=90)
            data = buf.getvalue()
        (mirror / BUCKET / key).write_bytes(data)
        vec = (rng.random(13) < 0.2).astype(float).tolist()
        rows.append({"image_url": f"s3://{BUCKET}/{key}",
                     "patient_details": f"{40 + i} year old {'male' if i % 2 else 'female'} "
                                        f"PA view, cough, case {i}",
                     "disease_classification_vector": json.dumps(vec),
                     "report": f"Findings: case {i}. The lungs are clear. No effusion."})
    pq = root / "features.parquet"
    pd.DataFrame(rows).to_parquet(pq)
    return root, mirror, pq


@pytest.fixture(scope="module")
def trained(feature_group):
    root, mirror, pq = feature_group
    old = dict(os.environ)
    os.environ.update(MMDX_FEATURES_PARQUET=str(pq), MMDX_S3_MIRROR=str(mirror),
                      AWS_S3_BUCKET_NAME=BUCKET, MMDX_MODEL_REGISTRY=str(root / "registry"),
                      MMDX_MODEL_DIR=str(root / "model"))
    try:
        torch.manual_seed(0)
        out = mmdx.training_pipeline.training_tests(
            num_steps=4, b_fusion=4, batch_size=8, text_model="bert-base-uncased@2",
            gen_kwargs=dict(max_new_tokens=6, min_new_tokens=2, num_beams=2), verbose=False)
        torch.cuda.synchronize()
        yield root, out
    finally:
        os.environ.clear()
        os.environ.update(old)


def test_training_tests_phases(trained):
    _, out = trained
    assert out["transform_shape"] == (3, 224, 224)                    # TP:823
    assert out["image_shapes"] == ((8, 1024), (8, 13))                 # TP:861-862
    assert out["text_ids_shape"] == (2, 96)                            # TP:898
    assert out["text_z_shape"] == (2, 512)                             # TP:921
    assert out["z_shapes"] == ((4, 1024), (4, 512))                    # TP:1006-1009
    assert tuple(out["disease_vectors"].shape) == (4, 13)              # TP:1088-1090
    assert out["gen_ids"].shape[0] == 4 and out["gen_ids"].shape[1] <= 7
    assert len(out["image_loss"]) == 2 and len(out["text_loss"]) == 6
    assert all(np.isfinite(v) for v in out["image_loss"] + out["text_loss"])
    assert all(np.isfinite(v) for row in out["fusion_loss"] for v in row[1:])
    # GradScaler: at most a few overflow back-offs in 4 fp16 steps, no growth yet
    assert 2.0 ** 12 <= out["grad_scale"] <= 65536.0
    assert out["registry_version"] == 1


def _oracle_modules(blob):
    cfg = blob["cfg"]
    ref_img = R.RefImageEncoderCNN("resnet50", 1024, 13)
    ref_img.load_state_dict(blob["image_state"])
    ref_txt = R.RefTextEncoderTransformer("bert-base-uncased", bert_layers=2, dropout=0.0)
    ref_txt.load_state_dict(blob["text_state"])
    ref_fus = R.RefFusion(1024, cfg["fusion"]["d_txt"], 1024, 13, dropout=0.0)
    ref_fus.load_state_dict({k: v for k, v in blob["fusion_state"].items()
                             if not k.startswith("report_model.")})
    for m in (ref_img, ref_txt, ref_fus):
        m.eval()
    return ref_img, ref_txt, ref_fus


def _views_rebuild(blob):
    """VW:196-256 on the mmdx classes (tokenizer fetches by name are out of scope)."""
    from mmdx.inference_pipeline import (FusionTransformerModel, ImageEncoderCNN,
                                         TextEncoderTransformer)
    required = {"cfg", "fusion_state", "image_state", "text_state", "t5_tokenizer_name",
                "bert_tokenizer_name"}
    assert not required.difference(blob.keys())
    cfg = blob["cfg"]
    f = cfg.get("fusion") or {}
    fusion = FusionTransformerModel(
        d_img=f.get("d_img", 1024), d_txt=f.get("d_txt", 512), n_disease=f.get("n_disease", 13),
        d_fuse_hidden=f.get("d_fuse_hidden", 1024), n_cond_tokens=f.get("n_cond_tokens", 4),
        model_name=(cfg.get("report_head") or {}).get("hf_model_name", "t5-small"),
        init_t5_from_config=True)
    fusion.load_state_dict(blob["fusion_state"])
    fusion.eval()
    image_encoder = ImageEncoderCNN()
    if blob["image_state"]:
        image_encoder.load_state_dict(blob["image_state"])
    image_encoder.eval()
    text_encoder = TextEncoderTransformer(
        model_name=(cfg.get("text_encoder") or {}).get("hf_model_name", "bert-base-uncased"),
        d_txt=f.get("d_txt", 512), n_disease=f.get("n_disease", 13))
    if blob["text_state"]:
        text_encoder.load_state_dict(blob["text_state"])
    text_encoder.eval()
    arts = cfg.get("artifacts") or {}
    return {"cfg": cfg, "fusion_model": fusion, "image_encoder": image_encoder,
            "text_encoder": text_encoder, "t5_tok": None, "bert_tok": None,
            "class_names": arts.get("class_names", list(mmdx.DISEASES)),
            "thresholds": arts.get("thresholds", [0.5] * 13), "version": 999}


def _check_probs(out, blob, pil, text):
    ref_img, ref_txt, ref_fus = _oracle_modules(blob)
    x = R.reference_transform(pil).unsqueeze(0)
    tok = dict(mmdx.tokenize_patient_details([text], max_len=96))
    probs, vec = R.inference_probs(ref_img, ref_txt, ref_fus, x,
                                   {k: tok[k] for k in ("input_ids", "attention_mask")})
    mine = torch.tensor([out["disease_probs"][c] for c in mmdx.DISEASES])
    err = (mine - probs).abs().max().item()
    assert err <= 1e-5, err
    for j in range(13):
        if abs(probs[j].item() - 0.5) > 1e-4:
            assert out["disease_vector"][j] == int(vec[j])
    return ref_img, ref_txt, ref_fus, x, tok


def test_views_bundle_rebuild_and_inference(trained):
    import time
    from transformers.modeling_outputs import BaseModelOutput
    from mmdx.inference_pipeline import inference
    root, _ = trained
    blob = torch.load(root / "model" / "model_bundle.pt", map_location="cpu", weights_only=True)
    bundle = _views_rebuild(blob)
    pil = Image.open(os.path.join(GOLD, "e1.jpg")).convert("RGB")
    with open(os.path.join(GOLD, "patient_details.json")) as f:
        text = json.load(f)["e1.jpg"]
    inference(bundle, pil, text, gen_kwargs={"max_new_tokens": 4})   # warm-up
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    out = inference(bundle, pil, text)                                # IP:190 settings
    dt = time.perf_counter() - t0
    print(f"inference() with the T5 report head (4 beams, 150-180 tokens): {dt * 1e3:.1f} ms, "
          f"{len(out['report_ids']) - 1} tokens")
    assert out["model_version"] == 999 and out["report_generated"]
    ref_img, ref_txt, ref_fus, x, tok = _check_probs(out, blob, pil, text)
    # the report: transformers' T5 on the same weights and condition tokens.  The device
    # step is checked along the reference's own 150-180-token search (BeamStepCheck; the
    # reference step runs on transformers' GPU copy of the model, every prefix re-run), and
    # the pipeline's ids must equal transformers' generate() when that search had no
    # candidate within the tolerance of a neighbour.
    from transformers import T5Config, T5ForConditionalGeneration
    from mmdx.t5 import T5Head, _DecodeState
    from parity_util import BeamStepCheck, hf_beam_stepper
    cfg = bundle["fusion_model"].report_model.config.to_dict()
    t5 = T5ForConditionalGeneration(T5Config(**cfg))
    t5.load_state_dict({k[len("report_model."):]: v for k, v in blob["fusion_state"].items()
                        if k.startswith("report_model.")})
    t5.eval()
    kw = dict(max_new_tokens=180, min_new_tokens=150, num_beams=4, no_repeat_ngram_size=3,
              length_penalty=1.1, early_stopping=True, eos_token_id=1, pad_token_id=0)
    with torch.no_grad():
        z_img = ref_img(x)["embeddings"]
        z_txt = ref_txt(input_ids=tok["input_ids"],
                        attention_mask=tok["attention_mask"])["embeddings"]
        z_fuse = ref_fus(z_img, z_txt)["z_fuse"]
        cond = ref_fus.cond_proj(z_fuse).view(1, 4, 512)
        want = t5.generate(encoder_outputs=BaseModelOutput(last_hidden_state=cond), **kw)
    t5g = copy.deepcopy(t5).to("cuda")
    head = T5Head(bundle["fusion_model"].report_model)
    condd = cond.to("cuda")
    dec = _DecodeState(head, condd.repeat_interleave(4, dim=0), torch.float32, 181)
    chk = BeamStepCheck(hf_beam_stepper(t5g, cond, 4, 8), dec, 1, 4, 8, tol=2e-5)
    replay = head.generate(condd, _stepper=chk, **kw)
    print(f"steps {chk.steps}, max err {chk.max_err:.2e}, min gap {chk.min_gap:.2e}, "
          f"near-ties {chk.ambiguous}")
    assert chk.steps >= 150
    assert 151 <= len(out["report_ids"]) <= 181 and out["report_ids"][0] == 0
    if chk.ambiguous == 0:
        assert torch.equal(replay, want)
        assert out["report_ids"] == want[0].tolist()


def test_registry_load_and_inference(trained):
    from mmdx.inference_pipeline import inference, load_model_from_hopsworks_model_registry
    root, _ = trained
    os.environ["MMDX_MODEL_REGISTRY"] = str(root / "registry")
    try:
        bundle = load_model_from_hopsworks_model_registry("fusion_model_T5")
    finally:
        del os.environ["MMDX_MODEL_REGISTRY"]
    assert bundle["version"] == 1 and bundle["t5_tok"] is not None
    pil = Image.open(os.path.join(GOLD, "e1.jpg")).convert("RGB")
    text = "44 year old female PA view , hypertension , cough"
    out = inference(bundle, pil, text, gen_kwargs={"max_new_tokens": 5, "min_new_tokens": 2})
    blob = torch.load(root / "model" / "model_bundle.pt", map_location="cpu", weights_only=True)
    _check_probs(out, blob, pil, text)
    assert out["report_text"] != "" and out["report_ids"][0] == 0
