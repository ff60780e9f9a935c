"""Drop-in for the hot-path part of backend/ml/pipelines/inference_pipeline.py ("IP").

`inference(model_bundle, image_pil, patient_details, device=None, gen_kwargs=None)` keeps
IP:151's signature, argument checks and return dict; the two towers and the disease head
run on the mmdx kernels.  The report text needs the T5 head (outside the hot path,
SURVEY §8(f)): it is generated only when the bundle's fusion model carries one, otherwise
`report_text` is "" and `report_generated` is False.

`load_model_bundle(path)` rebuilds the bundle from a local `model_bundle.pt` written by the
reference's save path (TP:773-796: keys cfg, fusion_state, image_state, text_state,
t5_tokenizer_name, bert_tokenizer_name, version), with the same key validation and errors
as the Django loader (VW:196-204).  Loading uses weights_only=True.  `save_model_bundle`
writes the same dict (atomically, TP:792-794), so bundles move both ways.
"""
from __future__ import annotations

import os

import torch

from .preprocess import preprocess_batch
from .training_pipeline import (DISEASES, FusionTransformerModel, ImageEncoderCNN,
                                TextEncoderTransformer, image_transfom_into_tensor,
                                tokenize_patient_details)

BUNDLE_KEYS = ("cfg", "fusion_state", "image_state", "text_state", "t5_tokenizer_name",
               "bert_tokenizer_name", "version")


def _text_model_name(raw):
    """The text architecture comes from cfg["text_encoder"]["hf_model_name"] (TP:701, the
    text encoder's model_name); the tokenizer name is only the fallback (same value in the
    reference's writer, TP:788)."""
    tc = (raw["cfg"] or {}).get("text_encoder", {}) or {}
    return tc.get("hf_model_name") or raw.get("bert_tokenizer_name") or "bert-base-uncased"


def _load_fusion_state(fusion, state):
    """Strict on every disease-branch key (fusion_mlp, disease_head, cond_proj): a mismatch
    raises instead of leaving randomly initialised heads (VW:221 loads strictly).  The T5
    `report_model.*` keys are loaded when the model carries a report head, else set aside."""
    has_t5 = getattr(fusion, "report_model", None) is not None
    fs = {k: v for k, v in state.items() if has_t5 or not k.startswith("report_model.")}
    res = fusion.load_state_dict(fs, strict=False)
    bad = [k for k in list(res.missing_keys) + list(res.unexpected_keys)
           if not k.startswith("report_model.")]
    if bad or (has_t5 and res.missing_keys):
        raise RuntimeError(f"fusion_state does not match the fusion model: "
                           f"missing {list(res.missing_keys)}, unexpected "
                           f"{list(res.unexpected_keys)}")


def load_model_bundle(path: str, device="cuda", compute_dtype=torch.float32):
    if not os.path.exists(path):
        raise FileNotFoundError(f"Model bundle not found at {path}")  # VW:178
    raw = torch.load(path, map_location="cpu", weights_only=True)
    missing = [k for k in BUNDLE_KEYS if k not in raw]
    if missing:
        raise ValueError(f"Bundle missing keys: {missing}")  # VW:204
    cfg = raw["cfg"] or {}
    fc = cfg.get("fusion", {}) or {}
    d_img = fc.get("d_img") or 1024
    d_txt = fc.get("d_txt") or 512  # VW:209 fallback (IP:74 uses 1024)
    fusion = FusionTransformerModel(d_img=d_img, d_txt=d_txt,
                                    d_fuse_hidden=fc.get("d_fuse_hidden") or 1024,
                                    n_disease=fc.get("n_disease") or 13,
                                    n_cond_tokens=fc.get("n_cond_tokens") or 4)
    _load_fusion_state(fusion, raw["fusion_state"])
    backbone = ((cfg.get("image_encoder", {}) or {}).get("backbone")) or "resnet50"
    image = ImageEncoderCNN(backbone, d_img, compute_dtype=compute_dtype)
    image.load_state_dict(raw["image_state"])
    text = TextEncoderTransformer(_text_model_name(raw), d_txt, compute_dtype=compute_dtype)
    text.load_state_dict(raw["text_state"])
    arts = cfg.get("artifacts", {}) or {}
    return {
        "cfg": cfg,
        "version": raw["version"],
        "fusion_model": fusion.to(device).eval(),
        "image_encoder": image.to(device).eval(),
        "text_encoder": text.to(device).eval(),
        "t5_tok": None,
        "bert_tok": None,
        "class_names": arts.get("class_names", DISEASES),
        "thresholds": arts.get("thresholds", [0.5] * len(DISEASES)),
    }


def bundle_config(fusion_model, image_encoder, text_encoder, artifacts=None,
                  hf_model_name=None):
    """The `configuration` dict of TP:682-720 (JSON-safe), built from the live modules."""
    from datetime import datetime, timezone
    rm = getattr(fusion_model, "report_model", None)
    bert_name = getattr(text_encoder, "model_name", None) or "bert-base-uncased"
    cfg = {
        "saved_at": datetime.now(timezone.utc).replace(tzinfo=None).isoformat() + "Z",
        "fusion": {
            "d_img": getattr(fusion_model, "d_img", None),
            "d_txt": getattr(fusion_model, "d_txt", None),
            "d_fuse_hidden": getattr(fusion_model, "d_fuse_hidden", None),
            "n_disease": getattr(fusion_model, "n_disease", None),
            "n_cond_tokens": getattr(fusion_model, "n_cond", None),
            "decoder_hidden": rm.config.d_model if rm is not None else None,
        },
        "report_head": {"hf_model_name": hf_model_name or (
            getattr(rm.config, "_name_or_path", None) if rm is not None else None)},
        "text_encoder": {"hf_model_name": bert_name,
                         "d_txt": getattr(fusion_model, "d_txt", None),
                         "pooling": getattr(text_encoder, "pooling", "masked_mean"),
                         "max_len": 96},
        "image_encoder": {"backbone": getattr(image_encoder, "backbone_name", None),
                          "d_img": getattr(fusion_model, "d_img", None),
                          "img_size": 224,
                          "normalize": {"mean": [0.485, 0.456, 0.406],
                                        "std": [0.229, 0.224, 0.225]}},
        "notes": "Fusion MLP + disease head (BCEWithLogits) + T5 report head (CE).",
    }
    if artifacts:
        cfg["artifacts"] = artifacts
    return cfg


def save_model_bundle(fusion_model, image_encoder, text_encoder, model_dir, version=1,
                      artifacts=None, hf_model_name=None, timestamped_copy=True):
    """Write `model_bundle.pt` exactly as the reference's local save does (TP:773-796):
    keys cfg, fusion_state, image_state, text_state, t5_tokenizer_name,
    bert_tokenizer_name, version; written to a .tmp file and moved into place with
    os.replace (atomic, TP:792-794), plus a timestamped copy (TP:779-780, TP:795).  The
    registry upload around it (TP:650-771) is out of scope.  State dicts are saved from
    CPU copies in the reference's layout (NCHW fp32 — the modules store it that way).
    Returns the path of the latest bundle."""
    import shutil
    from datetime import datetime, timezone
    from pathlib import Path
    d = Path(model_dir)
    d.mkdir(parents=True, exist_ok=True)
    cfg = bundle_config(fusion_model, image_encoder, text_encoder, artifacts, hf_model_name)

    def cpu_state(m):
        return {k: v.detach().cpu() for k, v in m.state_dict().items()}

    bundle = {
        "cfg": cfg,
        "fusion_state": cpu_state(fusion_model),
        "image_state": cpu_state(image_encoder),
        "text_state": cpu_state(text_encoder),
        "t5_tokenizer_name": cfg["report_head"]["hf_model_name"],
        "bert_tokenizer_name": cfg["text_encoder"]["hf_model_name"],
        "version": version,
    }
    latest = d / "model_bundle.pt"
    tmp = latest.with_suffix(".pt.tmp")
    torch.save(bundle, tmp)
    os.replace(tmp, latest)
    if timestamped_copy:
        stamp = datetime.now(timezone.utc).strftime("%Y%m%dT%H%M%SZ")
        shutil.copyfile(latest, d / f"model_bundle_{stamp}.pt")
    return str(latest)


@torch.no_grad()
def inference(model_bundle, image_pil, patient_details, device=None, gen_kwargs=None):
    if isinstance(device, torch.device):  # IP:152-159
        dev = device
    elif isinstance(device, str):
        dev = torch.device(device)
    elif device is None:
        dev = torch.device("cuda")
    else:
        raise TypeError(f"'device' must be str|torch.device|None, got {type(device)}")
    fusion = model_bundle["fusion_model"].to(dev)
    class_names = model_bundle["class_names"]
    thresholds = torch.tensor(model_bundle["thresholds"], device=dev)
    image_encoder = model_bundle["image_encoder"].to(dev).eval()
    text_encoder = model_bundle["text_encoder"].to(dev).eval()

    if dev.type == "cuda":  # IP:174 on the GPU (bit-exact with image_transfom_into_tensor)
        x_img = preprocess_batch([image_pil], dev)
    else:
        x_img = image_transfom_into_tensor(image_pil).unsqueeze(0).to(dev)
    tok = tokenize_patient_details([patient_details], max_len=96)       # IP:175
    tok = {k: v.to(dev) for k, v in tok.items()}
    z_img = image_encoder(x_img)["embeddings"]                          # IP:179
    z_txt = text_encoder(**tok)["embeddings"]                           # IP:180
    out = fusion(z_img=z_img, z_txt=z_txt, report_labels=None)          # IP:183
    logits = out["disease_logits"]
    probs = torch.sigmoid(logits.float())[0]                            # IP:185
    vector = (probs >= thresholds).int().tolist()                       # IP:186

    report = ""
    generated = False
    if getattr(fusion, "report_model", None) is not None and model_bundle.get("t5_tok"):
        t5_tok = model_bundle["t5_tok"]
        gen = dict(max_new_tokens=180, min_new_tokens=150, num_beams=4, no_repeat_ngram_size=3,
                   length_penalty=1.1, early_stopping=True, eos_token_id=t5_tok.eos_token_id,
                   pad_token_id=t5_tok.pad_token_id)  # IP:190
        if gen_kwargs:
            gen.update(gen_kwargs)
        fusion.report_model.to(dev)
        ids = fusion.generate(z_img, z_txt, **gen)
        report = t5_tok.batch_decode(ids, skip_special_tokens=True)[0]
        generated = True
    return {
        "report_text": report,
        "disease_probs": {class_names[j]: float(probs[j]) for j in range(len(class_names))},
        "disease_vector": vector,
        "model_version": model_bundle["version"],
        "report_generated": generated,
    }
