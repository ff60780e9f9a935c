"""`training_tests()` (TP:808-1127) and `save_model_to_hopsworks_model_registry` (TP:650-804)
on the mmdx kernels, fed from the local stand-ins of mmdx.registry instead of Hopsworks/S3.

`backend/api/management/commands/run_daily_training_pipeline.py:2` imports
`training_tests` from the training pipeline and calls it with no arguments; this one runs the
reference's phases in the reference's order on an MI355X:

1. feature-store read (TP:810) -> local parquet;
2. image transform check on one image (TP:820-824);
3. image tower phase 1 (frozen trunk, heads-only AdamW, ONE batch of 32, TP:846-863) and
   phase 2 (unfrozen, discriminative lrs, ONE batch, TP:866-880);
4. text tower phase 1 / phase 2 on the two hard-coded strings, 3 steps each (TP:885-939;
   TP:909's `model.train()` after freeze kept);
5. fusion (TP:943-1064): B_FUSION = 10 rows sampled with random_state=42, encoders in eval
   under no_grad, the fusion model WITH its T5 report head, AdamW over the four groups of
   TP:1018-1023, AMP on the GPU (TP:1025-1026: fp16 autocast + GradScaler; here the fusion
   model computes in fp16 and mmdx.GradScaler scales), clip 1.0 in the reference's place
   (TP:1058, before scaler.step), NUM_STEPS = 300;
6. generation demo (TP:1066-1099): beam search + disease predictions;
7. save (TP:1103-1127) into the local registry + local model_bundle.pt.

The arguments (all optional) only shrink the run for tests; the defaults are the reference's.
Report texts need a T5 tokenizer, which cannot be fetched offline: a deterministic
word-hash stand-in maps them to ids in the t5-small vocabulary (eos 1, pad 0) unless
MMDX_T5_SPM names a local sentencepiece model.
"""
from __future__ import annotations

import hashlib
import io
import os
import re
import shutil
import tempfile

import numpy as np
import torch

from . import registry as REG
from .amp import GradScaler
from .optim import AdamW, clip_grad_norm_


class _HashT5Tokenizer:
    """Offline stand-in for T5Tokenizer.from_pretrained("t5-small") (TP:967): words hashed
    into [3, 32100), then </s> = 1; pad 0.  NOT SentencePiece — ids differ from t5-small's."""

    eos_token_id = 1
    pad_token_id = 0
    V = 32100

    def __call__(self, texts, max_length=256, truncation=True, padding="max_length",
                 return_tensors="pt"):
        ids = torch.zeros((len(texts), max_length), dtype=torch.long)
        mask = torch.zeros_like(ids)
        for i, t in enumerate(texts):
            words = re.findall(r"\w+|[^\w\s]", t.lower())
            toks = [3 + int.from_bytes(hashlib.sha1(w.encode()).digest()[:4], "little")
                    % (self.V - 3) for w in words][: max_length - 1] + [self.eos_token_id]
            ids[i, : len(toks)] = torch.tensor(toks)
            mask[i, : len(toks)] = 1
        return {"input_ids": ids, "attention_mask": mask}

    def batch_decode(self, ids, skip_special_tokens=True):
        out = []
        for row in (ids.tolist() if torch.is_tensor(ids) else ids):
            toks = [t for t in row if not (skip_special_tokens and t in (0, 1))]
            out.append(" ".join(f"<{t}>" for t in toks))
        return out

    def save_pretrained(self, d):
        os.makedirs(d, exist_ok=True)
        with open(os.path.join(d, "MMDX_HASH_TOKENIZER"), "w") as f:
            f.write("word-hash stand-in for the t5-small tokenizer (offline)\n")


def t5_tokenizer():
    spm = os.environ.get("MMDX_T5_SPM")
    if spm:
        from transformers import T5Tokenizer
        return T5Tokenizer(vocab_file=spm)
    return _HashT5Tokenizer()


def _open_row_image(url):
    """An image_url of the feature group -> PIL RGB image: s3:// URLs through the S3 mirror
    (TP:957-960), other strings as local paths (relative to MMDX_IMAGE_ROOT)."""
    from PIL import Image
    from .data import open_image
    if url.startswith("s3://"):
        b, k = REG.parse_s3_url(url)
        return Image.open(io.BytesIO(REG.get_image_from_s3(b, k))).convert("RGB")
    return open_image(os.environ.get("MMDX_IMAGE_ROOT", ""), url).convert("RGB")


def _image_root_for(df):
    urls = df["image_url"].tolist()
    if urls and urls[0].startswith("s3://"):
        b, _ = REG.parse_s3_url(urls[0])
        return os.path.join(REG._env_path("MMDX_S3_MIRROR", "S3"),
                            os.environ.get("AWS_S3_BUCKET_NAME", b))
    return os.environ.get("MMDX_IMAGE_ROOT", "")


def save_model_to_hopsworks_model_registry(fusion_model, model_name="fusion_transformer",
                                           version=None, project_name=None,
                                           description="Fusion model with disease-head and T5 "
                                                       "report head",
                                           metrics=None, artifacts=None, image_encoder=None,
                                           text_encoder=None, t5_tokenizer=None,
                                           save_t5_weights=False, hf_model_name=None,
                                           model_dir=None):
    """TP:650-804 into the local registry: a staged folder with fusion_model.pt,
    image_encoder.pt, text_encoder.pt, config.json (TP:682-720 schema) and t5_assets/,
    saved as <registry>/<model_name>/<version>/ (version auto-increments), then the local
    model_bundle.pt (+ timestamped copy) written atomically (TP:773-796) into `model_dir`
    (env MMDX_MODEL_DIR, default <registry>/../model).  Returns the registry model."""
    from .inference_pipeline import bundle_config, save_model_bundle
    reg = REG.login(project_name).get_model_registry()
    temp_dir = tempfile.mkdtemp(prefix="fusion_reg_")
    try:
        def cpu_state(m):
            return {k: v.detach().cpu() for k, v in m.state_dict().items()}
        torch.save(cpu_state(fusion_model), os.path.join(temp_dir, "fusion_model.pt"))
        torch.save(cpu_state(image_encoder), os.path.join(temp_dir, "image_encoder.pt"))
        torch.save(cpu_state(text_encoder), os.path.join(temp_dir, "text_encoder.pt"))
        cfg = bundle_config(fusion_model, image_encoder, text_encoder, artifacts, hf_model_name)
        import json
        with open(os.path.join(temp_dir, "config.json"), "w") as f:
            json.dump(cfg, f, indent=2)
        t5_dir = os.path.join(temp_dir, "t5_assets")
        os.makedirs(t5_dir, exist_ok=True)
        if t5_tokenizer is not None and hasattr(t5_tokenizer, "save_pretrained"):
            t5_tokenizer.save_pretrained(t5_dir)
        if save_t5_weights and getattr(fusion_model, "report_model", None) is not None:
            fusion_model.report_model.save_pretrained(t5_dir)
        rm = reg.create_model(name=model_name, version=version, metrics=metrics or {},
                              description=description)
        rm.save(temp_dir)
        mdir = model_dir or os.environ.get("MMDX_MODEL_DIR") or str(
            REG.registry_root().parent / "model")
        save_model_bundle(fusion_model, image_encoder, text_encoder, mdir, version=rm.version,
                          artifacts=artifacts, hf_model_name=hf_model_name)
        return rm
    finally:
        shutil.rmtree(temp_dir, ignore_errors=True)


def training_tests(num_steps=300, b_fusion=10, batch_size=32, image_backbone="resnet50",
                   text_model="bert-base-uncased", gen_kwargs=None, save=True,
                   model_name="fusion_model_T5", device=None, verbose=True):
    """TP:808-1127 on mmdx (see the module docstring).  Returns a dict of what the reference
    prints: tensor shapes, per-step losses and the generated ids / disease vectors."""
    from PIL import Image
    from . import training_pipeline as TP
    from .data import LocalCXRBatches
    from .inference_pipeline import DISEASES

    log = print if verbose else (lambda *a, **k: None)
    dev = torch.device(device) if device is not None else torch.device("cuda")
    out = {}

    log("----------LOAD FEATURES/LABELS FROM FEATURE STORE (local parquet)---------")
    df = REG.load_features_labels_from_feature_store()
    out["n_rows"] = len(df)

    log("----------IMAGE ENCODER: IMAGE TRANSFORM TEST SINGLE IMAGE----------")
    pil = _open_row_image(df["image_url"].iloc[0])
    t = TP.image_transfom_into_tensor(pil)
    log(t.shape, t.dtype)
    out["transform_shape"] = tuple(t.shape)

    log("----------IMAGE ENCODER: DATASET / BATCHES----------")
    batches = LocalCXRBatches(df, _image_root_for(df), batch_size=batch_size, shuffle=True,
                              device=dev)
    imgs, _, y = next(iter(batches))
    log(f"batch img input shape: {tuple(imgs.shape)}, labels {tuple(y.shape)}")

    log("---------IMAGE ENCODER: CREATE IMAGE-ENCODER-CLASS----------")
    model = TP.ImageEncoderCNN(backbone_name=image_backbone, d_img=1024,
                               n_disease_classes=13).to(dev)
    criterion = TP.BCEWithLogitsLoss()
    out["image_loss"] = []
    for phase in (1, 2):
        if phase == 1:
            model.freeze_backbone()
            optim = model.build_optimizer(phase=1, lr_head=5e-4, weight_decay=1e-2)
        else:
            model.unfreeze_backbone()
            optim = model.build_optimizer(phase=2, lr_backbone=1e-4, lr_head=5e-4,
                                          weight_decay=1e-2)
        for imgs, _, y in batches:  # ONE batch per phase (break at TP:863 / TP:880)
            optim.zero_grad()
            o = model(imgs)
            loss = criterion(o["logits"], y)
            loss.backward()
            optim.step()
            log(f"phase {phase}: embeddings {tuple(o['embeddings'].shape)}, logits "
                f"{tuple(o['logits'].shape)}, loss {loss.item():.4f}")
            out["image_loss"].append(loss.item())
            out["image_shapes"] = (tuple(o["embeddings"].shape), tuple(o["logits"].shape))
            break

    log("----------TEXT ENCODER: TOKENIZE PATIENT DETAILS TEXT----------")
    texts = ["67M, smoker; dyspnea; CHF history.", "54F, no smoking; cough; asthma."]
    y_txt = torch.tensor([[0, 1, 0, 1, 0, 0, 0, 0, 1, 0, 1, 0, 0],
                          [1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 0, 0, 1]], dtype=torch.float32,
                         device=dev)
    tok = TP.tokenize_patient_details(texts, max_len=96)
    tok = {k: v.to(dev) for k, v in tok.items()}
    out["text_ids_shape"] = tuple(tok["input_ids"].shape)
    text_encoder_model = TP.TextEncoderTransformer(model_name=text_model, d_txt=512,
                                                   n_disease=13).to(dev)
    out["text_loss"] = []
    for phase in (1, 2):
        if phase == 1:
            text_encoder_model.freeze_encoder()
            optim = text_encoder_model.build_optimizer(phase=1, lr_head=5e-4)
            text_encoder_model.train()  # TP:909
        else:
            text_encoder_model.unfreeze_encoder()
            optim = text_encoder_model.build_optimizer(phase=2, lr_enc=2e-5, lr_head=5e-4,
                                                       weight_decay=1e-2)
        for step in range(3):
            optim.zero_grad()
            o = text_encoder_model(**tok)
            loss = criterion(o["logits"], y_txt)
            loss.backward()
            optim.step()
            log(f"text phase {phase} step {step}: z {tuple(o['embeddings'].shape)}, "
                f"loss {loss.item():.4f}")
            out["text_loss"].append(loss.item())
            out["text_z_shape"] = tuple(o["embeddings"].shape)

    log("----------FUSION MODEL----------")
    rows = df.sample(n=min(b_fusion, len(df)), random_state=42).reset_index(drop=True)
    from .preprocess import preprocess_batch
    imgs = preprocess_batch([_open_row_image(u) for u in rows["image_url"]], dev)
    y_multi = torch.tensor(np.stack([np.asarray(v, dtype=np.float32)
                                     for v in rows["disease_classification_vector"]]),
                           dtype=torch.float32, device=dev)
    tok_aligned = TP.tokenize_patient_details(rows["patient_details"].astype(str).tolist(),
                                              max_len=96)
    tok_aligned = {k: v.to(dev) for k, v in tok_aligned.items()}
    t5_tok = t5_tokenizer()
    rep = t5_tok(rows["report"].astype(str).tolist(), max_length=256, truncation=True,
                 padding="max_length", return_tensors="pt")
    report_labels = rep["input_ids"].clone()
    report_labels[rep["attention_mask"] == 0] = -100
    report_labels = report_labels.to(dev)

    image_encoder, text_encoder = model, text_encoder_model
    image_encoder.eval()
    text_encoder.eval()
    with torch.no_grad():
        z_img = image_encoder(imgs)["embeddings"]
        z_txt = text_encoder(**tok_aligned)["embeddings"]
    out["z_shapes"] = (tuple(z_img.shape), tuple(z_txt.shape))

    fusion_model = TP.FusionTransformerModel(d_img=1024, d_txt=512, n_disease=13,
                                             with_report_head=True).to(dev)
    optim_fuse = AdamW([
        {"params": fusion_model.fusion_mlp.parameters(), "lr": 5e-4},
        {"params": fusion_model.disease_head.parameters(), "lr": 5e-4},
        {"params": fusion_model.cond_proj.parameters(), "lr": 5e-4},
        {"params": fusion_model.report_model.parameters(), "lr": 2e-5},
    ], weight_decay=1e-2)
    use_amp = dev.type == "cuda"                           # TP:1025
    scaler = GradScaler(enabled=use_amp)                   # TP:1026
    amp_dtype = torch.float16 if use_amp else torch.float32  # autocast(fp16) on the GPU
    fusion_model.train()
    out["fusion_loss"] = []
    for step in range(1, num_steps + 1):
        optim_fuse.zero_grad(set_to_none=True)
        o = fusion_model(z_img=z_img.to(amp_dtype), z_txt=z_txt.to(amp_dtype),
                         report_input_ids=None, report_attention_mask=None,
                         report_labels=report_labels)
        loss_cls = criterion(o["disease_logits"].float(), y_multi)
        loss_gen = o["gen"].loss if o["gen"] is not None else 0.0
        loss = loss_cls + 1.0 * loss_gen
        scaler.scale(loss).backward()                                     # TP:1056
        clip_grad_norm_(fusion_model.parameters(), 1.0)                   # TP:1058
        scaler.step(optim_fuse)                                           # TP:1060
        scaler.update()                                                   # TP:1061
        if step % 25 == 0 or step == 1 or step == num_steps:
            out["fusion_loss"].append((step, loss_cls.item(), float(loss_gen), loss.item()))
            log(f"[FUSION][train] step {step:04d} | cls={loss_cls.item():.4f}  "
                f"gen={float(loss_gen):.4f}  total={loss.item():.4f}")
    out["grad_scale"] = scaler.get_scale()

    fusion_model.eval()
    gen = dict(max_new_tokens=180, min_new_tokens=150, num_beams=4, no_repeat_ngram_size=3,
               length_penalty=1.0, early_stopping=True, eos_token_id=t5_tok.eos_token_id,
               pad_token_id=t5_tok.pad_token_id)  # TP:1076-1083
    if gen_kwargs:
        gen.update(gen_kwargs)
    with torch.no_grad():
        gen_ids = fusion_model.generate(z_img, z_txt, **gen)
        d_logits = fusion_model(z_img=z_img, z_txt=z_txt, report_labels=None)["disease_logits"]
        d_probs = torch.sigmoid(d_logits.float())
        d_preds = (d_probs >= 0.5).int()
    out["gen_ids"] = gen_ids
    out["disease_vectors"] = d_preds.cpu()
    for i, s in enumerate(t5_tok.batch_decode(gen_ids, skip_special_tokens=True)):
        log(f"Example report #{i}: {s[:120]}")
        log("Disease vector:", d_preds[i].tolist())

    if save:
        rm = save_model_to_hopsworks_model_registry(
            fusion_model=fusion_model, text_encoder=text_encoder, image_encoder=image_encoder,
            model_name=model_name, description="CXR fusion: CNN+Text -> MLP; multi-label "
                                               "disease head; T5 report head.",
            metrics={"val_auroc_micro": 0.874, "val_rougeL": 0.214},  # TP:1112 placeholders
            artifacts={"class_names": list(DISEASES), "thresholds": [0.5] * 13},
            t5_tokenizer=t5_tok, save_t5_weights=False, hf_model_name="t5-small")
        log("model version in registry:", rm.version)
        out["registry_version"] = rm.version
    out["models"] = (image_encoder, text_encoder, fusion_model)
    return out
