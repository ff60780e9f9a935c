"""Drop-in replacement for the hot-path surface of backend/ml/pipelines/training_pipeline.py.

Same public names, constructor arguments, methods, return dicts and state_dict keys as the
reference (file:line citations below, "TP" = training_pipeline.py); the arithmetic runs on
the mmdx HIP kernels on an MI355X.  Out of scope: Hopsworks/S3 plumbing,
the T5 report generator (kept as an optional CPU-side submodule for state_dict/bundle
compatibility), the model registry.
"""
from __future__ import annotations

import hashlib
import os
import re
from types import SimpleNamespace

import numpy as np
import torch
import torch.nn as nn

from . import _lib as L
from . import functional as F
from . import text_encoders as TE
from .layers import Dropout, GELU, LayerNorm, Linear
from .optim import AdamW
from .resnet import ResNetTrunk
from .vit import VitTrunk

HOPS_PROJECT_NAME = "medical_ml_project"   # TP:60-62 (names kept; the services are local)
HOPS_FEATURE_GROUP_NAME = "cxr_features"
VERSION = 1
IMG_SIZE = 224  # TP:65
TEXT_ENCODER_MODEl_NAME = "bert-base-uncased"  # TP:66 (name kept verbatim)
IMAGENET_MEAN = (0.485, 0.456, 0.406)
IMAGENET_STD = (0.229, 0.224, 0.225)
DISEASES = [
    "No Finding", "Enlarged Cardiomediastinum", "Cardiomegaly", "Lung Opacity", "Lung Lesion",
    "Edema", "Consolidation", "Pneumonia", "Atelectasis", "Pneumothorax", "Pleural Effusion",
    "Pleural Other", "Fracture",
]  # TP:1115-1119

_DEFAULT_DTYPE = [torch.float32]


def set_compute_dtype(dtype: torch.dtype):
    """Process-wide default compute dtype for newly built towers (fp32 parity / bf16 speed)."""
    if dtype not in (torch.float32, torch.bfloat16, torch.float16):
        raise TypeError("compute dtype must be torch.float32, torch.bfloat16 or torch.float16 "
                        "(float16: the ViT / BERT towers, C5)")
    _DEFAULT_DTYPE[0] = dtype


def get_compute_dtype() -> torch.dtype:
    return _DEFAULT_DTYPE[0]


def BCEWithLogitsLoss():
    """`torch.nn.BCEWithLogitsLoss()` (mean reduction) on the mmdx kernel (TP:843, 1015)."""
    return F.bce_with_logits


# =====================================================================================
# Feature store / S3 / registry surface (TP:72-103, 122-152, 650-804, 808-1127): the same
# names over the local stand-ins of mmdx.registry (the cloud services are out of scope).
# =====================================================================================
from .registry import (get_image_from_s3, load_features_labels_from_feature_store,  # noqa: E402,F401
                       parse_s3_url)


def construct_input_label_pairs_for_image_encoder_dataset(df):  # TP:122-127
    from .data import construct_input_label_pairs_for_image_encoder_dataset as f
    return f(df)


class CXR_ImageDataset(torch.utils.data.Dataset):
    """TP:131-152: (image tensor, float32 label vector) pairs; image bytes via
    get_image_from_s3(bucket, key) — the local S3 mirror."""

    def __init__(self, img_s3_keys_input, bucket, labels=None, image_transform=None):
        self.img_s3_keys_input = img_s3_keys_input
        self.bucket = bucket
        self.labels = labels
        self.image_transform = image_transform

    def __len__(self):
        assert len(self.img_s3_keys_input) == len(self.labels)
        return len(self.img_s3_keys_input)

    def __getitem__(self, i):
        import io
        from PIL import Image
        img = Image.open(io.BytesIO(get_image_from_s3(self.bucket, self.img_s3_keys_input[i])))
        x = self.image_transform(img)
        y = torch.tensor(self.labels[i], dtype=torch.float32)
        return x, y


def save_model_to_hopsworks_model_registry(*args, **kwargs):  # TP:650-804
    from .training_driver import save_model_to_hopsworks_model_registry as f
    return f(*args, **kwargs)


def training_tests(*args, **kwargs):  # TP:808-1127
    from .training_driver import training_tests as f
    return f(*args, **kwargs)


# =====================================================================================
# Image preprocessing (TP:112-119): torchvision Resize(256, antialias) -> CenterCrop(224)
# -> ToTensor -> gray->RGB -> Normalize, restated on PIL (torchvision is not a dependency).
# =====================================================================================
def _resize_shorter(img, size):
    from PIL import Image
    w, h = img.size
    short, long = (w, h) if w <= h else (h, w)
    if short == size:
        return img
    new_short, new_long = size, int(size * long / short)
    nw, nh = (new_short, new_long) if w <= h else (new_long, new_short)
    return img.resize((nw, nh), Image.BILINEAR)


def _center_crop(img, size):
    w, h = img.size
    top = int(round((h - size) / 2.0))
    left = int(round((w - size) / 2.0))
    return img.crop((left, top, left + size, top + size))


def image_transfom_into_tensor(img) -> torch.Tensor:
    """PIL image -> float32 [3, 224, 224] normalised tensor (name misspelt as in TP:112)."""
    img = _center_crop(_resize_shorter(img, 256), IMG_SIZE)
    arr = np.asarray(img)
    if arr.ndim == 2:
        arr = arr[:, :, None]
    x = torch.from_numpy(np.array(arr, copy=True)).permute(2, 0, 1).float().div(255.0)
    if x.shape[0] == 1:
        x = x.repeat(3, 1, 1)
    mean = torch.tensor(IMAGENET_MEAN).view(3, 1, 1)
    std = torch.tensor(IMAGENET_STD).view(3, 1, 1)
    return ((x - mean) / std).contiguous()


# =====================================================================================
# Image encoder (TP:157-311)
# =====================================================================================
class ImageEncoderCNN(nn.Module):
    SUPPORTED = ("resnet50", "resnet18", "resnet34", "resnet101", "vit_b_16")

    def __init__(self, backbone_name="resnet50", d_img=1024, n_disease_classes=13,
                 use_warmup_classifier=True, pretrained_weights=None, compute_dtype=None):
        super().__init__()
        self.backbone_name = backbone_name
        self.d_img = d_img
        self.n_disease_classes = n_disease_classes
        self.use_warmup_classifier = use_warmup_classifier
        # The reference ignores this argument and always asks torchvision for
        # IMAGENET1K_V2 (TP:169); offline, a local state_dict path may be given instead.
        self.pretrained_weights = pretrained_weights
        self.compute_dtype = compute_dtype or get_compute_dtype()
        self.backbone = None
        self.proj = None
        self.classifier = None
        self.is_backbone_frozen = False
        self.load_pretrained_backbone()

    def load_pretrained_backbone(self):  # TP:176-197
        if self.backbone_name.lower() == "vit_b_16":  # build-defined
            self.backbone = VitTrunk()
            self.backbone.compute_dtype = self.compute_dtype
            feat_dim = self.backbone.feat_dim
        elif self.backbone_name.lower() in self.SUPPORTED:
            self.backbone = ResNetTrunk(self.backbone_name.lower())
            self.backbone.compute_dtype = self.compute_dtype
            feat_dim = self.backbone.feat_dim
        else:
            raise ValueError(f"Unsupported backbone model: {self.backbone}")
        if isinstance(self.pretrained_weights, str) and os.path.exists(self.pretrained_weights):
            sd = torch.load(self.pretrained_weights, map_location="cpu", weights_only=True)
            sd = {k: v for k, v in sd.items() if not k.startswith(("fc.", "heads."))}
            self.backbone.load_state_dict(sd if self.backbone_name.lower() == "vit_b_16"
                                          else _tv_to_seq(sd))
        self.proj = Linear(feat_dim, self.d_img)
        if self.use_warmup_classifier:
            self.classifier = Linear(self.d_img, self.n_disease_classes)
        self.is_backbone_frozen = False

    def set_compute_dtype(self, dtype):
        self.compute_dtype = dtype
        self.backbone.compute_dtype = dtype
        return self

    def freeze_backbone(self):  # TP:200-215
        for p in self.backbone.parameters():
            p.requires_grad = False
        self.is_backbone_frozen = True
        self.backbone.eval()
        self.proj.train()
        if self.classifier is not None:
            self.classifier.train()

    def unfreeze_backbone(self):  # TP:218-230
        for p in self.backbone.parameters():
            p.requires_grad = True
        self.is_backbone_frozen = False
        self.backbone.train()
        self.proj.train()
        if self.classifier is not None:
            self.classifier.train()

    def build_optimizer(self, phase, lr_backbone=1e-4, lr_head=5e-4, weight_decay=1e-2,
                        optimizer_cls=AdamW):  # TP:238-269
        if phase == 1:
            params = [{"params": self.proj.parameters(), "lr": lr_head}]
            if self.classifier is not None:
                params.append({"params": self.classifier.parameters(), "lr": lr_head})
            return optimizer_cls(params, weight_decay=weight_decay)
        elif phase == 2:
            params = []
            bb_params = [p for p in self.backbone.parameters() if p.requires_grad]
            if bb_params:
                params.append({"params": bb_params, "lr": lr_backbone})
            params.append({"params": self.proj.parameters(), "lr": lr_head})
            if self.classifier is not None:
                params.append({"params": self.classifier.parameters(), "lr": lr_head})
            return optimizer_cls(params, weight_decay=weight_decay)

    @torch.no_grad()
    def _backbone_forward_nograd(self, x):  # TP:277-281
        return self.backbone(x).flatten(1)

    def _backbone_forward_grad(self, x):  # TP:285-288
        return self.backbone(x).flatten(1)

    def encode(self, images):  # TP:291-302
        if self.is_backbone_frozen:
            feats = self._backbone_forward_nograd(images)
        else:
            feats = self._backbone_forward_grad(images)
        return self.proj(feats)

    def forward(self, images):  # TP:306-311
        z = self.encode(images)
        out = {"embeddings": z}
        if self.classifier is not None:
            out["logits"] = self.classifier(z, out_dtype=torch.float32)
        return out


def _tv_to_seq(sd):
    """torchvision resnet keys (conv1/bn1/layerN) -> Sequential indices (0/1/4..7)."""
    m = {"conv1.": "0.", "bn1.": "1.", "layer1.": "4.", "layer2.": "5.", "layer3.": "6.",
         "layer4.": "7."}
    out = {}
    for k, v in sd.items():
        for a, b in m.items():
            if k.startswith(a):
                k = b + k[len(a):]
                break
        out[k] = v
    return out


# =====================================================================================
# Text encoder (TP:316-508)
# =====================================================================================
_TOKENIZER = [None]


class _HashWordTokenizer:
    """Offline stand-in used ONLY when no BERT vocab is available locally: BERT-style
    basic tokenisation (lower-case, split on whitespace/punctuation), ids from a stable
    hash into [1000, 30522), [CLS]=101 ... [SEP]=102, [PAD]=0.  NOT WordPiece: ids differ
    from bert-base-uncased's; set MMDX_BERT_VOCAB to a vocab.txt for the real tokenizer."""

    def __call__(self, text_list, padding="max_length", truncation=True, return_tensors="pt",
                 max_length=96):
        ids = torch.zeros((len(text_list), max_length), dtype=torch.long)
        mask = torch.zeros_like(ids)
        for i, t in enumerate(text_list):
            words = re.findall(r"\w+|[^\w\s]", t.lower())
            toks = [101] + [1000 + int.from_bytes(hashlib.sha1(w.encode()).digest()[:4],
                                                  "little") % (30522 - 1000)
                            for w in words][: max_length - 2] + [102]
            ids[i, : len(toks)] = torch.tensor(toks)
            mask[i, : len(toks)] = 1
        return {"input_ids": ids, "token_type_ids": torch.zeros_like(ids),
                "attention_mask": mask}


class _WordPieceTokenizer:
    """bert-base-uncased's tokenizer (what AutoTokenizer builds at TP:323: BertTokenizerFast,
    lower-casing, BERT basic tokenisation, greedy longest-match WordPiece, [CLS] ... [SEP],
    truncation, [PAD] padding) from a local vocab.txt, on the `tokenizers` library that
    BertTokenizerFast wraps.  (transformers 5.x's BertTokenizerFast(vocab_file=...) no longer
    reads the file: it returned [UNK] for every word.)"""

    def __init__(self, vocab):
        from tokenizers import BertWordPieceTokenizer
        self.tok = BertWordPieceTokenizer(vocab, lowercase=True)
        self.pad_id = self.tok.token_to_id("[PAD]")

    def __call__(self, text_list, padding="max_length", truncation=True, return_tensors="pt",
                 max_length=96):
        if truncation:
            self.tok.enable_truncation(max_length)
        else:
            self.tok.no_truncation()
        if padding == "max_length":
            self.tok.enable_padding(length=max_length, pad_id=self.pad_id, pad_token="[PAD]")
        else:
            self.tok.enable_padding(pad_id=self.pad_id, pad_token="[PAD]")
        enc = self.tok.encode_batch(list(text_list))
        return {"input_ids": torch.tensor([e.ids for e in enc], dtype=torch.long),
                "token_type_ids": torch.tensor([e.type_ids for e in enc], dtype=torch.long),
                "attention_mask": torch.tensor([e.attention_mask for e in enc],
                                               dtype=torch.long)}


def _tokenizer():
    if _TOKENIZER[0] is None:
        vocab = os.environ.get("MMDX_BERT_VOCAB")
        if vocab:
            _TOKENIZER[0] = _WordPieceTokenizer(vocab)
        else:
            _TOKENIZER[0] = _HashWordTokenizer()
    return _TOKENIZER[0]


def tokenize_patient_details(text_list, max_len=96):  # TP:335-342
    return _tokenizer()(text_list, padding="max_length", truncation=True, return_tensors="pt",
                        max_length=max_len)


def _build_text_backbone(model_name):
    name = model_name.lower()
    if name.startswith("bert"):
        return TE.BertModel.from_name(model_name)
    if name in ("embed-mean", "embedding-mean", "embed_mean"):
        return TE.EmbedMeanEncoder()
    if name in ("bilstm", "bi-lstm", "lstm"):
        return TE.BiLSTMEncoder()
    raise ValueError(f"Unsupported text encoder: {model_name}")


class TextEncoderTransformer(nn.Module):
    def __init__(self, model_name="bert-base-uncased", d_txt=512, n_disease=13,
                 use_warmup_classifier=True, compute_dtype=None):  # TP:350-369
        super().__init__()
        self.model_name = model_name
        self.d_txt = d_txt
        self.n_disease = n_disease
        self.use_warmup_classifier = use_warmup_classifier
        self.encoder = _build_text_backbone(model_name)
        self.hyperparameters = self.encoder.config
        self.hidden_size = self.hyperparameters.hidden_size
        self.proj = Linear(self.hidden_size, self.d_txt)
        self.classifier = Linear(d_txt, n_disease) if self.use_warmup_classifier else None
        self.is_frozen = False
        self.set_compute_dtype(compute_dtype or get_compute_dtype())

    def set_compute_dtype(self, dtype):
        self.compute_dtype = dtype
        self.encoder.compute_dtype = dtype
        return self

    def freeze_encoder(self):  # TP:372-387
        for p in self.encoder.parameters():
            p.requires_grad = False
        self.is_frozen = True
        self.encoder.eval()
        self.proj.train()
        if self.classifier is not None:
            self.classifier.train()

    def unfreeze_encoder(self):  # TP:390-405
        for p in self.encoder.parameters():
            p.requires_grad = True
        self.is_frozen = False
        self.encoder.train()
        self.proj.train()
        if self.classifier is not None:
            self.classifier.train()

    def build_optimizer(self, phase, lr_enc=1e-4, lr_head=54 - 4, weight_decay=1e-2,
                        optimizer_cls=AdamW):  # TP:408-432 (lr_head default kept: 54-4 = 50)
        if phase == 1:
            params = [{"params": self.proj.parameters(), "lr": lr_head}]
            if self.classifier is not None:
                params.append({"params": self.classifier.parameters(), "lr": lr_head})
            return optimizer_cls(params, weight_decay=weight_decay)
        if phase == 2:
            enc_params = [p for p in self.encoder.parameters() if p.requires_grad]
            params = []
            if enc_params:
                params.append({"params": enc_params, "lr": lr_enc})
            params.append({"params": self.proj.parameters(), "lr": lr_head})
            if self.classifier is not None:
                params.append({"params": self.classifier.parameters(), "lr": lr_head})
            return optimizer_cls(params, weight_decay=weight_decay)

    def mean_pool(self, last_hidden_state, attention_mask):  # TP:452-459
        return F.masked_mean(last_hidden_state, attention_mask.long())

    def _pooled(self, input_ids, attention_mask, token_type_ids):
        if hasattr(self.encoder, "pooled_mean"):
            return self.encoder.pooled_mean(input_ids, attention_mask, token_type_ids)
        out = self.encoder(input_ids=input_ids, attention_mask=attention_mask,
                           token_type_ids=token_type_ids, return_dict=True)
        return self.mean_pool(out.last_hidden_state, attention_mask)

    def encode(self, input_ids, attention_mask, token_type_ids):  # TP:465-488
        input_ids = input_ids.long()
        attention_mask = attention_mask.long()
        if token_type_ids is not None:
            token_type_ids = token_type_ids.long()
        if self.is_frozen:
            with torch.no_grad():
                pooled = self._pooled(input_ids, attention_mask, token_type_ids)
        else:
            pooled = self._pooled(input_ids, attention_mask, token_type_ids)
        return self.proj(pooled)

    def forward(self, **batch):  # TP:503-508
        z = self.encode(batch["input_ids"], batch["attention_mask"], batch.get("token_type_ids"))
        out = {"embeddings": z}
        if self.classifier is not None:
            out["logits"] = self.classifier(z, out_dtype=torch.float32)
        return out


# =====================================================================================
# Fusion model (TP:516-618)
# =====================================================================================
class FusionTransformerModel(nn.Module):
    def __init__(self, d_img, d_txt, d_fuse_hidden=1024, n_disease=13, model_name="t5-small",
                 n_cond_tokens=4, dropout=0.1, init_t5_from_config=None, t5_assets_dir=None,
                 with_report_head=False):  # TP:518-569
        super().__init__()
        self.d_img, self.d_txt = d_img, d_txt
        self.d_fuse_hidden = d_fuse_hidden
        self.n_disease = n_disease
        self.model_name = model_name
        self.n_cond_tokens = n_cond_tokens
        self.dropout = dropout
        self.d_fuse = self.d_img + self.d_txt
        self.fusion_mlp = nn.Sequential(
            Linear(self.d_fuse, self.d_fuse_hidden),
            GELU(),
            Dropout(dropout),
            LayerNorm(self.d_fuse_hidden),
        )
        self.disease_head = Linear(self.d_fuse_hidden, n_disease)
        # T5 report head: outside the hot path.  Built only on
        # request, from a local config/assets dir (no network); d_model of t5-small = 512.
        self.report_model = None
        self.h_dec = 512
        if with_report_head or init_t5_from_config or t5_assets_dir:
            self.report_model = _build_t5(model_name, init_t5_from_config, t5_assets_dir)
            if self.report_model is not None:
                self.h_dec = self.report_model.config.d_model
        self.n_cond = self.n_cond_tokens
        self.cond_proj = nn.Sequential(Linear(self.d_fuse_hidden, self.h_dec * self.n_cond),
                                       GELU())

    def _fuse(self, z_img, z_txt):
        lin, _, drop, ln = self.fusion_mlp
        T = z_img.dtype
        h = F.fusion_linear(z_img.contiguous(), z_txt.to(T).contiguous(), lin.weight, lin.bias,
                            L.ACT_GELU)
        h = drop(h)
        return ln(h)

    def _t5(self):
        if self.report_model is None:
            raise NotImplementedError(
                "no T5 report head attached: build the fusion model with with_report_head=True, "
                "init_t5_from_config=True or t5_assets_dir (TP:561-569)")
        head = getattr(self, "_t5_head", None)
        if head is None or head.m is not self.report_model:
            from .t5 import T5Head
            head = self._t5_head = T5Head(self.report_model)
        return head

    def forward(self, z_img, z_txt, report_input_ids=None, report_attention_mask=None,
                report_labels=None):  # TP:584-610
        z_fuse = self._fuse(z_img, z_txt)
        disease_logits = self.disease_head(z_fuse, out_dtype=torch.float32)
        gen = None
        if (report_input_ids is not None) or (report_labels is not None):
            # T5 decoder conditioned on K tokens from z_fuse, teacher-forced CE on the labels
            # (TP:595-604; report_input_ids / mask are accepted and unused, as in the reference)
            head = self._t5()
            enc = self._make_encoder_outputs(z_fuse).last_hidden_state
            loss, logits = head.forward(enc, labels=report_labels, T=z_fuse.dtype)
            gen = SimpleNamespace(loss=loss, logits=logits)
        return {"z_fuse": z_fuse, "disease_logits": disease_logits, "gen": gen}

    def _make_encoder_outputs(self, z_fuse):  # TP:574-578
        from transformers.modeling_outputs import BaseModelOutput
        B = z_fuse.size(0)
        cond = self.cond_proj[0](z_fuse, act=L.ACT_GELU)
        cond = cond.view(B, self.n_cond, self.h_dec)
        return BaseModelOutput(last_hidden_state=cond)

    @torch.no_grad()
    def generate(self, z_img, z_txt, **gen_kwargs):  # TP:613-618
        """Beam-search report token ids (the reference's report_model.generate kwargs:
        num_beams, max_new_tokens, min_new_tokens, no_repeat_ngram_size, length_penalty,
        early_stopping, eos_token_id, pad_token_id) on the mmdx T5 decoder."""
        head = self._t5()
        z_fuse = self._fuse(z_img, z_txt)
        enc = self._make_encoder_outputs(z_fuse).last_hidden_state
        return head.generate(enc, T=z_fuse.dtype, **gen_kwargs)


def _build_t5(model_name, init_from_config, assets_dir):
    try:
        from transformers import T5Config, T5ForConditionalGeneration
    except ImportError:  # pragma: no cover
        return None
    if assets_dir:
        return T5ForConditionalGeneration.from_pretrained(assets_dir, local_files_only=True)
    # t5-small geometry (its config.json values) without any download
    cfg = T5Config(d_model=512, d_ff=2048, d_kv=64, num_layers=6, num_decoder_layers=6,
                   num_heads=8, vocab_size=32128, relative_attention_num_buckets=32,
                   relative_attention_max_distance=128, dropout_rate=0.1,
                   layer_norm_epsilon=1e-6, feed_forward_proj="relu", decoder_start_token_id=0,
                   eos_token_id=1, pad_token_id=0, tie_word_embeddings=True)
    return T5ForConditionalGeneration(cfg)
