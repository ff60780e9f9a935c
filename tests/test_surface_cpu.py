"""CPU: the mmdx operator surface mirrors the reference (names, kwargs, state_dict keys,
optimizer groups, errors, preprocessing) without touching a GPU."""
import os

import numpy as np
import pytest
import torch
from PIL import Image

import mmdx
from oracle import ref_cpu as R

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.mark.parametrize("arch", ["resnet18", "resnet50"])
def test_image_state_dict_keys(arch):
    ref = R.RefImageEncoderCNN(arch)
    mine = mmdx.ImageEncoderCNN(arch)
    assert list(ref.state_dict()) == list(mine.state_dict())
    for (k, a), (_, b) in zip(ref.state_dict().items(), mine.state_dict().items()):
        assert a.shape == b.shape and a.dtype == b.dtype, k
    mine.load_state_dict(ref.state_dict())  # strict round trip


@pytest.mark.parametrize("name,ref_name", [("bert-base-uncased@2", "bert-base-uncased"),
                                           ("embed-mean", "embed-mean"), ("bilstm", "bilstm")])
def test_text_state_dict_keys(name, ref_name):
    ref = R.RefTextEncoderTransformer(ref_name, bert_layers=2)
    mine = mmdx.TextEncoderTransformer(name)
    assert set(ref.state_dict()) == set(mine.state_dict())
    mine.load_state_dict(ref.state_dict())


def test_bert_full_key_set_matches_transformers():
    from transformers import BertConfig, BertModel
    hf = BertModel(BertConfig())
    mine = mmdx.text_encoders.BertModel()
    assert set(hf.state_dict()) == set(mine.state_dict())
    assert sum(p.numel() for p in mine.parameters()) == 109482240


def test_fusion_keys_and_forward_contract():
    fus = mmdx.FusionTransformerModel(d_img=1024, d_txt=512, n_disease=13)
    keys = set(fus.state_dict())
    for k in ("fusion_mlp.0.weight", "fusion_mlp.3.weight", "disease_head.weight",
              "cond_proj.0.weight"):
        assert k in keys
    assert fus.d_fuse == 1536 and fus.n_cond == 4


def test_unsupported_backbone_raises_valueerror():
    with pytest.raises(ValueError):
        mmdx.ImageEncoderCNN("vgg16")


def test_build_optimizer_groups_follow_reference():
    m = mmdx.ImageEncoderCNN("resnet18")
    m.freeze_backbone()
    o1 = m.build_optimizer(phase=1, lr_head=5e-4, weight_decay=1e-2)
    assert [g["lr"] for g in o1.param_groups] == [5e-4, 5e-4]
    m.unfreeze_backbone()
    o2 = m.build_optimizer(phase=2, lr_backbone=1e-4, lr_head=5e-4)
    assert [g["lr"] for g in o2.param_groups] == [1e-4, 5e-4, 5e-4]
    assert all(g["weight_decay"] == 1e-2 for g in o2.param_groups)
    t = mmdx.TextEncoderTransformer("embed-mean")
    t.unfreeze_encoder()
    o3 = t.build_optimizer(phase=2, lr_enc=2e-5, lr_head=5e-4)
    assert [g["lr"] for g in o3.param_groups] == [2e-5, 5e-4, 5e-4]
    # the reference's default lr_head is the literal 54-4 (=50), kept verbatim (TP:408)
    assert t.build_optimizer(phase=1).param_groups[0]["lr"] == 50


def test_image_transform_matches_oracle_on_sample():
    img = Image.open(os.path.join(HERE, "golden", "e1.jpg")).convert("RGB")
    a = mmdx.image_transfom_into_tensor(img)
    b = R.reference_transform(img)
    assert a.shape == (3, 224, 224) and a.dtype == torch.float32  # TP:823-824
    assert torch.allclose(a, b, atol=1e-6)
    gray = img.convert("L")
    g = mmdx.image_transfom_into_tensor(gray)
    assert g.shape == (3, 224, 224)


def test_tokenize_contract():
    tok = mmdx.tokenize_patient_details(["67M, smoker; dyspnea; CHF history.",
                                         "54F, no smoking; cough; asthma."], max_len=96)
    assert tuple(tok["input_ids"].shape) == (2, 96)  # TP:898-899
    assert (tok["input_ids"][:, 0] == 101).all()
    assert tok["attention_mask"].sum(1).min() >= 2


def test_cpu_tensors_fail_loudly():
    m = mmdx.TextEncoderTransformer("embed-mean")
    with pytest.raises(RuntimeError):
        m(input_ids=torch.randint(0, 100, (1, 8)), attention_mask=torch.ones(1, 8,
                                                                             dtype=torch.long))


def _write_bundle(path, drop=None):
    torch.manual_seed(0)
    img = mmdx.ImageEncoderCNN("resnet18", 1024, 13)
    txt = mmdx.TextEncoderTransformer("embed-mean", 512, 13)
    fus = mmdx.FusionTransformerModel(1024, 512, 1024, 13)
    bundle = {"cfg": {"fusion": {"d_img": 1024, "d_txt": 512},
                      "image_encoder": {"backbone": "resnet18"}},
              "fusion_state": fus.state_dict(), "image_state": img.state_dict(),
              "text_state": txt.state_dict(), "t5_tokenizer_name": "t5-small",
              "bert_tokenizer_name": "embed-mean", "version": 999}  # TP:783-791
    if drop:
        bundle.pop(drop)
    torch.save(bundle, path)
    return img, txt, fus


def test_bundle_roundtrip_and_key_validation(tmp_path):
    from mmdx.inference_pipeline import load_model_bundle
    with pytest.raises(FileNotFoundError):  # VW:178
        load_model_bundle(str(tmp_path / "missing.pt"), device="cpu")
    bad = tmp_path / "bad.pt"
    _write_bundle(bad, drop="text_state")
    with pytest.raises(ValueError):  # VW:204
        load_model_bundle(str(bad), device="cpu")
    good = tmp_path / "model_bundle.pt"
    img, txt, fus = _write_bundle(good)
    b = load_model_bundle(str(good), device="cpu")
    assert b["version"] == 999 and len(b["class_names"]) == 13 and b["thresholds"] == [0.5] * 13
    for mine, ref in ((b["image_encoder"], img), (b["text_encoder"], txt),
                      (b["fusion_model"], fus)):
        sd, rsd = mine.state_dict(), ref.state_dict()
        assert set(sd) == set(rsd)
        for k in rsd:
            assert torch.equal(sd[k], rsd[k]), k


def test_inference_rejects_bad_device_type():
    from mmdx.inference_pipeline import inference
    with pytest.raises(TypeError):  # IP:159
        inference({}, None, "x", device=3)


def test_vit_b_16_tower_keys_match_torchvision_layout():
    """vit_b_16 (C5, build-defined name): torchvision state_dict keys minus `heads`, and
    torchvision's parameter count (86,567,656 - 769,000 head parameters)."""
    m = mmdx.ImageEncoderCNN("vit_b_16", 1024, 13)
    r = R.RefImageEncoderCNN("vit_b_16")
    assert set(m.state_dict()) == set(r.state_dict())
    assert "backbone.encoder.layers.encoder_layer_11.self_attention.in_proj_weight" in m.state_dict()
    assert sum(p.numel() for p in m.backbone.parameters()) == 85798656
    assert m.backbone.feat_dim == 768 and m.proj.in_features == 768


def test_save_model_bundle_roundtrip(tmp_path):
    """save_model_bundle writes TP:773-796's dict atomically (no .tmp left behind, plus a
    timestamped copy) and load_model_bundle reads it back bit-identically."""
    from mmdx.inference_pipeline import load_model_bundle, save_model_bundle
    torch.manual_seed(0)
    img = mmdx.ImageEncoderCNN("resnet18", 1024, 13)
    txt = mmdx.TextEncoderTransformer("embed-mean", 512, 13)
    fus = mmdx.FusionTransformerModel(1024, 512, 1024, 13)
    path = save_model_bundle(fus, img, txt, tmp_path, version=7,
                             artifacts={"class_names": mmdx.DISEASES, "thresholds": [0.4] * 13})
    files = sorted(p.name for p in tmp_path.iterdir())
    assert "model_bundle.pt" in files and not any(f.endswith(".tmp") for f in files)
    assert any(f.startswith("model_bundle_") and f.endswith("Z.pt") for f in files)
    raw = torch.load(path, weights_only=True)
    assert list(raw) == ["cfg", "fusion_state", "image_state", "text_state",
                         "t5_tokenizer_name", "bert_tokenizer_name", "version"]
    cfg = raw["cfg"]
    assert cfg["fusion"] == {"d_img": 1024, "d_txt": 512, "d_fuse_hidden": 1024, "n_disease": 13,
                             "n_cond_tokens": 4, "decoder_hidden": None}
    assert cfg["text_encoder"]["hf_model_name"] == "embed-mean" == raw["bert_tokenizer_name"]
    assert cfg["image_encoder"]["backbone"] == "resnet18"
    b = load_model_bundle(path, device="cpu")
    assert b["version"] == 7 and b["thresholds"] == [0.4] * 13
    for mine, ref in ((b["image_encoder"], img), (b["text_encoder"], txt),
                      (b["fusion_model"], fus)):
        sd, rsd = mine.state_dict(), ref.state_dict()
        assert set(sd) == set(rsd)
        for k in rsd:
            assert torch.equal(sd[k], rsd[k]), k


def test_bundle_fusion_state_strict(tmp_path):
    """report_model.* keys (a reference bundle with its T5 head) load without a T5 head;
    any other fusion-key mismatch raises instead of running random heads.  The text
    architecture comes from cfg, not from bert_tokenizer_name."""
    from mmdx.inference_pipeline import load_model_bundle
    torch.manual_seed(0)
    img = mmdx.ImageEncoderCNN("resnet18", 1024, 13)
    txt = mmdx.TextEncoderTransformer("embed-mean", 512, 13)
    fus = mmdx.FusionTransformerModel(1024, 512, 1024, 13)
    fs = dict(fus.state_dict())
    fs["report_model.shared.weight"] = torch.zeros(4, 4)
    bundle = {"cfg": {"fusion": {"d_img": 1024, "d_txt": 512},
                      "image_encoder": {"backbone": "resnet18"},
                      "text_encoder": {"hf_model_name": "embed-mean"}},
              "fusion_state": fs, "image_state": img.state_dict(),
              "text_state": txt.state_dict(), "t5_tokenizer_name": "t5-small",
              "bert_tokenizer_name": "bert-base-uncased", "version": 3}
    ok = tmp_path / "ok.pt"
    torch.save(bundle, ok)
    b = load_model_bundle(str(ok), device="cpu", with_report_head=False)
    assert b["text_encoder"].model_name == "embed-mean"
    assert torch.equal(b["fusion_model"].disease_head.weight, fus.disease_head.weight)
    fs2 = dict(fs)
    fs2["disease_head.weight_renamed"] = fs2.pop("disease_head.weight")
    bundle["fusion_state"] = fs2
    bad = tmp_path / "bad.pt"
    torch.save(bundle, bad)
    with pytest.raises(RuntimeError):
        load_model_bundle(str(bad), device="cpu", with_report_head=False)


def test_bundle_with_t5_report_head_roundtrip(tmp_path):
    """A bundle written with the T5 report head (report_model.*: the reference's
    FusionTransformerModel state, TP:783-791) loads into the mmdx fusion model with its T5
    head, every key strictly, bit-identical."""
    from mmdx.inference_pipeline import load_model_bundle, save_model_bundle
    torch.manual_seed(0)
    img = mmdx.ImageEncoderCNN("resnet18", 1024, 13)
    txt = mmdx.TextEncoderTransformer("embed-mean", 512, 13)
    fus = mmdx.FusionTransformerModel(1024, 512, 1024, 13, init_t5_from_config=True)
    path = save_model_bundle(fus, img, txt, tmp_path, version=2, timestamped_copy=False)
    b = load_model_bundle(path, device="cpu")
    f2 = b["fusion_model"]
    assert f2.report_model is not None
    sd, rsd = f2.state_dict(), fus.state_dict()
    assert set(sd) == set(rsd)
    for k in rsd:
        assert torch.equal(sd[k], rsd[k]), k
