"""CPU: the reference's callers import the drop-in unchanged, and the local stand-ins of its
cloud I/O (S3, feature store, model registry) behave as the reference's calls expect.

* The exact import lines of backend/api/views.py:12-17, inference_pipeline.py:25-29 (inside
  the shim module) and run_daily_training_pipeline.py:2, executed in a fresh interpreter
  with only integration/backend on the path — no hopsworks, boto3, torchvision or django.
* parse_s3_url / get_image_from_s3 (TP:93-103) over a local mirror; a clear error without one.
* The local model registry: save_model_to_hopsworks_model_registry (TP:650-804) writes the
  files IP:53-139 reads, versions auto-increment, load_model_from_hopsworks_model_registry
  rebuilds every module with identical state, and the local model_bundle.pt carries the
  bundle keys VW:200-204 validates.  (Module construction and state loading only: no GPU.)
"""
import json
import os
import subprocess
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SHIM = os.path.join(ROOT, "integration", "backend")

CALLER_LINES = """
import torch
from ml.pipelines.inference_pipeline import load_model_from_hopsworks_model_registry, inference
from ml.pipelines.inference_pipeline import FusionTransformerModel, ImageEncoderCNN, TextEncoderTransformer

torch.serialization.add_safe_globals([FusionTransformerModel])
torch.serialization.add_safe_globals([ImageEncoderCNN])
torch.serialization.add_safe_globals([TextEncoderTransformer])
from ml.pipelines.training_pipeline import training_tests
import mmdx, sys
assert ImageEncoderCNN is mmdx.ImageEncoderCNN
assert FusionTransformerModel is mmdx.FusionTransformerModel
assert training_tests is mmdx.training_pipeline.training_tests
assert inference is mmdx.inference_pipeline.inference
for banned in ("hopsworks", "hsml", "boto3", "torchvision", "django"):
    assert banned not in sys.modules, banned
print("CALLERS-OK")
"""


def test_reference_callers_import_unchanged():
    env = dict(os.environ, PYTHONPATH=SHIM)
    env.pop("MMDX_HOME", None)
    r = subprocess.run([sys.executable, "-c", CALLER_LINES], env=env, cwd="/tmp",
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "CALLERS-OK" in r.stdout


def test_s3_mirror(tmp_path, monkeypatch):
    import mmdx
    from mmdx import registry as REG
    from mmdx.training_pipeline import get_image_from_s3, parse_s3_url
    assert parse_s3_url("s3://medical-ml-proj-bucket/chest-x-ray-images/a.jpg") == (
        "medical-ml-proj-bucket", "chest-x-ray-images/a.jpg")
    with pytest.raises(AssertionError):
        parse_s3_url("http://x/y")
    monkeypatch.delenv("MMDX_S3_MIRROR", raising=False)
    with pytest.raises(REG.OfflineServiceError, match="MMDX_S3_MIRROR"):
        get_image_from_s3("b", "k.jpg")
    (tmp_path / "b" / "dir").mkdir(parents=True)
    (tmp_path / "b" / "dir" / "k.jpg").write_bytes(b"\xff\xd8abc")
    monkeypatch.setenv("MMDX_S3_MIRROR", str(tmp_path))
    assert get_image_from_s3("b", "dir/k.jpg") == b"\xff\xd8abc"
    with pytest.raises(FileNotFoundError):
        get_image_from_s3("b", "missing.jpg")
    # keys from feature-store rows cannot leave the mirror
    (tmp_path.parent / "outside.jpg").write_bytes(b"secret")
    with pytest.raises(ValueError, match="outside the local mirror"):
        get_image_from_s3("b", "../../outside.jpg")
    with pytest.raises(ValueError, match="outside the local mirror"):
        get_image_from_s3("..", "outside.jpg")
    monkeypatch.delenv("MMDX_FEATURES_PARQUET", raising=False)
    with pytest.raises(REG.OfflineServiceError, match="MMDX_FEATURES_PARQUET"):
        mmdx.training_pipeline.load_features_labels_from_feature_store()


def test_registry_roundtrip(tmp_path, monkeypatch):
    import mmdx
    from mmdx.inference_pipeline import (BUNDLE_KEYS, latest_version,
                                         load_model_from_hopsworks_model_registry)
    from mmdx.registry import LocalModelRegistry
    monkeypatch.setenv("MMDX_MODEL_REGISTRY", str(tmp_path / "registry"))
    monkeypatch.setenv("MMDX_MODEL_DIR", str(tmp_path / "model"))
    torch.manual_seed(0)
    img = mmdx.ImageEncoderCNN("resnet18", 1024, 13)
    txt = mmdx.TextEncoderTransformer("embed-mean", 512, 13)
    fus = mmdx.FusionTransformerModel(1024, 512, 1024, 13, with_report_head=True)
    arts = {"class_names": list(mmdx.DISEASES), "thresholds": [0.5] * 13}
    rm1 = mmdx.training_pipeline.save_model_to_hopsworks_model_registry(
        fus, model_name="fusion_model_T5", image_encoder=img, text_encoder=txt,
        artifacts=arts, hf_model_name="t5-small")
    rm2 = mmdx.training_pipeline.save_model_to_hopsworks_model_registry(
        fus, model_name="fusion_model_T5", image_encoder=img, text_encoder=txt,
        artifacts=arts, hf_model_name="t5-small")
    assert (rm1.version, rm2.version) == (1, 2)
    reg = LocalModelRegistry()
    assert latest_version(reg, "fusion_model_T5") == 2
    d = tmp_path / "registry" / "fusion_model_T5" / "2"
    for f in ("fusion_model.pt", "image_encoder.pt", "text_encoder.pt", "config.json"):
        assert (d / f).is_file(), f
    assert (d / "t5_assets").is_dir()
    cfg = json.loads((d / "config.json").read_text())
    assert cfg["fusion"] == {"d_img": 1024, "d_txt": 512, "d_fuse_hidden": 1024,
                             "n_disease": 13, "n_cond_tokens": 4, "decoder_hidden": 512}
    assert cfg["image_encoder"]["backbone"] == "resnet18"
    assert cfg["artifacts"] == arts
    b = load_model_from_hopsworks_model_registry("fusion_model_T5")
    assert b["version"] == 2 and set(b) >= {"cfg", "fusion_model", "image_encoder",
                                            "text_encoder", "t5_tok", "bert_tok",
                                            "class_names", "thresholds", "dir"}
    for mine, theirs in ((b["fusion_model"], fus), (b["image_encoder"], img),
                         (b["text_encoder"], txt)):
        sa, sb = mine.state_dict(), theirs.state_dict()
        assert sa.keys() == sb.keys()
        assert all(torch.equal(sa[k], sb[k]) for k in sa)
    with pytest.raises(RuntimeError, match="No models named"):
        load_model_from_hopsworks_model_registry("nope")
    blob = torch.load(tmp_path / "model" / "model_bundle.pt", map_location="cpu",
                      weights_only=True)
    assert set(BUNDLE_KEYS) <= set(blob) and blob["version"] == 2


def test_adamw_refuses_late_parameters():
    import mmdx
    with pytest.raises(ValueError, match="per-parameter steps"):
        p = torch.nn.Parameter(torch.zeros(3))
        q = torch.nn.Parameter(torch.zeros(3))
        opt = mmdx.AdamW([p, q])
        sd = opt.state_dict()
        sd["state"] = {0: {"step": torch.tensor(3.0), "exp_avg": torch.zeros(3),
                           "exp_avg_sq": torch.zeros(3)},
                       1: {"step": torch.tensor(5.0), "exp_avg": torch.zeros(3),
                           "exp_avg_sq": torch.zeros(3)}}
        opt.load_state_dict(sd)


def test_registry_save_replaces_a_version_atomically(tmp_path, monkeypatch):
    """RegistryModel.save over an existing version: the new folder takes the name, the old
    one is gone, no temporary or renamed-aside folder is left behind."""
    from mmdx.registry import LocalModelRegistry
    monkeypatch.setenv("MMDX_MODEL_REGISTRY", str(tmp_path / "registry"))
    reg = LocalModelRegistry()
    for content in (b"v1", b"v2"):
        stage = tmp_path / f"stage_{content.decode()}"
        stage.mkdir()
        (stage / "weights.bin").write_bytes(content)
        rm = reg.create_model("m", version=1)
        rm.save(str(stage))
    d = tmp_path / "registry" / "m"
    assert (d / "1" / "weights.bin").read_bytes() == b"v2"
    assert sorted(p.name for p in d.iterdir()) == ["1"]
