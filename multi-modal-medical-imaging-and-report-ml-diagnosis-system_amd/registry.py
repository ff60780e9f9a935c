"""Local stand-ins for the reference's cloud I/O, so its callers run unchanged offline.

The reference reaches three services from the hot path's callers: the Hopsworks feature store
(TP:72-90), an S3 image bucket (TP:93-103, TP:142-152) and the Hopsworks model registry
(TP:650-804 save, IP:36-139 load).  Network I/O is out of scope, but the
function names, arguments, return values and on-disk formats are part of the drop-in
surface, so each is restated over a local directory:

* feature store  -> a parquet file (env MMDX_FEATURES_PARQUET) read by mmdx.data with the
  reference's type enforcement and event_time dedupe;
* S3             -> a local mirror (env MMDX_S3_MIRROR): s3://bucket/key is the file
  <mirror>/<bucket>/<key>;
* model registry -> a directory (env MMDX_MODEL_REGISTRY, default ./model_registry) holding
  <name>/<version>/ folders with exactly the files the reference uploads (TP:675-724:
  fusion_model.pt, image_encoder.pt, text_encoder.pt, config.json, t5_assets/) and the
  local `model_bundle.pt` written next to it (TP:773-796; env MMDX_MODEL_DIR).

When a variable is unset the functions raise with a message naming it — never a silent
fallback to random data.
"""
from __future__ import annotations

import json
import os
import shutil
from pathlib import Path


class OfflineServiceError(RuntimeError):
    """A cloud service of the reference (Hopsworks, S3) was asked for without a local
    stand-in configured."""


def _env_path(var, what):
    v = os.environ.get(var)
    if not v:
        raise OfflineServiceError(
            f"{what} is a cloud service in the reference and out of scope offline; set {var} "
            f"to a local stand-in")
    return v


# ----------------------------------------------------------------------------- S3
def parse_s3_url(url):
    """TP:99-103: 's3://bucket/key' -> (bucket, key); asserts the scheme as the reference."""
    assert url.startswith("s3://")
    bucket, key = url[5:].split("/", 1)
    return bucket, key


def get_image_from_s3(bucket, key):
    """TP:93-96: the object's bytes — read from <MMDX_S3_MIRROR>/<bucket>/<key>."""
    root = Path(_env_path("MMDX_S3_MIRROR", "S3 (get_image_from_s3)")).resolve()
    path = (root / bucket / key).resolve()
    # bucket / key come from feature-store rows: a '..' or absolute component must not read
    # outside the mirror
    if root != path and root not in path.parents:
        raise ValueError(f"s3://{bucket}/{key} resolves outside the local mirror ({root})")
    if not path.is_file():
        raise FileNotFoundError(f"s3://{bucket}/{key} not in the local mirror ({path})")
    return path.read_bytes()


# ----------------------------------------------------------------------------- feature store
def load_features_labels_from_feature_store():
    """TP:72-90: the feature group as a dataframe (image_url, patient_details,
    disease_classification_vector, report[, event_time]); latest row per image_url."""
    from .data import load_features_labels_local
    return load_features_labels_local(_env_path("MMDX_FEATURES_PARQUET",
                                                "The Hopsworks feature store"))


# ----------------------------------------------------------------------------- registry
def registry_root():
    return Path(os.environ.get("MMDX_MODEL_REGISTRY", os.path.join(os.getcwd(),
                                                                   "model_registry")))


class RegistryModel:
    """The slice of hsml's Model the reference uses: .name, .version, .download(), .save()."""

    def __init__(self, root, name, version, metrics=None, description=""):
        self.root = Path(root)
        self.name = name
        self.version = int(version)
        self.metrics = metrics or {}
        self.description = description

    @property
    def path(self):
        return self.root / self.name / str(self.version)

    def download(self):
        if not self.path.is_dir():
            raise FileNotFoundError(f"model {self.name} v{self.version} not in {self.root}")
        return str(self.path)

    def save(self, local_dir):
        """Upload (copy) a staged folder as this version, atomically (tmp + rename)."""
        dst = self.path
        dst.parent.mkdir(parents=True, exist_ok=True)
        tmp = dst.with_name(f".{dst.name}.tmp")
        if tmp.exists():
            shutil.rmtree(tmp)
        shutil.copytree(local_dir, tmp)
        with open(tmp / "model.json", "w") as f:
            json.dump({"name": self.name, "version": self.version, "metrics": self.metrics,
                       "description": self.description}, f, indent=2)
        # the old version is renamed aside (not deleted) before the new one takes its name,
        # so a crash at any point leaves either version on disk under a known name
        old = dst.with_name(f".{dst.name}.old")
        if old.exists():
            shutil.rmtree(old)
        if dst.exists():
            os.replace(dst, old)
        os.replace(tmp, dst)
        if old.exists():
            shutil.rmtree(old)
        return self


class LocalModelRegistry:
    """The slice of hsml's ModelRegistry the reference calls (get_models, get_model,
    create_model / python.create_model)."""

    def __init__(self, root=None):
        self.root = Path(root) if root is not None else registry_root()
        self.python = self

    def get_models(self, name):
        d = self.root / name
        if not d.is_dir():
            return []
        return [RegistryModel(self.root, name, v.name) for v in d.iterdir()
                if v.is_dir() and v.name.isdigit()]

    def get_model(self, name, version=None):
        if version is None:
            version = latest_version(self, name)
        return RegistryModel(self.root, name, version)

    def create_model(self, name, version=None, metrics=None, description="",
                     model_schema=None):
        if version is None:  # the registry auto-increments (TP:733-747)
            have = self.get_models(name)
            version = 1 + max((m.version for m in have), default=0)
        return RegistryModel(self.root, name, version, metrics, description)


def latest_version(model_reg, name: str) -> int:
    """IP:36-41."""
    models = model_reg.get_models(name=name)
    if not models:
        raise RuntimeError(f"No models named '{name}' found.")
    return max(m.version for m in models)


def login(project=None):
    """hopsworks.login stand-in: an object whose get_model_registry() is the local one."""

    class _Project:
        name = project

        @staticmethod
        def get_model_registry():
            return LocalModelRegistry()

    return _Project()
