"""Local dataset loader: the reference's Hopsworks feature group + S3
image bucket replaced by a local parquet file and a local image directory, feeding the same
(image, patient_details, disease vector) triples to the GPU train step.

Reference behaviour kept:
  * the raw-data schema and type enforcement of `feature_pipeline.enforce_raw_data_columns`
    (feature_pipeline.py:34-58): image_url / patient_details / report as str, the disease
    vector as 13 floats (a list or its JSON text), ValueError otherwise;
  * the feature-store read's dedupe (TP:86-88): with an `event_time` column, the latest row
    per image_url wins;
  * `construct_input_label_pairs_for_image_encoder_dataset` (TP:122-127): image keys from the
    image_url column (an s3://bucket/key URL keeps its key, TP:99-103; a plain path is used as
    is) and float32 label vectors;
  * `CXR_ImageDataset.__getitem__` (TP:142-152): image bytes -> PIL image -> the transform,
    label as a float32 tensor.

New: `LocalCXRBatches` decodes a batch on the host with PIL (as the reference does) and runs
the transform for the whole batch on the GPU in two HIP launches (`preprocess_batch`,
bit-exact with `image_transfom_into_tensor`), so the host cost per sample is the decode.
"""
from __future__ import annotations

import io
import json
import os

import numpy as np
import torch

RAW_DATA_COLUMNS = ["image_url", "patient_details", "disease_classification_vector", "report"]
N_DISEASES = 13


def _to_float_vector(x):
    """feature_pipeline.py:47-54: list/tuple/array or JSON text -> 13 floats."""
    if isinstance(x, (list, tuple, np.ndarray)):
        arr = np.asarray(x, dtype=float)
    else:
        arr = np.asarray(json.loads(str(x)), dtype=float)
    if arr.size != N_DISEASES:
        raise ValueError(f"Expected vector of length {N_DISEASES}, got {arr.size}")
    return arr


def enforce_raw_data_columns(df):
    """feature_pipeline.enforce_raw_data_columns (feature_pipeline.py:41-58)."""
    df["image_url"] = df["image_url"].astype(str)
    df["patient_details"] = df["patient_details"].astype(str)
    df["report"] = df["report"].astype(str)
    df["disease_classification_vector"] = df["disease_classification_vector"].map(
        _to_float_vector)
    return df


def load_features_labels_local(parquet_path: str):
    """Local stand-in for `load_raw_data` + `load_features_labels_from_feature_store`
    (feature_pipeline.py:61-66, TP:72-90): read the raw columns (plus `event_time` when
    present), enforce their types, keep the latest row per image_url."""
    import pandas as pd
    import pyarrow.parquet as pq
    names = set(pq.read_schema(parquet_path).names)
    missing = [c for c in RAW_DATA_COLUMNS if c not in names]
    if missing:
        raise ValueError(f"{parquet_path}: missing columns {missing}")
    cols = RAW_DATA_COLUMNS + (["event_time"] if "event_time" in names else [])
    df = pd.read_parquet(parquet_path, columns=cols, engine="pyarrow")
    df = enforce_raw_data_columns(df)
    if "event_time" in df.columns:  # TP:86-88
        df = (df.sort_values("event_time").groupby("image_url", as_index=False).tail(1)
              .reset_index(drop=True))
    return df


def parse_image_key(url: str) -> str:
    """TP:99-103 for s3:// URLs (the key part); any other string is a local path."""
    if url.startswith("s3://"):
        return url[5:].split("/", 1)[1]
    return url


def construct_input_label_pairs_for_image_encoder_dataset(df):
    """TP:122-127: image keys and float32 disease vectors, in row order."""
    keys = [parse_image_key(u) for u in df["image_url"].tolist()]
    labels = [np.asarray(v, dtype=np.float32) for v in df["disease_classification_vector"]]
    return keys, labels


def open_image(root, key):
    """Image bytes -> PIL image (TP:144-146), from `root/key` (or `key` if absolute)."""
    from PIL import Image
    path = key if os.path.isabs(key) or not root else os.path.join(root, key)
    with open(path, "rb") as f:
        img = Image.open(io.BytesIO(f.read()))
        img.load()
    return img


class CXR_ImageDataset(torch.utils.data.Dataset):
    """TP:131-152 with the S3 bucket replaced by a local directory `image_root` (image keys
    are paths relative to it).  `image_transform` as in the reference (e.g.
    training_pipeline.image_transfom_into_tensor); None returns the decoded PIL image."""

    def __init__(self, img_keys_input, image_root, labels=None, image_transform=None):
        self.img_keys_input = img_keys_input
        self.image_root = image_root
        self.labels = labels
        self.image_transform = image_transform

    def __len__(self):
        assert len(self.img_keys_input) == len(self.labels)
        return len(self.img_keys_input)

    def __getitem__(self, i):
        img = open_image(self.image_root, self.img_keys_input[i])
        x = self.image_transform(img) if self.image_transform is not None else img
        y = torch.tensor(self.labels[i], dtype=torch.float32)
        return x, y


class LocalCXRBatches:
    """Batches of (images [B,3,224,224] fp32 on the GPU, patient_details list[str],
    labels [B,13] fp32 on the GPU) from a feature dataframe and a local image root.  Images
    are decoded on the host (PIL, TP:146) and transformed on the GPU for the whole batch
    (`preprocess_batch`, identical to stacking `image_transfom_into_tensor` outputs).
    `shuffle` draws a seeded permutation per epoch; the last partial batch is kept unless
    `drop_last`."""

    def __init__(self, df, image_root, batch_size=32, shuffle=True, seed=0, drop_last=False,
                 device=None):
        self.keys, self.labels = construct_input_label_pairs_for_image_encoder_dataset(df)
        self.details = df["patient_details"].astype(str).tolist()
        self.image_root = image_root
        self.batch_size = int(batch_size)
        self.shuffle = shuffle
        self.rng = np.random.default_rng(seed)
        self.drop_last = drop_last
        self.device = device

    def __len__(self):
        n = len(self.keys)
        return n // self.batch_size if self.drop_last else -(-n // self.batch_size)

    def order(self):
        n = len(self.keys)
        return self.rng.permutation(n) if self.shuffle else np.arange(n)

    def __iter__(self):
        from .preprocess import preprocess_batch
        dev = self.device
        if dev is None:
            dev = torch.device("cuda", torch.cuda.current_device())
        order = self.order()
        for s in range(0, len(order), self.batch_size):
            idx = order[s:s + self.batch_size]
            if self.drop_last and len(idx) < self.batch_size:
                break
            imgs = [open_image(self.image_root, self.keys[i]) for i in idx]
            x = preprocess_batch(imgs, dev)
            y = torch.from_numpy(np.stack([self.labels[i] for i in idx])).to(dev)
            yield x, [self.details[i] for i in idx], y
