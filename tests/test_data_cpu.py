"""Local dataset loader (mmdx.data) vs the reference's data contract:
feature_pipeline.enforce_raw_data_columns (feature_pipeline.py:41-58), the feature-store
dedupe by event_time (TP:86-88), construct_input_label_pairs_for_image_encoder_dataset
(TP:122-127) and CXR_ImageDataset.__getitem__ (TP:142-152) with the reference transform."""
import json
import os

import numpy as np
import pandas as pd
import pytest
import torch

from mmdx import data as D
from oracle import ref_cpu as R

HERE = os.path.dirname(os.path.abspath(__file__))
E1 = os.path.join(HERE, "golden", "e1.jpg")


def _vec(i):
    v = np.zeros(13)
    v[i % 13] = 1.0
    return v


def _frame(tmp_path):
    rows = [
        # duplicate image_url: the later event_time wins (TP:86-88)
        dict(image_url="s3://bucket/cxr/a.jpg", patient_details="67M, smoker", report="r0",
             disease_classification_vector=json.dumps(_vec(0).tolist()),
             event_time=pd.Timestamp("2024-01-01")),
        dict(image_url="s3://bucket/cxr/a.jpg", patient_details="67M, smoker; CHF",
             report="r1", disease_classification_vector=json.dumps(_vec(1).tolist()),
             event_time=pd.Timestamp("2024-02-01")),
        dict(image_url="cxr/b.jpg", patient_details=54, report=None,
             disease_classification_vector=json.dumps(_vec(2).tolist()),
             event_time=pd.Timestamp("2024-01-15")),
    ]
    path = str(tmp_path / "dataset.parquet")
    df = pd.DataFrame(rows)
    df["patient_details"] = df["patient_details"].astype(str)
    df.to_parquet(path, engine="pyarrow")
    return path


def test_load_enforces_types_and_dedupes(tmp_path):
    df = D.load_features_labels_local(_frame(tmp_path))
    assert len(df) == 2
    a = df[df.image_url == "s3://bucket/cxr/a.jpg"].iloc[0]
    assert a.patient_details == "67M, smoker; CHF" and a.report == "r1"
    np.testing.assert_array_equal(a.disease_classification_vector, _vec(1))
    b = df[df.image_url == "cxr/b.jpg"].iloc[0]
    assert b.patient_details == "54" and b.report == "None"  # astype(str) as the reference


def test_bad_vector_length_and_missing_columns(tmp_path):
    p = str(tmp_path / "bad.parquet")
    pd.DataFrame([dict(image_url="x.jpg", patient_details="p", report="r",
                       disease_classification_vector="[1, 0]")]).to_parquet(p)
    with pytest.raises(ValueError, match="length"):
        D.load_features_labels_local(p)
    q = str(tmp_path / "nocol.parquet")
    pd.DataFrame([dict(image_url="x.jpg", report="r")]).to_parquet(q)
    with pytest.raises(ValueError, match="missing columns"):
        D.load_features_labels_local(q)


def test_pairs_and_dataset_item(tmp_path):
    os.makedirs(tmp_path / "cxr")
    for name in ("a.jpg", "b.jpg"):
        with open(E1, "rb") as src, open(tmp_path / "cxr" / name, "wb") as dst:
            dst.write(src.read())
    df = D.load_features_labels_local(_frame(tmp_path))
    keys, labels = D.construct_input_label_pairs_for_image_encoder_dataset(df)
    assert sorted(keys) == ["cxr/a.jpg", "cxr/b.jpg"]  # s3 key kept, local path as is
    assert all(l.dtype == np.float32 and l.shape == (13,) for l in labels)
    ds = D.CXR_ImageDataset(keys, str(tmp_path), labels, image_transform=R.reference_transform)
    assert len(ds) == 2
    x, y = ds[0]
    assert x.shape == (3, 224, 224) and x.dtype == torch.float32
    assert y.dtype == torch.float32 and torch.equal(y, torch.from_numpy(labels[0]))
    batches = D.LocalCXRBatches(df, str(tmp_path), batch_size=1, shuffle=True, seed=3)
    assert len(batches) == 2 and sorted(batches.order().tolist()) == [0, 1]
