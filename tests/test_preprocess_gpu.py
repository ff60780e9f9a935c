"""GPU image preprocessing (mmdx_image_preprocess) == the reference transform, bit for bit:
PIL Image.resize(BILINEAR) to shorter side 256 + CenterCrop(224) + ToTensor + gray->RGB +
Normalize (TP:112-119; oracle.ref_cpu.reference_transform), one batch of mixed sizes and
modes (the committed reference sample image, synthetic RGB/gray, up/down-scales, no-op)."""
import numpy as np
import pytest
import torch

import mmdx
from oracle import ref_cpu as R
from test_preprocess_cpu import images

pytestmark = pytest.mark.gpu


def test_preprocess_batch_bitwise(dev):
    ims = images()
    got = mmdx.preprocess_batch(ims, dev).cpu()
    want = torch.stack([R.reference_transform(im) for im in ims])
    assert got.shape == (len(ims), 3, 224, 224)
    assert torch.equal(got.view(torch.int32), want.view(torch.int32))


def test_preprocess_feeds_inference_path(dev):
    # the GPU tensor is the trunk input the reference would build on the CPU
    ims = images()[:2]
    x = mmdx.preprocess_batch(ims, dev)
    assert x.is_cuda and x.dtype == torch.float32 and x.is_contiguous()
    ref = torch.stack([mmdx.image_transfom_into_tensor(im) for im in ims])
    assert np.array_equal(x.cpu().numpy(), ref.numpy())


def test_local_batches_feed_gpu_transform(dev, tmp_path):
    """mmdx.data.LocalCXRBatches: host decode + GPU transform per batch
    == the reference transform of each decoded image, labels and details in batch order."""
    import pandas as pd
    from mmdx import data as D
    ims = images()
    keys = []
    for i, im in enumerate(ims):
        k = f"img{i}.png"
        im.save(tmp_path / k)
        keys.append(k)
    vecs = [np.eye(13)[i % 13].tolist() for i in range(len(keys))]
    df = pd.DataFrame(dict(image_url=keys, patient_details=[f"p{i}" for i in range(len(keys))],
                           disease_classification_vector=vecs, report=["r"] * len(keys)))
    df = D.enforce_raw_data_columns(df)
    it = D.LocalCXRBatches(df, str(tmp_path), batch_size=3, shuffle=True, seed=1, device=dev)
    order = D.LocalCXRBatches(df, str(tmp_path), batch_size=3, shuffle=True, seed=1).order()
    seen = 0
    for x, details, y in it:
        idx = order[seen:seen + x.shape[0]]
        want = torch.stack([R.reference_transform(ims[i]) for i in idx])
        assert torch.equal(x.cpu().view(torch.int32), want.view(torch.int32))
        assert details == [f"p{i}" for i in idx]
        assert torch.equal(y.cpu(), torch.tensor([vecs[i] for i in idx], dtype=torch.float32))
        seen += x.shape[0]
    assert seen == len(ims)
