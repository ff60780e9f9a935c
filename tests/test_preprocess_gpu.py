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
