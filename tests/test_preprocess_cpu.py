"""CPU: the GPU preprocessing plan (mmdx.preprocess: PIL resample geometry and 22-bit
coefficients for the 224 crop window) reproduces the reference transform bit for bit.

The kernel's integer arithmetic is emulated here in numpy on the very tables the host
uploads; the oracle is the reference's own path (oracle.ref_cpu.reference_transform: PIL
Image.resize(BILINEAR) + torchvision-rule crop/normalise, TP:112-119).  The committed sample
image (tests/golden/e1.jpg, from the reference's backend/sample_images) and synthetic sizes
(down/up-scales, odd aspect ratios, gray, no-op resize) are covered."""
import os

import numpy as np
import pytest
import torch
from PIL import Image

from mmdx import preprocess as PP
from oracle import ref_cpu as R

HERE = os.path.dirname(os.path.abspath(__file__))


def _emulate(arrays):
    """numpy restatement of mmdx_image_preprocess over plan_batch's tables."""
    descs, coef, temp_bytes, max_trows, _ = PP.plan_batch(arrays)
    coef = coef.astype(np.int64)
    mean = np.array([0.485, 0.456, 0.406], np.float32)
    std = np.array([0.229, 0.224, 0.225], np.float32)
    outs = []
    for a, d in zip(arrays, descs):
        h, w, c = a.shape
        trows, crop = int(d["trows"]), PP.CROP
        temp = np.zeros((trows, crop, c), np.int64)
        for r in range(trows):
            y = int(d["trow0"]) + r
            for j in range(crop):
                if not d["need_h"]:
                    temp[r, j] = a[y, int(d["left"]) + j]
                    continue
                k = coef[int(d["kh_off"]) + j * (int(d["ksize_h"]) + 2):][: int(d["ksize_h"]) + 2]
                xmin, n = int(k[0]), int(k[1])
                ss = (1 << 21) + (a[y, xmin:xmin + n].astype(np.int64) * k[2:2 + n, None]).sum(0)
                temp[r, j] = np.clip(ss >> 22, 0, 255)
        img = np.zeros((crop, crop, c), np.int64)
        for i in range(crop):
            if not d["need_v"]:
                img[i] = temp[int(d["top"]) + i - int(d["trow0"])]
                continue
            k = coef[int(d["kv_off"]) + i * (int(d["ksize_v"]) + 2):][: int(d["ksize_v"]) + 2]
            ymin, n = int(k[0]), int(k[1])
            ss = (1 << 21) + (temp[ymin:ymin + n] * k[2:2 + n, None, None]).sum(0)
            img[i] = np.clip(ss >> 22, 0, 255)
        f = img.astype(np.float32) / np.float32(255.0)
        if c == 1:
            f = np.repeat(f, 3, axis=2)
        outs.append(((f - mean) / std).transpose(2, 0, 1))
    return np.stack(outs)


def images():
    # the reference's two sample images (backend/sample_images/e1.jpg, e2.jpg)
    ims = [Image.open(os.path.join(HERE, "golden", f)).convert("RGB")
           for f in ("e1.jpg", "e2.jpg")]
    g = np.random.default_rng(0)
    for (w, h, mode) in ((512, 384, "RGB"), (300, 700, "L"), (256, 333, "RGB"),
                         (240, 231, "RGB"), (1023, 517, "L"), (256, 256, "RGB")):
        c = 3 if mode == "RGB" else 1
        px = g.integers(0, 256, size=(h, w, c), dtype=np.uint8)
        ims.append(Image.fromarray(px[:, :, 0] if c == 1 else px, mode))
    return ims


def test_plan_matches_reference_transform_bitwise():
    ims = images()
    arrays = [PP._as_array(im) for im in ims]
    got = _emulate(arrays)
    want = torch.stack([R.reference_transform(im) for im in ims]).numpy()
    assert got.shape == want.shape == (len(ims), 3, 224, 224)
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32))


def test_pil_coeffs_reproduce_pil_resize_rows():
    # one resized row of a random RGB image through the coefficient table == PIL's resize
    g = np.random.default_rng(1)
    a = g.integers(0, 256, size=(3, 517, 3), dtype=np.uint8)
    out_w = 260
    bounds, kk, _ = PP.pil_coeffs(517, out_w)
    want = np.asarray(Image.fromarray(a).resize((out_w, 3), Image.BILINEAR))
    for x in range(out_w):
        xmin, n = bounds[x]
        ss = (1 << 21) + (a[:, xmin:xmin + n].astype(np.int64) * kk[x, :n, None]).sum(1)
        assert np.array_equal(np.clip(ss >> 22, 0, 255), want[:, x])


def test_rejects_unsupported_modes():
    with pytest.raises(ValueError):
        PP._as_array(Image.new("RGBA", (300, 300)))
