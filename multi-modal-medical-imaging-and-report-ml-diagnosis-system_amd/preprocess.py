"""Batched GPU image preprocessing: the reference's per-image CPU
transform `image_transfom_into_tensor` (training_pipeline.py:112-119) —

    T.Resize(256, antialias=True)  on a PIL image  = PIL Image.resize(BILINEAR)
    T.CenterCrop(224)              top/left = int(round((size - 224) / 2))
    T.ToTensor()                   uint8 / 255, HWC -> CHW
    gray -> RGB                    x.repeat(3, 1, 1) when one channel
    T.Normalize(ImageNet mean/std)

— for a whole batch in two HIP launches (`mmdx_image_preprocess`), bit-exact with the CPU
transform.  JPEG decoding stays on the host with PIL, as in the reference
(CXR_ImageDataset.__getitem__, TP:146).  This module computes PIL's resampling geometry and
fixed-point coefficients on the host (PIL's own double-precision formulas, libImaging
Resample.c: precompute_coeffs + normalize_coeffs_8bpc) for the 224x224 crop window only, and
packs the decoded pixels; the GPU does the arithmetic.
"""
from __future__ import annotations

import math

import numpy as np
import torch

from . import _lib as L
from ._lib import call, ptr, stream

RESIZE, CROP = 256, 224
PRECISION_BITS = 22  # PIL: 32 - 8 - 2

# mirrors mmdx_img_desc (include/mmdx.h)
_DESC = np.dtype([("src_off", "<i8"), ("kh_off", "<i8"), ("kv_off", "<i8"), ("temp_off", "<i8"),
                  ("w", "<i4"), ("h", "<i4"), ("c", "<i4"), ("left", "<i4"), ("top", "<i4"),
                  ("need_h", "<i4"), ("need_v", "<i4"), ("ksize_h", "<i4"), ("ksize_v", "<i4"),
                  ("trow0", "<i4"), ("trows", "<i4")], align=True)


def resized_size(w: int, h: int, size: int = RESIZE):
    """torchvision _compute_resized_output_size for an int size (shorter side -> size)."""
    short, long = (w, h) if w <= h else (h, w)
    new_short, new_long = size, int(size * long / short)
    return (new_short, new_long) if w <= h else (new_long, new_short)


def _bilinear(x: float) -> float:
    if x < 0.0:
        x = -x
    return 1.0 - x if x < 1.0 else 0.0


def pil_coeffs(in_size: int, out_size: int):
    """PIL precompute_coeffs (box = whole axis) + normalize_coeffs_8bpc: per output index
    (xmin, count) and `ksize` int32 weights with 22 fractional bits."""
    scale = in_size / out_size
    filterscale = max(scale, 1.0)
    support = 1.0 * filterscale  # bilinear support 1.0
    ksize = int(math.ceil(support)) * 2 + 1
    bounds = np.zeros((out_size, 2), dtype=np.int64)
    kk = np.zeros((out_size, ksize), dtype=np.int64)
    ss = 1.0 / filterscale
    for xx in range(out_size):
        center = 0.0 + (xx + 0.5) * scale
        xmin = int(center - support + 0.5)
        if xmin < 0:
            xmin = 0
        xmax = int(center + support + 0.5)
        if xmax > in_size:
            xmax = in_size
        xmax -= xmin
        ws = []
        ww = 0.0
        for x in range(xmax):
            wgt = _bilinear((x + xmin - center + 0.5) * ss)
            ws.append(wgt)
            ww += wgt
        for x in range(xmax):
            v = ws[x] / ww if ww != 0.0 else ws[x]
            kk[xx, x] = int(-0.5 + v * (1 << PRECISION_BITS)) if v < 0 else \
                int(0.5 + v * (1 << PRECISION_BITS))
        bounds[xx] = (xmin, xmax)
    return bounds, kk, ksize


_COEF_CACHE: dict = {}


def _coeffs_cached(in_size, out_size):
    key = (in_size, out_size)
    c = _COEF_CACHE.get(key)
    if c is None:
        if len(_COEF_CACHE) > 256:
            _COEF_CACHE.clear()
        c = _COEF_CACHE[key] = pil_coeffs(in_size, out_size)
    return c


def _as_array(img):
    """PIL image (mode L or RGB) or HWC/HW uint8 array -> (H, W, C) uint8 contiguous."""
    if hasattr(img, "mode"):
        if img.mode not in ("L", "RGB"):
            raise ValueError(f"image mode {img.mode!r}: the transform expects L or RGB "
                             "(ToTensor + 3-channel Normalize)")
        a = np.asarray(img)
    else:
        a = np.asarray(img)
    if a.dtype != np.uint8:
        raise TypeError("decoded images must be uint8")
    if a.ndim == 2:
        a = a[:, :, None]
    if a.ndim != 3 or a.shape[2] not in (1, 3):
        raise ValueError(f"expected HxW or HxWx{{1,3}} pixels, got {a.shape}")
    return np.ascontiguousarray(a)


def plan_batch(arrays):
    """Descriptors + coefficient table + temp size for a list of HWC uint8 arrays."""
    descs = np.zeros(len(arrays), dtype=_DESC)
    coef_parts, coef_len = [], 0
    src_off = temp_off = 0
    max_trows = 1
    for b, a in enumerate(arrays):
        h, w, c = a.shape
        rw, rh = resized_size(w, h)
        if (rw, rh) == (w, h):      # torchvision returns the image unchanged
            need_h = need_v = False
        else:                        # PIL ImagingResampleInner pass selection
            need_h, need_v = rw != w, rh != h
        if rw < CROP or rh < CROP:
            raise ValueError("resized image smaller than the 224 crop")
        top = int(round((rh - CROP) / 2.0))
        left = int(round((rw - CROP) / 2.0))
        d = descs[b]
        d["src_off"], d["w"], d["h"], d["c"] = src_off, w, h, c
        d["left"], d["top"], d["need_h"], d["need_v"] = left, top, int(need_h), int(need_v)
        if need_h:
            bh, kh, ksh = _coeffs_cached(w, rw)
            rows = np.concatenate([bh[left:left + CROP], kh[left:left + CROP]], axis=1)
            d["kh_off"], d["ksize_h"] = coef_len, ksh
            coef_parts.append(rows.reshape(-1))
            coef_len += rows.size
        if need_v:
            bv, kv, ksv = _coeffs_cached(h, rh)
            bsel = bv[top:top + CROP].copy()
            trow0 = int(bsel[:, 0].min())
            trows = int((bsel[:, 0] + bsel[:, 1]).max()) - trow0
            bsel[:, 0] -= trow0
            rows = np.concatenate([bsel, kv[top:top + CROP]], axis=1)
            d["kv_off"], d["ksize_v"] = coef_len, ksv
            coef_parts.append(rows.reshape(-1))
            coef_len += rows.size
        else:
            trow0, trows = top, CROP
        d["trow0"], d["trows"], d["temp_off"] = trow0, trows, temp_off
        max_trows = max(max_trows, trows)
        src_off += a.nbytes
        temp_off += trows * CROP * c
    coef = (np.concatenate(coef_parts) if coef_parts else np.zeros(1, np.int64))
    if np.abs(coef).max() >= (1 << 31):
        raise ValueError("coefficient table overflow")
    return descs, coef.astype(np.int32), max(temp_off, 1), max_trows, src_off


def preprocess_batch(images, device=None) -> torch.Tensor:
    """PIL images (L/RGB, any sizes) -> [B, 3, 224, 224] fp32 on the GPU, identical to
    torch.stack([image_transfom_into_tensor(im) for im in images])."""
    if device is None:
        device = torch.device("cuda", torch.cuda.current_device())
    device = torch.device(device)
    if device.type != "cuda":
        raise RuntimeError("mmdx preprocessing runs on the GPU (HIP); there is no CPU path "
                           "here — use training_pipeline.image_transfom_into_tensor on CPU")
    arrays = [_as_array(im) for im in images]
    if not arrays:
        raise ValueError("empty batch")
    descs, coef, temp_bytes, max_trows, total = plan_batch(arrays)
    host = torch.empty(total, dtype=torch.uint8, pin_memory=True)
    hv = host.numpy()
    off = 0
    for a in arrays:
        hv[off:off + a.nbytes] = a.reshape(-1)
        off += a.nbytes
    px = host.to(device, non_blocking=True)
    d_desc = torch.from_numpy(descs.view(np.uint8).copy()).to(device, non_blocking=True)
    d_coef = torch.from_numpy(coef).to(device, non_blocking=True)
    temp = torch.empty(temp_bytes, dtype=torch.uint8, device=device)
    out = torch.empty((len(arrays), 3, CROP, CROP), dtype=torch.float32, device=device)
    with torch.cuda.device(device):
        call("mmdx_image_preprocess", ptr(px), ptr(d_desc), len(arrays), ptr(d_coef), max_trows,
             CROP, CROP, ptr(temp), ptr(out), stream())
        # the pinned staging buffer must outlive the asynchronous copy
        torch.cuda.current_stream().synchronize()
    return out


assert _DESC.itemsize == 80
