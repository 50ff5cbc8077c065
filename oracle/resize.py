"""ORACLE (test infrastructure only): PIL-exact bilinear resize 48x48 -> 224x224, u8.

Restates the input transform of the reference image path:
  Image.open(p).convert('RGB')                      inference/image_inference.py:112
  transforms.Resize((224, 224))  (PIL BILINEAR)      inference/image_inference.py:29
which calls Pillow's ImagingResample (src/libImaging/Resample.c): triangle filter,
support 1 (upscale), coefficients normalised then converted to 22-bit fixed point,
horizontal pass then vertical pass, each `clip8((sum(px*k) + 2^21) >> 22)` into a
uint8 intermediate. convert('RGB') replicates the gray channel, so the three channels
are identical and one plane is computed. Pinned bit-exact against PIL 12.2 by
tests/golden/image_resize.npz.
"""
import math

import numpy as np

PRECISION_BITS = 32 - 8 - 2


def coeffs(in_size: int, out_size: int):
    """Per output index: (xmin, n_taps, int32 taps[ksize]) exactly as Pillow's
    precompute_coeffs + normalize_coeffs_8bpc for the bilinear filter."""
    scale = in_size / out_size
    filterscale = max(scale, 1.0)
    support = 1.0 * filterscale
    ksize = int(math.ceil(support)) * 2 + 1
    xmins = np.zeros(out_size, np.int32)
    ns = np.zeros(out_size, np.int32)
    kk = np.zeros((out_size, ksize), np.int32)
    for xx in range(out_size):
        center = (xx + 0.5) * scale
        ss = 1.0 / filterscale
        xmin = int(center - support + 0.5)
        if xmin < 0:
            xmin = 0
        xmax = int(center + support + 0.5)
        if xmax > in_size:
            xmax = in_size
        xmax -= xmin
        ws = []
        for x in range(xmax):
            t = abs((x + xmin - center + 0.5) * ss)
            ws.append(1.0 - t if t < 1.0 else 0.0)
        ww = sum(ws)
        for x in range(xmax):
            w = ws[x] / ww if ww != 0.0 else ws[x]
            kk[xx, x] = int(-0.5 + w * (1 << PRECISION_BITS)) if w < 0 else int(0.5 + w * (1 << PRECISION_BITS))
        xmins[xx] = xmin
        ns[xx] = xmax
    return xmins, ns, kk


def _pass(src: np.ndarray, xmins, ns, kk, axis: int) -> np.ndarray:
    """One separable pass along `axis` (last axis = horizontal) of a [B,H,W] u8 array."""
    src = np.moveaxis(src, axis, -1).astype(np.int64)
    out_size = len(xmins)
    acc = np.full(src.shape[:-1] + (out_size,), 1 << (PRECISION_BITS - 1), np.int64)
    for xx in range(out_size):
        for x in range(int(ns[xx])):
            acc[..., xx] += src[..., xmins[xx] + x] * int(kk[xx, x])
    out = np.clip(acc >> PRECISION_BITS, 0, 255).astype(np.uint8)
    return np.moveaxis(out, -1, axis)


def resize_bilinear_u8(gray: np.ndarray, out_hw=(224, 224)) -> np.ndarray:
    """gray u8 [B,H,W] -> u8 [B,out_h,out_w], bit-exact with PIL BILINEAR."""
    gray = np.asarray(gray, np.uint8)
    B, H, W = gray.shape
    oh, ow = out_hw
    xc = coeffs(W, ow)
    yc = coeffs(H, oh)
    tmp = _pass(gray, *xc, axis=2)          # horizontal first (ImagingResampleInner)
    return _pass(tmp, *yc, axis=1)          # then vertical


def to_normalized_tensor(resized_u8: np.ndarray) -> np.ndarray:
    """ToTensor (/255) + Normalize(ImageNet) on the RGB-replicated image
    (inference/image_inference.py:30-31); returns float32 [B,3,224,224]."""
    mean = np.array([0.485, 0.456, 0.406], np.float32)
    std = np.array([0.229, 0.224, 0.225], np.float32)
    x = resized_u8.astype(np.float32) / np.float32(255.0)
    x = np.repeat(x[:, None], 3, axis=1)
    return ((x - mean[None, :, None, None]) / std[None, :, None, None]).astype(np.float32)
