"""CPU restatement of the reference's image preprocessing (the host data step).

TEST INFRASTRUCTURE ONLY.  Imported by `tests/` as the checker; the product path
(`projectiontrainer_amd.data`) never imports it.

The reference (`Stage1/train_projection_stage1.py:97-99`) does

    image = Image.open(path).convert('RGB')
    image = image.resize((img_size, img_size))          # Pillow default resample: BICUBIC
    pixel_values = processor(images=image).pixel_values  # SiglipImageProcessor: rescale 1/255,
                                                         # normalise mean = std = 0.5

and the trainer casts pixel_values to the vision tower's dtype (bf16) before the
tower (`Stage1/projector_trainer.py:158-171`).  The resampler is third-party
code absent from /root/reference: Pillow (12.2.0 in this image; the reference pins
no version), `src/libImaging/Resample.c`:
  * `precompute_coeffs`     — separable bicubic (a = -0.5, support 2) widened by the
                              downscale factor (antialiasing), weights normalised to 1;
  * `normalize_coeffs_8bpc` — weights to fixed point, PRECISION_BITS = 22, rounded
                              half away from zero;
  * `ImagingResampleHorizontal_8bpc` / `..._Vertical_8bpc` — horizontal pass first into
                              a uint8 image, then the vertical pass; each output
                              = clip8((2^21 + sum in * k) >> 22);
  * `ImagingResampleInner`  — a pass whose size does not change is skipped (the fixed-
                              point identity weights make that equal to running it).
The normalisation restates transformers' `image_transforms.rescale` (float64 multiply,
cast to float32) and `normalize` ((x - mean) / std in float32).

Pinned by `tests/test_image_ref.py` against Pillow and transformers' SiglipImageProcessor
themselves (both importable here): bit-exact on every tested size.
"""
from __future__ import annotations

import math

import numpy as np

PRECISION_BITS = 32 - 8 - 2
BICUBIC_SUPPORT = 2.0


def bicubic_filter(x: float) -> float:
    """Resample.c `bicubic_filter` (a = -0.5)."""
    a = -0.5
    if x < 0.0:
        x = -x
    if x < 1.0:
        return ((a + 2.0) * x - (a + 3.0)) * x * x + 1
    if x < 2.0:
        return (((x - 5) * x + 8) * x - 4) * a
    return 0.0


def precompute_coeffs(in_size: int, out_size: int):
    """Resample.c `precompute_coeffs` over the full box [0, in_size) + `normalize_coeffs_8bpc`.
    Returns (ksize, bounds int32 [out, 2] = (first tap, tap count), coeffs int32 [out, ksize])."""
    scale = float(in_size) / out_size
    filterscale = max(scale, 1.0)
    support = BICUBIC_SUPPORT * filterscale
    ksize = int(math.ceil(support)) * 2 + 1
    bounds = np.zeros((out_size, 2), np.int32)
    kk = np.zeros((out_size, ksize), np.float64)
    ss = 1.0 / filterscale
    for xx in range(out_size):
        center = (xx + 0.5) * scale
        xmin = max(int(center - support + 0.5), 0)          # C (int) truncates toward zero
        xmax = min(int(center + support + 0.5), in_size) - xmin
        w = [bicubic_filter((x + xmin - center + 0.5) * ss) for x in range(xmax)]
        ww = 0.0
        for v in w:
            ww += v
        for x in range(xmax):
            kk[xx, x] = w[x] / ww if ww != 0.0 else w[x]
        bounds[xx] = (xmin, xmax)
    one = float(1 << PRECISION_BITS)
    fixed = np.where(kk < 0, np.trunc(-0.5 + kk * one), np.trunc(0.5 + kk * one)).astype(np.int32)
    return ksize, bounds, fixed


def _clip8(acc: np.ndarray) -> np.ndarray:
    return np.clip(acc >> PRECISION_BITS, 0, 255).astype(np.uint8)


def resample_axis(img: np.ndarray, axis: int, out_size: int) -> np.ndarray:
    """One 8bpc pass along `axis` (1 = horizontal, 0 = vertical) of an [H, W, C] uint8 image."""
    _, bounds, k = precompute_coeffs(img.shape[axis], out_size)
    src = np.moveaxis(img, axis, 0).astype(np.int64)
    out = np.empty((out_size,) + src.shape[1:], np.uint8)
    for o in range(out_size):
        lo, n = int(bounds[o, 0]), int(bounds[o, 1])
        acc = np.full(src.shape[1:], 1 << (PRECISION_BITS - 1), np.int64)
        for t in range(n):
            acc += src[lo + t] * int(k[o, t])
        out[o] = _clip8(acc)
    return np.moveaxis(out, 0, axis)


def pil_resize_bicubic(img: np.ndarray, out_h: int, out_w: int) -> np.ndarray:
    """`Image.resize((out_w, out_h))` of an [H, W, C] uint8 image (ImagingResampleInner order:
    horizontal pass, then vertical; unchanged axes skipped)."""
    if img.ndim == 2:
        img = img[:, :, None]
    if img.shape[1] != out_w:
        img = resample_axis(img, 1, out_w)
    if img.shape[0] != out_h:
        img = resample_axis(img, 0, out_h)
    return img


def siglip_normalize_lut(rescale_factor: float = 1 / 255, mean: float = 0.5, std: float = 0.5) -> np.ndarray:
    """float32 pixel value for every uint8 input: transformers `rescale` (float64 multiply, cast to
    float32) then `normalize` ((x - mean) / std with float32 mean/std)."""
    x = (np.arange(256, dtype=np.float64) * rescale_factor).astype(np.float32)
    return (x - np.float32(mean)) / np.float32(std)


def to_bf16_bits(x: np.ndarray) -> np.ndarray:
    """float32 -> bf16 bit patterns, round to nearest even (torch's `.to(torch.bfloat16)`)."""
    u = np.ascontiguousarray(x, np.float32).view(np.uint32).astype(np.uint64)
    r = (u + 0x7FFF + ((u >> 16) & 1)) >> 16
    return r.astype(np.uint16)


def preprocess(img: np.ndarray, size: int, lut: np.ndarray | None = None) -> np.ndarray:
    """The reference's per-image pixel path: [H, W, C] uint8 (C = 1 for a greyscale JPEG, whose
    `.convert('RGB')` replicates the channel) -> float32 [3, size, size]."""
    lut = siglip_normalize_lut() if lut is None else lut
    r = pil_resize_bicubic(img, size, size)
    if r.shape[2] == 1:
        r = np.repeat(r, 3, axis=2)
    return lut[r].transpose(2, 0, 1).copy()
