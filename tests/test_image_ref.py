"""The image-preprocessing oracle (oracle/image_ref.py) pinned against the libraries the reference
calls (`Stage1/train_projection_stage1.py:97-99`): Pillow's `Image.resize` (default BICUBIC) and
transformers' SiglipImageProcessor (rescale + normalise).  CPU only; bit-exact."""
import numpy as np
import pytest

from oracle import image_ref as R

PIL = pytest.importorskip("PIL.Image")

SIZES = [(384, 384), (40, 52), (300, 200), (767, 1013), (1500, 1200), (385, 383), (96, 1200)]


def _img(h, w, c, seed):
    rng = np.random.default_rng(seed)
    base = rng.integers(0, 256, (h, w, c), dtype=np.uint8)
    # smooth regions + hard edges so both the negative lobes and clipping are exercised
    yy, xx = np.mgrid[0:h, 0:w]
    ramp = ((xx * 3 + yy * 5) % 256).astype(np.uint8)[..., None]
    return np.where(rng.random((h, w, 1)) < 0.5, base, ramp).astype(np.uint8)


@pytest.mark.parametrize("h,w", SIZES)
@pytest.mark.parametrize("c", [1, 3])
def test_resize_matches_pillow(h, w, c):
    img = _img(h, w, c, seed=h * 7 + w + c)
    pil = PIL.fromarray(img[..., 0] if c == 1 else img, "L" if c == 1 else "RGB").convert("RGB")
    ref = np.asarray(pil.resize((96, 96)))
    got = R.pil_resize_bicubic(img, 96, 96)
    if c == 1:
        got = np.repeat(got, 3, axis=2)
    np.testing.assert_array_equal(got, ref)


def test_coeffs_identity_and_sum():
    k, b, c = R.precompute_coeffs(384, 384)
    assert k == 5
    for o in range(384):
        taps = c[o, : b[o, 1]]
        assert (taps == np.eye(1, len(taps), o - b[o, 0], dtype=np.int32) * (1 << 22)).all()
    for n in (100, 1000, 3000):
        k, b, c = R.precompute_coeffs(n, 384)
        s = c.sum(1)
        assert np.abs(s - (1 << 22)).max() <= k   # fixed-point rounding of normalised weights


def test_normalize_lut_matches_siglip_processor():
    tr = pytest.importorskip("transformers")
    proc = tr.SiglipImageProcessor(size={"height": 8, "width": 32}, do_resize=True)
    img = np.arange(256, dtype=np.uint8).reshape(8, 32)
    pil = PIL.fromarray(img, "L").convert("RGB")
    ref = proc(images=pil, return_tensors="np")["pixel_values"][0]   # [3, 8, 32] float32
    lut = R.siglip_normalize_lut(proc.rescale_factor, proc.image_mean[0], proc.image_std[0])
    got = lut[img][None].repeat(3, 0)
    np.testing.assert_array_equal(got, ref)
    bits = R.to_bf16_bits(lut)
    import torch
    assert (torch.from_numpy(lut).bfloat16().view(torch.int16).numpy().view(np.uint16) == bits).all()


@pytest.mark.parametrize("n,s", [(384, 384), (40, 384), (3000, 384), (1013, 96), (385, 384), (2, 7)])
def test_capi_resize_coeffs_match_oracle(n, s):
    """libptk's host-side coefficient builder (no GPU) == the Resample.c restatement."""
    from projectiontrainer_amd import _lib as L
    lib = L.lib()
    k = lib.ptk_resize_ksize(n, s)
    ko, bo, co = R.precompute_coeffs(n, s)
    assert k == ko
    b = np.empty((s, 2), np.int32)
    c = np.empty((s, k), np.int32)
    assert lib.ptk_resize_coeffs(n, s, b.ctypes.data, c.ctypes.data) == k
    np.testing.assert_array_equal(b, bo)
    np.testing.assert_array_equal(c, co)


def test_pack_layout_without_gpu():
    """ImagePreprocessor.pack: descriptor offsets, coefficient tables and pixel bytes (host only)."""
    from projectiontrainer_amd import _lib as L
    from projectiontrainer_amd.data import ImagePreprocessor
    pre = ImagePreprocessor.__new__(ImagePreprocessor)
    pre.S, pre._coef_cache = 32, {}
    ims = [_img(50, 70, 1, 1), _img(20, 33, 3, 2)]
    buf, meta = pre.pack([im.copy() for im in ims])
    n, d_bytes, c_bytes, max_h, max_rb, tmp_bytes, total = meta
    assert (n, max_h, max_rb) == (2, 50, 99)
    raw = buf.numpy()
    descs = (L.ImageDesc * 2).from_buffer_copy(raw[: L.C.sizeof(L.ImageDesc) * 2].tobytes())
    coefs = raw[d_bytes: d_bytes + c_bytes].view(np.int32)
    for d, im in zip(descs, ims):
        h, w, c = im.shape
        assert (d.h, d.w, d.c) == (h, w, c)
        got = raw[d_bytes + c_bytes + d.src_off: d_bytes + c_bytes + d.src_off + im.size]
        np.testing.assert_array_equal(got, im.reshape(-1))
        kh, bh, ch = R.precompute_coeffs(w, 32)
        kv, bv, cv = R.precompute_coeffs(h, 32)
        assert (d.kh, d.kv) == (kh, kv)
        o = d.coef_off
        np.testing.assert_array_equal(coefs[o: o + 64].reshape(32, 2), bh)
        np.testing.assert_array_equal(coefs[o + 64: o + 64 + 32 * kh].reshape(32, kh), ch)
        o += 64 + 32 * kh
        np.testing.assert_array_equal(coefs[o: o + 64].reshape(32, 2), bv)
        np.testing.assert_array_equal(coefs[o + 64: o + 64 + 32 * kv].reshape(32, kv), cv)
    assert tmp_bytes >= 50 * 32 * 1 + 20 * 32 * 3
