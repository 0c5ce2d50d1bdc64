"""GPU pixel path of the host data step (`ptk_image_preprocess`) vs the reference's own libraries
and the oracle: bit-exact bf16 / f32 pixel_values.

The reference's per-image path (`Stage1/train_projection_stage1.py:97-99` +
`Stage1/projector_trainer.py:158-171`): Pillow `.convert('RGB').resize((S, S))`,
SiglipImageProcessor (rescale 1/255, normalise 0.5/0.5), cast to the tower dtype.
"""
import json
import os

import numpy as np
import pytest
import torch

from oracle import image_ref as R

pytestmark = pytest.mark.gpu
PIL = pytest.importorskip("PIL.Image")


def _img(h, w, c, seed):
    rng = np.random.default_rng(seed)
    yy, xx = np.mgrid[0:h, 0:w]
    smooth = ((np.sin(xx / 17.0) + np.cos(yy / 23.0)) * 60 + 128).astype(np.uint8)[..., None]
    noise = rng.integers(0, 256, (h, w, c), dtype=np.uint8)
    return np.where(rng.random((h, w, 1)) < 0.3, noise, smooth).astype(np.uint8)


def _pil_ref(img, S):
    pil = PIL.fromarray(img[..., 0] if img.shape[2] == 1 else img, "L" if img.shape[2] == 1 else "RGB")
    return np.asarray(pil.convert("RGB").resize((S, S)))          # [S, S, 3] uint8


# (h, w, c): downscale by up to ~8x, upscale, identity, non-square, 1 and 3 channels
SHAPES = [(3000, 2500, 1), (384, 384, 3), (384, 384, 1), (200, 150, 3), (1024, 768, 3), (2048, 2048, 1),
          (500, 4000, 1), (383, 385, 3)]


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_preprocess_bit_exact_vs_pillow(gpu, dtype):
    from projectiontrainer_amd.data import ImagePreprocessor
    S = 384
    imgs = [_img(h, w, c, i) for i, (h, w, c) in enumerate(SHAPES)]
    pre = ImagePreprocessor(S, gpu, dtype=dtype)
    out = pre([im.copy() for im in imgs])
    torch.cuda.synchronize()
    lut = R.siglip_normalize_lut()
    for i, im in enumerate(imgs):
        ref_u8 = _pil_ref(im, S)
        ref = torch.from_numpy(lut[ref_u8].transpose(2, 0, 1).copy()).to(dtype)
        got = out[i].cpu()
        if not torch.equal(got, ref):
            bad = (got != ref).nonzero()
            raise AssertionError(f"image {i} {im.shape}: {len(bad)} mismatches, first {bad[:4].tolist()}")


def test_preprocess_matches_oracle_small_target(gpu):
    """A non-384 target through the oracle's own resampler (independent of Pillow)."""
    from projectiontrainer_amd.data import ImagePreprocessor
    imgs = [_img(97, 131, 1, 5), _img(40, 29, 3, 6), _img(64, 64, 3, 7)]
    pre = ImagePreprocessor(56, gpu, dtype=torch.float32)
    out = pre([im.copy() for im in imgs]).cpu().numpy()
    for i, im in enumerate(imgs):
        np.testing.assert_array_equal(out[i], R.preprocess(im, 56))


def test_processor_constants_and_empty_batch(gpu):
    tr = pytest.importorskip("transformers")
    from projectiontrainer_amd.data import ImagePreprocessor
    proc = tr.SiglipImageProcessor(size={"height": 64, "width": 64})
    pre = ImagePreprocessor(64, gpu, processor=proc, dtype=torch.float32)
    im = _img(100, 80, 3, 9)
    pil = PIL.fromarray(im, "RGB").resize((64, 64))                  # the reference resizes before the processor
    ref = proc(images=pil, return_tensors="np")["pixel_values"][0]
    got = pre([im.copy()])[0].cpu().numpy()
    np.testing.assert_array_equal(got, ref)
    assert pre([]).shape == (0, 3, 64, 64)


class _Tok:
    """Minimal left-padding tokenizer with the HF call surface the dataset uses."""
    pad_token_id, bos_token_id = 0, 2

    def __call__(self, text, max_length, padding, truncation, return_tensors):
        ids = [self.bos_token_id] + [3 + (ord(ch) % 250) for ch in text][: max_length - 1]
        ids = [self.pad_token_id] * (max_length - len(ids)) + ids

        class _O:
            pass
        o = _O()
        o.input_ids = torch.tensor([ids])
        return o


def test_dataset_loader_prefetcher_end_to_end(gpu, tmp_path):
    """JPEG files + JSON -> XrayTextPairDataset (2 worker processes) -> DevicePrefetcher ->
    pixel_values identical to Pillow decode/resize + SiglipImageProcessor + bf16 cast."""
    tr = pytest.importorskip("transformers")
    from projectiontrainer_amd.data import (DevicePrefetcher, ImagePreprocessor, ThreadedImageLoader,
                                           XrayTextPairDataset, collate)
    root, root2 = tmp_path / "a", tmp_path / "b"
    root.mkdir()
    (root2 / "study7").mkdir(parents=True)
    samples = []
    for i in range(7):
        h, w = 300 + 37 * i, 260 + 53 * i
        im = _img(h, w, 1 if i % 2 == 0 else 3, 100 + i)
        pil = PIL.fromarray(im[..., 0], "L") if im.shape[2] == 1 else PIL.fromarray(im, "RGB")
        if i == 6:   # MIMIC-style directory under the second root
            pil.save(root2 / "study7" / "view.jpg", quality=90)
            samples.append({"image": "study7", "normal_caption": "no acute findings " * 3})
        else:
            pil.save(root / f"img{i}.jpg", quality=90)
            samples.append({"image": f"img{i}.jpg", "normal_caption": f"caption {i} lungs clear"})
    js = tmp_path / "s.json"
    js.write_text(json.dumps(samples))
    proc = tr.SiglipImageProcessor(size={"height": 384, "width": 384})
    ds = XrayTextPairDataset(str(root), str(js), proc, _Tok(), 384, max_length=32, image_root_2=str(root2))
    loader = torch.utils.data.DataLoader(ds, batch_size=3, shuffle=False, num_workers=2, collate_fn=collate)
    pre = ImagePreprocessor(384, gpu, processor=proc)
    got = []
    for b in DevicePrefetcher(loader, pre):
        got.append((b["pixel_values"].cpu(), b["token_ids"].cpu(), b["labels"].cpu()))
    pix = torch.cat([g[0] for g in got])
    ids = torch.cat([g[1] for g in got])
    # the threaded decode-into-pinned loader (the trainer's path) yields the same batches
    thr = [(b["pixel_values"].cpu(), b["token_ids"].cpu()) for b in
           ThreadedImageLoader(ds, [[0, 1, 2], [3, 4, 5], [6]], pre, threads=3)]
    assert torch.equal(torch.cat([t[0] for t in thr]), pix) and torch.equal(torch.cat([t[1] for t in thr]), ids)
    assert pix.shape == (7, 3, 384, 384) and pix.dtype == torch.bfloat16
    for i, s in enumerate(samples):
        path = ds.resolve_path(s["image"])
        image = PIL.open(path).convert("RGB").resize((384, 384))     # the reference's __getitem__
        ref = torch.from_numpy(proc(images=image, return_tensors="np")["pixel_values"][0]).bfloat16()
        assert torch.equal(pix[i], ref), (i, (pix[i] != ref).sum())
        tok = _Tok()(s["normal_caption"], 32, "max_length", True, "pt").input_ids[0]
        assert torch.equal(ids[i], tok)
    lab = torch.cat([g[2] for g in got])
    assert torch.equal(lab, torch.where(ids == 0, torch.full_like(ids, -100), ids))
