"""Host data step of Stage 1: dataset, batch packing and the GPU pixel path.

`XrayTextPairDataset` keeps the reference's constructor and path resolution
(`Stage1/train_projection_stage1.py:25-118`) but stops after the JPEG decode: an
item carries the decoded uint8 image (one channel for a greyscale X-ray) instead of
float32 pixel_values.  `ImagePreprocessor` then does, for a whole batch in one
host->device copy and two HIP kernels (`ptk_image_preprocess`):

    .convert('RGB').resize((S, S))   Pillow's antialiased bicubic, bit-exact (integer passes)
    processor(images=...)            rescale 1/255 + normalise (SiglipImageProcessor semantics)
    .to(vision dtype)                bf16 (or float32) planar [B, 3, S, S]

`DevicePrefetcher` overlaps that with the training step: worker processes decode, the
main process packs each batch into one pinned buffer, the copy and the kernels run on a
side stream, and the step's stream waits on an event only when it takes the batch.

Tokenisation is the reference's own call (`tokenizer(caption, max_length=..., padding=
"max_length", truncation=True)`), on the host.
"""
from __future__ import annotations

import json
import logging
import os

import numpy as np
import torch

from . import _lib as L

logger = logging.getLogger(__name__)

_ALIGN = 64


def _align(n: int) -> int:
    return (n + _ALIGN - 1) // _ALIGN * _ALIGN


def decode_image(path: str) -> np.ndarray:
    """JPEG/PNG decode on the host (Pillow, as the reference).  Greyscale stays one channel
    (`.convert('RGB')` of an "L" image replicates it, which the GPU pass does for free);
    every other mode goes through `.convert('RGB')` here."""
    from PIL import Image
    with Image.open(path) as im:
        if im.mode == "L":
            return np.array(im)[:, :, None]
        return np.array(im.convert("RGB"))


class XrayTextPairDataset(torch.utils.data.Dataset):
    """`Stage1/train_projection_stage1.py:25-118` with the pixel work moved to the GPU.
    Items: {"image": uint8 [H, W, C], "token_ids": int64 [max_length], "labels": int64 [max_length]}."""

    yields_images = True   # ProjectionTrainerStage1 routes such datasets through the GPU pixel path

    def __init__(self, image_root, json_file, processor, tokenizer, img_size, max_length=512, image_root_2=None):
        self.image_root, self.image_root_2 = image_root, image_root_2
        self.img_size, self.processor, self.tokenizer, self.max_length = img_size, processor, tokenizer, max_length
        self.samples = []
        if json_file:
            with open(json_file, "r", encoding="utf-8") as f:
                self.samples = json.load(f)

    def __len__(self):
        return len(self.samples)

    def resolve_path(self, name: str) -> str:
        """Primary root, else a MIMIC directory under the second root (first .jpg in it), else a
        file under the second root (`:62-95`)."""
        path = os.path.join(self.image_root, name)
        if os.path.exists(path) and not os.path.isdir(path):
            return path
        if not self.image_root_2:
            raise FileNotFoundError(f"Image not found in primary root and no secondary root provided: {path}")
        alt = os.path.join(self.image_root_2, name)
        if os.path.isdir(alt):
            jpgs = [f for f in os.listdir(alt) if f.lower().endswith(".jpg")]
            if not jpgs:
                raise FileNotFoundError(f"No .jpg file found in MIMIC directory: {alt}")
            alt = os.path.join(alt, jpgs[0])
        if not os.path.exists(alt) or os.path.isdir(alt):
            raise FileNotFoundError(f"Image path is invalid or a directory: {alt}")
        return alt

    def tokenize(self, caption: str):
        t = self.tokenizer(caption, max_length=self.max_length, padding="max_length", truncation=True,
                           return_tensors="pt")
        ids = t.input_ids.squeeze(0) if hasattr(t, "input_ids") else torch.as_tensor(t["input_ids"]).squeeze(0)
        labels = ids.clone()
        if self.tokenizer.pad_token_id is not None:
            labels[labels == self.tokenizer.pad_token_id] = -100
        return ids, labels

    def __getitem__(self, idx):
        s = self.samples[idx]
        path = self.resolve_path(s["image"])
        ids, labels = self.tokenize(s["normal_caption"])
        return {"image": decode_image(path), "token_ids": ids, "labels": labels}

    def open_item(self, idx):
        """(lazy Pillow image: header parsed, pixels not decoded yet, token_ids, labels)."""
        from PIL import Image
        s = self.samples[idx]
        ids, labels = self.tokenize(s["normal_caption"])
        return Image.open(self.resolve_path(s["image"])), ids, labels


def worker_init(_worker_id=None):
    """DataLoader worker setup: one intra-op thread per decode worker (the workers are the parallelism;
    the default thread count per worker oversubscribes the host cores)."""
    torch.set_num_threads(1)


def collate(items):
    """Batch of dataset items: images stay a list (ragged sizes) of uint8 tensors — tensors, not numpy
    arrays, so a DataLoader worker hands them over through shared memory instead of a pickle pipe —
    ids/labels are stacked."""
    out = {"images": [torch.from_numpy(np.ascontiguousarray(it["image"])) for it in items]}
    for k in ("token_ids", "labels"):
        out[k] = torch.stack([torch.as_tensor(it[k]) for it in items])
    return out


def normalize_lut(rescale_factor=1 / 255, mean=(0.5, 0.5, 0.5), std=(0.5, 0.5, 0.5), dtype=torch.bfloat16):
    """[3, 256] table: transformers `rescale` (float64 multiply -> float32) and `normalize`
    ((x - mean) / std in float32), then the cast to the tower dtype."""
    x = (np.arange(256, dtype=np.float64) * rescale_factor).astype(np.float32)
    rows = [(x - np.float32(m)) / np.float32(s) for m, s in zip(mean, std)]
    return torch.from_numpy(np.stack(rows)).to(dtype)


class ImagePreprocessor:
    """Batched resize + normalise of decoded uint8 images into pixel_values on the GPU."""

    def __init__(self, img_size: int, device, processor=None, dtype=torch.bfloat16):
        if dtype not in (torch.bfloat16, torch.float32):
            raise ValueError("pixel dtype must be bf16 or f32")
        self.S, self.device, self.dtype = int(img_size), torch.device(device), dtype
        mean, std, rf = (0.5, 0.5, 0.5), (0.5, 0.5, 0.5), 1 / 255
        if processor is not None:   # SiglipImageProcessor / a processor holding one
            ip = getattr(processor, "image_processor", processor)
            mean = tuple(getattr(ip, "image_mean", mean))
            std = tuple(getattr(ip, "image_std", std))
            rf = getattr(ip, "rescale_factor", rf)
        self.lut = normalize_lut(rf, mean, std, dtype).to(self.device)
        self._coef_cache: dict[tuple[int, int], np.ndarray] = {}
        self._tmp = None
        L.lib()

    def coeffs(self, in_size: int) -> tuple[int, np.ndarray]:
        """(ksize, int32 [S*2 + S*ksize]) bounds then weights for in_size -> S (host, cached)."""
        key = (in_size, self.S)
        hit = self._coef_cache.get(key)
        if hit is None:
            lib = L.lib()
            k = lib.ptk_resize_ksize(in_size, self.S)
            L.check(0 if k > 0 else -1, "resize_ksize")
            buf = np.empty(2 * self.S + self.S * k, np.int32)
            rc = lib.ptk_resize_coeffs(in_size, self.S, buf.ctypes.data, buf[2 * self.S:].ctypes.data)
            L.check(0 if rc == k else -1, "resize_coeffs")
            hit = self._coef_cache[key] = buf
        return (len(hit) - 2 * self.S) // self.S, hit

    def layout(self, shapes, out: torch.Tensor | None = None):
        """Lay a batch of [H, W, C] images out in one host buffer [descs | coefs | pixels] (pinned when
        CUDA is present); returns (buffer, meta, per-image uint8 views of the pixel section to fill)."""
        n, S = len(shapes), self.S
        descs = (L.ImageDesc * max(n, 1))()
        coef_parts, coef_off = [], 0
        src_off, tmp_off, max_h, max_rb = 0, 0, 0, 0
        offs = []
        for i, (h, w, c) in enumerate(shapes):
            if c not in (1, 3) or h <= 0 or w <= 0:
                raise ValueError(f"image {i}: need [H, W, 1|3], got {(h, w, c)}")
            kh, ch = self.coeffs(w)
            kv, cv = self.coeffs(h)
            descs[i].src_off, descs[i].h, descs[i].w, descs[i].c = src_off, h, w, c
            descs[i].kh, descs[i].kv, descs[i].coef_off, descs[i].tmp_off = kh, kv, coef_off, tmp_off
            coef_parts += [ch, cv]
            coef_off += len(ch) + len(cv)
            offs.append(src_off)
            src_off += _align(h * w * c)
            tmp_off += _align(h * S * c)
            max_h, max_rb = max(max_h, h), max(max_rb, w * c)
        d_bytes = _align(L.C.sizeof(descs))
        c_bytes = _align(coef_off * 4)
        total = d_bytes + c_bytes + src_off
        if out is None or out.numel() < total:
            out = torch.empty(max(total, 1), dtype=torch.uint8, pin_memory=torch.cuda.is_available())
        buf = out.numpy()
        buf[: L.C.sizeof(descs)] = np.frombuffer(descs, np.uint8)
        if coef_parts:
            buf[d_bytes: d_bytes + coef_off * 4] = np.concatenate(coef_parts).view(np.uint8)
        base = d_bytes + c_bytes
        views = [buf[base + o: base + o + h * w * c].reshape(h, w, c) for o, (h, w, c) in zip(offs, shapes)]
        return out, (n, d_bytes, c_bytes, max_h, max_rb, tmp_off, total), views

    def pack(self, images, out: torch.Tensor | None = None):
        """`layout` + copy of already decoded uint8 images ([H, W, C] arrays or tensors, or [H, W])."""
        arrs = []
        for i, im in enumerate(images):
            im = im.numpy() if isinstance(im, torch.Tensor) else np.asarray(im)
            im = im[:, :, None] if im.ndim == 2 else im
            if im.dtype != np.uint8 or im.ndim != 3:
                raise ValueError(f"image {i}: need uint8 [H, W, 1|3], got {im.dtype} {im.shape}")
            arrs.append(im)
        out, meta, views = self.layout([a.shape for a in arrs], out)
        for v, a in zip(views, arrs):
            v[...] = a
        return out, meta

    def launch(self, dev_buf: torch.Tensor, meta, out: torch.Tensor, stream=None):
        """Run the two passes over a packed batch already on the device."""
        n, d_bytes, c_bytes, max_h, max_rb, tmp_bytes, _ = meta
        if n == 0:
            return out
        if max_rb > 65536:
            raise ValueError(f"image rows of {max_rb} bytes exceed the 64 KiB LDS row stage")
        if self._tmp is None or self._tmp.numel() < tmp_bytes:
            self._tmp = torch.empty(max(tmp_bytes, 1 << 20), dtype=torch.uint8, device=self.device)
        base = dev_buf.data_ptr()
        st = (stream or torch.cuda.current_stream(self.device)).cuda_stream
        L.check(L.lib().ptk_image_preprocess(base + d_bytes + c_bytes, base + d_bytes, base, n, max_h, max_rb, self.S,
                                             self.lut.data_ptr(), int(self.dtype == torch.float32),
                                             self._tmp.data_ptr(), out.data_ptr(), st), "image_preprocess")
        return out

    def __call__(self, images) -> torch.Tensor:
        """Decoded uint8 images -> pixel_values [B, 3, S, S] on the device (current stream)."""
        images = list(images)
        host, meta = self.pack(images)
        dev = host[: meta[-1]].to(self.device, non_blocking=True)
        out = torch.empty(len(images), 3, self.S, self.S, dtype=self.dtype, device=self.device)
        return self.launch(dev, meta, out)


def image_shape(im) -> tuple[int, int, int]:
    """[H, W, C] that decode_into will produce for a lazily opened Pillow image."""
    return im.size[1], im.size[0], 1 if im.mode == "L" else 3


def decode_into(im, out: np.ndarray):
    """Decode a lazily opened Pillow image into `out` (uint8 [H, W, C]); Pillow releases the GIL
    while it decodes, so a thread pool decodes in parallel."""
    with im:
        im.load()
        a = np.asarray(im if im.mode == "L" else im.convert("RGB"))
    out.reshape(a.shape)[...] = a


class ThreadedImageLoader:
    """Batches of a decoding dataset (`open_item`) straight into device pixel_values.

    A producer thread opens each batch's images (headers only), lays the batch out
    (`ImagePreprocessor.layout`) in one of `depth` pinned slots and has a thread pool decode every
    image directly into its place there (one copy per image, no inter-process hand-over); the
    consumer copies the slot to the device and runs the resize/normalise kernels on a side stream.
    A slot is refilled only after its previous copy has landed."""

    def __init__(self, dataset, index_batches, pre: "ImagePreprocessor", threads: int = 8, depth: int = 3):
        self.ds, self.batches, self.pre = dataset, [list(b) for b in index_batches], pre
        self.threads, self.depth = max(1, threads), max(2, depth)

    def __iter__(self):
        import queue
        import threading
        from concurrent.futures import ThreadPoolExecutor
        pre, depth = self.pre, self.depth
        slots = [None] * depth
        slot_event = [None] * depth
        free = threading.Semaphore(depth)
        q: "queue.Queue" = queue.Queue()
        stop = threading.Event()

        def produce():
            try:
                with ThreadPoolExecutor(self.threads) as pool:
                    for k, idx in enumerate(self.batches):
                        free.acquire()
                        if stop.is_set():
                            return
                        s = k % depth
                        if slot_event[s] is not None:
                            slot_event[s].synchronize()
                        items = [self.ds.open_item(i) for i in idx]
                        shapes = [image_shape(it[0]) for it in items]
                        host, meta, views = pre.layout(shapes, slots[s])
                        slots[s] = host
                        list(pool.map(lambda a: decode_into(a[0][0], a[1]), zip(items, views)))
                        ids = torch.stack([it[1] for it in items])
                        labels = torch.stack([it[2] for it in items])
                        q.put((s, host, meta, ids, labels))
                q.put(None)
            except BaseException as e:   # surfaced in the consumer
                q.put(e)

        th = threading.Thread(target=produce, daemon=True)
        th.start()
        side = torch.cuda.Stream(pre.device)
        cur = torch.cuda.current_stream(pre.device)
        try:
            while True:
                got = q.get()
                if got is None:
                    break
                if isinstance(got, BaseException):
                    raise got
                s, host, meta, ids, labels = got
                with torch.cuda.stream(side):
                    dev = host[: meta[-1]].to(pre.device, non_blocking=True)
                    out = torch.empty(meta[0], 3, pre.S, pre.S, dtype=pre.dtype, device=pre.device)
                    pre.launch(dev, meta, out, side)
                    ids_d = ids.pin_memory().to(pre.device, non_blocking=True)
                    lab_d = labels.pin_memory().to(pre.device, non_blocking=True)
                    ev = torch.cuda.Event()
                    ev.record(side)
                slot_event[s] = ev
                free.release()
                cur.wait_event(ev)
                for t in (out, ids_d, lab_d, dev):
                    t.record_stream(cur)
                yield {"pixel_values": out, "token_ids": ids_d, "labels": lab_d}
        finally:
            stop.set()
            free.release()
            th.join(timeout=60)


class DevicePrefetcher:
    """Iterates collated batches (e.g. a multi-worker DataLoader with `collate`) and yields
    device batches {"pixel_values", "token_ids", "labels"}, the next batch's copy and pixel
    kernels running on a side stream while the caller's step runs."""

    def __init__(self, batches, pre: ImagePreprocessor, depth: int = 2):
        self.batches, self.pre, self.depth = batches, pre, max(1, depth)
        self.stream = torch.cuda.Stream(pre.device)
        self.pinned = [None] * self.depth
        self.done = [None] * self.depth

    def _stage(self, slot, b):
        pre = self.pre
        if self.done[slot] is not None:
            self.done[slot].synchronize()          # the pinned slot's previous copy has landed
        host, meta = pre.pack(b["images"], self.pinned[slot])
        self.pinned[slot] = host
        with torch.cuda.stream(self.stream):
            dev = host[: meta[-1]].to(pre.device, non_blocking=True)
            out = torch.empty(len(b["images"]), 3, pre.S, pre.S, dtype=pre.dtype, device=pre.device)
            pre.launch(dev, meta, out, self.stream)
            ids = b["token_ids"].pin_memory().to(pre.device, non_blocking=True)
            labels = b["labels"].pin_memory().to(pre.device, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(self.stream)
        self.done[slot] = ev
        return {"pixel_values": out, "token_ids": ids, "labels": labels, "_event": ev, "_keep": dev}

    def __iter__(self):
        it = iter(self.batches)
        queue, slot = [], 0
        for b in it:
            queue.append(self._stage(slot, b))
            slot = (slot + 1) % self.depth
            if len(queue) >= self.depth:
                yield self._hand_over(queue.pop(0))
        while queue:
            yield self._hand_over(queue.pop(0))

    def _hand_over(self, d):
        cur = torch.cuda.current_stream(self.pre.device)
        cur.wait_event(d.pop("_event"))
        keep = d.pop("_keep")
        for t in (d["pixel_values"], d["token_ids"], d["labels"], keep):
            t.record_stream(cur)
        return d
