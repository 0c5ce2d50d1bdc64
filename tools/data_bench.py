"""Host data step throughput: synthetic X-ray-sized JPEGs on disk ->
XrayTextPairDataset (worker processes decode) -> DevicePrefetcher (pinned pack, H2D and the
GPU resize/normalise on a side stream) -> bf16 pixel_values, against the reference's host
path (Pillow decode + resize + SiglipImageProcessor per image) timed on the same files.

    python tools/data_bench.py [--n 256] [--workers 8] [--size 2048x2500] [--batch 32]

Prints one JSON line: img/s of the GPU path end to end, of its decode-only leg, the GPU kernel
time per batch (HIP events on the side stream), and the reference host path's img/s per core.
"""
import argparse
import json
import os
import sys
import tempfile
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


class _Tok:
    pad_token_id = 0

    def __call__(self, text, max_length, padding, truncation, return_tensors):
        ids = [2] + [3 + (ord(c) % 250) for c in text][: max_length - 1]
        ids = [0] * (max_length - len(ids)) + ids

        class _O:
            pass
        o = _O()
        o.input_ids = torch.tensor([ids])
        return o


def make_files(d, n, h, w, seed=0):
    from PIL import Image
    rng = np.random.default_rng(seed)
    yy, xx = np.mgrid[0:h, 0:w].astype(np.float32)
    samples = []
    for i in range(min(n, 16)):   # 16 distinct images, reused by name (decode cost is per file read)
        base = 120 + 60 * np.sin(xx / (40 + i)) * np.cos(yy / (55 + i)) + rng.normal(0, 12, (h, w))
        Image.fromarray(np.clip(base, 0, 255).astype(np.uint8), "L").save(os.path.join(d, f"x{i}.jpg"), quality=92)
    for i in range(n):
        samples.append({"image": f"x{i % 16}.jpg", "normal_caption": "The lungs are clear. No effusion. " * 4})
    js = os.path.join(d, "s.json")
    json.dump(samples, open(js, "w"))
    return js


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=256)
    ap.add_argument("--workers", type=int, default=8)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--size", default="2048x2500")
    ap.add_argument("--ref-n", type=int, default=8)
    ap.add_argument("--one-thread", type=int, default=1)
    args = ap.parse_args()
    h, w = (int(v) for v in args.size.split("x"))
    from projectiontrainer_amd.data import DevicePrefetcher, ImagePreprocessor, XrayTextPairDataset, collate, worker_init
    dev = torch.device("cuda:0")
    with tempfile.TemporaryDirectory() as d:
        js = make_files(d, args.n, h, w)
        ds = XrayTextPairDataset(d, js, None, _Tok(), 384, max_length=128)
        mk = lambda: torch.utils.data.DataLoader(ds, batch_size=args.batch, num_workers=args.workers,
                                                 collate_fn=collate, persistent_workers=False, prefetch_factor=4,
                                                 worker_init_fn=worker_init if args.one_thread else None)
        # decode-only leg
        t0 = time.perf_counter()
        nd = sum(len(b["images"]) for b in mk())
        t_dec = time.perf_counter() - t0
        # end to end to device pixel_values
        pre = ImagePreprocessor(384, dev)
        pre([np.zeros((h, w, 1), np.uint8)])   # warm up the kernels / allocator
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        n = 0
        for b in DevicePrefetcher(mk(), pre):
            n += b["pixel_values"].shape[0]
        torch.cuda.synchronize()
        t_e2e = time.perf_counter() - t0
        # end to end through the threaded decode-into-pinned loader (the trainer's path)
        from projectiontrainer_amd.data import ThreadedImageLoader
        idx = [list(range(i, min(i + args.batch, args.n))) for i in range(0, args.n, args.batch)]
        thr = {}
        for nt in (8, 14):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            m = sum(b["pixel_values"].shape[0] for b in ThreadedImageLoader(ds, idx, pre, threads=nt))
            torch.cuda.synchronize()
            thr[nt] = round(m / (time.perf_counter() - t0), 1)
        # kernel time of one batch (events on the current stream)
        imgs = [np.asarray(ds[i]["image"]) for i in range(min(args.batch, args.n))]
        host, meta = pre.pack(imgs)
        dbuf = host[: meta[-1]].to(dev)
        out = torch.empty(len(imgs), 3, 384, 384, dtype=torch.bfloat16, device=dev)
        pre.launch(dbuf, meta, out)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            pre.launch(dbuf, meta, out)
        e1.record()
        torch.cuda.synchronize()
        k_ms = e0.elapsed_time(e1) / 10
        in_bytes = sum(im.size for im in imgs)
        # decode alone on one core (the part of the host path the GPU path keeps)
        from projectiontrainer_amd.data import decode_image
        t0 = time.perf_counter()
        for i in range(args.ref_n):
            decode_image(os.path.join(d, f"x{i % 16}.jpg"))
        t_d1 = (time.perf_counter() - t0) / args.ref_n
        # the reference's host path on one core
        from PIL import Image
        import transformers as tr
        proc = tr.SiglipImageProcessor(size={"height": 384, "width": 384})
        t0 = time.perf_counter()
        for i in range(args.ref_n):
            im = Image.open(os.path.join(d, f"x{i % 16}.jpg")).convert("RGB").resize((384, 384))
            proc(images=im, return_tensors="pt")
        t_ref = (time.perf_counter() - t0) / args.ref_n
    print(json.dumps({
        "image": f"{h}x{w} greyscale JPEG q92", "batch": args.batch, "workers": args.workers,
        "one_thread_per_worker": bool(args.one_thread),
        "threaded_e2e_img_s": thr, "e2e_img_s": round(n / t_e2e, 1), "decode_only_img_s": round(nd / t_dec, 1),
        "gpu_kernel_ms_per_batch": round(k_ms, 3), "gpu_kernel_img_s": round(len(imgs) / k_ms * 1e3, 1),
        "gpu_kernel_src_GBs": round(in_bytes / k_ms / 1e6, 1),
        "decode_ms_per_img_1core": round(t_d1 * 1e3, 2),
        "reference_host_path_ms_per_img_1core": round(t_ref * 1e3, 2),
    }))


if __name__ == "__main__":
    main()
