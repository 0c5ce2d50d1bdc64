"""Time the flash attention kernels at the cfg2 step's shapes (HIP events on the launch stream).

Gemma3-1B: 32 samples x 1 kv head x (704 positions x 4 query heads) rows, head_dim 256, causal,
sliding window 512 (5 of 6 layers) or full causal; key padding 703 -> 704.
SigLIP-L/16-384: 32 x 16 heads, 576 patches, head_dim 64, non-causal.
Run under `rocprofv3 --kernel-trace --stats` for per-kernel times of the backward."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from projectiontrainer_amd import kernels as Kn  # noqa: E402

dev = torch.device("cuda:0")


def pairs_gemma(S, G, window, nvalid):
    n = 0
    for p in range(nvalid):
        lo = max(0, p - window + 1) if window else 0
        n += p + 1 - lo
    return n * G


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--B", type=int, default=32)
    ap.add_argument("--what", default="fwd,bwd,siglip")
    args = ap.parse_args()
    B, S, G, D = args.B, 704, 4, 256
    g = torch.Generator(device=dev).manual_seed(0)
    rnd = lambda *s: torch.randn(*s, device=dev, generator=g).to(torch.bfloat16)
    Q, Kt, Vt, dO = rnd(B, S * G, D), rnd(B, S, D), rnd(B, S, D), rnd(B, S * G, D)
    kv = torch.ones(B, S, dtype=torch.int32, device=dev)
    kv[:, S - 1] = 0
    O = torch.zeros(B, S * G, D, dtype=torch.bfloat16, device=dev)
    lse = torch.zeros(B, S * G, dtype=torch.float32, device=dev)
    out = []
    for window in (512, 0):
        common = dict(rows=S * G, nkeys=S, head_dim=D, batch=B, batch_inner=1, zdiv=1, qdiv=G, causal=True,
                      window=window, key_valid=kv, scale=D ** -0.5)
        fwd = lambda: Kn.flash_attn(Q, Kt, Vt, O, lse=lse, ldq=D, ldk=D, ldo=D,
                                    strides=(S * G * D, 0, S * D, 0, S * G * D, 0), **common)
        fl = 4.0 * pairs_gemma(S, G, window, S - 1) * D * B
        if "fwd" in args.what:
            ms = timed(fwd, args.reps)
            out.append({"kernel": f"gemma_fwd_w{window}", "us": round(ms * 1e3, 1), "TFLOPs": round(fl / ms / 1e9, 1)})
        fwd()
        if "bwd" in args.what:
            bwd = lambda: Kn.flash_attn_bwd(Q, Kt, Vt, O, dO, lse, sO=(S * G * D, 0), **common)
            ms = timed(bwd, args.reps)
            out.append({"kernel": f"gemma_bwd_w{window}", "us": round(ms * 1e3, 1),
                        "TFLOPs_5prod": round(2.5 * fl / ms / 1e9, 1)})
    if "siglip" in args.what:
        N, H, hd = 576, 16, 64
        Dm = H * hd
        qkv = rnd(B * N, 3 * Dm)
        Os = torch.zeros(B * N, Dm, dtype=torch.bfloat16, device=dev)
        f = lambda: Kn.flash_attn(qkv, qkv[:, Dm:], qkv[:, 2 * Dm:], Os, rows=N, nkeys=N, head_dim=hd, ldq=3 * Dm,
                                  ldk=3 * Dm, ldo=Dm, batch=B * H, batch_inner=H, zdiv=H,
                                  strides=(N * 3 * Dm, hd, N * 3 * Dm, hd, N * Dm, hd), scale=hd ** -0.5)
        ms = timed(f, args.reps)
        fl = 4.0 * N * N * hd * B * H
        out.append({"kernel": "siglip_fwd", "us": round(ms * 1e3, 1), "TFLOPs": round(fl / ms / 1e9, 1)})
    for r in out:
        print(json.dumps(r))


if __name__ == "__main__":
    main()
