"""Split-K probe for the long-K, few-tile GEMMs of the unfrozen-LLM step (dW = dY^T X at K = tokens) and
the N = 1152 dX GEMMs: auto-dispatched single GEMM vs S-way split-K (batched 128x128 kernel, fp32
partials), HIP-event timed.  Prints one JSON line per shape and split."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from projectiontrainer_amd import kernels as K, _lib as L  # noqa: E402

dev = torch.device("cuda:0")
Mt = 16 * 896   # cfg4 token rows
SHAPES = [  # name, M (out rows), N (out cols), K
    ("dW_qkv", 1536, 1152, Mt), ("dW_o", 1152, 1024, Mt), ("dW_down", 1152, 6912, Mt),
    ("dW_gateup", 13824, 1152, Mt), ("dX_gateup_s2", Mt, 1152, 13824), ("down_fwd_s2", Mt, 1152, 6912),
    ("dX_gateup_s1", 32 * 704, 1152, 13824), ("dW_lmhead", 262144, 1152, 4096),
]


def timed(fn, reps=8):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


for name, m, n, k in SHAPES:
    A = torch.randn(m, k, device=dev).to(torch.bfloat16)
    B = (torch.randn(n, k, device=dev) * 0.05).to(torch.bfloat16)
    C = torch.empty(m, n, dtype=torch.float32, device=dev)
    fl = 2.0 * m * n * k
    ms = timed(lambda: K.gemm(A, B, C=C))
    print(json.dumps({"shape": name, "M": m, "N": n, "K": k, "split": 0, "ms": round(ms, 4),
                      "TFLOPs": round(fl / ms / 1e9, 1)}), flush=True)
    for S in (2, 4, 8, 16):
        kc = k // S // 64 * 64
        if kc < 256 or kc * S != k:
            continue
        P = torch.empty(S, m, n, dtype=torch.float32, device=dev)
        out = torch.empty(m, n, dtype=torch.float32, device=dev)

        def run():
            K.gemm(A, B, C=P, M=m, N=n, K=kc, lda=k, ldb=k, ldc=n, batch=S, strides=(kc, 0, kc, 0, m * n, 0))
            torch.sum(P, dim=0, out=out)      # the partial reduce (torch here: probe only)
        ms = timed(run)
        print(json.dumps({"shape": name, "split": S, "ms": round(ms, 4), "TFLOPs": round(fl / ms / 1e9, 1)}),
              flush=True)
    del A, B, C
    torch.cuda.empty_cache()
