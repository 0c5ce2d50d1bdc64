"""Time libptk GEMM shapes of the cfg2 step (HIP events, interleaved rounds in one
process) and print achieved TFLOP/s and effective HBM GB/s per shape/epilogue."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from projectiontrainer_amd import kernels as K, _lib as L  # noqa: E402

dev = torch.device("cuda:0")
M = 32 * 704
SHAPES = [  # name, M, N, K, act, out dtype
    ("gemma_gate_up_geglu", M, 13824, 1152, L.ACT_GEGLU, torch.bfloat16),
    ("gemma_gate_up_plain", M, 13824, 1152, L.ACT_NONE, torch.bfloat16),
    ("gemma_down", M, 1152, 6912, L.ACT_NONE, torch.bfloat16),
    ("gemma_dX_gate_up_f32", M, 1152, 13824, L.ACT_NONE, torch.float32),
    ("gemma_geglu_bwd", M, 6912, 1152, L.ACT_GEGLU_BWD, torch.bfloat16),
    ("gemma_qkv", M, 1536, 1152, L.ACT_NONE, torch.bfloat16),
    ("siglip_fc1_gelu", 18432, 4096, 1024, L.ACT_GELU_TANH, torch.bfloat16),
    ("siglip_fc2_f32", 18432, 1024, 4096, L.ACT_NONE, torch.float32),
    ("lm_head", 4096, 262144, 1152, L.ACT_NONE, torch.bfloat16),
    ("square_8192", 8192, 8192, 8192, L.ACT_NONE, torch.bfloat16),
]
SQUARE = [("sq4096", 4096, 4096, 4096, L.ACT_NONE, torch.bfloat16), ("sq8192", 8192, 8192, 8192, L.ACT_NONE, torch.bfloat16)]


def run(name, m, n, k, act, odt, reps=10):
    A = torch.randn(m, k, device=dev).to(torch.bfloat16)
    B = (torch.randn(n, k, device=dev) * 0.05).to(torch.bfloat16)
    kw = {}
    if act == L.ACT_GEGLU:
        kw = dict(aux=torch.empty(m, n // 2, dtype=torch.bfloat16, device=dev),
                  aux2=torch.empty(m, n // 2, dtype=torch.bfloat16, device=dev))
    if act == L.ACT_GEGLU_BWD:
        kw = dict(aux_in=torch.randn(m, n, device=dev).to(torch.bfloat16),
                  aux_in2=torch.randn(m, n, device=dev).to(torch.bfloat16))
    C = K.gemm(A, B, out_dtype=odt, act=act, **kw)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        K.gemm(A, B, C=C, out_dtype=odt, act=act, **kw)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    fl = 2.0 * m * n * k
    return {"name": name, "M": m, "N": n, "K": k, "ms": round(ms, 4), "TFLOPs": round(fl / ms / 1e9, 1)}


ALL = [  # every single-batch GEMM of the cfg2 step: name, M, N, K, act, out
    ("sig_patch", 18432, 1024, 768, L.ACT_NONE, torch.float32),
    ("sig_qkv", 18432, 3072, 1024, L.ACT_NONE, torch.bfloat16),
    ("sig_o", 18432, 1024, 1024, L.ACT_NONE, torch.float32),
    ("sig_fc1", 18432, 4096, 1024, L.ACT_GELU_TANH, torch.bfloat16),
    ("sig_fc2", 18432, 1024, 4096, L.ACT_NONE, torch.float32),
    ("proj_fc1", 18432, 11520, 1024, L.ACT_GELU_ERF, torch.bfloat16),
    ("proj_fc2", 18432, 1152, 11520, L.ACT_NONE, torch.float32),
    ("g_qkv", M, 1536, 1152, L.ACT_NONE, torch.bfloat16),
    ("g_o", M, 1152, 1024, L.ACT_NONE, torch.bfloat16),
    ("g_gu", M, 13824, 1152, L.ACT_GEGLU, torch.bfloat16),
    ("g_down", M, 1152, 6912, L.ACT_NONE, torch.bfloat16),
    ("g_lm", 4096, 262144, 1152, L.ACT_NONE, torch.bfloat16),
    ("g_dh", M, 6912, 1152, L.ACT_NONE, torch.bfloat16),
    ("g_dh_geglu_bwd", M, 6912, 1152, L.ACT_GEGLU_BWD, torch.bfloat16),
    ("g_dgu", M, 1152, 13824, L.ACT_NONE, torch.float32),
    ("g_dO", M, 1024, 1152, L.ACT_NONE, torch.bfloat16),
    ("g_dqkv", M, 1152, 1536, L.ACT_NONE, torch.float32),
    ("g_dao", M, 1152, 1024, L.ACT_NONE, torch.float32),
]

if __name__ == "__main__" and "--all" in sys.argv:
    for s in ALL + SQUARE:
        r = {}
        for mode in (2, 1, 4, 8, 2, 1, 4, 8):   # second round kept (warm)
            L.lib().ptk_gemm_force_small_tiles(mode)
            r[mode] = run(*s)
        L.lib().ptk_gemm_force_small_tiles(0)
        r[0] = run(*s)
        print(json.dumps({"name": s[0], "M": s[1], "N": s[2], "K": s[3], "big_TF": r[2]["TFLOPs"],
                          "small_TF": r[1]["TFLOPs"], "big2_TF": r[4]["TFLOPs"], "w4_TF": r[8]["TFLOPs"],
                          "auto_TF": r[0]["TFLOPs"]}),
              flush=True)
    sys.exit(0)

if __name__ == "__main__" and "--blas" not in sys.argv:
    res = []
    if "--small" in sys.argv:
        L.lib().ptk_gemm_force_small_tiles(1)
    for rnd in range(0 if "--sweep" in sys.argv else 2):
        for s in SHAPES:
            r = run(*s)
            if rnd == 1:
                res.append(r)
                print(json.dumps(r), flush=True)
    if "--sweep" in sys.argv:
        # fixed per-tile cost vs K-proportional cost (prologue/epilogue overhead)
        for n in (13824, 4096):
            for k in (256, 512, 1152, 2304, 4608):
                r = run(f"sweep_n{n}", M, n, k, L.ACT_NONE, torch.bfloat16)
                r["tiles"] = ((M + 255) // 256) * ((n + 255) // 256)
                print(json.dumps(r), flush=True)


def run_blas(name, m, n, k, reps=10):
    """torch.matmul (hipBLASLt) on the same shape, plain bf16 output: calibration only."""
    A = torch.randn(m, k, device=dev).to(torch.bfloat16)
    B = (torch.randn(n, k, device=dev) * 0.05).to(torch.bfloat16)
    C = torch.empty(m, n, device=dev, dtype=torch.bfloat16)
    torch.matmul(A, B.t(), out=C)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        torch.matmul(A, B.t(), out=C)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    return round(2.0 * m * n * k / ms / 1e9, 1)


if __name__ == "__main__" and "--blas" in sys.argv:
    for s in ALL + SQUARE:
        ours = [run(*s) for _ in range(2)][-1]["TFLOPs"]
        blas = [run_blas(*s[:4]) for _ in range(2)][-1]
        print(json.dumps({"name": s[0], "M": s[1], "N": s[2], "K": s[3], "ptk_TF": ours, "hipblaslt_TF": blas}),
              flush=True)
