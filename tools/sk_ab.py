"""Same-process A/B of the stream-K tail (gemm_w4.hip P8Tail) against the dispatch without it, on the GEMM shapes
of the cfg2 step (and cfg4's weight grads): HIP-event time per launch, interleaved rounds, median of rounds."""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from projectiontrainer_amd import kernels as K, _lib as L  # noqa: E402

dev = torch.device("cuda:0")
SHAPES = [  # name, M, N, K, out, epilogue kind
    ("g_qkv", 22528, 1536, 1152, "bf16", ""), ("g_dO", 22528, 1024, 1152, "bf16", ""),
    ("g_o", 22528, 1152, 1024, "f32", "resid"), ("g_dgu_dX", 22528, 1152, 13824, "bf16", ""),
    ("g_down", 22528, 1152, 6912, "bf16", ""), ("sig_o", 18432, 1024, 1024, "bf16", "siglip"),
    ("sig_fc2", 18432, 1024, 4096, "bf16", "siglip"), ("proj_fc2", 18432, 1152, 10240, "f32r", "bias"),
    ("proj_dW2", 1152, 10240, 18432, "f32", ""), ("proj_dW1", 10240, 1024, 18432, "f32", ""),
    ("s2_dW_qkv", 1536, 1152, 14336, "bf16", "acc"), ("s2_dW_gu", 13824, 1152, 14336, "bf16", "acc"),
    ("s2_dW_down", 1152, 6912, 14336, "bf16", "acc"), ("s2_down", 14336, 1152, 6912, "bf16", ""),
    ("s2_dgu_dX", 14336, 1152, 13824, "bf16", ""), ("s2_sig_fc2", 9216, 1024, 4096, "bf16", "siglip"),
    ("s2_sig_o", 9216, 1024, 1024, "bf16", "siglip"), ("s2b8_down", 7168, 1152, 6912, "bf16", ""),
]
only = sys.argv[1:]
tail = torch.zeros(L.lib().ptk_gemm_tail_scratch_bytes(), dtype=torch.uint8, device=dev)
for name, m, n, k, out, kind in SHAPES:
    if only and name not in only:
        continue
    A = torch.randn(m, k, device=dev).to(torch.bfloat16)
    B = (torch.randn(n, k, device=dev) * 0.05).to(torch.bfloat16)
    odt = torch.bfloat16 if out == "bf16" else torch.float32
    C = torch.empty(m, n, dtype=odt, device=dev)
    kw = {}
    if out == "f32r":
        kw["out_mode"] = L.OUT_F32_BF16ROUND
    if kind == "siglip":
        kw.update(bias=torch.randn(n, device=dev), resid16=C, bf16_linear=True)
    elif kind == "bias":
        kw.update(bias=torch.randn(n, device=dev))
    elif kind == "resid":
        kw.update(resid=C)
    elif kind == "acc":
        kw.update(resid16=C, bf16_linear=True)
    d = L.GemmDesc()
    d.M, d.N, d.K, d.act = m, n, k, L.ACT_NONE
    d.out = {"bf16": L.OUT_BF16, "f32": L.OUT_F32, "f32r": L.OUT_F32_BF16ROUND}[out]
    d.tail_ws = tail.data_ptr()
    gs = L.lib().ptk_gemm_tail_split(d)
    res = {"sk": [], "p8": [], "base": []}
    lib = L.lib()

    def launch(arm):
        if arm == "p8":
            lib.ptk_gemm_force_small_tiles(32)
        K.gemm(A, B, C=C, tail_ws=tail if arm == "sk" else None, **kw)
        if arm == "p8":
            lib.ptk_gemm_force_small_tiles(0)
    for arm in res:   # warm all
        launch(arm)
    arms = list(res)
    for rnd in range(5):
        for arm in arms if rnd % 2 == 0 else arms[::-1]:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(5):
                launch(arm)
            e1.record()
            torch.cuda.synchronize()
            res[arm].append(e0.elapsed_time(e1) / 5 * 1e3)
    L.gemm_path_counts(reset=True)
    K.gemm(A, B, C=C, tail_ws=tail, **kw)
    p_sk = sorted(L.gemm_path_counts(reset=True))
    K.gemm(A, B, C=C, **kw)
    p_b = sorted(L.gemm_path_counts(reset=True))
    s, p, b = (statistics.median(res[a]) for a in ("sk", "p8", "base"))
    fl = 2.0 * m * n * k
    print(f"{name:11s} M{m} N{n} K{k} split_over={gs:3d}  sk {s:7.1f} us ({fl / s / 1e6:5.0f} TF/s)  "
          f"p8 {p:7.1f} us ({fl / p / 1e6:5.0f})  base {b:7.1f} us ({fl / b / 1e6:5.0f}) {p_b}  "
          f"sk/p8 {s / p:.3f} sk/base {s / b:.3f}", flush=True)
