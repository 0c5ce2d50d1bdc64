"""Plain-GEMM shapes of the Stage-1 (cfg2) and Stage-2 (cfg4) steps through libptk's ptk_gemm, timed with
HIP events, plus a bitwise determinism check (3 launches must agree).  Run once with PTK_BLASLT=0 (the
hand-written MFMA kernels) and once with PTK_BLASLT=1 (hipBLASLt for plain GEMMs)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from projectiontrainer_amd import kernels as K  # noqa: E402

dev = torch.device("cuda:0")
M1, M2 = 32 * 704, 16 * 896
SHAPES = [  # name, M, N, K, out dtype
    ("s1_qkv", M1, 1536, 1152, torch.bfloat16), ("s1_o", M1, 1152, 1024, torch.bfloat16),
    ("s1_down", M1, 1152, 6912, torch.bfloat16), ("s1_dX_gateup", M1, 1152, 13824, torch.float32),
    ("s1_dO", M1, 1024, 1152, torch.bfloat16), ("s1_dX_qkv", M1, 1152, 1536, torch.float32),
    ("lm_head", 4096, 262144, 1152, torch.bfloat16), ("s1_dX_lmhead", 4096, 1152, 262144, torch.float32),
    ("s1_dX_qkv_b16", M1, 1152, 1536, torch.bfloat16), ("s1_dX_gateup_b16", M1, 1152, 13824, torch.bfloat16),
    ("s2_qkv", M2, 1536, 1152, torch.bfloat16), ("s2_down", M2, 1152, 6912, torch.bfloat16),
    ("s2_dX_gateup", M2, 1152, 13824, torch.float32), ("s2_o", M2, 1152, 1024, torch.bfloat16),
    ("s2_dO", M2, 1024, 1152, torch.bfloat16), ("s2_dX_qkv", M2, 1152, 1536, torch.float32),
    ("dW_qkv", 1536, 1152, M2, torch.float32), ("dW_o", 1152, 1024, M2, torch.float32),
    ("dW_down", 1152, 6912, M2, torch.float32), ("dW_gateup", 13824, 1152, M2, torch.float32),
    ("dW_lmhead", 262144, 1152, 4096, torch.float32),
]
tag = {"1": "blaslt", "0": "mfma"}.get(os.environ.get("PTK_BLASLT"), "rule")
only = set(sys.argv[1:])
for name, m, n, k, odt in SHAPES:
    if only and name not in only:
        continue
    A = torch.randn(m, k, device=dev).to(torch.bfloat16)
    B = (torch.randn(n, k, device=dev) * 0.05).to(torch.bfloat16)
    C = K.gemm(A, B, out_dtype=odt)
    torch.cuda.synchronize()
    ref = C.clone()
    same = True
    for _ in range(2):
        K.gemm(A, B, C=C, out_dtype=odt)
        torch.cuda.synchronize()
        same = same and torch.equal(C, ref)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 10
    e0.record()
    for _ in range(reps):
        K.gemm(A, B, C=C, out_dtype=odt)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    err = float((C.float() - (A.float() @ B.float().t())).norm() / (A.float() @ B.float().t()).norm())
    print(json.dumps({"impl": tag, "shape": name, "M": m, "N": n, "K": k, "ms": round(ms, 4),
                      "TFLOPs": round(2.0 * m * n * k / ms / 1e9, 1), "deterministic": same, "rel_err": err}),
          flush=True)
    del A, B, C, ref
    torch.cuda.empty_cache()
