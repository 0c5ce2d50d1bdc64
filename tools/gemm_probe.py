"""Run one GEMM shape on a forced tile path repeatedly (for rocprofv3 kernel traces / PMC passes).
usage: python tools/gemm_probe.py M N K [act] [mode] [reps]"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from projectiontrainer_amd import _lib as L  # noqa: E402
if os.environ.get("PTK_LIB"):   # diagnostic builds (build/libptk_abl*.so, build/libptk_stamps.so)
    L.LIB_PATH = os.path.join(ROOT, os.environ["PTK_LIB"])
from projectiontrainer_amd import kernels as K  # noqa: E402

m, n, k = (int(x) for x in sys.argv[1:4])
act = int(sys.argv[4]) if len(sys.argv) > 4 else L.ACT_NONE
mode = int(sys.argv[5]) if len(sys.argv) > 5 else 8
reps = int(sys.argv[6]) if len(sys.argv) > 6 else 20
dev = torch.device("cuda:0")
A = torch.randn(m, k, device=dev).to(torch.bfloat16)
B = (torch.randn(n, k, device=dev) * 0.05).to(torch.bfloat16)
kw = {}
if act == L.ACT_GEGLU:
    kw = dict(aux=torch.empty(m, n // 2, dtype=torch.bfloat16, device=dev),
              aux2=torch.empty(m, n // 2, dtype=torch.bfloat16, device=dev))
elif act == L.ACT_GEGLU_BWD:   # dh GEMM: saved g, u [m, n] in, interleaved dg|du [m, 2n] out
    kw = dict(aux_in=torch.randn(m, n, device=dev).to(torch.bfloat16),
              aux_in2=torch.randn(m, n, device=dev).to(torch.bfloat16))
L.lib().ptk_gemm_force_small_tiles(mode)
C = K.gemm(A, B, act=act, **kw)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(reps):
    K.gemm(A, B, C=C, act=act, **kw)
e1.record()
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / reps
print(f"M={m} N={n} K={k} act={act} mode={mode}: {ms:.4f} ms  {2.0 * m * n * k / ms / 1e9:.1f} TFLOP/s", flush=True)
