"""Diagnostic: where the ping-pong GEMM's k-steps go, from in-kernel s_memtime stamps (build/libptk_ppstamps.so,
`make -C projectiontrainer_amd/csrc ppstamps`).  Per role (consumer = the group running the K loop, producer =
the group issuing the LDS-DMA stream and draining its previous tile), the mean cycles per k-step between
barriers ("work") and inside the step-end wait + barrier ("wait").  Never used by tests or the bench.
usage: python tools/pp_stamps.py M N K [act]"""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from projectiontrainer_amd import _lib as L  # noqa: E402

L.LIB_PATH = os.path.join(ROOT, "build", "libptk_ppstamps.so")
from projectiontrainer_amd import kernels as K  # noqa: E402

lib = L.lib()
lib.ptk_debug_pp_stamps_read.argtypes = [ctypes.c_void_p, ctypes.c_size_t]

m, n, k = (int(x) for x in sys.argv[1:4])
act = int(sys.argv[4]) if len(sys.argv) > 4 else L.ACT_NONE
dev = torch.device("cuda:0")
A = torch.randn(m, k, device=dev).to(torch.bfloat16)
B = (torch.randn(n, k, device=dev) * 0.05).to(torch.bfloat16)
kw = {}
if act == L.ACT_GEGLU:
    kw = dict(aux=torch.empty(m, n // 2, dtype=torch.bfloat16, device=dev),
              aux2=torch.empty(m, n // 2, dtype=torch.bfloat16, device=dev))
elif act == L.ACT_GEGLU_BWD:
    kw = dict(aux_in=torch.randn(m, n, device=dev).to(torch.bfloat16),
              aux_in2=torch.randn(m, n, device=dev).to(torch.bfloat16))
lib.ptk_gemm_force_small_tiles(32)
for _ in range(3):
    K.gemm(A, B, act=act, **kw)
torch.cuda.synchronize()
buf = np.zeros((1024, 8, 6), dtype=np.uint64)
assert lib.ptk_debug_pp_stamps_read(buf.ctypes.data, buf.nbytes) == 0
g = min(1024, torch.cuda.get_device_properties(0).multi_processor_count)
b = buf[:g].astype(np.float64)
for role, name in ((0, "consumer"), (1, "producer")):
    work, wait, cnt = b[:, :, 3 * role], b[:, :, 3 * role + 1], b[:, :, 3 * role + 2]
    steps = cnt.sum()
    print(f"M={m} N={n} K={k} act={act} {name}: {steps / (g * 8):.0f} steps per wave, "
          f"work {work.sum() / steps:.0f} + wait {wait.sum() / steps:.0f} cycles per k-step", flush=True)
