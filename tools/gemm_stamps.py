"""Diagnostic: per-block phase timing of the 256x256 GEMM from in-kernel stamps
(build/libptk_stamps.so, `make -C projectiontrainer_amd/csrc stamps`).  Loads the
diagnostic library in place of libptk.so; never used by tests or the bench.
usage: python tools/gemm_stamps.py M N K [act]"""
import ctypes
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from projectiontrainer_amd import _lib as L  # noqa: E402

L.LIB_PATH = os.path.join(ROOT, "build", "libptk_stamps.so")
from projectiontrainer_amd import kernels as K  # noqa: E402

lib = L.lib()
lib.ptk_debug_stamps_read.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
lib.ptk_debug_epi_mode.argtypes = [ctypes.c_int]


def main():
    m, n, k = (int(x) for x in sys.argv[1:4])
    act = int(sys.argv[4]) if len(sys.argv) > 4 else L.ACT_NONE
    emode = int(sys.argv[5]) if len(sys.argv) > 5 else 0
    assert lib.ptk_debug_epi_mode(emode) == 0
    dev = torch.device("cuda:0")
    A = torch.randn(m, k, device=dev).to(torch.bfloat16)
    B = (torch.randn(n, k, device=dev) * 0.05).to(torch.bfloat16)
    kw = {}
    if act == L.ACT_GEGLU:
        kw = dict(aux=torch.empty(m, n // 2, dtype=torch.bfloat16, device=dev),
                  aux2=torch.empty(m, n // 2, dtype=torch.bfloat16, device=dev))
    C = K.gemm(A, B, act=act, **kw)
    for _ in range(50):    # >= ~50 ms of back-to-back launches so the clock settles
        K.gemm(A, B, C=C, act=act, **kw)
    torch.cuda.synchronize()
    nblk = ((m + 255) // 256) * ((n + 255) // 256)
    buf = np.zeros((1 << 15, 6), dtype=np.uint64)
    assert lib.ptk_debug_stamps_read(buf.ctypes.data, buf.nbytes) == 0
    s = buf[:nblk].astype(np.int64)
    t0 = s[:, 0].min()
    start, pro, loop, epi = s[:, 0] - t0, s[:, 1] - s[:, 0], s[:, 2] - s[:, 1], s[:, 3] - s[:, 2]
    clk = np.median((s[:, 3] - s[:, 0]) / np.maximum(s[:, 4] - s[:, 5], 1)) * 100.0   # MHz
    span = (s[:, 3].max() - t0)
    order = np.argsort(start)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        K.gemm(A, B, C=C, act=act, **kw)
    e1.record()
    torch.cuda.synchronize()
    out = {"M": m, "N": n, "K": k, "epi_mode": emode, "ms": round(e0.elapsed_time(e1) / 10, 4), "blocks": nblk, "clock_MHz": round(float(clk), 1),
           "prologue_cyc_med": int(np.median(pro)), "mainloop_cyc_med": int(np.median(loop)),
           "epilogue_cyc_med": int(np.median(epi)),
           "prologue_cyc_p90": int(np.percentile(pro, 90)), "epilogue_cyc_p90": int(np.percentile(epi, 90)),
           "mainloop_cyc_per_ktile": round(float(np.median(loop)) / (k // 64), 1),
           }
    print(json.dumps(out))


if __name__ == "__main__":
    main()
