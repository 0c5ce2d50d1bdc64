"""Diagnostic: per-segment phase timing of the persistent GEMMs (gemm_p8_kernel, gemm_w4_kernel) from in-kernel stamps
(ablibs/libptk_w4stamps.so: `make -C projectiontrainer_amd/csrc ablib AB_NAME=w4stamps AB_SRC=gemm_w4.hip
AB_DEFS=-DPTK_P8_STAMPS`).  Loads the diagnostic library in place of libptk.so; never used by tests or the bench.
Wave 0 of every workgroup stamps each segment (output tile): 0 start, 1 first K-tile done (its end-of-pair vmcnt
wait passed: after an epilogue that wait also drains the epilogue's stores, which were issued before that
K-tile's DMA pieces), 2 K loop done, 3 epilogue issued.  epi_mode 1 skips the epilogue (K-loop-only timing,
wrong results).
usage: python tools/p8_stamps.py M N K [epi_mode] [name] [p8|w4] [act]"""
import ctypes
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from projectiontrainer_amd import _lib as L  # noqa: E402

L.LIB_PATH = os.environ.get("PTK_STAMPS_LIB", os.path.join(ROOT, "ablibs", "libptk_w4stamps.so"))
from projectiontrainer_amd import kernels as Kn  # noqa: E402

lib = L.lib()
lib.ptk_debug_p8_stamps_read.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
lib.ptk_debug_p8_epi_mode.argtypes = [ctypes.c_int]


def main():
    m, n, k = (int(x) for x in sys.argv[1:4])
    emode = int(sys.argv[4]) if len(sys.argv) > 4 else 0
    name = sys.argv[5] if len(sys.argv) > 5 else f"{m}x{n}x{k}"
    kern = sys.argv[6] if len(sys.argv) > 6 else "p8"
    act = int(sys.argv[7]) if len(sys.argv) > 7 else L.ACT_NONE
    assert lib.ptk_debug_p8_epi_mode(emode) == 0
    L.check(lib.ptk_gemm_force_small_tiles(32 if kern == "p8" else 8), "force kernel")
    dev = torch.device("cuda:0")
    A = torch.randn(m, k, device=dev).to(torch.bfloat16)
    B = (torch.randn(n, k, device=dev) * 0.05).to(torch.bfloat16)
    kw = {"act": act}
    if act == L.ACT_GEGLU:
        kw.update(aux=torch.empty(m, n // 2, dtype=torch.bfloat16, device=dev),
                  aux2=torch.empty(m, n // 2, dtype=torch.bfloat16, device=dev))
    elif act == L.ACT_GEGLU_BWD:
        kw.update(aux_in=torch.randn(m, n, device=dev).to(torch.bfloat16),
                  aux_in2=torch.randn(m, n, device=dev).to(torch.bfloat16))
    C = Kn.gemm(A, B, **kw)
    L.gemm_path_counts(reset=True)
    for _ in range(30):    # back-to-back launches so the clock settles
        Kn.gemm(A, B, C=C, **kw)
    torch.cuda.synchronize()
    paths = L.gemm_path_counts(reset=True)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        Kn.gemm(A, B, C=C, **kw)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / 20 * 1e3
    buf = np.zeros((1024, 4, 64), dtype=np.uint32)
    assert lib.ptk_debug_p8_stamps_read(buf.ctypes.data, buf.nbytes) == 0
    ntile = ((m + 255) // 256) * ((n + 255) // 256)
    G = min(ntile, int(os.environ.get("PTK_GEMM_GRID", "256")))
    kt = k // 64
    rows = []
    for g in range(G):
        for s in range(64):
            st = buf[g, :, s].astype(np.int64)
            if st[0] == 0 and st[3] == 0:
                break
            d = lambda a, b: (st[b] - st[a]) & 0xffffffff
            rows.append((s, d(0, 1), d(1, 2), d(2, 3)))
    r = np.array(rows, dtype=np.int64)
    out = {"shape": name, "kernel": kern, "act": act, "M": m, "N": n, "K": k, "epi_mode": emode, "us": round(us, 1), "tiles": ntile,
           "paths": {f"{p}/{a}": c for (p, a), c in paths.items()},
           "rounds": round(ntile / 256, 2)}
    for s in range(int(r[:, 0].max()) + 1):
        x = r[r[:, 0] == s]
        out[f"seg{s}"] = {"n": int(len(x)), "first_ktile_cyc": int(np.median(x[:, 1])),
                          "rest_loop_cyc_per_ktile": round(float(np.median(x[:, 2])) / max(kt - 1, 1), 1),
                          "epilogue_issue_cyc": int(np.median(x[:, 3]))}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
