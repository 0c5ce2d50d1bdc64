"""Time the persistent 4-wave GEMM on the Stage-1 GEGLU shapes (gate|up with the GEGLU epilogue, dh with the
GEGLU-backward epilogue) and the plain down / o projections, HIP events around 20 launches each, one JSON line
per shape.  Diagnostic switches are read from the environment by the library (e.g. PTK_W4_STAGGER), so run
one process per setting:  for s in 0 8 16; do PTK_W4_STAGGER=$s python tools/w4_probe.py; done"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from projectiontrainer_amd import kernels as K, _lib as L  # noqa: E402

dev = torch.device("cuda:0")
M = 32 * 704


def timed(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def main():
    L.lib().ptk_gemm_force_small_tiles(8)   # the persistent kernel for every shape below
    X = torch.randn(M, 1152, device=dev).to(torch.bfloat16)
    Wgu = (torch.randn(13824, 1152, device=dev) * 0.03).to(torch.bfloat16)
    g = torch.empty(M, 6912, dtype=torch.bfloat16, device=dev)
    u = torch.empty_like(g)
    h = torch.empty_like(g)
    us = timed(lambda: K.gemm(X, Wgu, C=h, act=L.ACT_GEGLU, aux=g, aux2=u))
    out = {"stagger": os.environ.get("PTK_W4_STAGGER", "0"), "gate_up_us": round(us, 1),
           "gate_up_TF": round(2 * M * 13824 * 1152 / us / 1e6, 1)}
    dY = torch.randn(M, 1152, device=dev).to(torch.bfloat16)
    WdT = (torch.randn(6912, 1152, device=dev) * 0.03).to(torch.bfloat16)
    dgu = torch.empty(M, 13824, dtype=torch.bfloat16, device=dev)
    us = timed(lambda: K.gemm(dY, WdT, C=dgu, act=L.ACT_GEGLU_BWD, aux_in=g, aux_in2=u))
    out.update(dh_us=round(us, 1), dh_TF=round(2 * M * 6912 * 1152 / us / 1e6, 1))
    Wd = (torch.randn(1152, 6912, device=dev) * 0.03).to(torch.bfloat16)
    y = torch.empty(M, 1152, dtype=torch.bfloat16, device=dev)
    us = timed(lambda: K.gemm(h, Wd, C=y))
    out.update(down_us=round(us, 1), down_TF=round(2 * M * 6912 * 1152 / us / 1e6, 1))
    L.lib().ptk_gemm_force_small_tiles(0)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
