"""Which tiles of a TN stream-K weight grad differ from fp32 (debug probe)."""
import sys, os
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from projectiontrainer_amd import kernels as K, _lib as L

dev = torch.device("cuda:0")
G = torch.cuda.get_device_properties(dev).multi_processor_count
for Ny, Nx, rows in [(1536, 1152, 14336), (1152, 1024, 14336), (1024, 1024, 14336), (1280, 1024, 14336),
                     (1152, 1152, 14336)]:
    g = torch.Generator(device="cpu").manual_seed(0)
    dy = (torch.randn(rows, Ny, generator=g)).to(dev).bfloat16()
    x = (torch.randn(rows, Nx, generator=g) * 0.05).to(dev).bfloat16()
    g0 = torch.zeros(Ny, Nx, dtype=torch.bfloat16, device=dev)
    part = torch.empty(max(G * 2 * 8 * 8192, 8 * Ny * Nx), dtype=torch.float32, device=dev)
    out = K.weight_grad(dy, x, g0.clone(), part=part, mode=2)
    ref = (dy.float().t() @ x.float())
    torch.cuda.synchronize()
    err = (out.float() - ref).abs()
    tol = 0.02 * ref.abs().max().item()
    nbm, nbn = (Ny + 255) // 256, (Nx + 255) // 256
    bad = []
    for bm in range(nbm):
        for bn in range(nbn):
            e = err[bm * 256:(bm + 1) * 256, bn * 256:(bn + 1) * 256]
            if e.max().item() > tol:
                # which 128x64 wave sub-tiles
                sub = [(wr, c) for wr in range(2) for c in range(4)
                       if e[wr * 128:(wr + 1) * 128, c * 64:(c + 1) * 64].numel() and
                       e[wr * 128:(wr + 1) * 128, c * 64:(c + 1) * 64].max().item() > tol]
                bad.append((bm, bn, round(e.max().item(), 2), sub))
    print(f"Ny {Ny} Nx {Nx}: tiles {nbm}x{nbn}, bad {len(bad)}: {bad[:12]}", flush=True)
