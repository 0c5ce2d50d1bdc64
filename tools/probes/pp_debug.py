"""Ping-pong GEMM debug: mismatch pattern of mode 32 vs mode 8 on small shapes (diagnostic only)."""
import os, sys
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from projectiontrainer_amd import _lib as L, kernels as K
dev = torch.device("cuda:0")
for (M, N, Kd) in [(256, 128, 640), (256, 256, 640), (512, 128, 640), (256, 128 * 3, 640), (256, 128, 1024)]:
    g = torch.Generator().manual_seed(0)
    A = torch.randn(M, Kd, generator=g).to(dev).to(torch.bfloat16)
    B = (torch.randn(N, Kd, generator=g) * 0.05).to(dev).to(torch.bfloat16)
    ref = A.float() @ B.float().T
    L.lib().ptk_gemm_force_small_tiles(32)
    C = K.gemm(A, B, out_dtype=torch.float32)
    torch.cuda.synchronize()
    L.lib().ptk_gemm_force_small_tiles(0)
    bad = ((C - ref).abs() > 1e-3 * ref.abs().max()).nonzero()
    print(M, N, Kd, "bad", bad.shape[0], "of", C.numel(), flush=True)
    if bad.shape[0]:
        rows = sorted(set(bad[:, 0].tolist())); cols = sorted(set(bad[:, 1].tolist()))
        print("  rows", len(rows), rows[:40])
        print("  cols", len(cols), cols[:64])
        r, c = bad[0].tolist()
        # is the wrong value equal to some other element / a partial sum?
        print("  C", C[r, c].item(), "ref", ref[r, c].item())
        for kk in range(0, Kd, 32):
            part = (A[r, :kk + 32].float() @ B[c, :kk + 32].float()).item()
            if abs(part - C[r, c].item()) < 1e-3 * max(1, abs(part)):
                print("  equals partial sum through k", kk + 32)
