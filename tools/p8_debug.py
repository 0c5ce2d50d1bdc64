"""Debug: where p8 (mode 32) differs from w4 (mode 8)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from projectiontrainer_amd import kernels as K, _lib as L  # noqa: E402

dev = torch.device("cuda:0")
for (M, N, Kd) in [(22528, 1152, 1152), (4608, 13824, 1152), (2048, 2048, 1152), (512, 256, 1152), (1024, 256, 128),
                   (768, 256, 256)]:
    g = torch.Generator(device="cpu").manual_seed(0)
    A = torch.randn(M, Kd, generator=g).to(dev).to(torch.bfloat16)
    B = (torch.randn(N, Kd, generator=g) * 0.05).to(dev).to(torch.bfloat16)
    out = []
    for md in (8, 32):
        L.lib().ptk_gemm_force_small_tiles(md)
        out.append(K.gemm(A, B, out_dtype=torch.float32))
    L.lib().ptk_gemm_force_small_tiles(0)
    torch.cuda.synchronize()
    ref = A.float() @ B.float().T
    d = (out[0] - out[1]).abs()
    bad = d > 1e-3
    print(M, N, Kd, "w4-ref", float((out[0] - ref).abs().max()), "p8-ref", float((out[1] - ref).abs().max()),
          "nbad", int(bad.sum()), flush=True)
    if bad.any():
        nbm, nbn = (M + 255) // 256, (N + 255) // 256
        tb = bad[: nbm * 256 if M >= nbm * 256 else M]
        tiles = set()
        idx = bad.nonzero()
        for r, c in idx[:200000:997].tolist():
            tiles.add((r // 256, c // 256))
        print("  bad tiles (sample):", sorted(tiles)[:40], flush=True)
        sub = bad.float()
        rq = [float(sub[r::256].sum()) for r in (0, 64, 128, 192)]
        cq = [float(sub[:, c::256].sum()) for c in (0, 32, 64, 96, 128, 160, 192, 224)]
        print("  rows mod 256 at 0/64/128/192:", rq, " cols mod 256 step 32:", cq, flush=True)
        rr = bad.any(1).nonzero().flatten()
        print("  first bad rows", rr[:10].tolist(), "bad row count", int(rr.numel()), flush=True)
