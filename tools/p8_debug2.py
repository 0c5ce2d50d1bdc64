"""Debug: p8 second-tile error structure at small K (which k-steps the wrong tiles accumulated)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from projectiontrainer_amd import kernels as K, _lib as L  # noqa: E402

dev = torch.device("cuda:0")
for (M, N, Kd) in [(4608, 4096, 128), (4608, 4096, 256), (4608, 4096, 384)]:
    g = torch.Generator(device="cpu").manual_seed(0)
    A = torch.randn(M, Kd, generator=g).to(dev).to(torch.bfloat16)
    B = (torch.randn(N, Kd, generator=g) * 0.05).to(dev).to(torch.bfloat16)
    L.lib().ptk_gemm_force_small_tiles(32)
    C = K.gemm(A, B, out_dtype=torch.float32)
    L.lib().ptk_gemm_force_small_tiles(0)
    torch.cuda.synchronize()
    Af, Bf = A.float(), B.float()
    ref = Af @ Bf.T
    bad = (C - ref).abs() > 1e-3
    print(M, N, Kd, "nbad", int(bad.sum()), flush=True)
    if not bad.any():
        continue
    nks = Kd // 32
    # a few bad tiles: explain C_tile as sum_k w_k * A_k B_k^T over the tile's own k-steps and the k-steps of other
    # tiles' rows/cols (same rows, any column tile) via least squares on the tile's own k-steps
    idx = bad.nonzero()
    shown = 0
    for r, c in idx[:: max(1, idx.shape[0] // 5)].tolist()[:5]:
        bm, bn = r // 256, c // 256
        rs, cs = slice(bm * 256, bm * 256 + 256), slice(bn * 256, bn * 256 + 256)
        parts = [Af[rs, 32 * k:32 * k + 32] @ Bf[cs, 32 * k:32 * k + 32].T for k in range(nks)]
        X = torch.stack([p.flatten() for p in parts], 1)
        y = C[rs, cs].flatten()
        w = torch.linalg.lstsq(X, y.unsqueeze(1)).solution.flatten()
        res = (X @ w - y).norm() / y.norm()
        # quadrant pattern of the error within the tile
        e = (C[rs, cs] - ref[rs, cs]).abs() > 1e-3
        quad = [[int(e[i * 128:(i + 1) * 128, j * 64:(j + 1) * 64].sum()) for j in range(4)] for i in range(2)]
        print(f"  tile ({bm},{bn}) own-k-step weights {[round(float(x), 3) for x in w]} resid {float(res):.3e} "
              f"bad per wave quadrant {quad}", flush=True)
