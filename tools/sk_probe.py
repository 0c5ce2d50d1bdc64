"""Determinism probe of the stream-K tail GEMM: repeated launches of one shape, which 256x256 tiles differ
between launches (data-parallel rounds vs tail tiles) and by how much."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from projectiontrainer_amd import kernels as K, _lib as L  # noqa: E402

dev = torch.device("cuda:0")
M, N, Kd = (int(x) for x in (sys.argv[1:4] if len(sys.argv) > 3 else (22528, 1536, 1152)))
tail = torch.zeros(L.lib().ptk_gemm_tail_scratch_bytes(), dtype=torch.uint8, device=dev)
A = torch.randn(M, Kd, device=dev).to(torch.bfloat16)
B = (torch.randn(N, Kd, device=dev) * 0.05).to(torch.bfloat16)
d = L.GemmDesc()
d.M, d.N, d.K, d.act, d.out = M, N, Kd, L.ACT_NONE, L.OUT_BF16
d.tail_ws = tail.data_ptr()
gs = L.lib().ptk_gemm_tail_split(d)
ref = (A.float() @ B.float().T)
outs = [K.gemm(A, B, tail_ws=tail) for _ in range(6)]
C0 = K.gemm(A, B)
torch.cuda.synchronize()
nbm, nbn = (M + 255) // 256, (N + 255) // 256
ntile = nbm * nbn
print("shape", M, N, Kd, "tiles", ntile, "split over", gs, "counters zero:", not tail[:16384].any().item())
for i, C in enumerate(outs):
    diff = (C.float() - outs[0].float()).abs()
    err = (C.float() - ref).abs().max().item()
    bad = []
    for bm in range(nbm):
        for bn in range(nbn):
            t = diff[bm * 256:(bm + 1) * 256, bn * 256:(bn + 1) * 256]
            if t.max().item() > 0:
                bad.append((bm, bn, round(t.max().item(), 4), int((t > 0).sum().item())))
    print(f"launch {i}: max|C-ref| {err:.4f}  tiles differing from launch 0: {len(bad)} {bad[:12]}")
print("unsplit max|C0-ref|", (C0.float() - ref).abs().max().item())
