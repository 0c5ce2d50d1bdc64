"""Per-K-tile rate of the TN weight-grad kernel vs the 8-wave NT kernel on the same GEMM sizes (HIP events, one process)."""
import json, os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from projectiontrainer_amd import kernels as K, _lib as L

dev = torch.device("cuda:0")


def t_ms(fn, reps):
    fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


SIZES = [(8192, 8192, 8192), (4096, 4096, 16384), (12800, 1280, 13824), (6400, 6400, 1152)]
if len(sys.argv) > 1:   # e.g. 8192,8192,8192 (profiling passes: one size)
    SIZES = [tuple(int(v) for v in a.split(",")) for a in sys.argv[1:]]
for M, N, Kd in SIZES:
    # NT: C[M,N] = A[M,K] B[N,K]^T on the 8-wave kernel;  TN: grad[M,N] += dY[K,M]^T X[K,N] (one slice, no slab)
    A = torch.randn(M, Kd, device=dev).bfloat16()
    B = (torch.randn(N, Kd, device=dev) * 0.05).bfloat16()
    C = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
    dy = torch.randn(Kd, M, device=dev).bfloat16()
    x = (torch.randn(Kd, N, device=dev) * 0.05).bfloat16()
    g = torch.zeros(M, N, dtype=torch.bfloat16, device=dev)
    reps = max(3, int(3e12 / (2.0 * M * N * Kd)))
    L.lib().ptk_gemm_force_small_tiles(32)
    nt = min(t_ms(lambda: K.gemm(A, B, C=C), reps) for _ in range(3))
    L.lib().ptk_gemm_force_small_tiles(0)
    tn = min(t_ms(lambda: K.weight_grad(dy, x, g, mode=2), reps) for _ in range(3))
    tiles = ((M + 255) // 256) * ((N + 255) // 256)
    rounds = (tiles + 255) // 256
    kt = Kd // 64
    print(json.dumps({"M": M, "N": N, "K": Kd, "tiles": tiles, "rounds": rounds, "nt_us": round(nt * 1e3, 1),
                      "tn_us": round(tn * 1e3, 1), "nt_us_per_ktile_round": round(nt * 1e3 / (rounds * kt), 3),
                      "tn_us_per_ktile_round": round(tn * 1e3 / (rounds * kt), 3)}), flush=True)
    del A, B, C, dy, x, g
    torch.cuda.empty_cache()
