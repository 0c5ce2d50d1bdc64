import os, sys, torch
sys.path.insert(0, os.getcwd())
from tests.test_kernels_gpu import _qknorm_rope_ref, rnd
from projectiontrainer_amd import kernels as Kn
gpu = torch.device("cuda:0")
B, S, Hq, Hkv, D, eps = 1, 8, 4, 1, 256, 1e-6
G = Hq // Hkv
qkv = rnd(B * S, (Hq + 2 * Hkv) * D, dev=gpu, seed=41, scale=2.0)
qw = torch.zeros(D, device=gpu); kw = torch.zeros(D, device=gpu)
inv = 1.0 / (10000.0 ** (torch.arange(0, D, 2, device=gpu, dtype=torch.float32) / D))
ang = torch.arange(S, device=gpu, dtype=torch.float32)[:, None] * inv[None]
cos_h, sin_h = ang.cos().contiguous(), ang.sin().contiguous()
Q, K, V, rq, rk = Kn.qknorm_rope(qkv, qw, kw, cos_h, sin_h, batch=B, seq=S, heads=Hq, kv_heads=Hkv, head_dim=D, eps=eps)
qr, kr, vr = _qknorm_rope_ref(qkv.float(), qw, kw, cos_h, sin_h, B, S, Hq, Hkv, D, eps)
Qr = qr.view(B, S, Hkv, G, D).permute(0, 2, 1, 3, 4)
err = (Q.float() - Qr).abs()
print("max err per (s, j):"); print(err.amax(-1)[0, 0])
s, j = 7, 3
print("kernel", Q[0, 0, s, j, :6].float().tolist(), Q[0, 0, s, j, 128:134].float().tolist())
print("ref   ", Qr[0, 0, s, j, :6].tolist(), Qr[0, 0, s, j, 128:134].tolist())
x = qkv.float().view(B, S, Hq + 2 * Hkv, D)[0, s, j]
xn = x * torch.rsqrt(x.pow(2).mean() + eps)
print("xn    ", xn[:6].tolist(), xn[128:134].tolist())
print("rstd k/r", rq[s, j].item(), torch.rsqrt(x.pow(2).mean() + eps).item())
