"""Debug the d-256 attention forward: per-row error against torch at small shapes."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from projectiontrainer_amd import kernels as Kn  # noqa: E402

dev = torch.device("cuda:0")
torch.manual_seed(0)
for S, causal, kind in [(32, False, "randn"), (64, False, "randn"), (64, True, "randn"), (32, False, "ones_v"), (128, True, "randn")]:
    B, G, D = 1, 1, 256
    Q = torch.randn(B, S * G, D, device=dev).to(torch.bfloat16)
    Kt = torch.randn(B, S, D, device=dev).to(torch.bfloat16)
    Vt = torch.randn(B, S, D, device=dev).to(torch.bfloat16)
    if kind == "ones_v":
        Vt = torch.ones_like(Vt)
    O = torch.zeros(B, S * G, D, dtype=torch.bfloat16, device=dev)
    lse = torch.zeros(B, S * G, dtype=torch.float32, device=dev)
    Kn.flash_attn(Q, Kt, Vt, O, lse=lse, ldq=D, ldk=D, ldo=D, strides=(S * G * D, 0, S * D, 0, S * G * D, 0),
                  rows=S * G, nkeys=S, head_dim=D, batch=B, batch_inner=1, zdiv=1, qdiv=G, causal=causal,
                  window=0, key_valid=None, scale=D ** -0.5)
    s = (Q.float() @ Kt.float().transpose(1, 2)) * D ** -0.5
    if causal:
        i = torch.arange(S, device=dev)
        s = s.masked_fill(~(i[None, :] <= i[:, None]), float("-inf"))
    ref = torch.softmax(s, -1) @ Vt.float()
    lref = torch.logsumexp(s, -1)
    err = (O.float() - ref).abs().amax(-1)[0]
    lerr = (lse - lref).abs()[0]
    print(S, causal, kind, "max err", float(err.max()), "lse err", float(lerr.max()))
    print("  rows with err > 0.05:", [int(x) for x in torch.nonzero(err > 0.05).flatten()[:40]])
    print("  lse rows err > 1e-2:", [int(x) for x in torch.nonzero(lerr > 1e-2).flatten()[:40]])
    bad = torch.nonzero(err > 0.05).flatten()
    if len(bad):
        r = int(bad[0])
        d = (O.float() - ref)[0, r]
        print("  row", r, "err by d (first 64):", [round(float(x), 2) for x in d[:64]])
