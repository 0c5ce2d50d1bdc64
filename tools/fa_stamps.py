"""Diagnostic: per-workgroup phase timing of the d-256 attention kernels from in-kernel stamps
(build/libptk_fastamps.so, `make -C projectiontrainer_amd/csrc fastamps`), at the cfg2 step's shape.
Forward / dQ phases: 0 entry, 1 Q (dO, O) fragments + key masks, 2 first three K/V tiles landed + the first
tile's MFMAs, 3 main loop done, 4 epilogue stores issued.  dK/dV: 1 = 2 K/V fragments loaded, 3 chunk loop
done, 4 outputs stored.  usage: fa_stamps.py [window] [fwd|bwd|fwd64] (fwd64: SigLIP's
d-64 forward, stamps 1 Q + masks, 2 first two tiles staged, 3 loop done).  Never used by tests or the bench."""
import ctypes
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from projectiontrainer_amd import _lib as L  # noqa: E402

L.LIB_PATH = os.environ.get("FA_STAMPS_LIB", os.path.join(ROOT, "ablibs", "libptk_fastamps.so"))   # make ablib AB_NAME=fastamps AB_SRC=flash.hip AB_DEFS=-DPTK_FA_STAMPS
from projectiontrainer_amd import kernels as Kn  # noqa: E402

lib = L.lib()
lib.ptk_debug_fa_stamps_read.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
dev = torch.device("cuda:0")
B, S, G, D = 32, 704, 4, 256
if len(sys.argv) > 2 and sys.argv[2] == "fwd64":   # SigLIP: 32 images x 16 heads, 576 patches, d 64, no mask
    B, S, G, D = 512, 576, 1, 64
window = int(sys.argv[1]) if len(sys.argv) > 1 else 512
what = sys.argv[2] if len(sys.argv) > 2 else "fwd"
g = torch.Generator(device=dev).manual_seed(0)
rnd = lambda *s: torch.randn(*s, device=dev, generator=g).to(torch.bfloat16)
Q, Kt, Vt = rnd(B, S * G, D), rnd(B, S, D), rnd(B, S, D)
kv = torch.ones(B, S, dtype=torch.int32, device=dev)
kv[:, S - 1] = 0
O = torch.zeros(B, S * G, D, dtype=torch.bfloat16, device=dev)
lse = torch.zeros(B, S * G, dtype=torch.float32, device=dev)
f = lambda: Kn.flash_attn(Q, Kt, Vt, O, lse=lse, ldq=D, ldk=D, ldo=D, strides=(S * G * D, 0, S * D, 0, S * G * D, 0),
                          rows=S * G, nkeys=S, head_dim=D, batch=B, batch_inner=1, zdiv=1, qdiv=G,
                          causal=what != "fwd64", window=window if what != "fwd64" else 0,
                          key_valid=kv if what != "fwd64" else None, scale=D ** -0.5)
f()
if what == "bwd":
    dO = rnd(B, S * G, D)
    fw = f
    f = lambda: Kn.flash_attn_bwd(Q, Kt, Vt, O, dO, lse, sO=(S * G * D, 0), rows=S * G, nkeys=S, head_dim=D, batch=B,
                                  batch_inner=1, zdiv=1, qdiv=G, causal=True, window=window, key_valid=kv,
                                  scale=D ** -0.5)
for _ in range(100):
    f()
torch.cuda.synchronize()
buf = np.zeros((4, 1 << 13, 8), dtype=np.uint64)
assert lib.ptk_debug_fa_stamps_read(buf.ctypes.data, buf.nbytes) == 0


def summary(s, name):
    s = s[s[:, 0] > 0].astype(np.int64)
    t0 = s[:, 0].min()
    clk = np.median((s[:, 4] - s[:, 0]) / np.maximum(s[:, 6] - s[:, 5], 1)) * 100.0
    ph = [s[:, i + 1] - s[:, i] for i in range(4)]
    nt = s[:, 7]
    return {"kernel": name, "blocks": len(s), "clock_MHz": round(float(clk), 1),
            "span_cyc": int(s[:, 4].max() - t0),
            "prologue_cyc_med": int(np.median(ph[0])), "first_tiles_cyc_med": int(np.median(ph[1])),
            "loop_cyc_med": int(np.median(ph[2])), "epilogue_cyc_med": int(np.median(ph[3])),
            "loop_cyc_per_tile_med": round(float(np.median(ph[2] / np.maximum(nt - 1, 1))), 1),
            "tiles_med": int(np.median(nt)), "sum_block_cyc_per_cu": int((s[:, 4] - s[:, 0]).sum() / 256)}


e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(20):
    f()
e1.record()
torch.cuda.synchronize()
print(json.dumps({"what": what, "window": window, "us": round(e0.elapsed_time(e1) / 20 * 1e3, 1)}))
for kid, name in {"fwd": ((0, "fwd"),), "fwd64": ((3, "fwd64"),)}.get(what, ((1, "dq"), (2, "dkv"))):
    print(json.dumps(summary(buf[kid], name)))
