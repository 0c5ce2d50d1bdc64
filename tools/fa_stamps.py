"""Diagnostic: per-workgroup phase timing of the d-256 attention forward from in-kernel stamps
(build/libptk_fastamps.so, `make -C projectiontrainer_amd/csrc fastamps`), at the cfg2 step's shape.
Phases: 0 entry, 1 Q fragments + key masks, 2 first three K/V tiles landed + QK^T of the first tile,
3 main loop done, 4 epilogue stores issued.  Never used by tests or the bench."""
import ctypes
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from projectiontrainer_amd import _lib as L  # noqa: E402

L.LIB_PATH = os.path.join(ROOT, "build", "libptk_fastamps.so")
from projectiontrainer_amd import kernels as Kn  # noqa: E402

lib = L.lib()
lib.ptk_debug_fa_stamps_read.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
dev = torch.device("cuda:0")
B, S, G, D = 32, 704, 4, 256
window = int(sys.argv[1]) if len(sys.argv) > 1 else 512
g = torch.Generator(device=dev).manual_seed(0)
rnd = lambda *s: torch.randn(*s, device=dev, generator=g).to(torch.bfloat16)
Q, Kt, Vt = rnd(B, S * G, D), rnd(B, S, D), rnd(B, S, D)
kv = torch.ones(B, S, dtype=torch.int32, device=dev)
kv[:, S - 1] = 0
O = torch.zeros(B, S * G, D, dtype=torch.bfloat16, device=dev)
lse = torch.zeros(B, S * G, dtype=torch.float32, device=dev)
f = lambda: Kn.flash_attn(Q, Kt, Vt, O, lse=lse, ldq=D, ldk=D, ldo=D, strides=(S * G * D, 0, S * D, 0, S * G * D, 0),
                          rows=S * G, nkeys=S, head_dim=D, batch=B, batch_inner=1, zdiv=1, qdiv=G, causal=True,
                          window=window, key_valid=kv, scale=D ** -0.5)
for _ in range(200):
    f()
torch.cuda.synchronize()
nblk = B * ((S * G + 127) // 128)
buf = np.zeros((1 << 14, 8), dtype=np.uint64)
assert lib.ptk_debug_fa_stamps_read(buf.ctypes.data, buf.nbytes) == 0
s = buf[:nblk].astype(np.int64)
t0 = s[:, 0].min()
clk = np.median((s[:, 4] - s[:, 0]) / np.maximum(s[:, 6] - s[:, 5], 1)) * 100.0
ph = [s[:, i + 1] - s[:, i] for i in range(4)]
nt = s[:, 7]
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(20):
    f()
e1.record()
torch.cuda.synchronize()
print(json.dumps({"window": window, "us": round(e0.elapsed_time(e1) / 20 * 1e3, 1), "blocks": nblk,
                  "clock_MHz": round(float(clk), 1), "span_cyc": int(s[:, 4].max() - t0),
                  "q_mask_cyc_med": int(np.median(ph[0])), "first_tiles_cyc_med": int(np.median(ph[1])),
                  "loop_cyc_med": int(np.median(ph[2])), "epilogue_cyc_med": int(np.median(ph[3])),
                  "loop_cyc_per_tile_med": round(float(np.median(ph[2] / np.maximum(nt - 1, 1))), 1),
                  "tiles_med": int(np.median(nt)), "sum_block_cyc_per_cu": int((s[:, 4] - s[:, 0]).sum() / 256)}))
