"""lm_head forward shape (4096 x 262144 x 1152, bf16 out) on each GEMM family, same process, interleaved:
mode 2 = 8-wave 256^2 (the default for this shape), 8 = persistent 4-wave, 32 = persistent 8-wave."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import gemm_bench as gb  # noqa: E402

L = gb.L
s = [x for x in gb.ALL if x[0] == "g_lm"][0]
res = {}
for rnd in range(3):
    for mode in (2, 8, 32):
        L.lib().ptk_gemm_force_small_tiles(mode)
        r = gb.run(*s, reps=10)
        if rnd:
            res.setdefault(mode, []).append(r["ms"])
L.lib().ptk_gemm_force_small_tiles(0)
print(json.dumps({f"mode{m}_ms": v for m, v in res.items()}), flush=True)
