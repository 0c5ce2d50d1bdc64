"""Same-process timing of named step GEMM shapes (tools/gemm_bench.py ALL) on the default dispatch:
python tools/gemm_ab.py g_gu g_dh_geglu_bwd g_down ...   (PTK_LIB selects a diagnostic build)"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import gemm_bench as gb  # noqa: E402

names = sys.argv[1:] or ["g_gu", "g_dh_geglu_bwd", "g_down", "g_qkv", "g_dgu", "sig_fc1", "proj_fc1"]
shapes = {s[0]: s for s in gb.ALL}
out = {}
for rnd in range(2):
    for n in names:
        r = gb.run(*shapes[n], reps=20)
        if rnd == 1:
            out[n] = r["TFLOPs"]
print(json.dumps({"lib": os.environ.get("PTK_LIB", "default"), **out}), flush=True)
