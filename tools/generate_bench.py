"""Time the KV-cache decode (ptk_gemma3_generate) at the Stage-1 validation shape: Gemma3-1B (26 layers,
random-init), batch B, prompt of 575 projected patch embeddings, 64 new tokens sampled (top-k 50, temperature 1),
as Stage1/projector_trainer.py:386-393 calls generate.  Prints new tokens per second (all rows).
usage: python tools/generate_bench.py [B] [max_new_tokens]"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from projectiontrainer_amd.config import PRESETS  # noqa: E402
from projectiontrainer_amd.gemma3 import Gemma3CausalLM  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
NT = int(sys.argv[2]) if len(sys.argv) > 2 else 64
dev = torch.device("cuda:0")
cfg = PRESETS["cfg2"].text
lm = Gemma3CausalLM.random_init(cfg, dev, seed=1, max_pos=704)
x = torch.randn(B, 575, cfg.hidden_size, device=dev)
lm.generate(x, max_new_tokens=4, do_sample=True)
torch.cuda.synchronize()
res = []
for rep in range(3):
    t0 = time.perf_counter()
    ids = lm.generate(x, max_new_tokens=NT, do_sample=True, seed=rep)
    torch.cuda.synchronize()
    res.append(time.perf_counter() - t0)
s = min(res)
print(json.dumps({"what": "generate (KV-cache decode), Gemma3-1B, prompt 575", "batch": B, "new_tokens": NT,
                  "seconds": round(s, 4), "ms_per_step": round(s / NT * 1e3, 3),
                  "tokens_per_s": round(B * NT / s, 1), "returned": list(ids.shape)}))
