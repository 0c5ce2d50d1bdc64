"""Time Stage 2's validation generate (Stage2/trainer.py:596-626) on the stepwise decode: Gemma3-1B (26 layers,
random-init), B prompts of 575 projected image tokens + a 64-token question (left-padded by 0..15), num_beams 3,
do_sample, top_k 50, top_p 0.9, max_new_tokens N (no EOS, so every step runs).  Prints the new tokens per second
(B x N) and the per-step time.   usage: python tools/beam_bench.py [B] [N]"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from projectiontrainer_amd.config import PRESETS  # noqa: E402
from projectiontrainer_amd.gemma3 import Gemma3CausalLM  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 16
N = int(sys.argv[2]) if len(sys.argv) > 2 else 128
dev = torch.device("cuda:0")
cfg = PRESETS["cfg2"].text
lm = Gemma3CausalLM.random_init(cfg, dev, seed=1, max_pos=1280)
P = 575 + 64
x = torch.randn(B, P, cfg.hidden_size, device=dev)
mask = torch.ones(B, P, dtype=torch.int32, device=dev)
for b in range(B):
    mask[b, 575:575 + (b % 16)] = 0
lm.beam_generate(x, mask, num_beams=3, max_new_tokens=4, do_sample=True, top_k=50, top_p=0.9)
torch.cuda.synchronize()
res = []
for rep in range(2):
    t0 = time.perf_counter()
    out = lm.beam_generate(x, mask, num_beams=3, max_new_tokens=N, do_sample=True, top_k=50, top_p=0.9, seed=rep)
    torch.cuda.synchronize()
    res.append(time.perf_counter() - t0)
s = min(res)
print(json.dumps({"what": "Stage-2 validation generate, beam sample (3 beams, top_k 50, top_p 0.9), Gemma3-1B, "
                          "prompt 575 + 64", "batch": B, "new_tokens": N, "seconds": round(s, 4),
                  "ms_per_step": round(s / N * 1e3, 3), "tokens_per_s": round(B * N / s, 1),
                  "returned": list(out.shape)}))
