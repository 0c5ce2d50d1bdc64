"""GEMM dispatch census (kernel family, epilogue) per batch size for the two configs whose parity tests must
run the benchmarked dispatch: Stage 2 at cfg4 (bs 16: one micro-batch's forward, backward
and weight grads) and Stage 1 at cfg5 (bs 16, T 256).  The first batch in each list is the benchmarked one;
the dispatch depends on the token-row count, not on depth, so the probes run 2 SigLIP + 6 Gemma layers.
usage: python tools/census_probe2.py [stage2|cfg5] [bs ...]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from projectiontrainer_amd import _lib as L  # noqa: E402
from projectiontrainer_amd import weights as W  # noqa: E402
from projectiontrainer_amd.config import PRESETS  # noqa: E402

dev = torch.device("cuda:0")
which = sys.argv[1] if len(sys.argv) > 1 else "stage2"
sizes = [int(x) for x in sys.argv[2:]] or [16, 2, 4, 6, 8, 10, 12, 14]


def shallow(cfg, bs):
    return cfg.replace(vision=cfg.vision.__class__(**{**cfg.vision.__dict__, "num_hidden_layers": 2}),
                       text=cfg.text.__class__(**{**cfg.text.__dict__, "num_hidden_layers": 6}), batch_size=bs)


ref = None
for bs in sizes:
    if which == "stage2":
        from projectiontrainer_amd.stage2 import synthetic_engine
        cfg = shallow(PRESETS["cfg4"], bs)
        eng = synthetic_engine(cfg, dev, seed=0, total_steps=10)
        args = [torch.from_numpy(t).to(dev) for t in W.synthetic_vqa_batch(cfg, seed=17, padding_side="left")]
    else:
        from projectiontrainer_amd.stage1 import Stage1Engine
        cfg = shallow(PRESETS["cfg5"], bs)
        eng = Stage1Engine.synthetic(cfg, dev, seed=0)
        args = [torch.from_numpy(t).to(dev) for t in W.synthetic_batch(cfg, seed=7, max_pad=40)]
    eng.forward_backward(*args)
    L.gemm_path_counts(reset=True)
    eng.forward_backward(*args)
    torch.cuda.synchronize()
    got = set(L.gemm_path_counts(reset=True))
    if ref is None:
        ref = got
        print(which, bs, "census:", sorted(got), flush=True)
    print(which, bs, "missing vs first:", sorted(ref - got), "extra:", sorted(got - ref), flush=True)
    del eng
    torch.cuda.empty_cache()
