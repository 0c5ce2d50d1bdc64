"""GEMM dispatch census (kernel family, epilogue) of the full-depth cfg2 Stage-1 step per batch size:
which batch exercises every family the benchmarked bs-32 step launches (tests/test_stage1_gpu.py)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from projectiontrainer_amd import _lib as L  # noqa: E402
from projectiontrainer_amd import weights as W  # noqa: E402
from projectiontrainer_amd.config import PRESETS  # noqa: E402
from projectiontrainer_amd.stage1 import Stage1Engine  # noqa: E402

dev = torch.device("cuda:0")
ref = None
for bs in [int(x) for x in (sys.argv[1:] or ["32", "16", "18", "20", "23", "24", "26", "28", "30"])]:
    cfg = PRESETS["cfg2"].replace(batch_size=bs)
    eng = Stage1Engine.synthetic(cfg, dev, seed=0)
    px, ids, labels = W.synthetic_batch(cfg, seed=7, max_pad=40)
    args = [torch.from_numpy(t).to(dev) for t in (px, ids, labels)]
    eng.forward_backward(*args)
    L.gemm_path_counts(reset=True)
    eng.forward_backward(*args)
    torch.cuda.synchronize()
    got = set(L.gemm_path_counts(reset=True))
    if ref is None:
        ref = got
    print(bs, "missing vs first:", sorted(ref - got), "extra:", sorted(got - ref), flush=True)
    del eng
    torch.cuda.empty_cache()
