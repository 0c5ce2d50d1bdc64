"""Debug: graph_step after a reallocating eager step (tests/test_graph_gpu.py)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tests.test_graph_gpu import _engine  # noqa: E402
from projectiontrainer_amd import weights as W  # noqa: E402
from projectiontrainer_amd.config import PRESETS  # noqa: E402

gpu = torch.device("cuda:0")
cfg2, cfg4 = PRESETS["tiny"].replace(batch_size=2), PRESETS["tiny"].replace(batch_size=4)
b2 = [tuple(torch.from_numpy(a).to(gpu) for a in W.synthetic_batch(cfg2, seed=40 + s)) for s in range(3)]
b4 = tuple(torch.from_numpy(a).to(gpu) for a in W.synthetic_batch(cfg4, seed=50))
eager, graphed = _engine(cfg2, gpu), _engine(cfg2, gpu)
seq = [("e", b2[0]), ("g", b2[1]), ("e", b4), ("g", b2[2]), ("g", b2[0])]
for k, (mode, b) in enumerate(seq):
    le = float(eager.step(*b))
    lg = float(graphed.step(*b) if mode == "e" else graphed.graph_step(*b))
    torch.cuda.synchronize()
    print(k, mode, le, lg, "grad_eq", torch.equal(eager.proj.flat_grad, graphed.proj.flat_grad),
          "grad_nan", bool(graphed.proj.flat_grad.isnan().any()), "param_eq", torch.equal(eager.proj.flat, graphed.proj.flat),
          "param_nan", bool(graphed.proj.flat.isnan().any()), "exp_avg_nan", bool(graphed.exp_avg.isnan().any()),
          "gnorm", float(eager.grad_norm), float(graphed.grad_norm), flush=True)
