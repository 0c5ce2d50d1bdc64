"""Debug: which graph_step sequences give NaN grads (tests/test_graph_gpu.py)."""
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
V = {
    "V6_realloc_recapture": [("e", b2[0]), ("g", b2[1]), ("e", b4), ("g", b2[2]), ("g", b2[0]), ("g", b2[1])],
    "V7_key_recapture": [("e", b2[0]), ("g", b2[1]), ("rekey", None), ("g", b2[2]), ("g", b2[0]), ("g", b2[1])],
    "V1_forced_recapture": [("e", b2[0]), ("g", b2[1]), ("reset", None), ("g", b2[2]), ("g", b2[0]), ("g", b2[1])],
    "V2_realloc_first": [("e", b2[0]), ("e", b4), ("g", b2[1]), ("g", b2[2]), ("g", b2[0])],
    "V3_bs4_then_bs2": [("e", b4), ("g", b2[1]), ("g", b2[2]), ("g", b2[0])],
    "V4_same_bs_replays": [("e", b2[0]), ("g", b2[1]), ("g", b2[2]), ("g", b2[0]), ("g", b2[1])],
    "V5_bs4_graph": [("e", b4), ("g", b4), ("g", b4), ("g", b4)],
}
for name, seq in V.items():
    eager, graphed = _engine(cfg2, gpu), _engine(cfg2, gpu)
    out = []
    for k, (mode, b) in enumerate(seq):
        if mode == "reset":
            graphed._graph = None
            continue
        if mode == "rekey":
            graphed._graph_key = None
            continue
        le = float(eager.step(*b))
        lg = float(graphed.step(*b) if mode == "e" else graphed.graph_step(*b))
        torch.cuda.synchronize()
        torch.cuda.synchronize()   # (graph_step destroys a replaced graph; PTK_HIP_MEMSET=1 brings back the
                                   # memset nodes whose graphs broke after such a destroy)
        out.append(f"{mode}{b[1].shape[0]}:{'ok' if torch.equal(eager.proj.flat_grad, graphed.proj.flat_grad) else ('NAN' if graphed.proj.flat_grad.isnan().any() else 'diff')}")
    print(name, " ".join(out), flush=True)
