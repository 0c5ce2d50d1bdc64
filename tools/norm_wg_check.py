"""Stage-2 weight grads of one micro-batch at cfg4's widths (2 SigLIP + 6 Gemma3 layers, bs 2, as
tests/test_stage2_gpu.py::test_stage2_architecture_scale_vs_oracle builds it), saved as raw bf16 bits so
two library builds (e.g. PTK_NORM_WG=0 / 1 of an A/B build) can be compared bit for bit.
usage: python tools/norm_wg_check.py OUT.npz           (PTK_LIB / PTK_* env select the build)
       python tools/norm_wg_check.py --compare A.npz B.npz"""
import os
import sys

import numpy as np

if sys.argv[1] == "--compare":
    a, b = np.load(sys.argv[2]), np.load(sys.argv[3])
    assert sorted(a.files) == sorted(b.files)
    diff = [k for k in a.files if not np.array_equal(a[k], b[k])]
    print(f"{len(a.files)} grads, {len(diff)} differ" + ("" if diff else " (bit-identical)"))

    def f32(x):   # raw bf16 bits -> float32
        return (x.astype(np.int32) << 16).view(np.float32)
    for k in diff:
        x, y = f32(a[k]), f32(b[k])
        print(f"  {k}: rel-L2 {np.linalg.norm(x - y) / max(np.linalg.norm(y), 1e-30):.3e}, "
              f"{np.count_nonzero(a[k] != b[k])} of {x.size} elements differ")
    sys.exit(0)

import torch  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import golden_util as G  # noqa: E402
from projectiontrainer_amd import weights as W  # noqa: E402
from projectiontrainer_amd.config import PRESETS  # noqa: E402
from projectiontrainer_amd.gemma3 import Gemma3CausalLM  # noqa: E402
from projectiontrainer_amd.projectors import MLPProjector  # noqa: E402
from projectiontrainer_amd.siglip import SiglipVisionTower  # noqa: E402
from projectiontrainer_amd.stage2 import Stage2Engine  # noqa: E402

gpu = torch.device("cuda:0")
cfg = PRESETS["cfg4"]
cfg = cfg.replace(vision=cfg.vision.__class__(**{**cfg.vision.__dict__, "num_hidden_layers": 2}),
                  text=cfg.text.__class__(**{**cfg.text.__dict__, "num_hidden_layers": 6}), batch_size=2)
vp = {k: G.bf16_round(v) for k, v in W.siglip_vision_params(cfg.vision, seed=3).items()}
lp = {k: G.bf16_round(v) for k, v in W.gemma3_params(cfg.text, seed=4).items()}
pp = {k: G.bf16_round(v) for k, v in W.projector_params(cfg.vision.hidden_size, cfg.text.hidden_size,
                                                        seed=5).items()}
px, q, a = W.synthetic_vqa_batch(cfg, seed=17, padding_side="left")
proj = MLPProjector(cfg.vision.hidden_size, cfg.text.hidden_size)
proj.load_state_dict({k: torch.from_numpy(v) for k, v in pp.items()})
proj.to(gpu)
eng = Stage2Engine(SiglipVisionTower(cfg.vision, vp, gpu),
                   Gemma3CausalLM(cfg.text, lp, gpu, max_pos=Gemma3CausalLM.seq_pad(cfg.seq_len)), proj,
                   learning_rate=1e-4, weight_decay=0.01, max_grad_norm=1.0, warmup_steps=0, total_steps=10,
                   pad_token_id=cfg.text.pad_token_id)
for _ in range(2):   # two micro-batches: the second accumulates into the first's bf16 grads
    loss = float(eng.forward_backward(*(torch.from_numpy(t).to(gpu) for t in (px, q, a))))
torch.cuda.synchronize()
grads = {k: v.contiguous().view(torch.int16).cpu().numpy() for k, v in eng.state.state_dict_hf(grads=True).items()}
np.savez(sys.argv[1], **grads)
print(f"loss {loss:.6f}, {len(grads)} grads -> {sys.argv[1]}")
