"""One Stage-1 forward/backward at architecture-true Gemma3-1B dims (bs 2, S 703, 2 layers: one sliding-window and
one full-attention layer, so both dK/dV split plans run), results
saved to argv[1]. Run by tests/test_dkv_fused_gpu.py under PTK_DKV_REDUCE_SPLIT=0/1 and tests/test_ce_stats_gpu.py
under PTK_CE_TWO_PASS=0/1 (each switch is read
once per process, so each setting needs its own process)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from projectiontrainer_amd import weights as W  # noqa: E402
from projectiontrainer_amd.config import PRESETS  # noqa: E402
from projectiontrainer_amd.gemma3 import Gemma3CausalLM  # noqa: E402
from projectiontrainer_amd.projectors import MLPProjector  # noqa: E402
from projectiontrainer_amd.siglip import SiglipVisionTower  # noqa: E402
from projectiontrainer_amd.stage1 import Stage1Engine  # noqa: E402


def main(out_path):
    gpu = torch.device("cuda:0")
    cfg = PRESETS["cfg2"]
    cfg = cfg.replace(vision=cfg.vision.__class__(**{**cfg.vision.__dict__, "num_hidden_layers": 1}),
                      text=cfg.text.__class__(**{**cfg.text.__dict__, "num_hidden_layers": 2,
                                                          "sliding_window_pattern": 2}),
                      batch_size=2, text_len=128)
    vp = W.siglip_vision_params(cfg.vision, seed=3)
    lp = W.gemma3_params(cfg.text, seed=4)
    pp = W.projector_params(cfg.vision.hidden_size, cfg.text.hidden_size, seed=5)
    px, ids, labels = W.synthetic_batch(cfg, seed=7, max_pad=40)
    proj = MLPProjector(cfg.vision.hidden_size, cfg.text.hidden_size)
    proj.load_state_dict({k: torch.from_numpy(v) for k, v in pp.items()})
    proj.to(gpu)
    eng = Stage1Engine(SiglipVisionTower(cfg.vision, vp, gpu),
                       Gemma3CausalLM(cfg.text, lp, gpu, max_pos=Gemma3CausalLM.seq_pad(cfg.seq_len)), proj,
                       gradient_accumulation_steps=1)
    loss = eng.forward_backward(torch.from_numpy(px).to(gpu), torch.from_numpy(ids).to(gpu),
                                torch.from_numpy(labels).to(gpu))
    torch.cuda.synchronize()
    torch.save({"loss": torch.as_tensor(float(loss)), "dx": eng.dx.cpu(),
                "grads": [g.cpu() for g in eng.proj.grads()]}, out_path)


if __name__ == "__main__":
    main(sys.argv[1])
