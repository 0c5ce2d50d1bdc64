"""Worker bodies for the world-size-2 tests (spawned by tests/test_dist.py)."""
import os

import numpy as np
import torch
import torch.distributed as dist


def _init(rank, world, port, backend):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK="0")
    dist.init_process_group(backend, rank=rank, world_size=world)


def oracle_ddp(rank, world, port, out_dir):
    """CPU/gloo: per-rank oracle grads on the rank's half batch -> allreduce_grads_
    (the engine's collective) -> clip + AdamW (oracle); dump flat grads/params."""
    _init(rank, world, port, "gloo")
    torch.set_num_threads(2)
    from oracle import stage1_ref as R
    from projectiontrainer_amd import dist as D
    from projectiontrainer_amd import weights as W
    from projectiontrainer_amd.config import PRESETS
    cfg = PRESETS["tiny"].replace(batch_size=4)
    vp, lp = W.siglip_vision_params(cfg.vision), W.gemma3_params(cfg.text)
    pp = W.projector_params(cfg.vision.hidden_size, cfg.text.hidden_size)
    px, ids, labels = W.synthetic_batch(cfg, seed=21)
    sl = slice(2 * rank, 2 * rank + 2)
    st = R.init_state(pp)
    params = {k: v.clone().requires_grad_(True) for k, v in st.params.items()}
    loss, _, _ = R.stage1_forward_loss(vp, cfg.vision, lp, cfg.text, params, *(torch.as_tensor(t[sl])
                                                                                for t in (px, ids, labels)))
    loss.backward()
    flat = torch.cat([params[k].grad.reshape(-1) for k in pp])
    scale = D.allreduce_grads_(flat, world)
    np.save(os.path.join(out_dir, f"grad{rank}.npy"), (flat * scale).numpy())
    dist.destroy_process_group()


def engine_ddp(rank, world, port, out_dir):
    """GPU/gloo on one device: the real Stage1Engine with world_size 2."""
    _init(rank, world, port, "gloo")
    from projectiontrainer_amd import weights as W
    from projectiontrainer_amd.config import PRESETS
    from projectiontrainer_amd.gemma3 import Gemma3CausalLM
    from projectiontrainer_amd.projectors import MLPProjector
    from projectiontrainer_amd.siglip import SiglipVisionTower
    from projectiontrainer_amd.stage1 import Stage1Engine
    dev = torch.device("cuda:0")
    cfg = PRESETS["tiny"].replace(batch_size=4)
    vp, lp = W.siglip_vision_params(cfg.vision), W.gemma3_params(cfg.text)
    pp = W.projector_params(cfg.vision.hidden_size, cfg.text.hidden_size)
    px, ids, labels = W.synthetic_batch(cfg, seed=21)
    proj = MLPProjector(cfg.vision.hidden_size, cfg.text.hidden_size)
    proj.load_state_dict({k: torch.from_numpy(v) for k, v in pp.items()})
    proj.to(dev)
    eng = Stage1Engine(SiglipVisionTower(cfg.vision, vp, dev),
                       Gemma3CausalLM(cfg.text, lp, dev, max_pos=Gemma3CausalLM.seq_pad(cfg.seq_len)), proj,
                       world_size=world, total_steps=10)
    sl = slice(2 * rank, 2 * rank + 2)
    eng.step(*(torch.from_numpy(t[sl]).to(dev) for t in (px, ids, labels)))
    torch.cuda.synchronize()
    np.save(os.path.join(out_dir, f"grad{rank}.npy"), eng.proj.flat_grad.cpu().numpy())
    np.save(os.path.join(out_dir, f"param{rank}.npy"), eng.proj.flat.cpu().numpy())
    np.save(os.path.join(out_dir, f"sched{rank}.npy"), np.array([eng.sched_step, eng.last_lr]))
    dist.destroy_process_group()
