"""Data-parallel path (world size 2).  The reference uses DDP: each rank's
projector grads are the gradient of its own mean loss and DDP averages them
(Stage1/projector_trainer.py:237); the scheduler advances num_processes times
per optimizer step (ACC/scheduler.py:69-82)."""
import socket
import tempfile

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from tests import dist_worker


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_shard_batches_partition():
    from projectiontrainer_amd.dist import shard_batches
    for n, bs, world in ((10, 3, 2), (64, 8, 4), (7, 2, 3)):
        parts = [shard_batches(n, bs, r, world, epoch=1) for r in range(world)]
        allidx = torch.cat([torch.cat(p) for p in parts if p]).tolist()
        assert sorted(allidx) == list(range(n))
        counts = [len(p) for p in parts]
        assert max(counts) - min(counts) <= 1
    # deterministic per epoch, different across epochs
    assert torch.equal(torch.cat(shard_batches(20, 4, 0, 1, 0)), torch.cat(shard_batches(20, 4, 0, 1, 0)))
    assert not torch.equal(torch.cat(shard_batches(20, 4, 0, 1, 0)), torch.cat(shard_batches(20, 4, 0, 1, 1)))


def test_ddp_grad_average_gloo_cpu():
    """2 gloo ranks on CPU: all-reduced grads == mean of the per-rank (per-half-batch) grads."""
    from oracle import stage1_ref as R
    from projectiontrainer_amd import weights as W
    from projectiontrainer_amd.config import PRESETS
    with tempfile.TemporaryDirectory() as td:
        mp.spawn(dist_worker.oracle_ddp, args=(2, _port(), td), nprocs=2, join=True)
        g0, g1 = np.load(f"{td}/grad0.npy"), np.load(f"{td}/grad1.npy")
    np.testing.assert_array_equal(g0, g1)
    cfg = PRESETS["tiny"].replace(batch_size=4)
    vp, lp = W.siglip_vision_params(cfg.vision), W.gemma3_params(cfg.text)
    pp = W.projector_params(cfg.vision.hidden_size, cfg.text.hidden_size)
    px, ids, labels = W.synthetic_batch(cfg, seed=21)
    gs = []
    for r in range(2):
        sl = slice(2 * r, 2 * r + 2)
        params = {k: torch.as_tensor(v).clone().requires_grad_(True) for k, v in pp.items()}
        loss, _, _ = R.stage1_forward_loss(vp, cfg.vision, lp, cfg.text, params,
                                           *(torch.as_tensor(t[sl]) for t in (px, ids, labels)))
        loss.backward()
        gs.append(torch.cat([params[k].grad.reshape(-1) for k in pp]).numpy())
    np.testing.assert_allclose(g0, (gs[0] + gs[1]) / 2, rtol=1e-5, atol=1e-9)


@pytest.mark.gpu
def test_engine_ddp_two_ranks_one_gpu(gpu):
    """The real Stage1Engine at world size 2 (gloo over one device): replicas stay
    identical, grads are the sum of per-rank grads (1/W folded into AdamW), the
    scheduler advanced twice."""
    with tempfile.TemporaryDirectory() as td:
        mp.spawn(dist_worker.engine_ddp, args=(2, _port(), td), nprocs=2, join=True)
        g0, g1 = np.load(f"{td}/grad0.npy"), np.load(f"{td}/grad1.npy")
        p0, p1 = np.load(f"{td}/param0.npy"), np.load(f"{td}/param1.npy")
        s0 = np.load(f"{td}/sched0.npy")
    np.testing.assert_array_equal(g0, g1)
    np.testing.assert_array_equal(p0, p1)
    assert s0[0] == 2
    # single-process reconstruction: sum of the two half-batch grads
    from projectiontrainer_amd import weights as W
    from projectiontrainer_amd.config import PRESETS
    from projectiontrainer_amd.gemma3 import Gemma3CausalLM
    from projectiontrainer_amd.projectors import MLPProjector
    from projectiontrainer_amd.siglip import SiglipVisionTower
    from projectiontrainer_amd.stage1 import Stage1Engine
    cfg = PRESETS["tiny"].replace(batch_size=4)
    vp, lp = W.siglip_vision_params(cfg.vision), W.gemma3_params(cfg.text)
    pp = W.projector_params(cfg.vision.hidden_size, cfg.text.hidden_size)
    px, ids, labels = W.synthetic_batch(cfg, seed=21)
    proj = MLPProjector(cfg.vision.hidden_size, cfg.text.hidden_size)
    proj.load_state_dict({k: torch.from_numpy(v) for k, v in pp.items()})
    proj.to(gpu)
    eng = Stage1Engine(SiglipVisionTower(cfg.vision, vp, gpu),
                       Gemma3CausalLM(cfg.text, lp, gpu, max_pos=Gemma3CausalLM.seq_pad(cfg.seq_len)), proj)
    tot = None
    for r in range(2):
        sl = slice(2 * r, 2 * r + 2)
        eng.forward_backward(*(torch.from_numpy(t[sl]).to(gpu) for t in (px, ids, labels)))
        g = eng.proj.flat_grad.clone()
        tot = g if tot is None else tot + g
    np.testing.assert_allclose(g0, tot.cpu().numpy(), rtol=1e-6, atol=1e-12)
