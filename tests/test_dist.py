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


def test_shard_batches_even_batches():
    """accelerate's even_batches: every rank gets the same number of full batches (world > 1), every sample
    is covered, the filler indices come from the start of the permutation; world 1 keeps the short batch."""
    from projectiontrainer_amd.dist import batches_per_rank, shard_batches
    for n, bs, world in ((10, 3, 2), (64, 8, 4), (7, 2, 3), (5, 4, 3), (1, 2, 2), (16, 4, 4)):
        parts = [shard_batches(n, bs, r, world, epoch=1) for r in range(world)]
        counts = [len(p) for p in parts]
        assert len(set(counts)) == 1 and counts[0] == batches_per_rank(n, bs, world), (n, bs, world, counts)
        assert all(len(b) == bs for p in parts for b in p)
        allidx = torch.cat([torch.cat(p) for p in parts]).tolist()
        assert set(allidx) == set(range(n))
    one = shard_batches(7, 2, 0, 1, epoch=0)
    assert [len(b) for b in one] == [2, 2, 2, 1]
    # deterministic per epoch, different across epochs
    assert torch.equal(torch.cat(shard_batches(20, 4, 0, 1, 0)), torch.cat(shard_batches(20, 4, 0, 1, 0)))
    assert not torch.equal(torch.cat(shard_batches(20, 4, 0, 1, 0)), torch.cat(shard_batches(20, 4, 0, 1, 1)))


def test_shard_batches_matches_accelerate():
    """Index for index the batches accelerate's BatchSamplerShard (the reference's prepared DataLoader,
    Stage1/projector_trainer.py:100-102) yields for the same permutation."""
    from torch.utils.data import BatchSampler
    from accelerate.data_loader import BatchSamplerShard
    from projectiontrainer_amd.dist import shard_batches
    for n in range(0, 30):
        for bs in (1, 2, 3, 5):
            for world in (1, 2, 3, 4):
                order = torch.randperm(n, generator=torch.Generator().manual_seed(11)).tolist()
                for r in range(world):
                    ours = [b.tolist() for b in shard_batches(n, bs, r, world, epoch=0, seed=11)]
                    ref = ([list(b) for b in BatchSampler(order, bs, False)] if world == 1 else
                           [list(b) for b in BatchSamplerShard(BatchSampler(order, bs, False), world, r)])
                    assert ours == ref, (n, bs, world, r)


def test_uneven_dataset_world3_gloo_cpu():
    """7 samples, bs 2, world 3, 2 epochs: every rank runs the same number of steps (no rank left waiting
    in a collective), all batches are full, and the replicas stay identical."""
    with tempfile.TemporaryDirectory() as td:
        mp.spawn(dist_worker.oracle_even_loop, args=(3, _port(), td), nprocs=3, join=True)
        ps = [np.load(f"{td}/param{r}.npy") for r in range(3)]
        sz = [np.load(f"{td}/sizes{r}.npy") for r in range(3)]
        ls = [np.load(f"{td}/losses{r}.npy") for r in range(3)]
    for r in (1, 2):
        np.testing.assert_array_equal(ps[0], ps[r])
        np.testing.assert_array_equal(ls[0], ls[r])
    assert all(list(s) == [2, 2, 2, 2] for s in sz), sz


def test_from_accelerator_cpu():
    """An accelerate.Accelerator handed to the trainer (as train_projection_stage1.py:338 does) is wrapped
    with the fields the trainer reads."""
    from accelerate import Accelerator
    from projectiontrainer_amd.dist import from_accelerator
    acc = Accelerator(cpu=True, gradient_accumulation_steps=2)
    st = from_accelerator(acc)
    assert (st.num_processes, st.process_index, st.gradient_accumulation_steps) == (1, 0, 2)
    assert st.is_main_process and st.sync_gradients and st.device == torch.device("cpu")
    t = torch.tensor([1.5])
    assert torch.equal(st.gather(t), t)
    assert torch.equal(st.all_reduce_sum_(t.clone()), t)


@pytest.mark.parametrize("world", [2, 8])
def test_ddp_grad_average_gloo_cpu(world):
    """2 and 8 gloo ranks on CPU: all-reduced grads == mean of the per-rank grads (each rank 2 samples)."""
    from oracle import stage1_ref as R
    from projectiontrainer_amd import weights as W
    from projectiontrainer_amd.config import PRESETS
    with tempfile.TemporaryDirectory() as td:
        mp.spawn(dist_worker.oracle_ddp, args=(world, _port(), td), nprocs=world, join=True)
        gr = [np.load(f"{td}/grad{r}.npy") for r in range(world)]
    g0 = gr[0]
    for r in range(1, world):
        np.testing.assert_array_equal(g0, gr[r])
    cfg = PRESETS["tiny"].replace(batch_size=2 * world)
    vp, lp = W.siglip_vision_params(cfg.vision), W.gemma3_params(cfg.text)
    pp = W.projector_params(cfg.vision.hidden_size, cfg.text.hidden_size)
    px, ids, labels = W.synthetic_batch(cfg, seed=21)
    gs = []
    for r in range(world):
        sl = slice(2 * r, 2 * r + 2)
        params = {k: torch.as_tensor(v).clone().requires_grad_(True) for k, v in pp.items()}
        loss, _, _ = R.stage1_forward_loss(vp, cfg.vision, lp, cfg.text, params,
                                           *(torch.as_tensor(t[sl]) for t in (px, ids, labels)))
        loss.backward()
        gs.append(torch.cat([params[k].grad.reshape(-1) for k in pp]).numpy())
    # fp32 sums of W terms in another order (gloo's ring vs a Python sum): cancellation near zero, hence an
    # absolute bar at the grads' scale
    ref = sum(gs) / world
    np.testing.assert_allclose(g0, ref, rtol=1e-5, atol=1e-6 * np.abs(ref).max())


def test_chunked_exchange_matches_single_allreduce_gloo_cpu():
    """world 2, gloo: the projector grads exchanged in the overlapped path's pieces (dW2 | db2, then dW1 | db1;
    SURVEY §8(e)) equal one all-reduce of the whole buffer bit for bit, and the pieces tile the buffer."""
    with tempfile.TemporaryDirectory() as td:
        mp.spawn(dist_worker.chunked_exchange, args=(2, _port(), td), nprocs=2, join=True)
        r = [np.load(f"{td}/chunk{k}.npy") for k in range(2)]
    assert all(x.all() for x in r), r


@pytest.mark.gpu
def test_rccl_comm_world1(gpu):
    """libptk's RCCL communicator (ptk_comm_*) at world 1 on the GPU: sum / average are the identity, and a
    Stage1Engine whose exchange runs inside the projector backward on the comm stream
    (ptk_projector_bwd_allreduce) trains bit-identically to the engine without it."""
    with tempfile.TemporaryDirectory() as td:
        mp.spawn(dist_worker.rccl_comm_world1, args=(1, _port(), td), nprocs=1, join=True)
        r = np.load(f"{td}/rcclcomm.npy")
    assert r.all(), r


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 4, 8])
def test_engine_ddp_ranks_one_gpu(gpu, world):
    """The real Stage1Engine at world size 2, 4 and 8 (gloo over one device; the 8-GPU benchmark's data-parallel
    path, cfg3, at the ranks count it runs): replicas stay identical; the exchanged grads are the sum of the per-rank
    grads of each rank's 2 samples (DDP's average of per-rank means, Stage1/projector_trainer.py:237, with the 1/W
    folded into clip + AdamW); the post-AdamW params equal the oracle's clip_grad_norm_(5) + AdamW on that sum / W;
    the scheduler advanced W times (F7); the loss gather returns every rank's loss in rank order."""
    from oracle import stage1_ref as R
    with tempfile.TemporaryDirectory() as td:
        mp.spawn(dist_worker.engine_ddp, args=(world, _port(), td), nprocs=world, join=True)
        g = [np.load(f"{td}/grad{r}.npy") for r in range(world)]
        p = [np.load(f"{td}/param{r}.npy") for r in range(world)]
        s0 = np.load(f"{td}/sched0.npy")
        ls = [np.load(f"{td}/loss{r}.npy") for r in range(world)]
    for r in range(1, world):
        np.testing.assert_array_equal(g[0], g[r])
        np.testing.assert_array_equal(p[0], p[r])
        np.testing.assert_array_equal(ls[0], ls[r])
    assert s0[0] == world
    # single-process reconstruction: the sum of the per-rank grads, each rank's loss
    from projectiontrainer_amd import weights as W
    from projectiontrainer_amd.config import PRESETS
    from projectiontrainer_amd.gemma3 import Gemma3CausalLM
    from projectiontrainer_amd.projectors import MLPProjector
    from projectiontrainer_amd.siglip import SiglipVisionTower
    from projectiontrainer_amd.stage1 import Stage1Engine
    cfg = PRESETS["tiny"].replace(batch_size=2 * world)
    vp, lp = W.siglip_vision_params(cfg.vision), W.gemma3_params(cfg.text)
    pp = W.projector_params(cfg.vision.hidden_size, cfg.text.hidden_size)
    px, ids, labels = W.synthetic_batch(cfg, seed=21)
    proj = MLPProjector(cfg.vision.hidden_size, cfg.text.hidden_size)
    proj.load_state_dict({k: torch.from_numpy(v) for k, v in pp.items()})
    proj.to(gpu)
    eng = Stage1Engine(SiglipVisionTower(cfg.vision, vp, gpu),
                       Gemma3CausalLM(cfg.text, lp, gpu, max_pos=Gemma3CausalLM.seq_pad(cfg.seq_len)), proj)
    tot, losses = None, []
    for r in range(world):
        sl = slice(2 * r, 2 * r + 2)
        eng.forward_backward(*(torch.from_numpy(t[sl]).to(gpu) for t in (px, ids, labels)))
        gr = eng.proj.flat_grad.clone()
        tot = gr if tot is None else tot + gr
        losses.append(float(eng.loss))
    # fp32 sums of W terms in another order (gloo's ring vs this loop): an absolute bar at the grads' scale
    tot = tot.cpu().numpy()
    np.testing.assert_allclose(g[0], tot, rtol=1e-5, atol=1e-6 * np.abs(tot).max())
    np.testing.assert_allclose(ls[0], np.array(losses, dtype=np.float32), rtol=1e-6)
    # clip + AdamW on the exchanged sum with the 1/W average (oracle, fp32 CPU), lr = lr0 * lambda(0)
    st = R.init_state(pp)
    grads, o = {}, 0
    for k in pp:
        n = st.params[k].numel()
        grads[k] = torch.from_numpy(g[0][o:o + n] / world).view(st.params[k].shape).clone()
        o += n
    R.clip_grad_norm_(list(grads.values()), 5.0)
    R.adamw_step(st, grads, float(s0[1]))
    ref = torch.cat([st.params[k].reshape(-1) for k in pp]).numpy()
    np.testing.assert_allclose(p[0], ref, rtol=1e-6, atol=1e-9)


@pytest.mark.gpu
def test_trainer_uneven_dataset_world3(gpu):
    """The real ProjectionTrainerStage1 at world 3 (gloo, one device) on 7 samples at bs 2: it finishes,
    every rank ran 2 steps per epoch, the replicas are identical, and the epoch loss is divided by the
    per-rank batch count (len(train_loader) after prepare)."""
    with tempfile.TemporaryDirectory() as td:
        mp.spawn(dist_worker.trainer_even, args=(3, _port(), td), nprocs=3, join=True)
        ps = [np.load(f"{td}/param{r}.npy") for r in range(3)]
        st = [np.load(f"{td}/steps{r}.npy") for r in range(3)]
        ep = np.load(f"{td}/eploss0.npy")
    for r in (1, 2):
        np.testing.assert_array_equal(ps[0], ps[r])
    assert all(int(s[0]) == 4 and int(s[1]) == 12 for s in st), st
    assert len(ep) == 2 and all(5.0 < e < 7.5 for e in ep), ep   # mean of per-step losses (~ln 512)


@pytest.mark.gpu
def test_nccl_backend_world1(gpu):
    """RCCL ("nccl" backend) initialised at world 1 on the GPU; the grad all-reduce and loss gather run on it."""
    with tempfile.TemporaryDirectory() as td:
        mp.spawn(dist_worker.nccl_world1, args=(1, _port(), td), nprocs=1, join=True)
        r = np.load(f"{td}/nccl.npy")
    assert r[0] == 1 and r[1] == 3.0 and r[2] == 0.0 and r[3] == 1 and r[4] == 1, r


def _bf16(x):
    return x.to(torch.bfloat16).to(torch.float32)


def test_bf16_ring_sum_w8_within_twin_noise():
    """Stage 2's ZeRO-1 reduce-scatter sums the bf16 grad store over 8 ranks in bf16 (RCCL's ring: each hop adds
    one rank's bf16 chunk to the running bf16 partial in fp32 and rounds back, 7 roundings per element).  The
    reference's DDP all-reduce of its bf16 .grad buckets (torch DDP: div_ by W, then the NCCL ring) rounds the same
    7 times, so both are one draw of the same noise.  Emulated here on grads whose per-rank scale varies 4x (as
    micro-batch losses do): the ring sum's rel-L2 to the exact fp32 sum must stay far below the 2e-2 twin-noise bar
    of the Stage-2 parity tests (measured 3.2e-3).  Pre-dividing by W = 8 is exact in bf16 (a power of two, no
    underflow at these magnitudes), so the reference's order gives the identical sums."""
    W = 8
    g = torch.Generator().manual_seed(0)
    n = 1 << 16
    base = torch.randn(n, generator=g) * 1e-3
    grads = [_bf16(base + torch.randn(n, generator=g) * 1e-3 * (0.5 + 1.5 * r / (W - 1))) for r in range(W)]
    exact = torch.stack(grads).double().sum(0)

    def ring(gs, start):
        acc = gs[start % W]
        for h in range(1, W):
            acc = _bf16(acc + gs[(start + h) % W])
        return acc

    rel = lambda x: float((x.double() - exact).norm() / exact.norm())
    ours = torch.cat([ring([t[c::W] for t in grads], c + 1) for c in range(W)])
    ours = torch.empty(n).index_copy_(0, torch.cat([torch.arange(c, n, W) for c in range(W)]), ours)
    ref = torch.cat([ring([_bf16(t[c::W] / W) for t in grads], c + 1) * W for c in range(W)])
    ref = torch.empty(n).index_copy_(0, torch.cat([torch.arange(c, n, W) for c in range(W)]), ref)
    assert rel(ours) < 5e-3, rel(ours)
    assert rel(ref) < 5e-3, rel(ref)
    assert torch.equal(ours, ref)
