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
    torch.set_num_threads(1 if world > 2 else 2)
    from oracle import stage1_ref as R
    from projectiontrainer_amd import dist as D
    from projectiontrainer_amd import weights as W
    from projectiontrainer_amd.config import PRESETS
    cfg = PRESETS["tiny"].replace(batch_size=2 * world)
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
    """GPU/gloo on one device: the real Stage1Engine at world_size `world`, 2 samples per rank (the batch of
    2 * world cut by rank), one step; the gathered per-rank losses (accelerator.gather, DistState.gather)."""
    _init(rank, world, port, "gloo")
    from projectiontrainer_amd import dist as D
    from projectiontrainer_amd import weights as W
    from projectiontrainer_amd.config import PRESETS
    from projectiontrainer_amd.gemma3 import Gemma3CausalLM
    from projectiontrainer_amd.projectors import MLPProjector
    from projectiontrainer_amd.siglip import SiglipVisionTower
    from projectiontrainer_amd.stage1 import Stage1Engine
    dev = torch.device("cuda:0")
    cfg = PRESETS["tiny"].replace(batch_size=2 * world)
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
    acc = D.DistState(1, backend="gloo", device=dev)
    losses = acc.gather(eng.loss.detach().cpu())
    np.save(os.path.join(out_dir, f"grad{rank}.npy"), eng.proj.flat_grad.cpu().numpy())
    np.save(os.path.join(out_dir, f"param{rank}.npy"), eng.proj.flat.cpu().numpy())
    np.save(os.path.join(out_dir, f"sched{rank}.npy"), np.array([eng.sched_step, eng.last_lr]))
    np.save(os.path.join(out_dir, f"loss{rank}.npy"), losses.numpy())
    dist.destroy_process_group()


def oracle_even_loop(rank, world, port, out_dir):
    """CPU/gloo, world 3: the trainer's per-batch collective sequence (grad all-reduce, loss gather) over
    a 7-sample dataset at bs 2 for 2 epochs, batches dealt by dist.shard_batches (accelerate even_batches).
    Uneven per-rank batch counts would leave one rank blocked in a collective; equal counts finish."""
    _init(rank, world, port, "gloo")
    torch.set_num_threads(1)
    from oracle import stage1_ref as R
    from projectiontrainer_amd import dist as D
    from projectiontrainer_amd import weights as W
    from projectiontrainer_amd.config import PRESETS
    acc = D.DistState(1, backend="gloo", device="cpu")
    cfg = PRESETS["tiny"].replace(batch_size=7)
    vp, lp = W.siglip_vision_params(cfg.vision), W.gemma3_params(cfg.text)
    pp = W.projector_params(cfg.vision.hidden_size, cfg.text.hidden_size)
    px, ids, labels = W.synthetic_batch(cfg, seed=33)
    st = R.init_state(pp)
    sizes, losses = [], []
    for epoch in range(2):
        for idx in D.shard_batches(7, 2, acc.process_index, acc.num_processes, epoch):
            sizes.append(len(idx))
            params = {k: v.clone().requires_grad_(True) for k, v in st.params.items()}
            loss, _, _ = R.stage1_forward_loss(vp, cfg.vision, lp, cfg.text, params,
                                               *(torch.as_tensor(t[idx.numpy()]) for t in (px, ids, labels)))
            loss.backward()
            flat = torch.cat([params[k].grad.reshape(-1) for k in pp])
            scale = D.allreduce_grads_(flat, acc.num_processes)
            flat *= scale
            grads, o = {}, 0
            for k in pp:
                n = st.params[k].numel()
                grads[k] = flat[o:o + n].view(st.params[k].shape).clone()
                o += n
            R.clip_grad_norm_(list(grads.values()), 5.0)
            R.adamw_step(st, grads, 1e-3)
            losses.append(float(acc.gather(loss.detach().reshape(1)).mean()))
    np.save(os.path.join(out_dir, f"param{rank}.npy"), torch.cat([st.params[k].reshape(-1) for k in pp]).numpy())
    np.save(os.path.join(out_dir, f"sizes{rank}.npy"), np.array(sizes))
    np.save(os.path.join(out_dir, f"losses{rank}.npy"), np.array(losses))
    dist.destroy_process_group()


def trainer_even(rank, world, port, out_dir):
    """GPU (one device shared by the ranks) / gloo: the real ProjectionTrainerStage1 on a 7-sample dataset,
    bs 2, 2 epochs, world 3 (7 samples -> 4 batches -> 2 full batches per rank under even_batches)."""
    _init(rank, world, port, "gloo")
    from projectiontrainer_amd import dist as D
    from projectiontrainer_amd import weights as W
    from projectiontrainer_amd.config import PRESETS
    from projectiontrainer_amd.gemma3 import Gemma3CausalLM
    from projectiontrainer_amd.projector_trainer import ProjectionTrainerStage1
    from projectiontrainer_amd.projectors import MLPProjector
    from projectiontrainer_amd.siglip import SiglipVisionTower
    import types
    dev = torch.device("cuda:0")
    cfg = PRESETS["tiny"].replace(batch_size=7)
    vp, lp = W.siglip_vision_params(cfg.vision), W.gemma3_params(cfg.text)
    pp = W.projector_params(cfg.vision.hidden_size, cfg.text.hidden_size)
    px, ids, labels = W.synthetic_batch(cfg, seed=33)
    data = [{"pixel_values": torch.from_numpy(px[i]), "token_ids": torch.from_numpy(ids[i]),
             "labels": torch.from_numpy(labels[i])} for i in range(7)]
    proj = MLPProjector(cfg.vision.hidden_size, cfg.text.hidden_size)
    proj.load_state_dict({k: torch.from_numpy(v) for k, v in pp.items()})
    logs = []
    tr = ProjectionTrainerStage1(D.DistState(1, backend="gloo", device=dev), SiglipVisionTower(cfg.vision, vp, dev),
                                 Gemma3CausalLM(cfg.text, lp, dev, max_pos=Gemma3CausalLM.seq_pad(cfg.seq_len)),
                                 proj, None, types.SimpleNamespace(pad_token_id=0, eos_token_id=1), data, None,
                                 output_dir=os.path.join(out_dir, f"o{rank}"), batch_size=2, learning_rate=1e-3,
                                 num_epochs=2, log_fn=lambda d, s: logs.append(d))
    tr.train()
    torch.cuda.synchronize()
    np.save(os.path.join(out_dir, f"param{rank}.npy"), tr.projection_layer.flat.cpu().numpy())
    np.save(os.path.join(out_dir, f"steps{rank}.npy"), np.array([tr.global_step, tr.engine.sched_step]))
    ep = [x["train/epoch_loss"] for x in logs if "train/epoch_loss" in x]
    np.save(os.path.join(out_dir, f"eploss{rank}.npy"), np.array(ep))
    dist.destroy_process_group()


def nccl_world1(rank, world, port, out_dir):
    """RCCL ("nccl" backend) at world 1 on the GPU: init, all-reduce, and one Stage1Engine step whose grad
    all-reduce goes through it."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    t = torch.full((4,), 3.0, device=dev)
    dist.all_reduce(t)
    from projectiontrainer_amd import dist as D
    from projectiontrainer_amd import weights as W
    from projectiontrainer_amd.config import PRESETS
    from projectiontrainer_amd.gemma3 import Gemma3CausalLM
    from projectiontrainer_amd.projectors import MLPProjector
    from projectiontrainer_amd.siglip import SiglipVisionTower
    from projectiontrainer_amd.stage1 import Stage1Engine
    acc = D.DistState(1)
    cfg = PRESETS["tiny"]
    vp, lp = W.siglip_vision_params(cfg.vision), W.gemma3_params(cfg.text)
    pp = W.projector_params(cfg.vision.hidden_size, cfg.text.hidden_size)
    px, ids, labels = W.synthetic_batch(cfg, seed=5)
    proj = MLPProjector(cfg.vision.hidden_size, cfg.text.hidden_size)
    proj.load_state_dict({k: torch.from_numpy(v) for k, v in pp.items()})
    proj.to(dev)
    eng = Stage1Engine(SiglipVisionTower(cfg.vision, vp, dev),
                       Gemma3CausalLM(cfg.text, lp, dev, max_pos=Gemma3CausalLM.seq_pad(cfg.seq_len)), proj,
                       world_size=1)
    eng.forward_backward(*(torch.from_numpy(x).to(dev) for x in (px, ids, labels)))
    g = eng.proj.flat_grad.clone()
    D.allreduce_grads_(eng.proj.flat_grad, 2)       # forces the RCCL all_reduce path (world arg > 1)
    loss = acc.gather(eng.loss)
    torch.cuda.synchronize()
    np.save(os.path.join(out_dir, "nccl.npy"),
            np.array([dist.get_backend() == "nccl", float(t[0]), float((eng.proj.flat_grad - g).abs().max()),
                      loss.numel(), acc.num_processes]))
    dist.destroy_process_group()


def stage2_zero(rank, world, port, out_dir):
    """GPU (one device shared) / gloo, world 2 / 4 / 8: Stage2Engine with ZeRO-1 sharding; each rank runs its 2
    samples of a batch of 2 * world, then the sharded optimizer step.  Saves the replica's flat parameters."""
    _init(rank, world, port, "gloo")
    import math
    from projectiontrainer_amd import weights as W
    from projectiontrainer_amd.config import PRESETS
    from projectiontrainer_amd.stage2 import synthetic_engine
    dev = torch.device("cuda:0")
    cfg = PRESETS["tiny"].replace(batch_size=2 * world, text_len=8 + 12, question_len=8)
    torch.manual_seed(0)
    eng = synthetic_engine(cfg, dev, seed=3, world_size=world, rank=rank, learning_rate=1e-3, total_steps=10)
    px, q, a = (torch.from_numpy(t).to(dev) for t in W.synthetic_vqa_batch(cfg, seed=9))
    sl = slice(2 * rank, 2 * rank + 2)
    eng.forward_backward(px[sl], q[sl], a[sl])
    eng.optimizer_step()
    torch.cuda.synchronize()
    np.save(os.path.join(out_dir, f"s2param{rank}.npy"), eng.state.flat.float().cpu().numpy())
    np.save(os.path.join(out_dir, f"s2norm{rank}.npy"), eng.grad_norm.cpu().numpy())
    torch.save(eng.optimizer_state(), os.path.join(out_dir, f"opt{rank}.pt"))
    dist.destroy_process_group()


def stage2_rccl_world1(rank, world, port, out_dir):
    """RCCL at world 1: Stage2Engine with zero1=True (reduce-scatter / all-gather / norm all-reduce through
    the nccl process group) vs zero1=False, same batch, one optimizer step each."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    from projectiontrainer_amd import weights as W
    from projectiontrainer_amd.config import PRESETS
    from projectiontrainer_amd.stage2 import synthetic_engine
    cfg = PRESETS["tiny"].replace(batch_size=2, text_len=8 + 12, question_len=8)
    px, q, a = (torch.from_numpy(t).to(dev) for t in W.synthetic_vqa_batch(cfg, seed=9))
    out = []
    for z in (True, False):
        torch.manual_seed(0)
        eng = synthetic_engine(cfg, dev, seed=3, learning_rate=1e-3, total_steps=10, zero1=z)
        eng.forward_backward(px, q, a)
        eng.optimizer_step()
        torch.cuda.synchronize()
        out.append((eng.state.flat.clone(), eng.exp_avg.clone(), eng.grad_norm.clone()))
    ok = [dist.get_backend() == "nccl", torch.equal(out[0][0], out[1][0]) and torch.equal(out[0][1], out[1][1]),
          torch.equal(out[0][2], out[1][2])]
    np.save(os.path.join(out_dir, "rccl.npy"), np.array(ok, dtype=np.int64))
    dist.destroy_process_group()


def chunked_exchange(rank, world, port, out_dir):
    """CPU/gloo: the projector grad exchange piece by piece (grad_exchange_chunks order) vs one all-reduce."""
    _init(rank, world, port, "gloo")
    from projectiontrainer_amd import dist as D
    from projectiontrainer_amd.projectors import MLPProjector
    proj = MLPProjector(32, 48, expansion_factor=3)
    g = torch.Generator().manual_seed(100 + rank)
    flat = torch.randn(proj.flat.numel(), generator=g)
    a, b = flat.clone(), flat.clone()
    s1 = D.allreduce_grads_(a, world)
    s2 = D.allreduce_grads_chunked_(b, D.grad_exchange_chunks(proj), world)
    chunks = D.grad_exchange_chunks(proj)
    covered = sorted((o, o + n) for o, n in chunks)
    ok = [torch.equal(a, b), s1 == s2, covered == [(0, covered[0][1]), (covered[0][1], flat.numel())]]
    np.save(os.path.join(out_dir, f"chunk{rank}.npy"), np.array(ok, dtype=np.int64))
    dist.destroy_process_group()


def rccl_comm_world1(rank, world, port, out_dir):
    """RCCL at world 1 through libptk's communicator: ptk_comm_allreduce_sum / _avg on a buffer, and a
    Stage1Engine step with the exchange overlapped inside the projector backward (comm=True) against the
    same step without it (comm=False)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    from projectiontrainer_amd import _lib as L
    from projectiontrainer_amd import dist as D
    from projectiontrainer_amd import weights as W
    from projectiontrainer_amd.config import PRESETS
    from projectiontrainer_amd.gemma3 import Gemma3CausalLM
    from projectiontrainer_amd.projectors import MLPProjector
    from projectiontrainer_amd.siglip import SiglipVisionTower
    from projectiontrainer_amd.stage1 import Stage1Engine
    comm = D.RcclComm()
    t = torch.arange(1000, dtype=torch.float32, device=dev)
    u = t.clone()
    comm.allreduce_sum_(u, L.stream_ptr(dev))
    L.check(L.lib().ptk_comm_allreduce_avg(comm.handle, u.data_ptr(), u.numel(), L.stream_ptr(dev)), "avg")
    torch.cuda.synchronize()
    ok = [L.lib().ptk_comm_world(comm.handle) == 1, torch.equal(t, u)]
    comm.close()
    cfg = PRESETS["tiny"]
    vp, lp = W.siglip_vision_params(cfg.vision), W.gemma3_params(cfg.text)
    pp = W.projector_params(cfg.vision.hidden_size, cfg.text.hidden_size)
    px, ids, labels = (torch.from_numpy(x).to(dev) for x in W.synthetic_batch(cfg, seed=5))
    res = []
    for use in (True, False):
        proj = MLPProjector(cfg.vision.hidden_size, cfg.text.hidden_size)
        proj.load_state_dict({k: torch.from_numpy(v) for k, v in pp.items()})
        proj.to(dev)
        eng = Stage1Engine(SiglipVisionTower(cfg.vision, vp, dev),
                           Gemma3CausalLM(cfg.text, lp, dev, max_pos=Gemma3CausalLM.seq_pad(cfg.seq_len)), proj,
                           world_size=1, comm=use, total_steps=10)
        for _ in range(2):
            eng.step(px, ids, labels)
        torch.cuda.synchronize()
        res.append((eng.proj.flat.clone(), eng.proj.flat_grad.clone(), eng.comm is not None))
    ok += [res[0][2] and not res[1][2], torch.equal(res[0][0], res[1][0]), torch.equal(res[0][1], res[1][1])]
    np.save(os.path.join(out_dir, "rcclcomm.npy"), np.array(ok, dtype=np.int64))
    dist.destroy_process_group()
