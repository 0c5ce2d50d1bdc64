"""Process-group plumbing: one process per GPU, torch.distributed over RCCL
("nccl" backend on ROCm) on the GPU box, gloo for CPU tests.

`DistState` exposes the subset of `accelerate.Accelerator` the reference's
trainer touches (`Stage1/accelerator_setup.py:7-54`):
`device, is_main_process, process_index, num_processes,
gradient_accumulation_steps, sync_gradients, gather`.
"""
from __future__ import annotations

import math
import os

import torch
import torch.distributed as dist


class DistState:
    def __init__(self, gradient_accumulation_steps: int = 1, backend: str | None = None, device=None):
        self.gradient_accumulation_steps = gradient_accumulation_steps
        self.sync_gradients = True          # Stage 1 never enters accumulate()
        world = int(os.environ.get("WORLD_SIZE", "1"))
        if world > 1 and not dist.is_initialized():
            if backend is None:
                backend = "nccl" if torch.cuda.is_available() else "gloo"
            local = int(os.environ.get("LOCAL_RANK", "0"))
            if backend == "nccl":
                torch.cuda.set_device(local)
                dist.init_process_group(backend, device_id=torch.device("cuda", local))
            else:
                dist.init_process_group(backend)
        self.initialized = dist.is_initialized()
        self.num_processes = dist.get_world_size() if self.initialized else 1
        self.process_index = dist.get_rank() if self.initialized else 0
        if device is None:
            device = (torch.device("cuda", int(os.environ.get("LOCAL_RANK", "0"))) if torch.cuda.is_available()
                      else torch.device("cpu"))
        self.device = torch.device(device)

    @property
    def is_main_process(self) -> bool:
        return self.process_index == 0

    def all_reduce_sum_(self, t):
        if self.num_processes > 1:
            dist.all_reduce(t, op=dist.ReduceOp.SUM)
        return t

    def gather(self, t):
        """accelerator.gather for a scalar / 1-D tensor (all_gather_into_tensor)."""
        t = t.reshape(-1)
        if self.num_processes == 1:
            return t
        if dist.get_backend() == "gloo":        # CPU tests: gloo has no all_gather_into_tensor
            parts = [torch.empty_like(t) for _ in range(self.num_processes)]
            dist.all_gather(parts, t.contiguous())
            return torch.cat(parts)
        out = torch.empty(self.num_processes * t.numel(), dtype=t.dtype, device=t.device)
        dist.all_gather_into_tensor(out, t.contiguous())
        return out

    def wait_for_everyone(self):
        if self.num_processes > 1:
            dist.barrier()

    def gather_object(self, obj):
        """accelerate.utils.gather_object for a list: every rank's list, concatenated in rank order."""
        if self.num_processes == 1:
            return list(obj)
        parts = [None] * self.num_processes
        dist.all_gather_object(parts, obj)
        return [x for part in parts for x in part]


def from_accelerator(acc) -> DistState:
    """Wrap an accelerate.Accelerator (process group already initialised by it)."""
    st = DistState.__new__(DistState)
    st.gradient_accumulation_steps = getattr(acc, "gradient_accumulation_steps", 1)
    st.sync_gradients = True
    st.initialized = dist.is_initialized()
    st.num_processes = acc.num_processes
    st.process_index = acc.process_index
    st.device = torch.device(acc.device)
    st.all_reduce_sum_ = DistState.all_reduce_sum_.__get__(st)
    st.gather_object = DistState.gather_object.__get__(st)
    return st


def shard_batches(n_items: int, batch_size: int, rank: int, world: int, epoch: int, seed: int = 0,
                  shuffle: bool = True):
    """Index batches for this rank, as the reference's prepared DataLoader
    yields them (`Stage1/projector_trainer.py:100-102` -> accelerate
    `BatchSamplerShard` with its defaults `even_batches=True`, `drop_last=False`,
    `split_batches=False`; ACC/data_loader.py:213-271).

    One seeded permutation (the same on every rank, as accelerate's synchronised
    sampler generator) is cut into batches of `batch_size`; batch i goes to rank
    i % world.  With world > 1 every rank gets the SAME number of FULL batches:
    the short last batch is completed, and missing batches are created, from the
    start of the permutation (indices of the first `world` batches, repeated as
    needed).  With world == 1 accelerate does not shard, so the short last batch
    is kept as the plain DataLoader yields it."""
    g = torch.Generator().manual_seed(seed + epoch)
    order = (torch.randperm(n_items, generator=g) if shuffle else torch.arange(n_items)).tolist()
    batches = [order[i:i + batch_size] for i in range(0, n_items, batch_size)]
    if world == 1:
        return [torch.tensor(b, dtype=torch.int64) for b in batches]
    out, to_yield = [], None
    initial = [i for b in batches[:world] for i in b]   # ACC :218-223 (first `world` batches)
    for idx, b in enumerate(batches):
        if idx % world == rank:
            to_yield = b
        if idx % world == world - 1 and len(b) == batch_size:
            out.append(to_yield)
            to_yield = None
    if batches:
        if to_yield is not None and len(to_yield) == batch_size:
            out.append(to_yield)
        while len(initial) < world * batch_size:         # degenerate: dataset smaller than one round
            initial = initial + initial
        idx, last = len(batches) - 1, list(batches[-1])
        if len(last) == batch_size:
            last, idx = [], idx + 1
        cyc = 0
        while idx % world != 0 or len(last) > 0:          # ACC :256-271: fill up to a multiple of world
            end = cyc + batch_size - len(last)
            last = last + initial[cyc:end]
            if idx % world == rank:
                out.append(last)
            cyc, last, idx = end, [], idx + 1
    return [torch.tensor(b, dtype=torch.int64) for b in out]


def batches_per_rank(n_items: int, batch_size: int, world: int) -> int:
    """len() of the prepared DataLoader on each rank (ACC/data_loader.py:170-186, even_batches)."""
    n = math.ceil(n_items / batch_size)
    return n if world == 1 else math.ceil(n / world)


def allreduce_grads_(flat_grad, world: int, group=None):
    """DDP gradient semantics (projector_trainer.py:237 -> DDP reducer): sum the
    flat fp32 grads over ranks in ONE collective; the 1/world average is folded
    into the fused clip+AdamW kernel (grad_scale), so this returns the scale."""
    if world > 1:
        dist.all_reduce(flat_grad, op=dist.ReduceOp.SUM, group=group)
    return 1.0 / world


def grad_exchange_chunks(proj):
    """(offset, count) pieces of the projector's flat grad [dW1 | db1 | dW2 | db2] in exchange order: dW2 | db2
    (computed first by the backward, so its all-reduce overlaps the dA / dW1 GEMMs), then dW1 | db1
    (ptk_projector_bwd_allreduce; SURVEY §8(e): the 89 MB all-reduce split to pipeline with the dW GEMMs)."""
    Dv, I, Dl = proj.vision_dim, proj.inter_dim, proj.llm_dim
    n1 = I * Dv + I
    return [(n1, Dl * I + Dl), (0, n1)]


def allreduce_grads_chunked_(flat_grad, chunks, world: int, group=None):
    """allreduce_grads_ piece by piece in the given order (the collective-library path of the overlapped
    RCCL exchange; gloo on CPU): the same sums, element for element."""
    if world > 1:
        for off, n in chunks:
            dist.all_reduce(flat_grad[off:off + n], op=dist.ReduceOp.SUM, group=group)
    return 1.0 / world


class RcclComm:
    """libptk's RCCL communicator (ptk_comm_*) over the ranks of an initialised torch process group: rank 0
    creates the unique id, the group broadcasts it, every rank joins on `device` (default: the current one)."""

    def __init__(self, group=None, device=None):
        import ctypes

        from . import _lib as L
        self._L = L
        lib = L.lib()
        nb = lib.ptk_comm_unique_id_bytes()
        world, rank = dist.get_world_size(group), dist.get_rank(group)
        uid = (ctypes.c_char * nb)()
        if rank == 0:
            L.check(lib.ptk_comm_get_unique_id(uid), "ptk_comm_get_unique_id")
        obj = [bytes(uid) if rank == 0 else None]
        dist.broadcast_object_list(obj, src=dist.get_global_rank(group, 0) if group is not None else 0, group=group)
        uid = (ctypes.c_char * nb).from_buffer_copy(obj[0])
        self.handle = ctypes.c_void_p()
        # ptk_comm_init joins RCCL on the current HIP device: make that the engine's device
        with torch.cuda.device(device if device is not None else torch.cuda.current_device()):
            L.check(lib.ptk_comm_init(ctypes.byref(self.handle), uid, world, rank), "ptk_comm_init")
        self.world, self.rank = world, rank

    def allreduce_sum_(self, t, stream):
        self._L.check(self._L.lib().ptk_comm_allreduce_sum(self.handle, t.data_ptr(), t.numel(), stream),
                      "ptk_comm_allreduce_sum")
        return t

    def close(self):
        if getattr(self, "handle", None) is not None and self.handle.value:
            self._L.lib().ptk_comm_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
