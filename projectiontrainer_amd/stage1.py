"""Stage1Engine: one reference Stage-1 training iteration on MI355X.

The body of `for batch in progress_bar:` (Stage1/projector_trainer.py:152-245):

  pixels f32 -> bf16 (:168)             ptk_cast_f32_bf16
  SigLIP fwd, drop patch 0 (:158-173)   ptk_siglip_fwd (patch 0 is skipped by the projector's row map)
  projector fwd (:180)                  ptk_projector_fwd -> writes the LLM input's vision rows
  embed + cat + mask + labels (:183-220)  inside ptk_gemma3_loss_fwd_bwd
  Gemma3 fwd + loss + backward (:226-237) ptk_gemma3_loss_fwd_bwd (loss scaled 1/gas^2)
  projector bwd                         ptk_gather_vision_grad + ptk_projector_bwd
  DDP grad all-reduce                   ptk_projector_bwd_allreduce (RCCL via libptk, overlapped with the
                                        projector backward); gloo: torch.distributed, same pieces
  clip_grad_norm_(5) + AdamW (:240-242) ptk_clip_adamw, then bf16 shadow refresh
  lr_scheduler.step() x num_processes   host-side cosine lambda (no device sync)

All buffers are allocated once per (batch, text_len); a step issues no host
synchronisation, so the loss is returned as a device tensor.

Vision prefetch: the SigLIP tower is frozen, so the vision features of the NEXT
batch do not depend on this step's update.  `step(..., next_pixel_values=...)`
runs the next batch's SigLIP forward on a side stream as soon as this step's
projector forward has consumed its own features; it overlaps the Gemma3
forward/backward (filling the CUs its GEMM tail waves and HBM-bound passes
leave idle), and the next step waits only on its event.  Vision features and
pixels are double-buffered; a buffer is reused only after the projector
backward that reads it has run.
"""
from __future__ import annotations

import contextlib
import math
import os

import torch

from . import _lib as L
from . import kernels as K
from .config import Stage1Config
from .dist import RcclComm, allreduce_grads_chunked_, grad_exchange_chunks
from .gemma3 import Gemma3CausalLM
from .projectors import MLPProjector
from .siglip import SiglipVisionTower


def cosine_lambda(step, warmup, total, num_cycles=0.5):
    """get_cosine_schedule_with_warmup lambda (TF/optimization.py:134-140)."""
    if step < warmup:
        return float(step) / float(max(1, warmup))
    prog = float(step - warmup) / float(max(1, total - warmup))
    return max(0.0, 0.5 * (1.0 + math.cos(math.pi * float(num_cycles) * 2.0 * prog)))


class Stage1Engine:
    def __init__(self, vision: SiglipVisionTower, llm: Gemma3CausalLM, projector: MLPProjector, *,
                 learning_rate=1e-4, weight_decay=0.01, gradient_accumulation_steps=1, max_grad_norm=5.0,
                 warmup_steps=0, total_steps=1, betas=(0.9, 0.999), eps=1e-8, process_group=None,
                 world_size=1, comm="auto"):
        self.vision, self.llm, self.proj = vision, llm, projector
        self.device = vision.device
        self.lr0, self.wd, self.gas, self.max_norm = learning_rate, weight_decay, gradient_accumulation_steps, max_grad_norm
        self.warmup, self.total, self.betas, self.eps = warmup_steps, total_steps, betas, eps
        self.pg, self.world = process_group, world_size
        # text key mask `token_ids != tokenizer.pad_token_id` (projector_trainer.py:207-209): the trainer
        # sets the tokenizer's id (-1 = tokenizer without a pad token: every text key attends); None = the
        # LM config's pad_token_id
        self.pad_token_id = None
        self.opt_step = 0        # optimizer steps (AdamW bias correction)
        self.sched_step = 0      # LambdaLR steps (advanced num_processes times per step, F7)
        n = projector.flat.numel()
        self.exp_avg = torch.zeros(n, dtype=torch.float32, device=self.device)
        self.exp_avg_sq = torch.zeros(n, dtype=torch.float32, device=self.device)
        self._partial = torch.empty(1024, dtype=torch.float32, device=self.device)
        self.grad_norm = torch.zeros(1, dtype=torch.float32, device=self.device)
        self._shape = None
        self.last_lr = learning_rate * cosine_lambda(0, warmup_steps, total_steps)
        self.vstream = None        # side stream of the vision prefetch
        self._prefetched = None    # event: the current buffer's features were computed ahead
        self._vision_ready = False  # encode_vision ran this step's tower on the main stream
        self._graph = None         # graph_step: captured forward_backward, its input key and static inputs
        self._graph_key = None
        self._graph_in = None
        # DDP exchange of the projector grads.  Default: the process group's collective (RCCL under the nccl
        # backend, gloo on CPU), piece by piece in a fixed order after the backward (allreduce_grads_chunked_,
        # checked bit for bit at world 2 / 3).  comm=True (or comm="auto" with PTK_RCCL_OVERLAP=1 on an nccl
        # group): libptk's own RCCL communicator with the dW2 | db2 all-reduce overlapped with the dA / dW1
        # GEMMs (ptk_projector_bwd_allreduce).  The overlapped path has run on hardware at world 1 only (one
        # GPU per box here), so it is opt-in until a world >= 2 run has compared it with the collective path.
        self.comm, self._comm_stream, self._exchanged = None, None, False
        use = comm is True or (comm == "auto" and os.environ.get("PTK_RCCL_OVERLAP") == "1" and world_size > 1
                               and torch.distributed.is_initialized()
                               and torch.distributed.get_backend(process_group) == "nccl")
        if use:
            self.comm = RcclComm(process_group, device=self.device)
            self._comm_stream = torch.cuda.Stream(self.device)

    def _buffers(self, B, T):
        """Step buffers are allocated for the largest batch seen at this text length; a smaller batch
        (the short last batch of an epoch) runs on leading views of them, so nothing is reallocated and
        then reallocated back (the kernels take the row counts explicitly)."""
        if self._shape == (B, T):
            return
        vc, tc = self.vision.cfg, self.llm.cfg
        N, Dv, Dl, I = vc.num_patches, vc.hidden_size, tc.hidden_size, self.proj.inter_dim
        S = (N - 1) + T
        Sp = Gemma3CausalLM.seq_pad(S)
        dev, bf = self.device, torch.bfloat16
        if self._prefetched is not None:
            raise RuntimeError("Stage1Engine: the batch shape changed while a vision prefetch was pending")
        if getattr(self, "_cap", None) is None or self._cap[1] != T or self._cap[0] < B:
            C = B
            self._full = dict(
                px=[torch.empty((C, vc.num_channels, vc.image_size, vc.image_size), dtype=bf, device=dev)
                    for _ in range(2)],
                vis=[torch.empty((C * N, Dv), dtype=bf, device=dev) for _ in range(2)],
                a=torch.empty((C * N, I), dtype=bf, device=dev),
                h=torch.empty((C * N, I), dtype=bf, device=dev),
                x=torch.empty((C * Sp, Dl), dtype=torch.float32, device=dev),
                dx=torch.empty((C * Sp, Dl), dtype=torch.float32, device=dev),
                dy=torch.empty((C * N, Dl), dtype=bf, device=dev))
            self.proj_ws = torch.empty(self.proj.workspace_bytes(C * N), dtype=torch.uint8, device=dev)
            self.vision.workspace(C)
            self.llm.workspace(C, T, Sp)
            self._cap = (C, T)
            self._cur = 0
            self._released = [None, None]   # event per buffer: the projector backward reading it has run
        f = self._full
        self.N, self.Sp = N, Sp
        self.px_bufs = [t[:B] for t in f["px"]]
        self.vis_bufs = [t[:B * N] for t in f["vis"]]
        self.px, self.vis = self.px_bufs[self._cur], self.vis_bufs[self._cur]
        self.a, self.h, self.dy = f["a"][:B * N], f["h"][:B * N], f["dy"][:B * N]
        self.x, self.dx = f["x"][:B * Sp], f["dx"][:B * Sp]
        if getattr(self, "loss", None) is None:
            self.loss = torch.zeros(1, dtype=torch.float32, device=dev)
        self._shape = (B, T)

    # ---------------------------------------------------------------- pieces
    def _vision(self, pixel_values, i):
        """pixels -> bf16 px_bufs[i] -> SigLIP features vis_bufs[i], on the current stream."""
        px = self.px_bufs[i]
        if tuple(pixel_values.shape) != tuple(px.shape):
            raise ValueError(f"pixel_values {tuple(pixel_values.shape)} do not match the vision tower's "
                             f"input {tuple(px.shape)}")
        if pixel_values.device != px.device:
            raise ValueError(f"pixel_values on {pixel_values.device}, the vision tower runs on {px.device}")
        with L.stage("vision", self.device):
            if pixel_values.dtype == torch.bfloat16:
                px.copy_(pixel_values)
            else:
                K.cast_bf16(pixel_values.contiguous(), px)
            self.vision.forward_into(px, self.vis_bufs[i])

    def forward_backward(self, pixel_values, token_ids, labels, next_pixel_values=None):
        """Everything up to (and including) the projector grads; returns loss (device [1]).
        next_pixel_values: the following step's pixels, whose SigLIP forward then runs on the side stream
        during this step's Gemma3 forward/backward (that step must pass the same pixels)."""
        B, T = token_ids.shape
        self._buffers(B, T)
        main = torch.cuda.current_stream(self.device)
        i = self._cur
        if self._prefetched is not None:
            main.wait_event(self._prefetched)
            self._prefetched = None
        elif self._vision_ready:
            self._vision_ready = False       # encode_vision already ran this batch's tower
        else:
            self._vision(pixel_values, i)
        self.px, self.vis = self.px_bufs[i], self.vis_bufs[i]
        # projector rows (b, i) -> LLM rows b*Sp + i - 1; patch 0 dropped (projector_trainer.py:173)
        self.proj.fwd_into(self.vis, self.a, self.h, self.x, out_map=(self.N, 1, self.Sp, -1), round_bf16=True)
        if next_pixel_values is not None:
            j = 1 - i
            consumed = torch.cuda.Event()
            consumed.record(main)   # SigLIP workspace and this step's features consumed by the projector
            if self.vstream is None:
                self.vstream = torch.cuda.Stream(self.device)
            self.vstream.wait_event(consumed)
            if self._released[j] is not None:
                self.vstream.wait_event(self._released[j])
            next_pixel_values.record_stream(self.vstream)
            with torch.cuda.stream(self.vstream):
                self._vision(next_pixel_values, j)
                ready = torch.cuda.Event()
                ready.record(self.vstream)
            self._prefetched = ready
            self._cur = j
        with L.stage("llm", self.device):
            self.llm.loss_and_input_grad(self.x, self.dx, token_ids, labels, self.N - 1,
                                         1.0 / float(self.gas * self.gas), self.loss, pad_token_id=self.pad_token_id)
        L.check(L.lib().ptk_gather_vision_grad(self.dx.data_ptr(), B, self.N, self.Sp, self.llm.cfg.hidden_size,
                                               self.dy.data_ptr(), L.stream_ptr(self.device)), "gather_vision_grad")
        if self.comm is not None:
            # the communicator's device must be the current HIP device (comm.cpp checks it), whichever device
            # the caller left current
            with torch.cuda.device(self.device):
                L.check(L.lib().ptk_projector_bwd_allreduce(self.proj.desc(), self.vis.shape[0], self.vis.data_ptr(),
                                                            self.a.data_ptr(), self.h.data_ptr(), self.dy.data_ptr(),
                                                            self.proj.flat_grad.data_ptr(), self.proj_ws.data_ptr(),
                                                            self.proj_ws.numel(), self.comm.handle,
                                                            self._comm_stream.cuda_stream, L.stream_ptr(self.device)),
                        "ptk_projector_bwd_allreduce")
            self._exchanged = True
        else:
            self.proj.bwd_into(self.vis, self.a, self.h, self.dy, self.proj_ws)
            self._exchanged = False
        if not torch.cuda.is_current_stream_capturing():   # (graph_step never prefetches)
            rel = torch.cuda.Event()
            rel.record(main)
            self._released[i] = rel
        return self.loss

    def forward_loss(self, pixel_values, token_ids, labels):
        """Loss only (the validation pass, projector_trainer.py:292-340 under no_grad): SigLIP, projector
        forward and the Gemma3 forward + CE (ptk_gemma3_loss_fwd); no backward, no exchange, grads untouched."""
        B, T = token_ids.shape
        self._buffers(B, T)
        if self._prefetched is not None:
            raise RuntimeError("Stage1Engine.forward_loss: a vision prefetch is pending")
        i = self._cur
        self._vision(pixel_values, i)
        self.px, self.vis = self.px_bufs[i], self.vis_bufs[i]
        self.proj.fwd_into(self.vis, self.a, self.h, self.x, out_map=(self.N, 1, self.Sp, -1), round_bf16=True)
        self.llm.loss_and_input_grad(self.x, None, token_ids, labels, self.N - 1, 1.0, self.loss,
                                     pad_token_id=self.pad_token_id)
        return self.loss

    def encode_vision(self, pixel_values, token_ids):
        """This step's SigLIP forward on its own, ahead of forward_backward (which then skips it): the
        trainer's skip-batch boundary (projector_trainer.py:158-176 logs a vision-tower exception and
        `continue`s before the projector runs).  An exception here leaves no projector state touched."""
        B, T = token_ids.shape
        self._buffers(B, T)
        if self._prefetched is not None:
            raise RuntimeError("Stage1Engine.encode_vision: a vision prefetch is pending")
        self._vision(pixel_values, self._cur)
        self._vision_ready = True

    def join_prefetch(self):
        """Make the current stream wait for an outstanding vision prefetch (end of a timed region)."""
        if self._prefetched is not None:
            torch.cuda.current_stream(self.device).wait_event(self._prefetched)

    def optimizer_step(self):
        """DDP all-reduce (sum; 1/W folded into the update), clip + AdamW, schedule."""
        if self._exchanged:      # summed over the ranks inside the backward (RCCL, overlapped)
            grad_scale = 1.0 / self.world
        else:
            with L.stage("grad_exchange", self.device) if self.world > 1 else contextlib.nullcontext():
                grad_scale = allreduce_grads_chunked_(self.proj.flat_grad, grad_exchange_chunks(self.proj),
                                                      self.world, self.pg)
        self._exchanged = False
        lr = self.lr0 * cosine_lambda(self.sched_step, self.warmup, self.total)
        self.opt_step += 1
        b1, b2 = self.betas
        with L.stage("optimizer", self.device):
            L.check(L.lib().ptk_clip_adamw(self.proj.flat.data_ptr(), self.proj.flat_grad.data_ptr(),
                                           self.exp_avg.data_ptr(), self.exp_avg_sq.data_ptr(),
                                           self.proj.flat.numel(), grad_scale, self.max_norm, lr, b1, b2, self.eps,
                                           self.wd, self.opt_step, self._partial.data_ptr(),
                                           self.grad_norm.data_ptr(), L.stream_ptr(self.device)), "clip_adamw")
            self.proj.refresh_shadows()
        self.sched_step += self.world
        self.last_lr = lr
        return lr

    def step(self, pixel_values, token_ids, labels, next_pixel_values=None):
        loss = self.forward_backward(pixel_values, token_ids, labels, next_pixel_values)
        self.optimizer_step()
        return loss

    def graph_step(self, pixel_values, token_ids, labels):
        """step() with forward_backward replayed from a HIP graph.  The ~900 kernel launches of the SigLIP,
        projector and Gemma3 passes are captured once per input shape and then replayed as one launch: at a
        small batch (cfg1: bs 2) the step is bound by launch latency, not by the kernels.  Capture needs every
        lazy initialisation (step buffers, workspaces, the projector's bf16 shadows) done, so at least one eager step()
        at this shape must precede the first call.  Inputs are copied into static buffers that the graph reads.
        The optimizer step stays eager: its learning rate and step count are kernel arguments that change every
        step (and the DDP all-reduce runs there).  Same kernels in the same order: bit-identical to step()."""
        if self._prefetched is not None or self._vision_ready:
            raise RuntimeError("Stage1Engine.graph_step: a vision prefetch / encode_vision is pending")
        if self.comm is not None:
            raise RuntimeError("Stage1Engine.graph_step: not with the RCCL exchange inside the backward")
        self._buffers(*token_ids.shape)
        # the graph replays the device pointers it was captured with: key it on every buffer it touches, so
        # a reallocation in between (an eager step at a larger batch or another text length, a grown
        # workspace) forces a new capture instead of replaying into freed memory
        key = (tuple(pixel_values.shape), pixel_values.dtype, tuple(token_ids.shape), tuple(labels.shape),
               self._buffer_fingerprint())
        if self._graph is None or self._graph_key != key:
            # a replaced graph is destroyed.  (Until round 4 it was kept alive: destroying one and capturing
            # another made the new graph's second and later replays compute NaN grads.  Root cause: the step's
            # three hipMemsetAsync calls became memset nodes of the captured graph; with them replaced by a
            # zero-fill kernel (csrc/misc.hip launch_zero) every destroy / re-capture sequence of
            # tools/graph_debug.py is bit-identical to eager, and with PTK_HIP_MEMSET=1 (memset nodes back)
            # the NaNs return -- profiles/r04_graph_memset_ab.txt.)
            self._graph = None
            self._graph_in = None
            static = (pixel_values.clone(), token_ids.clone(), labels.clone())
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):      # capture only: nothing runs until replay
                self.forward_backward(*static)
            self._graph, self._graph_key, self._graph_in = g, key, static
        else:
            for dst, src in zip(self._graph_in, (pixel_values, token_ids, labels)):
                dst.copy_(src)
        self._graph.replay()
        self.optimizer_step()
        return self.loss

    def _buffer_fingerprint(self):
        """Device addresses of everything forward_backward reads or writes (step buffers, workspaces,
        projector shadows) and the vision double-buffer index."""
        f = self._full
        ptrs = [t.data_ptr() for k in ("px", "vis") for t in f[k]]
        ptrs += [f[k].data_ptr() for k in ("a", "h", "x", "dx", "dy")]
        p = self.proj
        ptrs += [self.proj_ws.data_ptr(), self.loss.data_ptr(), p.flat.data_ptr(), p.flat_grad.data_ptr()]
        ptrs += [t.data_ptr() if t is not None else 0 for t in (getattr(p, "_w1b", None), getattr(p, "_w2b", None),
                                                               getattr(p, "_w2t", None))]
        ptrs += [self.vision._ws.data_ptr() if self.vision._ws is not None else 0,
                 self.llm._ws.data_ptr() if self.llm._ws is not None else 0]
        return (self._cur, self._cap) + tuple(ptrs)

    # ---------------------------------------------------------------- builders
    @classmethod
    def synthetic(cls, cfg: Stage1Config, device="cuda", seed=0, **kw):
        """Random-init towers of the named architecture (benchmark; no checkpoints offline)."""
        vision = SiglipVisionTower.random_init(cfg.vision, device, seed)
        llm = Gemma3CausalLM.random_init(cfg.text, device, seed + 1,
                                         max_pos=Gemma3CausalLM.seq_pad(cfg.seq_len))
        torch.manual_seed(seed + 2)
        proj = MLPProjector(cfg.vision.hidden_size, cfg.text.hidden_size, cfg.expansion_factor, device=device)
        return cls(vision, llm, proj, **kw)
