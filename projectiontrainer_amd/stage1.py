"""Stage1Engine: one reference Stage-1 training iteration on MI355X.

The body of `for batch in progress_bar:` (Stage1/projector_trainer.py:152-245):

  pixels f32 -> bf16 (:168)             ptk_cast_f32_bf16
  SigLIP fwd, drop patch 0 (:158-173)   ptk_siglip_fwd (patch 0 is skipped by the projector's row map)
  projector fwd (:180)                  ptk_projector_fwd -> writes the LLM input's vision rows
  embed + cat + mask + labels (:183-220)  inside ptk_gemma3_loss_fwd_bwd
  Gemma3 fwd + loss + backward (:226-237) ptk_gemma3_loss_fwd_bwd (loss scaled 1/gas^2)
  projector bwd                         ptk_gather_vision_grad + ptk_projector_bwd
  DDP grad all-reduce                   torch.distributed.all_reduce (RCCL) on the flat fp32 grads
  clip_grad_norm_(5) + AdamW (:240-242) ptk_clip_adamw, then bf16 shadow refresh
  lr_scheduler.step() x num_processes   host-side cosine lambda (no device sync)

All buffers are allocated once per (batch, text_len); a step issues no host
synchronisation, so the loss is returned as a device tensor.
"""
from __future__ import annotations

import math

import torch

from . import _lib as L
from . import kernels as K
from .config import Stage1Config
from .dist import allreduce_grads_
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
                 world_size=1):
        self.vision, self.llm, self.proj = vision, llm, projector
        self.device = vision.device
        self.lr0, self.wd, self.gas, self.max_norm = learning_rate, weight_decay, gradient_accumulation_steps, max_grad_norm
        self.warmup, self.total, self.betas, self.eps = warmup_steps, total_steps, betas, eps
        self.pg, self.world = process_group, world_size
        self.opt_step = 0        # optimizer steps (AdamW bias correction)
        self.sched_step = 0      # LambdaLR steps (advanced num_processes times per step, F7)
        n = projector.flat.numel()
        self.exp_avg = torch.zeros(n, dtype=torch.float32, device=self.device)
        self.exp_avg_sq = torch.zeros(n, dtype=torch.float32, device=self.device)
        self._partial = torch.empty(1024, dtype=torch.float32, device=self.device)
        self.grad_norm = torch.zeros(1, dtype=torch.float32, device=self.device)
        self._shape = None
        self.last_lr = learning_rate * cosine_lambda(0, warmup_steps, total_steps)

    def _buffers(self, B, T):
        if self._shape == (B, T):
            return
        vc, tc = self.vision.cfg, self.llm.cfg
        N, Dv, Dl, I = vc.num_patches, vc.hidden_size, tc.hidden_size, self.proj.inter_dim
        S = (N - 1) + T
        Sp = Gemma3CausalLM.seq_pad(S)
        dev, bf = self.device, torch.bfloat16
        self.N, self.Sp = N, Sp
        self.px = torch.empty((B, vc.num_channels, vc.image_size, vc.image_size), dtype=bf, device=dev)
        self.vis = torch.empty((B * N, Dv), dtype=bf, device=dev)
        self.a = torch.empty((B * N, I), dtype=bf, device=dev)
        self.h = torch.empty((B * N, I), dtype=bf, device=dev)
        self.x = torch.empty((B * Sp, Dl), dtype=torch.float32, device=dev)
        self.dx = torch.empty((B * Sp, Dl), dtype=torch.float32, device=dev)
        self.dy = torch.empty((B * N, Dl), dtype=bf, device=dev)
        self.loss = torch.zeros(1, dtype=torch.float32, device=dev)
        self.proj_ws = torch.empty(self.proj.workspace_bytes(B * N), dtype=torch.uint8, device=dev)
        self.vision.workspace(B)
        self.llm.workspace(B, T, Sp)
        self._shape = (B, T)

    # ---------------------------------------------------------------- pieces
    def forward_backward(self, pixel_values, token_ids, labels):
        """Everything up to (and including) the projector grads; returns loss (device [1])."""
        B, T = token_ids.shape
        self._buffers(B, T)
        if pixel_values.dtype == torch.bfloat16:
            self.px.copy_(pixel_values)
        else:
            K.cast_bf16(pixel_values.contiguous(), self.px)
        self.vision.forward_into(self.px, self.vis)
        # projector rows (b, i) -> LLM rows b*Sp + i - 1; patch 0 dropped (projector_trainer.py:173)
        self.proj.fwd_into(self.vis, self.a, self.h, self.x, out_map=(self.N, 1, self.Sp, -1), round_bf16=True)
        self.llm.loss_and_input_grad(self.x, self.dx, token_ids, labels, self.N - 1,
                                     1.0 / float(self.gas * self.gas), self.loss)
        L.check(L.lib().ptk_gather_vision_grad(self.dx.data_ptr(), B, self.N, self.Sp, self.llm.cfg.hidden_size,
                                               self.dy.data_ptr(), L.stream_ptr(self.device)), "gather_vision_grad")
        self.proj.bwd_into(self.vis, self.a, self.h, self.dy, self.proj_ws)
        return self.loss

    def optimizer_step(self):
        """DDP all-reduce (sum; 1/W folded into the update), clip + AdamW, schedule."""
        grad_scale = allreduce_grads_(self.proj.flat_grad, self.world, self.pg)
        lr = self.lr0 * cosine_lambda(self.sched_step, self.warmup, self.total)
        self.opt_step += 1
        b1, b2 = self.betas
        L.check(L.lib().ptk_clip_adamw(self.proj.flat.data_ptr(), self.proj.flat_grad.data_ptr(),
                                       self.exp_avg.data_ptr(), self.exp_avg_sq.data_ptr(), self.proj.flat.numel(),
                                       grad_scale, self.max_norm, lr, b1, b2, self.eps, self.wd, self.opt_step,
                                       self._partial.data_ptr(), self.grad_norm.data_ptr(),
                                       L.stream_ptr(self.device)), "clip_adamw")
        self.proj.refresh_shadows()
        self.sched_step += self.world
        self.last_lr = lr
        return lr

    def step(self, pixel_values, token_ids, labels):
        loss = self.forward_backward(pixel_values, token_ids, labels)
        self.optimizer_step()
        return loss

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
