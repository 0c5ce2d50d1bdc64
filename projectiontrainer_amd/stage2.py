"""Stage 2 (VQA fine-tune, BASELINE cfg4) on MI355X: the unfrozen Gemma3 step.

The body of `with self.accelerator.accumulate(...)` in VQATrainerStage2.train
(Stage2/trainer.py:299-444) with the cfg4 flags (`--unfreeze_llm`; projector
and vision encoder frozen; no QLoRA):

  SigLIP fwd (frozen, :313-332)          ptk_siglip_fwd
  projector fwd (frozen, :336-337)       ptk_projector_fwd -> the LLM input's vision rows
  [proj ‖ E[q]·s ‖ E[a]·s], mask, labels (:339-396)   inside ptk_gemma3_train_fwd_bwd
  Gemma3 fwd + manual CE (:398-418)      ptk_gemma3_train_fwd_bwd (label_offset = question length)
  accelerator.backward(loss / gas) (:421-423)   same call: dX and EVERY weight grad, accumulated into
                                         the bf16 .grad buffer (loss scaled 1/gas^2)
  sync: DDP grad reduce                  ZeRO-1: RCCL reduce-scatter of the flat bf16 grads
  clip_grad_norm_(llm, 1.0) + AdamW (:426-442)   ptk_bf16_grad_scale_sumsq + all-reduce of the sum of
                                         squares + ptk_adamw_bf16 on the rank's shard, then RCCL
                                         all-gather of the updated parameters
  lr_scheduler.step() x num_processes    host-side cosine-with-warmup lambda

Parameter store: every Gemma3 parameter lives in ONE flat bf16 buffer in the kernel layouts (q|k|v fused,
gate/up interleaved per 16 rows), the layer tensors being views of it; the grads in a second buffer of the
same layout.  Under `--mixed_precision bf16` the reference loads the LLM in bf16
(train_vqa_stage2.py:141-147,180-187), so its parameters, grads and AdamW moments are bf16 tensors: the
store keeps exactly that (no fp32 master copy), and the optimizer rounds every tensor op to bf16 as
torch's AdamW does on bf16 parameters.  The transposed copies the dX GEMMs read and the fp32 copies of the
norm weights the norm kernels read are refreshed after each optimizer step.
"""
from __future__ import annotations

import math

import torch
import torch.distributed as dist

from . import _lib as L
from . import kernels as K
from .gemma3 import Gemma3CausalLM
from .projectors import MLPProjector
from .siglip import SiglipVisionTower
from .stage1 import cosine_lambda

LAYER_KEYS = ("wqkv", "wo", "wgu", "wd", "ln_in", "ln_post_attn", "ln_pre_ff", "ln_post_ff", "q_norm", "k_norm")
NORM_KEYS = ("ln_in", "ln_post_attn", "ln_pre_ff", "ln_post_ff", "q_norm", "k_norm")
HF_NORM = {"ln_in": "input_layernorm", "ln_post_attn": "post_attention_layernorm",
           "ln_pre_ff": "pre_feedforward_layernorm", "ln_post_ff": "post_feedforward_layernorm",
           "q_norm": "self_attn.q_norm", "k_norm": "self_attn.k_norm"}


def deinterleave_gate_up(wgu):
    """[2I, H] interleaved per 16 rows -> gate [I, H], up [I, H] (inverse of gemma3.interleave_gate_up)."""
    I2, H = wgu.shape
    v = wgu.view(I2 // 32, 2, 16, H)
    return v[:, 0].reshape(I2 // 2, H), v[:, 1].reshape(I2 // 2, H)


class Gemma3TrainState:
    """Flat bf16 parameter / grad store of an unfrozen Gemma3CausalLM (rebinds the model's tensors)."""

    ALIGN = 64   # elements: every segment 128-B aligned

    def __init__(self, llm: Gemma3CausalLM, world_size: int = 1):
        self.llm, self.world = llm, world_size
        cfg, dev = llm.cfg, llm.device
        # matrices first, then every norm weight in one contiguous region (its fp32 mirror, which the norm
        # kernels read, is refreshed with one copy)
        segs = [("embed", tuple(llm.embed.shape))]
        for i, lay in enumerate(llm.layers):
            segs += [(f"{i}.{k}", tuple(lay[k].shape)) for k in ("wqkv", "wo", "wgu", "wd")]
        norm_segs = [("final_norm", (cfg.hidden_size,))]
        for i, lay in enumerate(llm.layers):
            norm_segs += [(f"{i}.{k}", tuple(lay[k].shape)) for k in NORM_KEYS]
        off, self.offsets = 0, {}
        for j, (name, shape) in enumerate(segs + norm_segs):
            if j == len(segs):
                self.norm_lo = off
            self.offsets[name] = (off, shape)
            n = math.prod(shape)
            off += (n + self.ALIGN - 1) // self.ALIGN * self.ALIGN
        self.norm_hi = off
        unit = self.ALIGN * world_size
        self.numel = (off + unit - 1) // unit * unit          # equal ZeRO shards
        self.flat = torch.zeros(self.numel, dtype=torch.bfloat16, device=dev)
        self.grad = torch.zeros(self.numel, dtype=torch.bfloat16, device=dev)
        # copy the current weights in (bf16 matrices as they are; norm weights rounded to bf16, as the
        # reference's bf16-loaded model holds them), then rebind the model onto views of the store
        self.view("embed").copy_(llm.embed)
        self.view("final_norm").copy_(llm.final_norm)
        for i, lay in enumerate(llm.layers):
            for k in LAYER_KEYS:
                self.view(f"{i}.{k}").copy_(lay[k])
        llm.embed = self.view("embed")
        self.norm32 = torch.zeros(self.norm_hi - self.norm_lo, dtype=torch.float32, device=dev)
        n32 = lambda name: self.norm32[self.offsets[name][0] - self.norm_lo:][:math.prod(self.offsets[name][1])]
        llm.final_norm = n32("final_norm")
        for i, lay in enumerate(llm.layers):
            for k in ("wqkv", "wo", "wgu", "wd"):
                lay[k] = self.view(f"{i}.{k}")
            for k in NORM_KEYS:
                lay[k] = n32(f"{i}.{k}").view(self.offsets[f"{i}.{k}"][1])
        self.refresh()
        llm._build_c()
        self._build_grads_c()

    def view(self, name, buf=None):
        off, shape = self.offsets[name]
        return (self.flat if buf is None else buf)[off:off + math.prod(shape)].view(shape)

    def grad_view(self, name):
        return self.view(name, self.grad)

    def _build_grads_c(self):
        arr = (L.Gemma3LayerGradsC * len(self.llm.layers))()
        for i in range(len(self.llm.layers)):
            arr[i] = L.Gemma3LayerGradsC(*[self.grad_view(f"{i}.{k}").data_ptr() for k in LAYER_KEYS])
        self._c_layer_grads = arr
        self.c_grads = L.Gemma3GradsC(self.grad_view("embed").data_ptr(), self.grad_view("final_norm").data_ptr(),
                                      arr)

    def refresh(self):
        """Derived copies the kernels read: transposed matrices (dX GEMMs) and fp32 norm weights."""
        llm = self.llm
        self.norm32.copy_(self.flat[self.norm_lo:self.norm_hi])
        for lay in llm.layers:
            for k in ("wqkv", "wo", "wgu", "wd"):
                K.transpose(lay[k], out=lay[k + "_t"])
        K.transpose(llm.embed, out=llm.embed_t)

    def zero_grad(self):
        self.grad.zero_()

    def shard(self, rank):
        n = self.numel // self.world
        return rank * n, n

    def state_dict_hf(self, grads=False):
        """HF Gemma3ForCausalLM names (lm_head tied, not listed), bf16 tensors on the device."""
        cfg = self.llm.cfg
        v = self.grad_view if grads else self.view
        Dq, Dkv = cfg.q_dim, cfg.kv_dim
        sd = {"model.embed_tokens.weight": v("embed")}
        for i in range(len(self.llm.layers)):
            p = f"model.layers.{i}."
            wqkv = v(f"{i}.wqkv")
            sd[p + "self_attn.q_proj.weight"] = wqkv[:Dq]
            sd[p + "self_attn.k_proj.weight"] = wqkv[Dq:Dq + Dkv]
            sd[p + "self_attn.v_proj.weight"] = wqkv[Dq + Dkv:]
            sd[p + "self_attn.o_proj.weight"] = v(f"{i}.wo")
            g, u = deinterleave_gate_up(v(f"{i}.wgu"))
            sd[p + "mlp.gate_proj.weight"], sd[p + "mlp.up_proj.weight"] = g, u
            sd[p + "mlp.down_proj.weight"] = v(f"{i}.wd")
            for k in NORM_KEYS:
                sd[p + HF_NORM[k] + ".weight"] = v(f"{i}.{k}")
        sd["model.norm.weight"] = v("final_norm")
        return sd


class Stage2Engine:
    """One VQATrainerStage2 micro-batch (forward_backward) and optimizer step (optimizer_step)."""

    def __init__(self, vision: SiglipVisionTower, llm: Gemma3CausalLM, projector: MLPProjector, *,
                 learning_rate=1e-4, weight_decay=0.01, gradient_accumulation_steps=1, max_grad_norm=1.0,
                 warmup_steps=0, total_steps=1, betas=(0.9, 0.999), eps=1e-8, world_size=1, rank=0,
                 process_group=None, pad_token_id=None, zero1=None):
        self.vision, self.llm, self.proj = vision, llm, projector
        self.device = vision.device
        self.lr0, self.wd, self.gas, self.max_norm = learning_rate, weight_decay, gradient_accumulation_steps, max_grad_norm
        self.warmup, self.total, self.betas, self.eps = warmup_steps, total_steps, betas, eps
        self.world, self.rank, self.pg = world_size, rank, process_group
        self.pad_token_id = llm.cfg.pad_token_id if pad_token_id is None else pad_token_id
        # zero1: reduce-scatter / sharded AdamW / all-gather through the process group (default: world > 1;
        # True at world 1 runs the same collectives on a one-rank group, which tests the RCCL path on one GPU)
        self.zero1 = world_size > 1 if zero1 is None else bool(zero1)
        if world_size > 1 and not self.zero1:
            # the optimizer step exchanges grads only through the reduce-scatter / all-gather of ZeRO-1; without
            # it every rank would update from its own grads and the replicas would drift apart
            raise ValueError("Stage2Engine: zero1=False is not supported with world_size > 1")
        self.state = Gemma3TrainState(llm, world_size)
        o, n = self.state.shard(rank)
        self.shard_lo, self.shard_n = o, n
        self.exp_avg = torch.zeros(n, dtype=torch.bfloat16, device=self.device)
        self.exp_avg_sq = torch.zeros(n, dtype=torch.bfloat16, device=self.device)
        self._shard_grad = torch.empty(n, dtype=torch.bfloat16, device=self.device) if self.zero1 else None
        self._shard_param = torch.empty(n, dtype=torch.bfloat16, device=self.device) if self.zero1 else None
        self._partial = torch.empty(L.lib().ptk_bf16_sumsq_partial_floats(), dtype=torch.float32, device=self.device)
        self.sumsq = torch.zeros(1, dtype=torch.float32, device=self.device)
        self.grad_norm = torch.zeros(1, dtype=torch.float32, device=self.device)
        self.loss = torch.zeros(1, dtype=torch.float32, device=self.device)
        self.opt_step = 0
        self.sched_step = 0
        self.last_lr = learning_rate * cosine_lambda(0, warmup_steps, total_steps)
        self._shape = None

    def _buffers(self, B, T):
        if self._shape == (B, T):
            return
        vc, tc = self.vision.cfg, self.llm.cfg
        N, Dv, Dl, I = vc.num_patches, vc.hidden_size, tc.hidden_size, self.proj.inter_dim
        Sp = Gemma3CausalLM.seq_pad(N - 1 + T)
        dev, bf = self.device, torch.bfloat16
        self.N, self.Sp = N, Sp
        self.px = torch.empty((B, vc.num_channels, vc.image_size, vc.image_size), dtype=bf, device=dev)
        self.vis = torch.empty((B * N, Dv), dtype=bf, device=dev)
        self.a = torch.empty((B * N, I), dtype=bf, device=dev)
        self.h = torch.empty((B * N, I), dtype=bf, device=dev)
        self.x = torch.empty((B * Sp, Dl), dtype=torch.float32, device=dev)
        self.dx = torch.empty((B * Sp, Dl), dtype=torch.float32, device=dev)
        self.vision.workspace(B)
        n = L.lib().ptk_gemma3_train_workspace_bytes(self.llm.c_cfg, B, T, Sp)
        if getattr(self, "_ws", None) is None or self._ws.numel() < n:
            self._ws = None
            self._ws = torch.empty(n, dtype=torch.uint8, device=dev)
        self._shape = (B, T)

    def _inputs(self, pixel_values, question_ids, answer_ids):
        """Vision + projector rows of x, token ids and labels, and the batch descriptor."""
        B, Tq = question_ids.shape
        Ta = answer_ids.shape[1]
        T = Tq + Ta
        self._buffers(B, T)
        if tuple(pixel_values.shape) != tuple(self.px.shape):
            raise ValueError(f"pixel_values {tuple(pixel_values.shape)} do not match the vision tower's input "
                             f"{tuple(self.px.shape)}")
        if pixel_values.dtype == torch.bfloat16:
            self.px.copy_(pixel_values)
        else:
            K.cast_bf16(pixel_values.contiguous(), self.px)
        self.vision.forward_into(self.px, self.vis)
        self.proj.fwd_into(self.vis, self.a, self.h, self.x, out_map=(self.N, 1, self.Sp, -1), round_bf16=True)
        ids = torch.cat([question_ids, answer_ids], dim=1).contiguous()
        labels = answer_ids.masked_fill(answer_ids == self.pad_token_id, -100).contiguous()
        cfg = self.llm.c_cfg
        if self.pad_token_id != cfg.pad_token_id:
            cfg = L.Gemma3ConfigC.from_buffer_copy(cfg)
            cfg.pad_token_id = int(self.pad_token_id)
        bt = L.Gemma3BatchC(B, T, self.N - 1, self.Sp, ids.data_ptr(), labels.data_ptr(), self.x.data_ptr(),
                            self.dx.data_ptr(), 1.0 / float(self.gas * self.gas), self.loss.data_ptr(), Tq)
        self._ids, self._labels = ids, labels     # alive until the stream has consumed them
        return cfg, bt

    def forward_backward(self, pixel_values, question_ids, answer_ids):
        """One micro-batch: loss (device [1], the mean CE over answer tokens) and grads accumulated
        (scaled 1/gas^2: the trainer's loss / gas and Accelerator.backward's / gas)."""
        cfg, bt = self._inputs(pixel_values, question_ids, answer_ids)
        L.check(L.lib().ptk_gemma3_train_fwd_bwd(cfg, self.llm.c_w, bt, self.state.c_grads, self._ws.data_ptr(),
                                                 self._ws.numel(), L.stream_ptr(self.device)),
                "ptk_gemma3_train_fwd_bwd")
        return self.loss

    def forward_loss(self, pixel_values, question_ids, answer_ids):
        """Validation loss under no_grad (Stage2/trainer.py:518-591): forward + CE only, no grads touched."""
        cfg, bt = self._inputs(pixel_values, question_ids, answer_ids)
        L.check(L.lib().ptk_gemma3_loss_fwd(cfg, self.llm.c_w, bt, self._ws.data_ptr(), self._ws.numel(),
                                            L.stream_ptr(self.device)), "ptk_gemma3_loss_fwd")
        return self.loss

    def optimizer_step(self):
        """DDP grad average (ZeRO-1 reduce-scatter), clip_grad_norm_(max_norm), AdamW, all-gather, schedule."""
        st, stream = self.state, L.stream_ptr(self.device)
        lo, n = self.shard_lo, self.shard_n
        if self.zero1:
            reduce_scatter_(self._shard_grad, st.grad, self.world, self.rank, self.pg)
            g, scale = self._shard_grad, 1.0 / self.world
        else:
            g, scale = st.grad, 1.0
        L.check(L.lib().ptk_bf16_grad_scale_sumsq(g.data_ptr(), n, scale, self._partial.data_ptr(),
                                                  self.sumsq.data_ptr(), stream), "grad_scale_sumsq")
        if self.zero1:
            dist.all_reduce(self.sumsq, op=dist.ReduceOp.SUM, group=self.pg)
        lr = self.lr0 * cosine_lambda(self.sched_step, self.warmup, self.total)
        self.opt_step += 1
        b1, b2 = self.betas
        p = st.flat[lo:lo + n]
        L.check(L.lib().ptk_adamw_bf16(p.data_ptr(), g.data_ptr(), self.exp_avg.data_ptr(),
                                       self.exp_avg_sq.data_ptr(), n, self.sumsq.data_ptr(), self.max_norm, lr, b1,
                                       b2, self.eps, self.wd, self.opt_step, self.grad_norm.data_ptr(), stream),
                "adamw_bf16")
        if self.zero1:
            self._shard_param.copy_(p)
            all_gather_(st.flat, self._shard_param, self.world, self.pg)
        st.refresh()
        st.zero_grad()
        self.sched_step += self.world
        self.last_lr = lr       # the LR this optimizer step used (param_groups[0]["lr"] during .step())
        return lr

    @property
    def scheduler_lr(self):
        """lr_scheduler.get_last_lr()[0]: the LR after the scheduler stepped num_processes times per optimizer
        step, i.e. the next step's LR -- what the reference logs as train/learning_rate
        (Stage2/trainer.py:446-452)."""
        return self.lr0 * cosine_lambda(self.sched_step, self.warmup, self.total)

    # ------------------------------------------------------------------ optimizer state (ZeRO-1 shards)
    def optimizer_state(self):
        """This rank's optimizer shard (moments of params [shard_lo, shard_lo + shard_n) of the flat store)
        plus the step / schedule counters: every rank's file together is the full AdamW state."""
        return {"exp_avg": self.exp_avg.cpu(), "exp_avg_sq": self.exp_avg_sq.cpu(), "step": self.opt_step,
                "sched_step": self.sched_step, "shard": (self.shard_lo, self.shard_n), "world": self.world,
                "rank": self.rank, "numel": self.state.numel}

    def load_optimizer_state(self, sd):
        if (sd["world"], sd["rank"], sd["numel"]) != (self.world, self.rank, self.state.numel):
            raise ValueError(f"optimizer shard of world {sd['world']} rank {sd['rank']} (store {sd['numel']}) does "
                             f"not match this engine (world {self.world} rank {self.rank} store {self.state.numel})")
        self.exp_avg.copy_(sd["exp_avg"])
        self.exp_avg_sq.copy_(sd["exp_avg_sq"])
        self.opt_step, self.sched_step = int(sd["step"]), int(sd["sched_step"])


def synthetic_engine(cfg, device="cuda", seed=0, **kw):
    """Stage2Engine over random-init towers of the named architecture (benchmark; no checkpoints offline)."""
    vision = SiglipVisionTower.random_init(cfg.vision, device, seed)
    llm = Gemma3CausalLM.random_init(cfg.text, device, seed + 1, max_pos=Gemma3CausalLM.seq_pad(cfg.seq_len))
    torch.manual_seed(seed + 2)
    proj = MLPProjector(cfg.vision.hidden_size, cfg.text.hidden_size, cfg.expansion_factor, device=device)
    return Stage2Engine(vision, llm, proj, **kw)


def reduce_scatter_(out_shard, flat, world, rank, group=None):
    """Sum of `flat` over ranks, this rank's contiguous shard into out_shard (RCCL reduce-scatter; gloo
    has none: all-reduce and slice)."""
    if dist.get_backend(group) == "gloo":
        t = flat.float()            # gloo has no bf16 sum: fp32 sum of the bf16 values, one rounding
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
        n = out_shard.numel()
        out_shard.copy_(t[rank * n:(rank + 1) * n])
    else:
        dist.reduce_scatter_tensor(out_shard, flat, op=dist.ReduceOp.SUM, group=group)
    return out_shard


def all_gather_(flat, shard, world, group=None):
    if dist.get_backend(group) == "gloo":
        parts = [torch.empty(shard.shape, dtype=torch.float32, device=shard.device) for _ in range(world)]
        dist.all_gather(parts, shard.float(), group=group)     # bf16 -> fp32 -> bf16 is exact
        flat.copy_(torch.cat(parts))
    else:
        dist.all_gather_into_tensor(flat, shard, group=group)
    return flat
