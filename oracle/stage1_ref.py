"""CPU restatement of the reference Stage-1 step (pure torch, fp32 by default).

TEST INFRASTRUCTURE ONLY.  Imported by `tests/`, `__graft_entry__.smoke()` and
`bench.py`'s `cpu_baseline` leg as the checker / CPU baseline; the product path
(`projectiontrainer_amd`) never imports it.

Pinned against fixtures produced by the reference itself
(`tests/golden/make_golden.py` drives `Stage1/projector_trainer.py` with HF
transformers 5.15 SigLIP/Gemma3 modules).  Each function cites what it restates.
No transformers / reference import here: this is an independent restatement.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import torch
import torch.nn.functional as F

from projectiontrainer_amd.config import Gemma3TextConfig, SiglipVisionConfig

IGNORE = -100


def _t(p, name, dtype):
    return torch.as_tensor(p[name]).to(dtype)


# --------------------------------------------------------------------------- SigLIP
def siglip_vision_forward(p, cfg: SiglipVisionConfig, pixel_values, dtype=torch.float32,
                          prefix="vision_model."):
    """`SiglipVisionModel.forward` minus the unused MAP head
    (TF/models/siglip/modeling_siglip.py:576-619): conv patch embed + learned
    positions (:175-186), pre-LN encoder layers (:335-357; attention :271-307
    with scale head_dim**-0.5; MLP :318-322 with gelu_pytorch_tanh), post-LN."""
    W = lambda n: _t(p, prefix + n, dtype)
    x = pixel_values.to(dtype)
    B = x.shape[0]
    D, H = cfg.hidden_size, cfg.num_attention_heads
    hd = D // H
    e = F.conv2d(x, W("embeddings.patch_embedding.weight"), W("embeddings.patch_embedding.bias"),
                 stride=cfg.patch_size)
    h = e.flatten(2).transpose(1, 2) + W("embeddings.position_embedding.weight")[None]
    N = h.shape[1]
    eps = cfg.layer_norm_eps
    for i in range(cfg.num_hidden_layers):
        L = f"encoder.layers.{i}."
        r = h
        a = F.layer_norm(h, (D,), W(L + "layer_norm1.weight"), W(L + "layer_norm1.bias"), eps)
        q = F.linear(a, W(L + "self_attn.q_proj.weight"), W(L + "self_attn.q_proj.bias"))
        k = F.linear(a, W(L + "self_attn.k_proj.weight"), W(L + "self_attn.k_proj.bias"))
        v = F.linear(a, W(L + "self_attn.v_proj.weight"), W(L + "self_attn.v_proj.bias"))
        q, k, v = (t.view(B, N, H, hd).transpose(1, 2) for t in (q, k, v))
        s = torch.matmul(q, k.transpose(2, 3)) * hd ** -0.5
        o = torch.matmul(torch.softmax(s.float(), dim=-1).to(dtype), v)
        o = o.transpose(1, 2).reshape(B, N, D)
        h = r + F.linear(o, W(L + "self_attn.out_proj.weight"), W(L + "self_attn.out_proj.bias"))
        r = h
        a = F.layer_norm(h, (D,), W(L + "layer_norm2.weight"), W(L + "layer_norm2.bias"), eps)
        a = F.gelu(F.linear(a, W(L + "mlp.fc1.weight"), W(L + "mlp.fc1.bias")), approximate="tanh")
        h = r + F.linear(a, W(L + "mlp.fc2.weight"), W(L + "mlp.fc2.bias"))
    return F.layer_norm(h, (D,), W("post_layernorm.weight"), W("post_layernorm.bias"), eps)


# --------------------------------------------------------------------------- projector
def projector_forward(pp, x):
    """`MLPProjector.forward` (Stage1/projectors.py:16-29):
    Linear -> GELU (erf, nn.GELU default) -> Linear."""
    h = F.gelu(F.linear(x, pp["model.0.weight"], pp["model.0.bias"]))
    return F.linear(h, pp["model.2.weight"], pp["model.2.bias"])


# --------------------------------------------------------------------------- Gemma3
def rms_norm(x, w, eps):
    """Gemma3RMSNorm (TF/models/gemma3/modeling_gemma3.py:136-150): fp32 math,
    scale (1 + w), cast back to the input dtype."""
    xf = x.float()
    o = xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps)
    return (o * (1.0 + w.float())).type_as(x)


def rope_cos_sin(cfg: Gemma3TextConfig, seq_len: int, sliding: bool):
    """Gemma3RotaryEmbedding (:156-205): inv_freq = 1/theta^(2i/d) (linear
    scaling divides it by `factor` on full-attention layers), emb = [f, f]."""
    d = cfg.head_dim
    theta = cfg.rope_local_base_freq if sliding else cfg.rope_theta
    inv = 1.0 / (theta ** (torch.arange(0, d, 2, dtype=torch.int64).float() / d))
    if not sliding and cfg.rope_linear_factor != 1.0:
        inv = inv / cfg.rope_linear_factor
    pos = torch.arange(seq_len, dtype=torch.float32)
    f = pos[:, None] * inv[None, :]
    emb = torch.cat([f, f], dim=-1)
    return emb.cos(), emb.sin()


def _rotate_half(x):
    x1, x2 = x[..., : x.shape[-1] // 2], x[..., x.shape[-1] // 2:]
    return torch.cat((-x2, x1), dim=-1)


def attention_mask_4d(attention_mask, sliding_window: int | None):
    """Boolean [B,1,S,S] mask: causal & key-padding (& kv > q - window).
    TF/masking_utils.py:92-101 (sliding overlay), :168-177 (padding)."""
    B, S = attention_mask.shape
    q = torch.arange(S)[:, None]
    k = torch.arange(S)[None, :]
    m = k <= q
    if sliding_window is not None:
        m = m & (k > q - sliding_window)
    return m[None, None] & attention_mask.bool()[:, None, None, :]


def gemma3_forward(p, cfg: Gemma3TextConfig, inputs_embeds, attention_mask, dtype=torch.float32, position_ids=None):
    """`Gemma3TextModel.forward` with inputs_embeds (:511-578); decoder layer
    :399-429 (sandwich norms), attention :341-383 (q/k RMSNorm, RoPE, GQA via
    repeat_kv, scale query_pre_attn_scalar**-0.5), gated GELU-tanh MLP :131-133.
    position_ids = arange(S) (not pad-adjusted; the training forward), or [B, S] (generate: HF derives them from the
    attention mask).  Returns the final-norm output."""
    W = lambda n: _t(p, n, dtype)
    x = inputs_embeds.to(dtype)
    B, S, Hd = x.shape
    hd, nq, nkv = cfg.head_dim, cfg.num_attention_heads, cfg.num_key_value_heads
    eps = cfg.rms_norm_eps
    scale = cfg.query_pre_attn_scalar ** -0.5
    if position_ids is None:
        rope = {s: rope_cos_sin(cfg, S, s) for s in (True, False)}
    else:
        pid = torch.as_tensor(position_ids).long()
        n = int(pid.max()) + 1
        rope = {s: tuple(t[pid][:, None] for t in rope_cos_sin(cfg, n, s)) for s in (True, False)}
    masks = {True: attention_mask_4d(attention_mask, cfg.sliding_window),
             False: attention_mask_4d(attention_mask, None)}
    for i in range(cfg.num_hidden_layers):
        L = f"model.layers.{i}."
        sl = cfg.is_sliding(i)
        r = x
        a = rms_norm(x, W(L + "input_layernorm.weight"), eps)
        q = F.linear(a, W(L + "self_attn.q_proj.weight")).view(B, S, nq, hd).transpose(1, 2)
        k = F.linear(a, W(L + "self_attn.k_proj.weight")).view(B, S, nkv, hd).transpose(1, 2)
        v = F.linear(a, W(L + "self_attn.v_proj.weight")).view(B, S, nkv, hd).transpose(1, 2)
        q = rms_norm(q, W(L + "self_attn.q_norm.weight"), eps)
        k = rms_norm(k, W(L + "self_attn.k_norm.weight"), eps)
        cos, sin = rope[sl]
        q = q * cos + _rotate_half(q) * sin
        k = k * cos + _rotate_half(k) * sin
        k = k.repeat_interleave(nq // nkv, dim=1)
        v = v.repeat_interleave(nq // nkv, dim=1)
        s = torch.matmul(q, k.transpose(2, 3)) * scale
        s = s.masked_fill(~masks[sl], torch.finfo(s.dtype).min)
        o = torch.matmul(torch.softmax(s.float(), dim=-1).to(dtype), v)
        o = o.transpose(1, 2).reshape(B, S, nq * hd)
        o = F.linear(o, W(L + "self_attn.o_proj.weight"))
        x = r + rms_norm(o, W(L + "post_attention_layernorm.weight"), eps)
        r = x
        a = rms_norm(x, W(L + "pre_feedforward_layernorm.weight"), eps)
        g = F.gelu(F.linear(a, W(L + "mlp.gate_proj.weight")), approximate="tanh")
        m = F.linear(g * F.linear(a, W(L + "mlp.up_proj.weight")), W(L + "mlp.down_proj.weight"))
        x = r + rms_norm(m, W(L + "post_feedforward_layernorm.weight"), eps)
    return rms_norm(x, W("model.norm.weight"), eps)


def causal_lm_loss(hidden, embed_weight, labels):
    """Tied lm_head (:642-651) + `ForCausalLMLoss` (TF/loss/loss_utils.py:49-67):
    logits in fp32, shift labels left by one, mean CE over labels != -100.
    Only rows whose shifted label is valid are projected (same value as the
    reference's all-position lm_head)."""
    shift = F.pad(labels, (0, 1), value=IGNORE)[:, 1:]
    sel = shift != IGNORE
    logits = F.linear(hidden[sel], embed_weight.to(hidden.dtype)).float()
    return F.cross_entropy(logits, shift[sel], reduction="mean")


def embed_tokens(p, cfg: Gemma3TextConfig, token_ids, dtype=torch.float32):
    """Gemma3TextScaledWordEmbedding (:106-117): E[ids] * sqrt(H) cast to the
    weight dtype (bf16 weights -> 34.0 at H=1152)."""
    E = _t(p, "model.embed_tokens.weight", dtype)
    scale = torch.tensor(cfg.hidden_size ** 0.5, dtype=torch.float32).to(dtype)
    return E[token_ids] * scale


def greedy_generate(p, cfg: Gemma3TextConfig, prompt_embeds, max_new_tokens, eos_token_id=None, pad_token_id=0,
                    force_ids=None, dtype=torch.float32, embed_dtype=torch.bfloat16):
    """`GenerationMixin._sample` with do_sample=False over `Gemma3ForCausalLM` from inputs_embeds and an all-ones
    attention mask, as the reference's validation calls generate (Stage1/projector_trainer.py:386-393; greedy, so
    deterministic): each step's logits are the tied lm_head of the last position's final-norm output (recomputed
    over the whole sequence, no cache), the token is their argmax; a row that produced eos_token_id emits
    pad_token_id afterwards and the loop stops once every row has.  New tokens enter as their embedding, the bf16
    weight row times bf16(sqrt H) rounded to bf16 (Gemma3TextScaledWordEmbedding on bf16 weights).  force_ids
    [B, max_new_tokens]: teacher forcing (step t appends force_ids[:, t-1]).  Returns (tokens [B, n], logits
    [n, B, V] fp32)."""
    B, P, _ = prompt_embeds.shape
    E = _t(p, "model.embed_tokens.weight", dtype)
    x = prompt_embeds.to(dtype)
    unfinished = torch.ones(B, dtype=torch.bool)
    toks, logs = [], []
    for t in range(max_new_tokens):
        h = gemma3_forward(p, cfg, x, torch.ones(B, x.shape[1], dtype=torch.long), dtype)
        lg = F.linear(h[:, -1], E).float()
        tok = lg.argmax(-1)
        tok = torch.where(unfinished, tok, torch.full_like(tok, pad_token_id))
        toks.append(tok)
        logs.append(lg)
        if eos_token_id is not None:
            unfinished &= tok != eos_token_id
            if not unfinished.any():
                break
        feed = tok if force_ids is None else torch.as_tensor(force_ids)[:, t]
        e = embed_tokens(p, cfg, feed[:, None], embed_dtype).to(dtype)   # (fp32 for an fp32 HF model)
        x = torch.cat([x, e], dim=1)
    return torch.stack(toks, 1), torch.stack(logs, 0)


# --------------------------------------------------------------------------- step
@dataclass
class TrainState:
    """Projector params + AdamW moments (fp32), LR-scheduler step counter."""
    params: dict
    exp_avg: dict
    exp_avg_sq: dict
    step: int = 0          # optimizer steps taken
    sched_step: int = 0    # LambdaLR steps taken (accelerate steps it num_processes times)


def init_state(proj_params):
    P = {k: torch.as_tensor(v).float().clone() for k, v in proj_params.items()}
    return TrainState(P, {k: torch.zeros_like(v) for k, v in P.items()},
                      {k: torch.zeros_like(v) for k, v in P.items()})


def cosine_lambda(step, warmup, total, num_cycles=0.5):
    """`_get_cosine_schedule_with_warmup_lr_lambda` (TF/optimization.py:134-140).
    No clamp of progress past 1: the LR rises again after reaching 0."""
    if step < warmup:
        return float(step) / float(max(1, warmup))
    prog = float(step - warmup) / float(max(1, total - warmup))
    return max(0.0, 0.5 * (1.0 + math.cos(math.pi * float(num_cycles) * 2.0 * prog)))


def clip_grad_norm_(grads, max_norm):
    """torch.nn.utils.clip_grad_norm_ (foreach, norm_type 2): total = ||(||g_i||)||,
    coef = clamp(max_norm / (total + 1e-6), max=1)."""
    total = torch.linalg.vector_norm(torch.stack([torch.linalg.vector_norm(g) for g in grads]))
    coef = torch.clamp(max_norm / (total + 1e-6), max=1.0)
    for g in grads:
        g.mul_(coef)
    return total


def adamw_step(state: TrainState, grads, lr, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.01):
    """torch.optim.AdamW single-tensor math (decoupled decay, bias correction);
    the optimizer built at Stage1/projector_trainer.py:75-79."""
    state.step += 1
    b1, b2 = betas
    bc1 = 1 - b1 ** state.step
    bc2 = 1 - b2 ** state.step
    for k, g in grads.items():
        p, m, v = state.params[k], state.exp_avg[k], state.exp_avg_sq[k]
        p.mul_(1 - lr * weight_decay)
        m.lerp_(g, 1 - b1)
        v.mul_(b2).addcmul_(g, g, value=1 - b2)
        denom = (v.sqrt() / math.sqrt(bc2)).add_(eps)
        p.addcdiv_(m, denom, value=-(lr / bc1))


@dataclass
class StepConfig:
    """Trainer knobs that change the arithmetic (Stage1/projector_trainer.py:19-38,
    train_projection_stage1.py:138-161)."""
    learning_rate: float = 1e-4
    weight_decay: float = 0.01
    gradient_accumulation_steps: int = 2
    max_grad_norm: float = 5.0
    warmup_steps: int = 0
    total_steps: int = 1
    num_processes: int = 1


def stage1_forward_loss(vp, vcfg, lp, lcfg, proj_params, pixel_values, token_ids, labels,
                        dtype=torch.float32, embed_dtype=None):
    """Forward of one Stage-1 batch (Stage1/projector_trainer.py:152-233).
    Returns (loss, patch_embeddings, projected_embeds)."""
    with torch.no_grad():
        patch = siglip_vision_forward(vp, vcfg, pixel_values, dtype)[:, 1:, :]   # :173 drops patch 0
    proj = projector_forward(proj_params, patch.float())
    with torch.no_grad():
        text = embed_tokens(lp, lcfg, token_ids, embed_dtype or dtype).float()
    x = torch.cat([proj, text], dim=1)                                        # :195
    B, Nv = proj.shape[:2]
    mask = torch.cat([torch.ones(B, Nv, dtype=torch.long),
                      (token_ids != lcfg.pad_token_id).long()], dim=1)        # :201-212
    lm_labels = torch.cat([torch.full((B, Nv), IGNORE, dtype=labels.dtype), labels], dim=1)  # :215-220
    hidden = gemma3_forward(lp, lcfg, x, mask, dtype)
    loss = causal_lm_loss(hidden, _t(lp, "model.embed_tokens.weight", dtype), lm_labels)
    return loss, patch, proj


def stage1_step(vp, vcfg, lp, lcfg, state: TrainState, batch, sc: StepConfig,
                dtype=torch.float32, embed_dtype=None):
    """One reference trainer iteration (Stage1/projector_trainer.py:152-245) with
    the accelerate quirks of SURVEY F7: loss/gas twice (trainer :236 and
    `Accelerator.backward`), optimizer step every micro-batch, scheduler stepped
    `num_processes` times.  Returns a dict of observables."""
    pixel_values, token_ids, labels = (torch.as_tensor(t) for t in batch)
    params = {k: v.clone().requires_grad_(True) for k, v in state.params.items()}
    loss, patch, proj = stage1_forward_loss(vp, vcfg, lp, lcfg, params, pixel_values,
                                            token_ids, labels, dtype, embed_dtype)
    gas = sc.gradient_accumulation_steps
    proj.retain_grad()
    ((loss / gas) / gas).backward()
    grads = {k: v.grad.detach().clone() for k, v in params.items()}
    raw = {k: g.clone() for k, g in grads.items()}
    lr = sc.learning_rate * cosine_lambda(state.sched_step, sc.warmup_steps, sc.total_steps)
    total_norm = clip_grad_norm_(list(grads.values()), sc.max_grad_norm)
    adamw_step(state, grads, lr, weight_decay=sc.weight_decay)
    state.sched_step += sc.num_processes
    return {"loss": loss.detach(), "patch": patch.detach(), "proj": proj.detach(),
            "d_proj": proj.grad.detach(), "grads": raw, "clipped": grads,
            "grad_norm": total_norm, "lr": lr}
