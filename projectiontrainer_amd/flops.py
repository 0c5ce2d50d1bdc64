"""Algorithmic FLOP count of one Stage-1 step per image.

Counts only what the math requires: dense 2·M·N·K on real tokens (no padding),
causal / sliding-window attention pairs only, the SigLIP MAP head excluded
(its output is discarded), lm_head on the T text-predicting rows only, the
frozen models' backward as dX only -- and the last Gemma3 layer's MLP on the
loss rows only: its other rows feed nothing but logits the loss never reads,
so libptk skips them (csrc/models.cpp gemma_run, `lossmap`: the last layer's
gate|up, down and their dX GEMMs run on the B·(T - label_offset) loss rows).
cfg2 -> 2.582 TFLOP/img (2.637 with the skipped rows, as rounds 1-5 counted).
"""
from __future__ import annotations

from .config import Stage1Config


def attention_pairs(S: int, window: int | None) -> int:
    """Number of (q, k) pairs with k <= q (and k > q - window)."""
    if window is None or window >= S:
        return S * (S + 1) // 2
    return window * (window + 1) // 2 + (S - window) * window


def attn_proj_flops_per_row(t) -> int:
    """q|k|v and o projections of one Gemma3 layer, one token row: 2·H·(q + 2 kv) + 2·q·H."""
    return 2 * t.hidden_size * (t.q_dim + 2 * t.kv_dim) + 2 * t.q_dim * t.hidden_size


def mlp_flops_per_row(t) -> int:
    """gate|up (2·H·2I) and down (2·I·H) of one Gemma3 layer, one token row."""
    return 2 * t.hidden_size * 2 * t.intermediate_size + 2 * t.intermediate_size * t.hidden_size


def gemma_dense_flops(cfg: Stage1Config, loss_rows: int) -> int:
    """Dense projection FLOPs of one Gemma3 pass (forward, or the dX backward, which has the same shapes) per
    image: every layer's q|k|v / o on all S rows, the MLP of layers 0..L-2 on all S rows and of the last layer on
    the `loss_rows` rows whose hidden state reaches the loss (models.cpp gemma_run: R = B·(T - label_offset))."""
    t, S = cfg.text, cfg.seq_len
    L = t.num_hidden_layers
    return L * S * attn_proj_flops_per_row(t) + ((L - 1) * S + loss_rows) * mlp_flops_per_row(t)


def flops_per_image(cfg: Stage1Config, loss_rows: int | None = None) -> dict:
    """Stage-1 step per image.  loss_rows: token rows per image whose last-layer state reaches the loss (Stage 1:
    all T text rows, position Nv-1+t predicts text token t; Stage 2: the answer rows)."""
    v, t = cfg.vision, cfg.text
    if loss_rows is None:
        loss_rows = cfg.text_len
    N, D, I = v.num_patches, v.hidden_size, v.intermediate_size
    vit = 2 * N * v.patch_dim * D
    vit += v.num_hidden_layers * (2 * N * D * 3 * D + 2 * 2 * N * N * D + 2 * N * D * D + 2 * 2 * N * D * I)
    Nv, Ip = cfg.num_vision_tokens, D * cfg.expansion_factor
    proj_f = 2 * Nv * (D * Ip + Ip * t.hidden_size)
    proj_b = 2 * Nv * (t.hidden_size * Ip) * 2 + 2 * Nv * Ip * D      # dW2, dH, dW1 (no dX)
    S, H = cfg.seq_len, t.hidden_size
    dense = gemma_dense_flops(cfg, loss_rows)
    attn = 0
    for i in range(t.num_hidden_layers):
        pairs = attention_pairs(S, t.sliding_window if t.is_sliding(i) else None)
        attn += 2 * 2 * pairs * t.head_dim * t.num_attention_heads
    head = 2 * loss_rows * H * t.vocab_size
    g_f = dense + attn + head
    g_b = dense + 2 * attn + head
    total = vit + proj_f + proj_b + g_f + g_b
    skipped = 2 * (S - loss_rows) * mlp_flops_per_row(t)     # the last layer's MLP rows no loss reads, fwd + dX
    return dict(vit_fwd=vit, proj_fwd=proj_f, proj_bwd=proj_b, llm_fwd=g_f, llm_bwd=g_b, total=total,
                skipped_last_mlp=skipped)


def geglu_gemm_flops(cfg: Stage1Config) -> float:
    """One Gemma3 gate|up projection launch (the step's largest kernel): 2·(B·S)·(2I)·H."""
    t = cfg.text
    return 2.0 * cfg.batch_size * cfg.seq_len * 2 * t.intermediate_size * t.hidden_size


def geglu_step_flops(cfg: Stage1Config) -> float:
    """Algorithmic FLOPs of all gate|up launches of one step: layers 0..L-2 on all B·S rows, the
    last layer on the B·T loss rows only (its other rows never reach the loss: libptk skips them)."""
    t = cfg.text
    per_row = 2.0 * 2 * t.intermediate_size * t.hidden_size
    return per_row * cfg.batch_size * (cfg.seq_len * (t.num_hidden_layers - 1) + cfg.text_len)


def geglu_algo_bytes(cfg: Stage1Config) -> float:
    """Algorithmic HBM bytes of one full-size gate|up launch: read the normed input xn [B*S, H] and the
    interleaved weight [2I, H] once, write h and the two saved GEGLU-backward factors [B*S, I] (bf16)."""
    t = cfg.text
    rows = cfg.batch_size * cfg.seq_len
    return 2.0 * (rows * t.hidden_size + 2 * t.intermediate_size * t.hidden_size + 3 * rows * t.intermediate_size)


def stage2_flops_per_image(cfg: Stage1Config) -> dict:
    """Algorithmic FLOPs of one Stage-2 (unfrozen LLM) micro-batch per image: frozen SigLIP and projector
    forward; Gemma3 forward with the lm_head and the last layer's MLP on the answer rows (the question rows carry
    no target, Stage2/trainer.py:390-396); backward = dX (as Stage 1) + every weight's dW = dY^T X (the dense
    GEMMs on the rows the forward ran them on, the tied lm_head on the answer rows).  The optimizer is
    HBM-bound and not counted."""
    Ta = cfg.text_len - cfg.question_len
    f = flops_per_image(cfg, loss_rows=Ta)
    t = cfg.text
    head = 2 * Ta * t.hidden_size * t.vocab_size
    g_f = f["llm_fwd"]
    g_b = f["llm_bwd"] + gemma_dense_flops(cfg, Ta) + head
    total = f["vit_fwd"] + f["proj_fwd"] + g_f + g_b
    return dict(vit_fwd=f["vit_fwd"], proj_fwd=f["proj_fwd"], llm_fwd=g_f, llm_bwd=g_b, total=total)
