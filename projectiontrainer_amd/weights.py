"""Deterministic synthetic weights and batches (no checkpoints are reachable offline).

Every tensor is keyed by the HF state-dict name the reference would load
(`SiglipModel.vision_model.*`, `Gemma3ForCausalLM.*`, `MLPProjector.model.*`),
so the same dict feeds the reference (fixture generation), the CPU oracle and
the HIP path.  Values come from numpy's PCG64 stream seeded per tensor name, so
they are reproducible without storing them.
"""
from __future__ import annotations

import zlib

import numpy as np

from .config import Gemma3TextConfig, SiglipVisionConfig, Stage1Config


def _rng(seed: int, name: str) -> np.random.Generator:
    return np.random.default_rng([seed, zlib.crc32(name.encode())])


def _normal(seed, name, shape, std, mean=0.0):
    return (mean + std * _rng(seed, name).standard_normal(shape, dtype=np.float32)).astype(np.float32)


def siglip_vision_params(cfg: SiglipVisionConfig, seed: int = 0, prefix: str = "vision_model."):
    """HF-named SigLIP vision-tower weights.  Linear/conv/pos ~ N(0, 0.02²);
    LayerNorm weight 1+N(0,0.1²), biases N(0, 0.02²) (non-trivial affine so the
    fixtures exercise every term)."""
    D, I = cfg.hidden_size, cfg.intermediate_size
    p = {}
    e = prefix + "embeddings."
    p[e + "patch_embedding.weight"] = _normal(seed, e + "pw", (D, cfg.num_channels, cfg.patch_size, cfg.patch_size), 0.02)
    p[e + "patch_embedding.bias"] = _normal(seed, e + "pb", (D,), 0.02)
    p[e + "position_embedding.weight"] = _normal(seed, e + "pos", (cfg.num_patches, D), 0.02)
    for i in range(cfg.num_hidden_layers):
        L = f"{prefix}encoder.layers.{i}."
        for ln in ("layer_norm1", "layer_norm2"):
            p[L + ln + ".weight"] = _normal(seed, L + ln + "w", (D,), 0.1, 1.0)
            p[L + ln + ".bias"] = _normal(seed, L + ln + "b", (D,), 0.02)
        for proj in ("q_proj", "k_proj", "v_proj", "out_proj"):
            p[L + f"self_attn.{proj}.weight"] = _normal(seed, L + proj + "w", (D, D), 0.02)
            p[L + f"self_attn.{proj}.bias"] = _normal(seed, L + proj + "b", (D,), 0.02)
        p[L + "mlp.fc1.weight"] = _normal(seed, L + "fc1w", (I, D), 0.02)
        p[L + "mlp.fc1.bias"] = _normal(seed, L + "fc1b", (I,), 0.02)
        p[L + "mlp.fc2.weight"] = _normal(seed, L + "fc2w", (D, I), 0.02)
        p[L + "mlp.fc2.bias"] = _normal(seed, L + "fc2b", (D,), 0.02)
    p[prefix + "post_layernorm.weight"] = _normal(seed, prefix + "plnw", (D,), 0.1, 1.0)
    p[prefix + "post_layernorm.bias"] = _normal(seed, prefix + "plnb", (D,), 0.02)
    return p


def gemma3_params(cfg: Gemma3TextConfig, seed: int = 1):
    """HF-named Gemma3ForCausalLM weights (lm_head tied to embed_tokens).
    Linear/embedding ~ N(0, 0.02²); RMSNorm weights N(0, 0.1²) around the
    HF zero init so the (1+w) scale is exercised."""
    H, I = cfg.hidden_size, cfg.intermediate_size
    p = {"model.embed_tokens.weight": _normal(seed, "embed", (cfg.vocab_size, H), 0.02)}
    for i in range(cfg.num_hidden_layers):
        L = f"model.layers.{i}."
        p[L + "self_attn.q_proj.weight"] = _normal(seed, L + "q", (cfg.q_dim, H), 0.02)
        p[L + "self_attn.k_proj.weight"] = _normal(seed, L + "k", (cfg.kv_dim, H), 0.02)
        p[L + "self_attn.v_proj.weight"] = _normal(seed, L + "v", (cfg.kv_dim, H), 0.02)
        p[L + "self_attn.o_proj.weight"] = _normal(seed, L + "o", (H, cfg.q_dim), 0.02)
        p[L + "self_attn.q_norm.weight"] = _normal(seed, L + "qn", (cfg.head_dim,), 0.1)
        p[L + "self_attn.k_norm.weight"] = _normal(seed, L + "kn", (cfg.head_dim,), 0.1)
        p[L + "mlp.gate_proj.weight"] = _normal(seed, L + "g", (I, H), 0.02)
        p[L + "mlp.up_proj.weight"] = _normal(seed, L + "u", (I, H), 0.02)
        p[L + "mlp.down_proj.weight"] = _normal(seed, L + "d", (H, I), 0.02)
        for n in ("input_layernorm", "post_attention_layernorm",
                  "pre_feedforward_layernorm", "post_feedforward_layernorm"):
            p[L + n + ".weight"] = _normal(seed, L + n, (H,), 0.1)
    p["model.norm.weight"] = _normal(seed, "final_norm", (H,), 0.1)
    return p


def projector_params(vision_dim: int, llm_dim: int, expansion_factor: int = 10, seed: int = 2):
    """MLPProjector (`Stage1/projectors.py:13-20`) state dict.  nn.Linear's
    default init is U(-1/sqrt(fan_in), 1/sqrt(fan_in)) for weight and bias."""
    inter = vision_dim * expansion_factor
    b1, b2 = 1.0 / np.sqrt(vision_dim), 1.0 / np.sqrt(inter)
    u = lambda n, shape, b: _rng(seed, n).uniform(-b, b, shape).astype(np.float32)
    return {"model.0.weight": u("w1", (inter, vision_dim), b1),
            "model.0.bias": u("b1", (inter,), b1),
            "model.2.weight": u("w2", (llm_dim, inter), b2),
            "model.2.bias": u("b2", (llm_dim,), b2)}


def synthetic_batch(cfg: Stage1Config, seed: int = 1234, max_pad: int | None = None):
    """(pixel_values f32 [B,3,H,W] in [-1,1), token_ids i64 [B,T], labels i64 [B,T]).

    Mirrors the batch contract of `XrayTextPairDataset.__getitem__`
    (`Stage1/train_projection_stage1.py:105-118`): left padding with the pad id,
    BOS first, labels = ids with pad -> -100.  SURVEY §8(d) recipe."""
    v, t = cfg.vision, cfg.text
    B, T = cfg.batch_size, cfg.text_len
    rng = np.random.default_rng(seed)
    px = rng.uniform(-1.0, 1.0, (B, v.num_channels, v.image_size, v.image_size)).astype(np.float32)
    max_pad = T // 4 if max_pad is None else max_pad
    ids = rng.integers(3, t.vocab_size, (B, T), dtype=np.int64)
    for b in range(B):
        k = int(rng.integers(0, max_pad + 1))
        ids[b, :k] = t.pad_token_id
        ids[b, k] = t.bos_token_id
    labels = ids.copy()
    labels[ids == t.pad_token_id] = -100
    return px, ids, labels


def synthetic_vqa_items(cfg: Stage1Config, n: int, seed: int = 21, q_len=(3, 8), a_len=(4, 12)):
    """n VQA samples in the reference's Stage-2 item format (Stage2/dataset.py:115-119): pixel_values
    f32 [3,H,W] in [-1,1), question ids (tokenised without special tokens, :98-103) of length in q_len,
    answer ids (with special tokens: BOS first, :106-110) of 1 + length in a_len."""
    import torch
    rng = np.random.default_rng(seed)
    v, t = cfg.vision, cfg.text
    px = rng.uniform(-1.0, 1.0, (n, v.num_channels, v.image_size, v.image_size)).astype(np.float32)
    items = []
    for i in range(n):
        q = rng.integers(3, t.vocab_size, int(rng.integers(q_len[0], q_len[1] + 1)), dtype=np.int64)
        a = np.concatenate([[t.bos_token_id],
                            rng.integers(3, t.vocab_size, int(rng.integers(a_len[0], a_len[1] + 1)), dtype=np.int64)])
        items.append({"pixel_values": torch.from_numpy(px[i]), "question_input_ids": torch.from_numpy(q),
                      "answer_input_ids": torch.from_numpy(a.astype(np.int64))})
    return items


def synthetic_vqa_batch(cfg: Stage1Config, seed: int = 1234, padding_side: str = "left"):
    """One collated Stage-2 batch (vqa_collate_fn output, Stage2/trainer.py:18-61) at cfg's shapes:
    pixel_values f32 [B,3,H,W], question ids [B, question_len], answer ids [B, text_len - question_len]
    (BOS first), each sample's tokens covering 3/4..all of the padded length (pad id elsewhere)."""
    v, t = cfg.vision, cfg.text
    B, Tq = cfg.batch_size, cfg.question_len
    Ta = cfg.text_len - Tq
    rng = np.random.default_rng(seed)
    px = rng.uniform(-1.0, 1.0, (B, v.num_channels, v.image_size, v.image_size)).astype(np.float32)
    q = np.full((B, Tq), t.pad_token_id, dtype=np.int64)
    a = np.full((B, Ta), t.pad_token_id, dtype=np.int64)
    for b in range(B):
        nq = int(rng.integers(max(1, 3 * Tq // 4), Tq + 1))
        na = int(rng.integers(max(2, 3 * Ta // 4), Ta + 1))
        qq = rng.integers(3, t.vocab_size, nq, dtype=np.int64)
        aa = np.concatenate([[t.bos_token_id], rng.integers(3, t.vocab_size, na - 1, dtype=np.int64)])
        if padding_side == "left":
            q[b, Tq - nq:], a[b, Ta - na:] = qq, aa
        else:
            q[b, :nq], a[b, :na] = qq, aa
    return px, q, a
