"""Model/step configurations for the Stage-1 projector path.

Field names follow the HF configs the reference loads by name
(`Stage1/train_projection_stage1.py:179-210`): `SiglipVisionConfig` and
`Gemma3TextConfig`.  Presets are the public architectures the benchmark names
(BASELINE.json configs) plus tiny variants used by the parity fixtures.
"""
from __future__ import annotations

import dataclasses
from dataclasses import dataclass, field


@dataclass(frozen=True)
class SiglipVisionConfig:
    """SigLIP vision tower (TF/models/siglip/configuration_siglip.py)."""
    image_size: int = 384
    patch_size: int = 16
    num_channels: int = 3
    hidden_size: int = 1024
    num_attention_heads: int = 16
    intermediate_size: int = 4096
    num_hidden_layers: int = 24
    layer_norm_eps: float = 1e-6

    @property
    def num_patches(self) -> int:
        return (self.image_size // self.patch_size) ** 2

    @property
    def head_dim(self) -> int:
        return self.hidden_size // self.num_attention_heads

    @property
    def patch_dim(self) -> int:
        return self.num_channels * self.patch_size * self.patch_size


@dataclass(frozen=True)
class Gemma3TextConfig:
    """Gemma3 decoder (TF/models/gemma3/configuration_gemma3.py)."""
    vocab_size: int = 262144
    hidden_size: int = 1152
    intermediate_size: int = 6912
    num_hidden_layers: int = 26
    num_attention_heads: int = 4
    num_key_value_heads: int = 1
    head_dim: int = 256
    sliding_window: int = 512
    sliding_window_pattern: int = 6          # layer i is full attention iff (i+1) % pattern == 0
    rope_theta: float = 1_000_000.0          # full-attention layers
    rope_local_base_freq: float = 10_000.0   # sliding layers
    rope_linear_factor: float = 1.0          # linear RoPE scaling on full layers (4B: 8.0)
    query_pre_attn_scalar: int = 256
    rms_norm_eps: float = 1e-6
    pad_token_id: int = 0
    eos_token_id: int = 1
    bos_token_id: int = 2

    def is_sliding(self, layer: int) -> bool:
        return (layer + 1) % self.sliding_window_pattern != 0

    @property
    def q_dim(self) -> int:
        return self.num_attention_heads * self.head_dim

    @property
    def kv_dim(self) -> int:
        return self.num_key_value_heads * self.head_dim

    @property
    def group(self) -> int:
        return self.num_attention_heads // self.num_key_value_heads


@dataclass(frozen=True)
class Stage1Config:
    """One Stage-1 step: SigLIP fwd -> projector -> Gemma3 fwd/bwd -> AdamW."""
    vision: SiglipVisionConfig = field(default_factory=SiglipVisionConfig)
    text: Gemma3TextConfig = field(default_factory=Gemma3TextConfig)
    expansion_factor: int = 10               # Stage1/projectors.py:13
    batch_size: int = 32
    text_len: int = 128
    # Stage 2 (VQA): the first question_len text tokens are the question (no targets), the rest the answer
    # (Stage2/trainer.py:370-396); Stage 1: 0 (every text token is a target)
    question_len: int = 0

    @property
    def num_vision_tokens(self) -> int:
        # patch 0 is dropped at Stage1/projector_trainer.py:173 (SigLIP has no CLS token)
        return self.vision.num_patches - 1

    @property
    def seq_len(self) -> int:
        return self.num_vision_tokens + self.text_len

    def replace(self, **kw) -> "Stage1Config":
        return dataclasses.replace(self, **kw)


# ---- presets ---------------------------------------------------------------

SIGLIP_L16_384 = SiglipVisionConfig()
SIGLIP_B16_224 = SiglipVisionConfig(image_size=224, patch_size=16, hidden_size=768,
                                    num_attention_heads=12, intermediate_size=3072,
                                    num_hidden_layers=12)
GEMMA3_1B = Gemma3TextConfig()
GEMMA3_4B = Gemma3TextConfig(vocab_size=262208, hidden_size=2560, intermediate_size=10240,
                             num_hidden_layers=34, num_attention_heads=8, num_key_value_heads=4,
                             head_dim=256, sliding_window=1024, rope_linear_factor=8.0)

# Tiny shapes for golden fixtures (every dim a multiple of 64, as the GEMM wants).
SIGLIP_TINY = SiglipVisionConfig(image_size=32, patch_size=8, hidden_size=128,
                                 num_attention_heads=2, intermediate_size=256,
                                 num_hidden_layers=2)
GEMMA3_TINY = Gemma3TextConfig(vocab_size=512, hidden_size=128, intermediate_size=256,
                               num_hidden_layers=3, num_attention_heads=2,
                               num_key_value_heads=1, head_dim=64, sliding_window=8,
                               sliding_window_pattern=3, query_pre_attn_scalar=64)
GEMMA3_TINY_GQA = Gemma3TextConfig(vocab_size=512, hidden_size=128, intermediate_size=256,
                                   num_hidden_layers=3, num_attention_heads=4,
                                   num_key_value_heads=2, head_dim=64, sliding_window=8,
                                   sliding_window_pattern=3, query_pre_attn_scalar=64,
                                   rope_linear_factor=8.0)

PRESETS = {
    # BASELINE.json configs[1]: the headline single-GPU workload
    "cfg2": Stage1Config(vision=SIGLIP_L16_384, text=GEMMA3_1B, batch_size=32, text_len=128),
    # BASELINE.json configs[0]: the reference's CPU-runnable plumbing case
    "cfg1": Stage1Config(vision=SIGLIP_B16_224, text=GEMMA3_1B, batch_size=2, text_len=64),
    # BASELINE.json configs[4]
    "cfg5": Stage1Config(vision=SIGLIP_L16_384, text=GEMMA3_4B, batch_size=16, text_len=256),
    # BASELINE.json configs[3]: Stage 2 VQA fine-tune, Gemma3-1B unfrozen, 576 vis + 64 Q + 256 A tokens
    "cfg4": Stage1Config(vision=SIGLIP_L16_384, text=GEMMA3_1B, batch_size=16, text_len=64 + 256, question_len=64),
    # cfg2 WIDTHS at reduced depth for reference-generated fixtures (tests/golden/make_golden.py: the reference's own
    # train() at SigLIP-L/16-384 + Gemma3-1B widths, 2 + 6 layers with one global Gemma layer, bs 2, T 128 -- S 703
    # > the 512-key sliding window, the step's per-layer shapes at bs 2)
    "cfg2w": Stage1Config(vision=SiglipVisionConfig(num_hidden_layers=2),
                          text=Gemma3TextConfig(num_hidden_layers=6), batch_size=2, text_len=128),
    # cfg5 WIDTHS at reduced depth (the same recipe at SigLIP-L/16-384 + Gemma3-4B widths: hidden 2560, GQA 8:4,
    # linear RoPE x8 on the one global layer of 6, vocab 262 208; bs 1, T 256 as cfg5's caption length)
    "cfg5w": Stage1Config(vision=SiglipVisionConfig(num_hidden_layers=2),
                          text=GEMMA3_4B.__class__(**{**GEMMA3_4B.__dict__, "num_hidden_layers": 6}), batch_size=1,
                          text_len=256),
    "tiny": Stage1Config(vision=SIGLIP_TINY, text=GEMMA3_TINY, batch_size=3, text_len=16),
    "tiny_gqa": Stage1Config(vision=SIGLIP_TINY, text=GEMMA3_TINY_GQA, batch_size=3, text_len=16),
}


def to_hf_dicts(cfg: Stage1Config):
    """kwargs for transformers' SiglipVisionConfig / Gemma3TextConfig (fixture generation)."""
    v, t = cfg.vision, cfg.text
    vis = dict(image_size=v.image_size, patch_size=v.patch_size, num_channels=v.num_channels,
               hidden_size=v.hidden_size, num_attention_heads=v.num_attention_heads,
               intermediate_size=v.intermediate_size, num_hidden_layers=v.num_hidden_layers,
               layer_norm_eps=v.layer_norm_eps, hidden_act="gelu_pytorch_tanh")
    full_rope = {"rope_type": "default", "rope_theta": t.rope_theta}
    if t.rope_linear_factor != 1.0:
        full_rope = {"rope_type": "linear", "rope_theta": t.rope_theta, "factor": t.rope_linear_factor}
    txt = dict(vocab_size=t.vocab_size, hidden_size=t.hidden_size,
               intermediate_size=t.intermediate_size, num_hidden_layers=t.num_hidden_layers,
               num_attention_heads=t.num_attention_heads,
               num_key_value_heads=t.num_key_value_heads, head_dim=t.head_dim,
               sliding_window=t.sliding_window, query_pre_attn_scalar=t.query_pre_attn_scalar,
               rms_norm_eps=t.rms_norm_eps, pad_token_id=t.pad_token_id,
               eos_token_id=t.eos_token_id, bos_token_id=t.bos_token_id,
               layer_types=["sliding_attention" if t.is_sliding(i) else "full_attention"
                            for i in range(t.num_hidden_layers)],
               rope_parameters={"sliding_attention": {"rope_type": "default",
                                                      "rope_theta": t.rope_local_base_freq},
                                "full_attention": full_rope},
               hidden_activation="gelu_pytorch_tanh")
    return vis, txt
