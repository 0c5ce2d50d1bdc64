"""Gemma3CausalLM.from_hf reads both HF config shapes: transformers 4.51 (the reference's pin,
requirements.txt:6: sliding_window_pattern / rope_theta / rope_local_base_freq / rope_scaling) and the
installed 5.x (layer_types / rope_parameters); quantised or QLoRA LMs are rejected with a clear error."""
import types

import pytest

from projectiontrainer_amd.config import GEMMA3_1B, GEMMA3_4B, to_hf_dicts, Stage1Config
from projectiontrainer_amd.gemma3 import Gemma3CausalLM


def _v451(cfg, rope_scaling):
    return types.SimpleNamespace(vocab_size=cfg.vocab_size, hidden_size=cfg.hidden_size,
                                 intermediate_size=cfg.intermediate_size, num_hidden_layers=cfg.num_hidden_layers,
                                 num_attention_heads=cfg.num_attention_heads,
                                 num_key_value_heads=cfg.num_key_value_heads, head_dim=cfg.head_dim,
                                 sliding_window=cfg.sliding_window, sliding_window_pattern=6,
                                 rope_theta=1_000_000.0, rope_local_base_freq=10_000.0, rope_scaling=rope_scaling,
                                 query_pre_attn_scalar=cfg.query_pre_attn_scalar, rms_norm_eps=cfg.rms_norm_eps,
                                 pad_token_id=0)


@pytest.mark.parametrize("cfg,scaling", [(GEMMA3_1B, None), (GEMMA3_4B, {"rope_type": "linear", "factor": 8.0})])
def test_config_transformers_451_shape(cfg, scaling):
    assert Gemma3CausalLM.config_from_hf(_v451(cfg, scaling)) == cfg


@pytest.mark.parametrize("cfg", [GEMMA3_1B, GEMMA3_4B])
def test_config_transformers_5_shape(cfg):
    import transformers
    _, txt = to_hf_dicts(Stage1Config(text=cfg))
    hf = transformers.Gemma3TextConfig(**txt)
    got = Gemma3CausalLM.config_from_hf(hf)
    assert got == cfg.__class__(**{**cfg.__dict__, "eos_token_id": got.eos_token_id,
                                   "bos_token_id": got.bos_token_id})


def test_unsupported_rope_scaling_rejected():
    with pytest.raises(ValueError, match="rope_scaling"):
        Gemma3CausalLM.config_from_hf(_v451(GEMMA3_1B, {"rope_type": "yarn", "factor": 4.0}))


@pytest.mark.parametrize("attrs", [{"is_loaded_in_4bit": True}, {"peft_config": {}},
                                   {"config": types.SimpleNamespace(quantization_config={"load_in_4bit": True})}])
def test_quantised_lm_rejected(attrs):
    m = types.SimpleNamespace(config=types.SimpleNamespace(quantization_config=None))
    for k, v in attrs.items():
        setattr(m, k, v)
    with pytest.raises(ValueError, match="QLoRA"):
        Gemma3CausalLM.from_hf(m, device="cpu")
