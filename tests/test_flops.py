"""The algorithmic FLOP count behind `step_mfma_frac` follows the work the kernels do: the last
Gemma3 layer's MLP runs on the loss rows only (csrc/models.cpp gemma_run, `lossmap`), so it is counted on those
rows only.  The enumeration below restates gemma_run's GEMM calls (rows, N, K) one by one, independently of
flops.py's closed form."""
import pytest

from projectiontrainer_amd.config import PRESETS
from projectiontrainer_amd.flops import attention_pairs, flops_per_image, stage2_flops_per_image


def _gemma_gemms(cfg, loss_rows_per_img):
    """(rows, N, K) of every dense GEMM gemma_run issues in the forward for one image (padding rows excluded):
    per layer q|k|v and o on all S rows; gate|up and down on all S rows below the last layer and on the R loss
    rows in the last (models.cpp: `if (l + 1 < nl) ... else { ... R ... g.amap = lossmap }`); lm_head on R."""
    t, S = cfg.text, cfg.seq_len
    H, I, Dq, Dqkv = t.hidden_size, t.intermediate_size, t.q_dim, t.q_dim + 2 * t.kv_dim
    R = loss_rows_per_img
    out = []
    for l in range(t.num_hidden_layers):
        out += [(S, Dqkv, H), (S, H, Dq)]
        rows = S if l + 1 < t.num_hidden_layers else R
        out += [(rows, 2 * I, H), (rows, H, I)]
    out.append((R, t.vocab_size, H))
    return out


def _attn(cfg):
    t, S = cfg.text, cfg.seq_len
    return sum(2 * 2 * attention_pairs(S, t.sliding_window if t.is_sliding(i) else None) * t.head_dim *
               t.num_attention_heads for i in range(t.num_hidden_layers))


@pytest.mark.parametrize("name", ["cfg1", "cfg2", "cfg5"])
def test_stage1_llm_flops_follow_the_dispatched_rows(name):
    cfg = PRESETS[name]
    f = flops_per_image(cfg)
    dense = sum(2 * m * n * k for m, n, k in _gemma_gemms(cfg, cfg.text_len))
    # forward: the GEMMs + attention pairs; backward dX: the same GEMM shapes transposed + twice the pairs
    assert f["llm_fwd"] == dense + _attn(cfg)
    assert f["llm_bwd"] == dense + 2 * _attn(cfg)
    # what rounds 1-5 counted on top: the last layer's MLP on the S - T rows no loss reads, forward and dX
    t = cfg.text
    extra = 2 * (cfg.seq_len - cfg.text_len) * (2 * t.hidden_size * 2 * t.intermediate_size +
                                                 2 * t.intermediate_size * t.hidden_size)
    assert f["skipped_last_mlp"] == extra


def test_cfg2_flops_pinned():
    """cfg2 (SigLIP-L/16-384 + Gemma3-1B, T 128): 2.582 TFLOP per image (2.637 before the skipped rows came
    out; VERDICT r05 weak item 5: 54.9 GF/img credited but never executed)."""
    f = flops_per_image(PRESETS["cfg2"])
    assert round(f["total"] / 1e12, 3) == 2.582
    assert round(f["skipped_last_mlp"] / 1e9, 1) == 54.9
    assert round((f["total"] + f["skipped_last_mlp"]) / 1e12, 3) == 2.637
    # the declared target: step fraction 0.40 at 2.5 PFLOP/s dense bf16 = 387 img/s
    assert round(0.40 * 2.5e15 / f["total"]) == 387


def test_stage2_flops_follow_the_dispatched_rows():
    """cfg4: the last layer's MLP, the lm_head and their weight grads on the answer rows only."""
    cfg = PRESETS["cfg4"]
    Ta = cfg.text_len - cfg.question_len
    f = stage2_flops_per_image(cfg)
    dense = sum(2 * m * n * k for m, n, k in _gemma_gemms(cfg, Ta))
    s1 = flops_per_image(cfg, loss_rows=Ta)
    assert f["llm_fwd"] == dense + _attn(cfg)
    # dX + every weight grad (the same GEMM shapes once more, lm_head included)
    assert f["llm_bwd"] == dense + 2 * _attn(cfg) + dense
    assert f["total"] == s1["vit_fwd"] + s1["proj_fwd"] + f["llm_fwd"] + f["llm_bwd"]
