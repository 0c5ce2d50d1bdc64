"""CPU restatement of the stepwise decode with beam search (test infrastructure only: imported by tests/, never by
the product path).

* `decode_logits`: the logits a decode row sees at each step, recomputed over the whole sequence (no cache) with
  the oracle's Gemma3 forward (stage1_ref.gemma3_forward) and the position ids transformers' generate derives from
  the attention mask (GenerationMixin._prepare_position_ids_for_generation: cumsum(mask) - 1, masked -> 0; the
  generated tokens continue from the row's valid count).
* `beam_candidates`: one selection of GenerationMixin._get_top_k_continuations (transformers 5.x
  generation/utils.py; reached from Stage2/trainer.py:626 through generate(num_beams=3, do_sample=True, top_k=50,
  top_p=0.9)): log_softmax of the fp32 logits, with sampling the warpers TemperatureLogitsWarper, TopKLogitsWarper
  (keep >= the k-th largest, k >= min_tokens_to_keep) and TopPLogitsWarper (ascending sort, cumulative softmax,
  drop <= 1 - top_p, keep the last min_tokens_to_keep) on the log probs, + the running beam score; greedy: the
  n_cand largest over beams x vocab; sampling: the processed joint distribution (for distribution checks).
Parity pinned by tests/test_beam_cpu.py against transformers' own beam search on a tiny Gemma3ForCausalLM.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from oracle import stage1_ref as R


def generate_positions(mask):
    """[B, P] 0/1 -> HF's position ids for the prompt (cumsum - 1, 0 where masked) and each row's valid count."""
    m = torch.as_tensor(mask).long()
    pos = (m.cumsum(-1) - 1).masked_fill(m == 0, 0)
    return pos, m.sum(-1)


def decode_logits(p, cfg, prompt_embeds, prompt_mask, tokens, dtype=torch.float32, embed_dtype=torch.bfloat16):
    """Last-position logits [B, V] (fp32) of prompts [B, P, H] (mask [B, P]) followed by the tokens [B, t].
    embed_dtype: the embedding's weight dtype (bf16 as the device holds it; fp32 for an fp32 HF model, whose
    Gemma3TextScaledWordEmbedding scales by sqrt(H) unrounded)."""
    B, P, _ = prompt_embeds.shape
    mask = torch.as_tensor(prompt_mask).long()
    pos, nval = generate_positions(mask)
    x = prompt_embeds.to(dtype)
    t = tokens.shape[1] if tokens is not None else 0
    if t:
        e = R.embed_tokens(p, cfg, tokens, embed_dtype).to(dtype)
        x = torch.cat([x, e], 1)
        mask = torch.cat([mask, torch.ones(B, t, dtype=torch.long)], 1)
        pos = torch.cat([pos, nval[:, None] + torch.arange(t)[None]], 1)
    h = R.gemma3_forward(p, cfg, x, mask, dtype, position_ids=pos)
    E = R._t(p, "model.embed_tokens.weight", dtype)
    return F.linear(h[:, -1], E).float()


def processed_log_probs(logits, do_sample, top_k=0, top_p=1.0, temperature=1.0, min_keep=1):
    """[rows, V] fp32 logits -> the log probs after HF's warpers (-inf where filtered)."""
    lp = F.log_softmax(logits.float(), -1)
    if not do_sample:
        return lp
    if temperature != 1.0:
        lp = lp / temperature
    if top_k and top_k > 0:
        k = min(max(top_k, min_keep), lp.shape[-1])
        thr = torch.topk(lp, k, -1).values[..., -1:]
        lp = lp.masked_fill(lp < thr, float("-inf"))
    if top_p < 1.0:
        srt, idx = torch.sort(lp, descending=False)
        cum = srt.softmax(-1).cumsum(-1)
        drop = cum <= (1 - top_p)
        drop[..., -min_keep:] = False
        lp = lp.masked_fill(drop.scatter(-1, idx, drop), float("-inf"))
    return lp


def beam_candidates(logits, beam_scores, beams, n_cand, do_sample=False, top_k=0, top_p=1.0, temperature=1.0,
                    min_keep=1):
    """Greedy: (tokens, beam, accumulated) [B, n_cand] by descending accumulated log prob.  With do_sample the
    joint accumulated scores [B, beams * V] are returned as the 4th value (softmax of them = the draw's law)."""
    V = logits.shape[-1]
    lp = processed_log_probs(logits, do_sample, top_k, top_p, temperature, min_keep)
    acc = (lp + beam_scores.float()[:, None]).reshape(-1, beams * V)
    val, idx = torch.topk(acc, n_cand, -1)
    return idx % V, idx // V, val, acc
