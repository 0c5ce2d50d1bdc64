"""Beam search of the stepwise decode, CPU side: the host bookkeeping (projectiontrainer_amd/beam.py) and the
oracle (oracle/beam_ref.py) against transformers' own GenerationMixin._beam_search on a tiny random-init
Gemma3ForCausalLM -- the generate Stage 2's validation calls (Stage2/trainer.py:596-626) with a padded question in
the prompt (attention mask 0 on the pads).  Greedy beam search (do_sample=False) is deterministic, so the token
sequences must be equal; beam sampling draws from the same law and is checked on the GPU as a distribution.

Position ids: HF derives the prompt's from the mask (cumsum - 1) and continues from there.  transformers 4.51 (the
reference's pin) recomputes cumsum(mask) - 1 every step; 5.x (installed here) adds 1 to the last prompt position.
The two agree whenever the prompt's last token is not a pad -- always, with the left-padded question of the
reference's collate -- and the decode follows that value (the row's valid count + step - 1).  A right-padded
prompt would restart at position 1 under 5.x, an artefact of its update rule; it is not reproduced."""
import pytest
import torch

from projectiontrainer_amd import weights as W
from projectiontrainer_amd.beam import BeamSearch
from projectiontrainer_amd.config import PRESETS, to_hf_dicts


def _hf(name="tiny"):
    from transformers import Gemma3ForCausalLM, Gemma3TextConfig
    cfg = PRESETS[name]
    _, txt = to_hf_dicts(cfg)
    llm = Gemma3ForCausalLM(Gemma3TextConfig(**txt)).float().eval()
    lp = W.gemma3_params(cfg.text)
    res = llm.load_state_dict({k: torch.from_numpy(v) for k, v in lp.items()}, strict=False)
    assert set(res.missing_keys) <= {"lm_head.weight"}, res
    return cfg.text, {k: torch.from_numpy(v) for k, v in lp.items()}, llm


def _prompt(cfg, B=2, P=12, seed=0):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(B, P, cfg.hidden_size, generator=g)
    mask = torch.ones(B, P, dtype=torch.long)
    mask[0, 8:10] = 0      # [image tokens | pad pad | question]: Gemma's tokenizer pads on the left, so the
    if B > 1:              # collate (Stage2/trainer.py:18-60) puts the question's pads right after the image
        mask[1, 8:11] = 0
    return x, mask


def test_oracle_positions_match_hf_forward():
    """The oracle's forward with HF's generate position ids (cumsum(mask) - 1) equals the HF model's forward with
    those ids and the same mask (the prefill of a padded prompt, and a prompt + 3 tokens)."""
    from oracle import beam_ref as BR
    cfg, lp, llm = _hf()
    x, mask = _prompt(cfg)
    pos, nval = BR.generate_positions(mask)
    with torch.no_grad():
        ref = llm(inputs_embeds=x, attention_mask=mask, position_ids=pos).logits[:, -1].float()
    got = BR.decode_logits(lp, cfg, x, mask, None)
    torch.testing.assert_close(got, ref, rtol=1e-4, atol=1e-4)
    toks = torch.tensor([[5, 7, 9], [11, 3, 2]])
    emb = llm.get_input_embeddings()(toks)
    with torch.no_grad():
        ref = llm(inputs_embeds=torch.cat([x, emb], 1), attention_mask=torch.cat([mask, torch.ones(2, 3, dtype=torch.long)], 1),
                  position_ids=torch.cat([pos, nval[:, None] + torch.arange(3)], 1)).logits[:, -1].float()
    got = BR.decode_logits(lp, cfg, x, mask, toks, embed_dtype=torch.float32)
    torch.testing.assert_close(got, ref, rtol=1e-4, atol=1e-4)


def _run_beam(cfg, lp, x, mask, beams, max_new, eos, pad, length_penalty=1.0, early_stopping=False):
    """BeamSearch driven by the oracle's full-recompute logits and greedy candidates."""
    from oracle import beam_ref as BR
    B = x.shape[0]
    bs = BeamSearch(B, beams, max_new, eos, pad, length_penalty, early_stopping)
    xr, mr = x.repeat_interleave(beams, 0), mask.repeat_interleave(beams, 0)
    seqs = [[] for _ in range(B * beams)]
    logits = BR.decode_logits(lp, cfg, xr, mr, None, embed_dtype=torch.float32)
    while True:
        tok, beam, acc, _ = BR.beam_candidates(logits, bs.run_score.reshape(-1), beams, 2 * beams)
        ids, rows = bs.step(tok, beam, acc)
        if bs.finished:
            break
        seqs = [seqs[int(rows[r])] + [int(ids[r])] for r in range(B * beams)]
        logits = BR.decode_logits(lp, cfg, xr, mr, torch.tensor(seqs), embed_dtype=torch.float32)
    return bs.result()


@pytest.mark.parametrize("beams,max_new,eos_rank,lp_", [(3, 6, None, 1.0), (3, 8, 0, 1.0), (2, 7, 1, 0.5)])
def test_beam_search_matches_transformers(beams, max_new, eos_rank, lp_):
    """Greedy beam search: the same token sequences as transformers' generate(num_beams, do_sample=False) on the
    same prompts and mask.  eos_rank: the EOS id is the token the first beam step ranks there (so hypotheses finish
    early and the finished-hypothesis path, the length penalty and the early-stop heuristic all run)."""
    from oracle import beam_ref as BR
    cfg, lp, llm = _hf()
    x, mask = _prompt(cfg)
    eos = None
    if eos_rank is not None:
        lg = BR.decode_logits(lp, cfg, x, mask, None)
        eos = int(torch.argsort(lg[0], descending=True)[eos_rank])
    with torch.no_grad():
        ref = llm.generate(inputs_embeds=x, attention_mask=mask, max_new_tokens=max_new, num_beams=beams,
                           do_sample=False, eos_token_id=eos, pad_token_id=0, length_penalty=lp_,
                           early_stopping=False)
    got = _run_beam(cfg, lp, x, mask, beams, max_new, eos, 0, length_penalty=lp_)
    assert torch.equal(got, ref), (got, ref)


def test_beam_state_fill_value_quirk():
    """Unused positions hold `pad_token_id or eos_token_id` (HF's fill): a pad id of 0 falls through to eos."""
    assert BeamSearch(1, 2, 4, eos_token_id=1, pad_token_id=0).fill == 1
    assert BeamSearch(1, 2, 4, eos_token_id=1, pad_token_id=3).fill == 3


@pytest.mark.parametrize("eos_rank", [None, 0])
def test_oracle_greedy_generate_matches_transformers(eos_rank):
    """Stage 1's validation decode semantics (Stage1/projector_trainer.py:386-393 -> GenerationMixin._sample) pinned
    against transformers itself: the oracle's cache-free greedy decode (oracle/stage1_ref.py greedy_generate, which
    the GPU decode is checked against) gives the same tokens as generate(inputs_embeds=, attention_mask=ones,
    do_sample=False) on a tiny fp32 Gemma3ForCausalLM, including the finished-row padding and the stop step when an
    EOS id is set."""
    from oracle import stage1_ref as R
    cfg, lp, llm = _hf()
    g = torch.Generator().manual_seed(3)
    x = torch.randn(3, 12, cfg.hidden_size, generator=g)
    eos = None
    if eos_rank is not None:
        lg = torch.nn.functional.linear(R.gemma3_forward(lp, cfg, x, torch.ones(3, 12, dtype=torch.long))[:, -1],
                                        lp["model.embed_tokens.weight"])
        eos = int(lg[0].argmax())            # row 0 stops at once, the others run on
    with torch.no_grad():
        ref = llm.generate(inputs_embeds=x, attention_mask=torch.ones(3, 12, dtype=torch.long), max_new_tokens=6,
                           do_sample=False, eos_token_id=eos, pad_token_id=0)
    got, _ = R.greedy_generate(lp, cfg, x, 6, eos_token_id=eos, pad_token_id=0, embed_dtype=torch.float32)
    assert torch.equal(got, ref), (got, ref)
