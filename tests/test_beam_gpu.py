"""Stepwise KV-cache decode and beam search on the GPU (ptk_gemma3_decode_prefill / _step, ptk_beam_candidates,
Gemma3CausalLM.beam_generate): Stage 2's validation generate (Stage2/trainer.py:596-626 -> GenerationMixin.
_beam_search with num_beams 3, do_sample, top_k 50, top_p 0.9) over a prompt of projected image tokens and a
left-padded question.

* decode steps against the oracle's cache-free recompute (oracle/beam_ref.py decode_logits, HF's position ids),
  with prompt masks, prompts repeated over beams and the cache rows re-ordered every step as beam search does;
* the candidate kernel against the oracle: greedy selection equal, sampled draws inside HF's processed support
  (temperature / top-k / top-p with min_tokens_to_keep), without replacement, distributed as softmax of the joint
  accumulated scores;
* beam_generate end to end: deterministic when greedy, HF's output crop and EOS handling, and Stage 2's
  evaluate writing the reference's example files.
The host bookkeeping itself is pinned against transformers' beam search in tests/test_beam_cpu.py."""
import numpy as np
import pytest
import torch

from tests.golden_util import bf16_round

pytestmark = pytest.mark.gpu


def _model(name, gpu, max_pos=128):
    from projectiontrainer_amd import weights as W
    from projectiontrainer_amd.config import PRESETS
    from projectiontrainer_amd.gemma3 import Gemma3CausalLM
    cfg = PRESETS[name].text
    lp = W.gemma3_params(cfg, seed=4)
    lm = Gemma3CausalLM(cfg, lp, gpu, max_pos=max_pos)
    return cfg, {k: torch.from_numpy(bf16_round(v)) for k, v in lp.items()}, lm


def _rel(a, b):
    a, b = a.double().ravel(), b.double().ravel()
    return float((a - b).norm() / b.norm().clamp(min=1e-30))


@pytest.mark.parametrize("name", ["tiny", "tiny_gqa"])
def test_decode_steps_with_masks_and_reorder_vs_oracle(gpu, name):
    """2 prompts x 2 rows each (P 20 > the sliding window 8; left-padded questions of 2 and 3 pads), 6 steps with
    random tokens and random beam re-orders inside each prompt's rows: every step's logits match the oracle's
    recompute of each row's own sequence (rel-L2 2e-2, cos 0.999 -- the Stage-1 parity bar)."""
    from oracle import beam_ref as BR
    from tests.test_stage1_gpu import record
    cfg, lpb, lm = _model(name, gpu)
    B, R, P, steps = 2, 2, 20, 6
    g = torch.Generator().manual_seed(1)
    x = torch.randn(B, P, cfg.hidden_size, generator=g)
    mask = torch.ones(B, P, dtype=torch.long)
    mask[0, 14:16] = 0
    mask[1, 13:16] = 0
    torch.set_num_threads(min(16, torch.get_num_threads()))
    rows = B * R
    prompt_of = torch.arange(rows) // R
    logits = lm.decode_begin(x.to(gpu), mask.to(gpu), repeat=R, max_new_tokens=steps + 1)
    seqs = [[] for _ in range(rows)]
    for t in range(steps + 1):
        ref = BR.decode_logits(lpb, cfg, x[prompt_of], mask[prompt_of],
                               torch.tensor(seqs) if t else None)
        got = logits.float().cpu()
        for r in range(rows):
            rl = _rel(got[r], ref[r])
            cos = float(torch.nn.functional.cosine_similarity(got[r].double(), ref[r].double(), dim=0))
            record(f"decode[{name}]", f"step{t}_row{r}", rel_l2=rl, cos=cos, tol_rel_l2=2e-2, tol_cos=0.999)
            assert rl <= 2e-2 and cos >= 0.999, (t, r, rl, cos)
        if t == steps:
            break
        ids = torch.randint(0, cfg.vocab_size, (rows,), generator=g)
        src = torch.stack([torch.randint(0, R, (1,), generator=g)[0] + R * (r // R) for r in range(rows)])
        seqs = [seqs[int(src[r])] + [int(ids[r])] for r in range(rows)]
        logits = lm.decode_next(t + 1, ids.to(gpu), src.to(torch.int32).to(gpu))


def test_decode_gemma3_1b_dims_stage2_prompt(gpu):
    """Gemma3-1B dims at 6 layers (one full-attention layer), the Stage-2 prompt shape: 575 image tokens + a
    16-token question left-padded by 3 and 5 (positions past the 512-key window), 2 prompts x 3 beams, 3 steps with
    beam re-orders: logits against the oracle's recompute (the Stage-1 parity bar)."""
    from oracle import beam_ref as BR
    from projectiontrainer_amd import weights as W
    from projectiontrainer_amd.config import PRESETS
    from projectiontrainer_amd.gemma3 import Gemma3CausalLM
    cfg = PRESETS["cfg2"].text
    cfg = cfg.__class__(**{**cfg.__dict__, "num_hidden_layers": 6})
    lp = W.gemma3_params(cfg, seed=4)
    lm = Gemma3CausalLM(cfg, lp, gpu, max_pos=704)
    lpb = {k: torch.from_numpy(bf16_round(v)) for k, v in lp.items()}
    B, R, P = 2, 3, 591
    g = torch.Generator().manual_seed(2)
    x = torch.randn(B, P, cfg.hidden_size, generator=g)
    mask = torch.ones(B, P, dtype=torch.long)
    mask[0, 575:578] = 0
    mask[1, 575:580] = 0
    torch.set_num_threads(min(16, torch.get_num_threads()))
    rows = B * R
    prompt_of = torch.arange(rows) // R
    logits = lm.decode_begin(x.to(gpu), mask.to(gpu), repeat=R, max_new_tokens=4)
    seqs = [[] for _ in range(rows)]
    for t in range(4):
        got = logits.float().cpu()
        if t == 0:   # the prefill gives every row of a prompt that prompt's logits
            assert all(torch.equal(got[r], got[R * (r // R)]) for r in range(rows))
        for r in range(rows):
            if r % R:      # the oracle recompute at 1B dims is slow: one row per prompt
                continue
            ref = BR.decode_logits(lpb, cfg, x[prompt_of[r:r + 1]], mask[prompt_of[r:r + 1]],
                                   torch.tensor([seqs[r]]) if t else None)[0]
            rl = _rel(got[r], ref)
            cos = float(torch.nn.functional.cosine_similarity(got[r].double(), ref.double(), dim=0))
            assert rl <= 2e-2 and cos >= 0.999, (t, r, rl, cos)
        if t == 3:
            break
        ids = torch.randint(0, cfg.vocab_size, (rows,), generator=g)
        src = torch.tensor([R * (r // R) + (r + t + 1) % R for r in range(rows)])
        seqs = [seqs[int(src[r])] + [int(ids[r])] for r in range(rows)]
        logits = lm.decode_next(t + 1, ids.to(gpu), src.to(torch.int32).to(gpu))


def _distinct_logits(rows, V, seed):
    """bf16 logits whose values in each row are all different (a permutation of V distinct bf16 values)."""
    g = torch.Generator().manual_seed(seed)
    vals = (torch.arange(V).float() / 16.0 - V / 32.0).to(torch.bfloat16)   # exact in bf16 for V <= 256
    return torch.stack([vals[torch.randperm(V, generator=g)] for _ in range(rows)])


@pytest.mark.parametrize("V", [256, 262144])
def test_beam_candidates_greedy_vs_oracle(gpu, V):
    """do_sample=False: the 2K best (beam, token) continuations over beams x vocab, by accumulated log prob
    (log_softmax + the running beam score), in descending order -- torch.topk on the oracle's scores."""
    from oracle import beam_ref as BR
    cfg, _, lm = _model("tiny", gpu)
    B, K = 5, 3
    lg = _distinct_logits(B * K, V, 3)
    if V > 256:   # distinct within the top region at least: bf16 ties elsewhere do not reach the top 6
        lg = (torch.randn(B * K, V, generator=torch.Generator().manual_seed(2)) * 2).to(torch.bfloat16)
    bs = torch.tensor([0.0, -0.7, -1.3] * B)
    tok, bi, sc = lm.beam_candidates(lg.to(gpu), bs, K, 2 * K, False, 0, 1.0, 1.0, 0, 0, 1)
    rt, rb, rs, _ = BR.beam_candidates(lg.float(), bs, K, 2 * K + 1)
    torch.testing.assert_close(sc.cpu(), rs[:, :-1], rtol=0, atol=2e-4)
    # a candidate's place is pinned where its score is apart from both neighbours' (bf16 logits tie often at
    # V = 262 144; torch.topk orders ties arbitrarily)
    apart = (rs[:, :-1] - rs[:, 1:]) > 1e-3
    pinned = apart[:, :] & torch.cat([torch.ones(rs.shape[0], 1, dtype=torch.bool), apart[:, :-1]], 1)
    same = (tok.cpu() == rt[:, :-1]) & (bi.cpu().long() == rb[:, :-1])
    assert bool(same[pinned].all()) and pinned.float().mean() > 0.5, (tok, rt, bi, rb)


def test_beam_candidates_sampling_law(gpu):
    """do_sample (T 0.8, top_k 50, top_p 0.9, min_tokens_to_keep 2, 2 beams, 4 draws): every candidate lies in
    HF's processed support, no (beam, token) repeats within an item, the first draw is distributed as
    softmax(accumulated) over the joint support (TV within 3x its expectation over 4096 items), the same seed
    repeats the draws and another changes them."""
    from oracle import beam_ref as BR
    cfg, _, lm = _model("tiny", gpu)
    K, V, N = 2, cfg.vocab_size, 4096
    g = torch.Generator().manual_seed(9)
    one = (torch.randn(K, V, generator=g) * 1.5).to(torch.bfloat16)
    lg = one.repeat(N, 1).to(gpu)
    bs = torch.tensor([0.0, -0.5]).repeat(N)
    kw = dict(do_sample=True, top_k=50, top_p=0.9, temperature=0.8, min_tokens_to_keep=2)
    tok, bi, sc = lm.beam_candidates(lg, bs, K, 4, kw["do_sample"], kw["top_k"], kw["top_p"], kw["temperature"],
                                     11, 0, kw["min_tokens_to_keep"])
    tok, bi = tok.cpu(), bi.cpu().long()
    _, _, _, acc = BR.beam_candidates(one.float(), bs[:K], K, 4, True, 50, 0.9, 0.8, 2)
    acc = acc[0]                                          # [K * V] joint accumulated scores
    flat = bi * V + tok
    assert (tok >= 0).all()
    assert torch.isfinite(acc[flat]).all(), "a draw outside the processed support"
    assert all(len(set(row.tolist())) == 4 for row in flat[:64]), "drawn twice"
    torch.testing.assert_close(sc.cpu(), acc[flat], rtol=0, atol=2e-4)
    p = torch.softmax(acc.double(), -1)
    emp = torch.bincount(flat[:, 0], minlength=K * V).double() / N
    tv = 0.5 * float((emp - p).abs().sum())
    bar = 3.0 * 0.5 * float((2.0 * p * (1 - p) / (np.pi * N)).sqrt().sum())
    assert tv < bar, (tv, bar)
    again = lm.beam_candidates(lg, bs, K, 4, True, 50, 0.9, 0.8, 11, 0, 2)[0].cpu()
    other = lm.beam_candidates(lg, bs, K, 4, True, 50, 0.9, 0.8, 12, 0, 2)[0].cpu()
    assert torch.equal(again, tok) and not torch.equal(other, tok)


def test_beam_generate_end_to_end(gpu):
    """Greedy beam search twice: identical; the output is the best finished hypothesis per prompt, cropped to the
    longest (HF), with the EOS run: a sequence that holds eos_token_id ends there (the rest is the fill value);
    beam sampling runs to a result of the same shape rules and depends on the seed."""
    cfg, lpb, lm = _model("tiny", gpu)
    g = torch.Generator().manual_seed(5)
    x = torch.randn(3, 20, cfg.hidden_size, generator=g).to(gpu)
    mask = torch.ones(3, 20, dtype=torch.long)
    mask[1, 16:18] = 0
    a = lm.beam_generate(x, mask.to(gpu), num_beams=3, max_new_tokens=10, do_sample=False)
    b = lm.beam_generate(x, mask.to(gpu), num_beams=3, max_new_tokens=10, do_sample=False)
    assert torch.equal(a, b) and a.shape == (3, 10)
    eos = int(a[0, 2])
    c = lm.beam_generate(x, mask.to(gpu), num_beams=3, max_new_tokens=10, do_sample=False, eos_token_id=eos,
                         pad_token_id=0).cpu()
    assert c.shape[0] == 3 and c.shape[1] <= 10
    for row in c:
        hit = (row == eos).nonzero()
        if hit.numel():
            assert (row[int(hit[0]) + 1:] == eos).all()   # fill = pad or eos, pad 0 -> eos (HF's quirk)
    s1 = lm.beam_generate(x, mask.to(gpu), num_beams=3, max_new_tokens=8, do_sample=True, top_k=50, top_p=0.9,
                          seed=1)
    s2 = lm.beam_generate(x, mask.to(gpu), num_beams=3, max_new_tokens=8, do_sample=True, top_k=50, top_p=0.9,
                          seed=2)
    assert s1.shape == (3, 8) and not torch.equal(s1, s2)


def test_stage2_evaluate_writes_generated_examples(gpu, tmp_path):
    """VQATrainerStage2.evaluate with a decoding tokenizer: val/loss and the reference's example files
    (validation_examples/epoch_1_examples.txt, all_validation_examples.txt; Stage2/trainer.py:672-700) with one
    example per validation sample, the predictions from beam_generate on [projected image | question]."""
    from projectiontrainer_amd import dist as D
    from projectiontrainer_amd import weights as W
    from projectiontrainer_amd.config import PRESETS
    from projectiontrainer_amd.gemma3 import Gemma3CausalLM
    from projectiontrainer_amd.projectors import MLPProjector
    from projectiontrainer_amd.siglip import SiglipVisionTower
    from projectiontrainer_amd.vqa_trainer import VQATrainerStage2
    cfg = PRESETS["tiny"]
    vp, lp = W.siglip_vision_params(cfg.vision), W.gemma3_params(cfg.text)
    proj = MLPProjector(cfg.vision.hidden_size, cfg.text.hidden_size)
    proj.load_state_dict({k: torch.from_numpy(v)
                          for k, v in W.projector_params(cfg.vision.hidden_size, cfg.text.hidden_size).items()})
    data = W.synthetic_vqa_items(cfg, 3, seed=21)

    class Tok:
        pad_token_id, eos_token_id, padding_side = 0, 1, "left"

        def batch_decode(self, seqs, skip_special_tokens=True):
            return [" ".join(f"w{int(t)}" for t in s if not (skip_special_tokens and int(t) in (0, 1)))
                    for s in np.asarray(seqs)]

    logs = []
    tr = VQATrainerStage2(D.DistState(1), SiglipVisionTower(cfg.vision, vp, gpu),
                          Gemma3CausalLM(cfg.text, lp, gpu, max_pos=1024), proj, Tok(), data, data, str(tmp_path), 2,
                          1e-3, 0.01, 1, 1, 0.0, freeze_vision_encoder=True, freeze_projection_layer=True,
                          freeze_llm=False, enable_qlora=False, train_ve_first_epoch=False, wandb_project="x",
                          log_fn=lambda d, s: logs.append(d), generate_max_new_tokens=6)
    v = tr.evaluate(0, 0)
    torch.cuda.synchronize()
    assert 0.0 < v < 20.0 and any("val/loss" in d for d in logs)
    text = (tmp_path / "validation_examples" / "epoch_1_examples.txt").read_text()
    assert text.startswith("Validation Examples for Epoch 1")
    assert text.count("Prediction: ") == len(data) and text.count("Question: ") == len(data)
    assert (tmp_path / "validation_examples" / "all_validation_examples.txt").exists()
