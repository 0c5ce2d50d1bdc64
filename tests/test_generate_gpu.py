"""KV-cache decode (`Gemma3CausalLM.generate`, `ptk_gemma3_generate`): the validation `generate` of the reference's
trainer (Stage1/projector_trainer.py:386-393 -> GenerationMixin._sample over Gemma3ForCausalLM with a cache).

Against the oracle's cache-free greedy decode (oracle/stage1_ref.py greedy_generate: the whole sequence recomputed
at every step), teacher-forced so both see the same tokens: every step's logits within the bf16-vs-fp32 bar of the
Stage-1 parity tests, and the argmax equal wherever the oracle's top-two margin is not a near-tie.  The configs put
decode positions past the sliding window (tiny: window 8, prompt 20; Gemma3-1B dims: window 512, prompt 575), so the
cache window start is exercised.  Sampling: HF's processors for do_sample (temperature, then top-k with ties kept)
and a softmax draw, checked as a distribution over many rows."""
import numpy as np
import pytest
import torch

from tests.golden_util import bf16_round

pytestmark = pytest.mark.gpu


def _model(name, gpu, max_pos=128, layers=None):
    from projectiontrainer_amd import weights as W
    from projectiontrainer_amd.config import PRESETS
    from projectiontrainer_amd.gemma3 import Gemma3CausalLM
    cfg = PRESETS[name].text
    if layers is not None:
        cfg = cfg.__class__(**{**cfg.__dict__, "num_hidden_layers": layers})
    lp = W.gemma3_params(cfg, seed=4)
    lm = Gemma3CausalLM(cfg, lp, gpu, max_pos=max_pos)
    return cfg, {k: bf16_round(v) for k, v in lp.items()}, lm   # the oracle on the bf16 weights the device holds


def _rel(a, b):
    a, b = a.double().ravel(), b.double().ravel()
    return float((a - b).norm() / b.norm().clamp(min=1e-30))


def _teacher_forced(cfg, lpb, lm, gpu, B, P, steps, seed=0, scale=1.0):
    from oracle import stage1_ref as R
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(B, P, cfg.hidden_size, generator=g) * scale
    torch.set_num_threads(min(16, torch.get_num_threads()))
    tok_o, log_o = R.greedy_generate({k: torch.from_numpy(v) for k, v in lpb.items()}, cfg, x, steps)
    ids, log_h = lm.generate(x.to(gpu).contiguous(), max_new_tokens=steps, do_sample=False, force_ids=tok_o,
                             return_logits=True)
    torch.cuda.synchronize()
    return tok_o, log_o, ids.cpu(), log_h.float().cpu()


def _check(tok_o, log_o, ids, log_h, rel_bar=2e-2, test="", margin=0.02):
    from tests.test_stage1_gpu import record
    steps = tok_o.shape[1]
    for t in range(steps):
        r = _rel(log_h[t], log_o[t])
        cos = torch.nn.functional.cosine_similarity(log_h[t].double().ravel(), log_o[t].double().ravel(), dim=0)
        record(test, f"step{t}_logits", rel_l2=r, cos=float(cos), tol_rel_l2=rel_bar, tol_cos=0.999)
        assert r <= rel_bar, (t, r)
        assert cos >= 0.999, (t, float(cos))
    # greedy tokens: the argmax of the HIP logits of each (teacher-forced) step; equal to the oracle's wherever the
    # oracle's best two logits are more than 2 % of their spread apart
    top2 = log_o.topk(2, dim=-1).values                              # [steps, B, 2]
    clear = (top2[..., 0] - top2[..., 1]) > margin * log_o.std(-1)
    agree = ids.t() == tok_o.t()
    record(test, "greedy_agreement", frac=float(agree.float().mean()), clear_frac=float(clear.float().mean()))
    assert bool(agree[clear].all()), (agree, clear)
    assert float(agree.float().mean()) >= 0.8, agree


@pytest.mark.parametrize("name", ["tiny", "tiny_gqa"])
def test_generate_teacher_forced_vs_oracle(gpu, name):
    """tiny: 3 layers (2 sliding with window 8, 1 full), prompt 20 > window, 10 new tokens; tiny_gqa: 4 q / 2 kv heads,
    linear RoPE x8 on the full layer."""
    cfg, lpb, lm = _model(name, gpu)
    tok_o, log_o, ids, log_h = _teacher_forced(cfg, lpb, lm, gpu, B=3, P=20, steps=10)
    _check(tok_o, log_o, ids, log_h, test=f"generate[{name}]")


def test_generate_teacher_forced_many_rows(gpu):
    """80 decode rows: past the skinny decode GEMM's 64, so every decode projection and the lm_head run as a 64-row
    and a 16-row chunk; teacher-forced logits against the oracle as above.  With 320 greedy picks a top-two gap of
    2 % of the logit spread still admitted a bf16 flip, so the argmax check uses 5 % here (measured: 98.75 % of
    all picks equal, every pick with a gap above 5 % equal; 90 % of the picks have one)."""
    cfg, lpb, lm = _model("tiny", gpu)
    tok_o, log_o, ids, log_h = _teacher_forced(cfg, lpb, lm, gpu, B=80, P=20, steps=4, seed=2)
    _check(tok_o, log_o, ids, log_h, test="generate[tiny-80rows]", margin=0.05)


@pytest.mark.slow
def test_generate_teacher_forced_gemma3_1b_dims(gpu):
    """Gemma3-1B dims (hidden 1152, GQA 4:1, head_dim 256, vocab 262 144, window 512) at 6 layers (one full): the
    reference's prompt of 575 projected patch embeddings, so decode positions 575.. sit past the 512-key window;
    4 new tokens, batch 2."""
    cfg, lpb, lm = _model("cfg2", gpu, max_pos=704, layers=6)
    tok_o, log_o, ids, log_h = _teacher_forced(cfg, lpb, lm, gpu, B=2, P=575, steps=4, seed=3)
    _check(tok_o, log_o, ids, log_h, test="generate[gemma3-1b-L6-P575]")


def test_generate_eos_and_stop(gpu):
    """A row that produced eos_token_id emits pad_token_id afterwards, and the returned length is the step at which
    every row had produced it (GenerationMixin._sample's unfinished_sequences / stopping rule); greedy decode is
    deterministic."""
    cfg, lpb, lm = _model("tiny", gpu)
    g = torch.Generator().manual_seed(5)
    x = torch.randn(4, 20, cfg.hidden_size, generator=g).to(gpu)
    free = lm.generate(x, max_new_tokens=12, do_sample=False)
    again = lm.generate(x, max_new_tokens=12, do_sample=False)
    assert torch.equal(free, again) and free.shape == (4, 12)
    eos, pad = int(free[0, 2]), 511
    out = lm.generate(x, max_new_tokens=12, do_sample=False, eos_token_id=eos, pad_token_id=pad).cpu()
    ref = free.cpu()
    hit = [(ref[b] == eos).nonzero() for b in range(4)]
    first = [int(h[0]) if h.numel() else None for h in hit]
    n = 12 if any(f is None for f in first) else max(first) + 1
    assert out.shape == (4, n), (out.shape, first)
    for b in range(4):
        f = first[b]
        if f is None:
            assert torch.equal(out[b], ref[b, :n])
        else:
            assert torch.equal(out[b, :f + 1], ref[b, :f + 1])
            assert (out[b, f + 1:] == pad).all()


def test_generate_sampling_distribution(gpu):
    """do_sample: 4096 rows with the same prompt draw the first token from the same logits; the draws stay inside
    the top-k set (logits >= the k-th largest, TopKLogitsWarper) and their histogram matches
    softmax(logits / temperature) over that set (total variation within 3x its expectation); without top-k the draws
    reach past it; the same seed repeats the draws, another seed changes them."""
    cfg, lpb, lm = _model("tiny", gpu)
    g = torch.Generator().manual_seed(7)
    x = (torch.randn(1, 20, cfg.hidden_size, generator=g)).expand(4096, 20, cfg.hidden_size).contiguous().to(gpu)
    T, k = 0.7, 50
    ids, logits = lm.generate(x, max_new_tokens=1, do_sample=True, top_k=k, temperature=T, seed=11,
                              return_logits=True)
    ids = ids[:, 0].cpu()
    lg = logits[0, 0].float().cpu()
    thr = lg.topk(k).values[-1]
    keep = lg >= thr
    assert keep[ids].all()
    p = torch.softmax(torch.where(keep, lg / T, torch.tensor(-float("inf"))), -1)
    emp = torch.bincount(ids, minlength=lg.numel()).float() / ids.numel()
    tv = 0.5 * float((emp - p).abs().sum())
    # three times the expected total variation of N multinomial draws, 0.5 sum sqrt(2 p (1 - p) / (pi N))
    bar = 3.0 * 0.5 * float((2.0 * p * (1 - p) / (np.pi * ids.numel())).sqrt().sum())
    assert tv < bar, (tv, bar)
    same = lm.generate(x, max_new_tokens=1, do_sample=True, top_k=k, temperature=T, seed=11)[:, 0].cpu()
    other = lm.generate(x, max_new_tokens=1, do_sample=True, top_k=k, temperature=T, seed=12)[:, 0].cpu()
    assert torch.equal(same, ids) and not torch.equal(other, ids)
    wide = lm.generate(x, max_new_tokens=1, do_sample=True, top_k=0, temperature=3.0, seed=13)[:, 0].cpu()
    assert (~keep[wide]).any()


def test_generate_sampling_top_p(gpu):
    """do_sample with top_k 64 and top_p 0.95 (the public gemma-3-1b-it generation config) and T 0.8: the draws stay
    inside HF's processed support (TopKLogitsWarper then TopPLogitsWarper, min_tokens_to_keep 1) and their
    histogram matches softmax over it (TV within 3x its expectation, 4096 rows)."""
    from oracle import beam_ref as BR
    cfg, lpb, lm = _model("tiny", gpu)
    g = torch.Generator().manual_seed(8)
    x = (torch.randn(1, 20, cfg.hidden_size, generator=g)).expand(4096, 20, cfg.hidden_size).contiguous().to(gpu)
    ids, logits = lm.generate(x, max_new_tokens=1, do_sample=True, top_k=64, top_p=0.95, temperature=0.8, seed=5,
                              return_logits=True)
    ids = ids[:, 0].cpu()
    lp = BR.processed_log_probs(logits[0, 0:1].float().cpu(), True, 64, 0.95, 0.8, 1)[0]
    assert torch.isfinite(lp[ids]).all()
    p = torch.softmax(lp.double(), -1)
    emp = torch.bincount(ids, minlength=lp.numel()).double() / ids.numel()
    tv = 0.5 * float((emp - p).abs().sum())
    bar = 3.0 * 0.5 * float((2.0 * p * (1 - p) / (np.pi * ids.numel())).sqrt().sum())
    assert tv < bar, (tv, bar)
    assert int(torch.isfinite(lp).sum()) < 64     # top-p removed part of the top-k set


def test_trainer_validation_generate(gpu, tmp_path):
    """ProjectionTrainerStage1 with a validation set and a tokenizer that decodes: the reference's validation logs
    (projector_trainer.py:423-431) -- validation/loss and validation/last_word_accuracy -- from generate on the
    projected embeddings; a tokenizer without batch_decode gives the loss only."""
    import types
    from projectiontrainer_amd import weights as W
    from projectiontrainer_amd.config import PRESETS
    from projectiontrainer_amd.gemma3 import Gemma3CausalLM
    from projectiontrainer_amd.projector_trainer import ProjectionTrainerStage1
    from projectiontrainer_amd.projectors import MLPProjector
    from projectiontrainer_amd.siglip import SiglipVisionTower
    cfg = PRESETS["tiny"].replace(batch_size=4)
    vp, lp = W.siglip_vision_params(cfg.vision), W.gemma3_params(cfg.text)
    pp = W.projector_params(cfg.vision.hidden_size, cfg.text.hidden_size)
    px, ids, labels = W.synthetic_batch(cfg, seed=41)
    data = [{"pixel_values": torch.from_numpy(px[i]), "token_ids": torch.from_numpy(ids[i]),
             "labels": torch.from_numpy(labels[i])} for i in range(4)]

    class Tok:
        pad_token_id, eos_token_id = 0, 1

        def batch_decode(self, seqs, skip_special_tokens=True):
            out = []
            for s in np.asarray(seqs):
                out.append(" ".join(f"w{int(t) % 3}" for t in s if not (skip_special_tokens and int(t) in (0, 1, 2))))
            return out

    for tok, want_acc in ((Tok(), True), (types.SimpleNamespace(pad_token_id=0, eos_token_id=1), False)):
        proj = MLPProjector(cfg.vision.hidden_size, cfg.text.hidden_size)
        proj.load_state_dict({k: torch.from_numpy(v) for k, v in pp.items()})
        logs = []
        tr = ProjectionTrainerStage1(None, SiglipVisionTower(cfg.vision, vp, gpu),
                                     Gemma3CausalLM(cfg.text, lp, gpu, max_pos=cfg.seq_len + 64 + 64), proj, None, tok,
                                     data, data, output_dir=str(tmp_path), batch_size=2, num_epochs=1,
                                     log_fn=lambda d, s: logs.append(d), generate_max_new_tokens=8)
        tr.train()
        torch.cuda.synchronize()
        val = [d for d in logs if "validation/loss" in d]
        assert len(val) == 1 and 0.0 < val[0]["validation/loss"] < 20.0
        if want_acc:
            a = val[0]["validation/last_word_accuracy"]
            assert 0.0 <= a <= 100.0
        else:
            assert "validation/last_word_accuracy" not in val[0]


def test_generate_defaults_from_hf_generation_config(gpu):
    """Gemma3CausalLM.from_hf keeps the checkpoint's generation_config (top_k, top_p, temperature) as generate()'s
    defaults, as HF's generate does when the reference calls it with do_sample=True and no sampling arguments
    (Stage1/projector_trainer.py:386-393): with top_k 5 / top_p 0.6 set there, every draw lies in that processed
    support; an explicit argument still wins."""
    from transformers import Gemma3ForCausalLM, Gemma3TextConfig
    from oracle import beam_ref as BR
    from projectiontrainer_amd import weights as W
    from projectiontrainer_amd.config import PRESETS, to_hf_dicts
    from projectiontrainer_amd.gemma3 import Gemma3CausalLM
    cfg = PRESETS["tiny"]
    _, txt = to_hf_dicts(cfg)
    hf = Gemma3ForCausalLM(Gemma3TextConfig(**txt))
    hf.load_state_dict({k: torch.from_numpy(v) for k, v in W.gemma3_params(cfg.text).items()}, strict=False)
    hf.generation_config.top_k, hf.generation_config.top_p, hf.generation_config.temperature = 5, 0.6, 1.0
    lm = Gemma3CausalLM.from_hf(hf, gpu, max_pos=128)
    assert lm.generation_defaults == {"top_k": 5, "top_p": 0.6, "temperature": 1.0}
    g = torch.Generator().manual_seed(4)
    x = torch.randn(1, 20, cfg.text.hidden_size, generator=g).expand(512, 20, cfg.text.hidden_size).contiguous().to(gpu)
    ids, logits = lm.generate(x, max_new_tokens=1, do_sample=True, seed=3, return_logits=True)
    lp = BR.processed_log_probs(logits[0, 0:1].float().cpu(), True, 5, 0.6, 1.0, 1)[0]
    assert torch.isfinite(lp[ids[:, 0].cpu()]).all() and int(torch.isfinite(lp).sum()) <= 5
    wide = lm.generate(x, max_new_tokens=1, do_sample=True, seed=3, top_k=0, top_p=1.0, temperature=3.0)
    assert (~torch.isfinite(lp[wide[:, 0].cpu()])).any()
