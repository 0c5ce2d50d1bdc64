"""Pin the Stage-2 CPU oracle (oracle/stage2_ref.py) to the reference's own VQA trainer.

`tests/golden/s2_tiny.npz` comes from running Stage2/trainer.py:VQATrainerStage2.train() on CPU in fp32
with the LLM unfrozen (tests/golden/make_golden_stage2.py): 6 samples, bs 2, gradient_accumulation_steps
2, 2 epochs -> 6 micro-batches, 4 optimizer steps (the first under warmup, the second and fourth at the
end of an epoch).  fp32 restatement vs fp32 reference: losses rtol 1e-4; accumulated grads rtol 1e-3 with
an absolute floor of 2e-4 x the tensor's rms; LR exact; params after AdamW within 0.05 lr."""
import ast
import math

import numpy as np
import pytest
import torch

from oracle import stage2_ref as S
from projectiontrainer_amd import weights as W
from projectiontrainer_amd.config import PRESETS
from tests import golden_util as G


def load(name):
    d = np.load(f"{G.GOLDEN}/{name}.npz", allow_pickle=False)
    return d, ast.literal_eval(str(d["meta"]))


def fixture_batches(d, meta):
    """The collated micro-batches the reference's prepared loader yielded, grouped per epoch."""
    cfg = PRESETS["tiny"]
    items = W.synthetic_vqa_items(cfg, meta["n_items"], meta["seed"])
    px = torch.stack([it["pixel_values"] for it in items])
    per_epoch = math.ceil(meta["n_items"] / meta["batch_size"])
    out = []
    for m in range(meta["micro_batches"]):
        b = {"pixel_values": px[d[f"m{m}_order"]], "question_input_ids": torch.from_numpy(d[f"m{m}_question_input_ids"]),
             "answer_input_ids": torch.from_numpy(d[f"m{m}_answer_input_ids"])}
        if m % per_epoch == 0:
            out.append([])
        out[-1].append(b)
    return out


def rms(t):
    return float(t.double().pow(2).mean().sqrt())


@pytest.mark.parametrize("name", ["s2_tiny", "s2_tiny_bf16"])
def test_stage2_fixture_contract(name):
    """Weights regenerate bit-identically; each recorded batch is vqa_collate_fn of the samples in the
    recorded order (per-batch padding on the tokenizer's side)."""
    d, meta = load(name)
    cfg = PRESETS["tiny"]
    vp, lp = W.siglip_vision_params(cfg.vision), W.gemma3_params(cfg.text)
    pp = W.projector_params(cfg.vision.hidden_size, cfg.text.hidden_size, cfg.expansion_factor)
    np.testing.assert_array_equal(G.fingerprint(vp, lp, pp), d["weight_fingerprint"])
    items = W.synthetic_vqa_items(cfg, meta["n_items"], meta["seed"])
    for m in range(meta["micro_batches"]):
        b = S.collate([items[i] for i in d[f"m{m}_order"]], cfg.text.pad_token_id, meta["padding_side"])
        np.testing.assert_array_equal(b["question_input_ids"].numpy(), d[f"m{m}_question_input_ids"])
        np.testing.assert_array_equal(b["answer_input_ids"].numpy(), d[f"m{m}_answer_input_ids"])


def test_stage2_oracle_matches_reference():
    torch.set_num_threads(8)
    d, meta = load("s2_tiny")
    cfg = PRESETS["tiny"]
    vp, lp = W.siglip_vision_params(cfg.vision), W.gemma3_params(cfg.text)
    pp = {k: torch.from_numpy(v) for k, v in W.projector_params(cfg.vision.hidden_size, cfg.text.hidden_size).items()}
    total = meta["max_train_steps"]
    warmup = math.ceil(meta["warmup_ratio"] * total)
    losses, steps, st = S.train({k: torch.from_numpy(v) for k, v in vp.items()}, cfg.vision, lp, cfg.text, pp,
                                fixture_batches(d, meta), gas=meta["gas"], lr0=meta["lr"], warmup=warmup,
                                total=total, pad_id=cfg.text.pad_token_id)
    assert len(losses) == meta["micro_batches"] and len(steps) == meta["opt_steps"]
    for m, l in enumerate(losses):
        np.testing.assert_allclose(l, float(d[f"m{m}_loss"]), rtol=1e-4)
    for o, rec in enumerate(steps):
        np.testing.assert_allclose(rec["lr"], float(d[f"o{o}_lr"]), rtol=1e-12)
        np.testing.assert_allclose(rec["grad_norm"], float(d[f"o{o}_grad_norm"]), rtol=1e-4)
        for n in meta["param_names"]:
            g = rec["grads"][n]
            G.check_tensor(d, f"o{o}_grad.{n}", g, 1e-3, max(1e-8, 2e-4 * rms(g)))
            G.check_tensor(d, f"o{o}_param.{n}", rec["params"][n], 1e-5, 0.05 * meta["lr"])
