"""CPU restatement of the reference Stage-2 VQA training step (pure torch, fp32).

TEST INFRASTRUCTURE ONLY.  Imported by `tests/` as the checker; the product
path (`projectiontrainer_amd`) never imports it.

Pinned against `tests/golden/s2_tiny.npz`, produced by running the reference's
`Stage2/trainer.py:VQATrainerStage2.train()` (tests/golden/make_golden_stage2.py).
Restates, with the BASELINE cfg4 flags (LLM unfrozen, projector and vision
encoder frozen, no QLoRA):
  * `vqa_collate_fn` (Stage2/trainer.py:18-61): per-batch padding of question
    and answer ids to the longest in the batch, on the tokenizer's padding side;
  * the step body (:299-444): frozen SigLIP (no grad), frozen projector, Gemma3
    input = [projected ‖ E[q]·scale ‖ E[a]·scale] (:345-370), attention mask
    1 ‖ q≠pad ‖ a≠pad (:379-385), labels -100 ‖ -100 ‖ a with pad -> -100
    (:390-396), logits in fp32, shifted mean CrossEntropyLoss (:407-418);
  * `accelerator.accumulate`: loss / gas twice (:422 and Accelerator.backward),
    gradients summed over micro-batches, an optimizer step when (micro+1) % gas
    == 0 or at the end of the loader; clip_grad_norm_(llm, 1.0), AdamW over the
    LLM parameters, the cosine-with-warmup schedule stepped num_processes times
    per optimizer step (:426-444).
"""
from __future__ import annotations

import math

import torch

from oracle import stage1_ref as R

IGNORE = -100


def collate(items, pad_id: int, padding_side: str):
    """vqa_collate_fn (Stage2/trainer.py:18-61)."""
    def pad(seqs):
        n = max(len(s) for s in seqs)
        out = []
        for s in seqs:
            p = torch.full((n - len(s),), pad_id, dtype=torch.long)
            out.append(torch.cat([p, s]) if padding_side == "left" else torch.cat([s, p]))
        return torch.stack(out)
    return {"pixel_values": torch.stack([it["pixel_values"] for it in items]),
            "question_input_ids": pad([it["question_input_ids"] for it in items]),
            "answer_input_ids": pad([it["answer_input_ids"] for it in items])}


def stage2_inputs(proj, E, q_ids, a_ids, pad_id, embed_scale):
    """inputs_embeds, attention mask and labels of one VQA batch (Stage2/trainer.py:339-396)."""
    x = torch.cat([proj, E[q_ids] * embed_scale, E[a_ids] * embed_scale], dim=1)
    B, Nv = proj.shape[:2]
    mask = torch.cat([torch.ones(B, Nv, dtype=torch.long), (q_ids != pad_id).long(), (a_ids != pad_id).long()], 1)
    alab = a_ids.clone()
    alab[alab == pad_id] = IGNORE
    labels = torch.cat([torch.full((B, Nv + q_ids.shape[1]), IGNORE, dtype=torch.long), alab], 1)
    return x, mask, labels


def stage2_loss(vp, vcfg, llm_params, lcfg, pp, pixel_values, q_ids, a_ids, pad_id):
    """Mean shifted CE over the answer tokens; llm_params may require grad (unfrozen LLM)."""
    with torch.no_grad():
        patch = R.siglip_vision_forward(vp, vcfg, pixel_values)[:, 1:, :]
        proj = R.projector_forward(pp, patch.float())
    E = llm_params["model.embed_tokens.weight"]
    x, mask, labels = stage2_inputs(proj, E, q_ids, a_ids, pad_id, math.sqrt(lcfg.hidden_size))
    hidden = R.gemma3_forward(llm_params, lcfg, x, mask)
    return R.causal_lm_loss(hidden, E, labels)


class Stage2State:
    """fp32 LLM parameters + AdamW moments, optimizer / scheduler counters."""
    def __init__(self, llm_params):
        self.params = {k: torch.as_tensor(v).float().clone().requires_grad_(True) for k, v in llm_params.items()}
        self.exp_avg = {k: torch.zeros_like(v) for k, v in self.params.items()}
        self.exp_avg_sq = {k: torch.zeros_like(v) for k, v in self.params.items()}
        self.step = 0
        self.sched_step = 0


def optimizer_step(st: Stage2State, lr0, warmup, total, weight_decay=0.01, max_norm=1.0, num_processes=1):
    """clip_grad_norm_(llm.parameters(), 1.0) + AdamW + scheduler (Stage2/trainer.py:426-444)."""
    grads = {k: p.grad.detach().clone() for k, p in st.params.items()}
    raw = {k: g.clone() for k, g in grads.items()}
    norm = R.clip_grad_norm_(list(grads.values()), max_norm)
    lr = lr0 * R.cosine_lambda(st.sched_step, warmup, total)
    ts = R.TrainState({k: p.detach() for k, p in st.params.items()}, st.exp_avg, st.exp_avg_sq, st.step)
    with torch.no_grad():
        R.adamw_step(ts, grads, lr, weight_decay=weight_decay)
    st.step = ts.step
    st.sched_step += num_processes
    for p in st.params.values():
        p.grad = None
    return {"lr": lr, "grad_norm": float(norm), "grads": raw}


def train(vp, vcfg, lp, lcfg, pp, batches, *, gas, lr0, warmup, total, pad_id, weight_decay=0.01, max_norm=1.0,
          epoch_lengths=None):
    """Replays collated micro-batches (a list per epoch) through the accumulate loop.  Returns the
    per-micro-batch losses, the per-step records and the final state."""
    st = Stage2State(lp)
    losses, steps = [], []
    for epoch_batches in batches:
        for i, b in enumerate(epoch_batches):
            loss = stage2_loss(vp, vcfg, st.params, lcfg, pp, b["pixel_values"], b["question_input_ids"],
                               b["answer_input_ids"], pad_id)
            ((loss / gas) / gas).backward()
            losses.append(float(loss.detach()))
            sync = (i + 1) % gas == 0 or i + 1 == len(epoch_batches)
            if sync:
                rec = optimizer_step(st, lr0, warmup, total, weight_decay, max_norm)
                rec["params"] = {k: p.detach().clone() for k, p in st.params.items()}
                steps.append(rec)
    return losses, steps, st
