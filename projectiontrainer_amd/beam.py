"""Beam-search bookkeeping of the stepwise decode (Stage 2's validation generate).

The reference's `VQATrainerStage2.evaluate` (Stage2/trainer.py:596-626) calls
`generate(inputs_embeds=, attention_mask=, max_new_tokens=512, do_sample=True, num_beams=3, top_p=0.9, top_k=50,
eos_token_id=, pad_token_id=)`, i.e. transformers' `GenerationMixin._beam_search` (beam sampling).  Per step that
loop (a) scores every (beam, token) continuation, (b) keeps 2 x num_beams candidates per item (sampled without
replacement, or the best), (c) continues the best num_beams that did not just stop, (d) offers the stopped ones
among the first num_beams candidates to the item's finished hypotheses (score / length ** length_penalty), and (e)
stops when no running beam can beat the worst finished one (early_stopping False: judged at the current length),
or when every candidate has stopped.

(a) and (b) run on the GPU (`ptk_beam_candidates`: log_softmax, the warpers, the joint draw); this module is the
small per-item state of (c)-(e), on the host: a few [batch, 2 x beams] tensors per step, against the
[rows, vocab] logits that stay on the device.  `BeamSearch.step` takes the candidates of one step and returns the
tokens and source rows of the next; `result` the best finished hypothesis per item, cropped like HF's output.
"""
from __future__ import annotations

import torch

NEG = -1.0e9   # HF's "never" score (running beams 1.. at the start, masked candidates)


class BeamSearch:
    """State of one beam search over `batch` items x `beams` rows (row b * beams + k), `max_len` new tokens."""

    def __init__(self, batch: int, beams: int, max_len: int, eos_token_id: int | None, pad_token_id: int | None,
                 length_penalty: float = 1.0, early_stopping: bool | str = False):
        self.B, self.K, self.T = batch, beams, max_len
        self.eos = eos_token_id
        self.lp = float(length_penalty)
        self.early = early_stopping
        # HF fills unused positions with `pad_token_id or eos_token_id` (a pad id of 0 falls through to eos)
        fill = pad_token_id if pad_token_id else (eos_token_id if eos_token_id is not None else -1)
        self.fill = int(fill) if fill is not None else -1
        self.run_seq = torch.full((batch, beams, max_len), self.fill, dtype=torch.int64)
        self.run_score = torch.zeros(batch, beams)
        self.run_score[:, 1:] = NEG
        self.fin_seq = self.run_seq.clone()
        self.fin_score = torch.full((batch, beams), NEG)
        self.fin_len = torch.zeros(batch, beams, dtype=torch.int64)
        self.fin_done = torch.zeros(batch, beams, dtype=torch.bool)
        self.unsat = torch.ones(batch, dtype=torch.bool)   # an open beam may still beat the worst finished one
        self.cur = 0
        self.finished = False

    def step(self, tok: torch.Tensor, beam: torch.Tensor, acc: torch.Tensor):
        """One step's candidates ([B, 2K] token, source beam, accumulated log prob; the first K in draw / score
        order): returns (next tokens [B*K], source rows [B*K]) for the next decode step."""
        B, K, T, t = self.B, self.K, self.T, self.cur
        tok, beam, acc = tok.cpu().long(), beam.cpu().long(), acc.cpu().float()
        invalid = tok < 0                        # fewer candidates than 2K with a finite score
        tok = tok.clamp(min=0)
        beam = beam.clamp(min=0)
        acc = torch.where(invalid, torch.full_like(acc, float("-inf")), acc)
        cand_seq = torch.gather(self.run_seq, 1, beam[:, :, None].expand(-1, -1, T)).clone()
        cand_seq[:, :, t] = tok
        hits = invalid | (t + 1 >= T)
        if self.eos is not None:
            hits = hits | (tok == self.eos)
        # (c) the best K candidates that did not stop continue
        masked = acc + hits.float() * NEG
        keep = torch.topk(masked, K, dim=1).indices
        self.run_seq = torch.gather(cand_seq, 1, keep[:, :, None].expand(-1, -1, T))
        self.run_score = torch.gather(masked, 1, keep)
        src_beam = torch.gather(beam, 1, keep)
        # (d) stopped candidates among the first K offered to the finished hypotheses
        first_k = torch.zeros_like(hits)
        first_k[:, :K] = True
        just = hits & first_k
        score = acc / float(t + 1) ** self.lp
        if self.early is True:
            score = score + (self.fin_done.all(1, keepdim=True)).float() * NEG
        score = score + (~self.unsat)[:, None].float() * NEG
        score = score + (~just).float() * NEG
        m_seq = torch.cat([self.fin_seq, cand_seq], 1)
        m_score = torch.cat([self.fin_score, score], 1)
        m_len = torch.cat([self.fin_len, torch.full_like(tok, t + 1)], 1)
        m_done = torch.cat([self.fin_done, just], 1)
        top = torch.topk(m_score, K, dim=1).indices
        self.fin_seq = torch.gather(m_seq, 1, top[:, :, None].expand(-1, -1, T))
        self.fin_score = torch.gather(m_score, 1, top)
        self.fin_len = torch.gather(m_len, 1, top)
        self.fin_done = torch.gather(m_done, 1, top)
        # (e) stopping
        self.cur = t + 1
        if self.early == "never" and self.lp > 0.0:
            best_len = T
        else:
            best_len = self.cur
        best_running = self.run_score[:, 0] / float(best_len) ** self.lp
        worst = torch.where(self.fin_done, self.fin_score.min(1, keepdim=True).values, torch.full_like(self.fin_score, NEG))
        self.unsat = self.unsat & (best_running[:, None] > worst).any(1)
        open_beam = not (bool(self.fin_done.all()) and self.early is True)
        self.finished = not (bool(self.unsat.any()) and open_beam and not bool(hits.all()))
        rows = (torch.arange(B)[:, None] * K + src_beam).reshape(-1).to(torch.int32)
        return self.run_seq[:, :, t].reshape(-1).clone(), rows

    def result(self) -> torch.Tensor:
        """The best finished hypothesis per item [B, n], n = the longest of them (HF's crop)."""
        n = int(self.fin_len[:, 0].max().clamp(min=1))
        return self.fin_seq[:, 0, :n].clone()
