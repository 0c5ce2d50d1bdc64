"""VQATrainerStage2 — the reference's Stage-2 trainer API (`Stage2/trainer.py:63-769`)
running its step on libptk (`stage2.Stage2Engine`).

Same constructor signature, `.train()`, `.evaluate(epoch, global_step)`,
`.save_model(path)` and the module-level `vqa_collate_fn(batch, tokenizer)`.
Supported configuration: BASELINE cfg4 — the LLM unfrozen (`freeze_llm=False`,
no QLoRA), projector and vision encoder frozen; anything else raises
NotImplementedError (QLoRA/peft needs 4-bit kernels; a trainable vision
encoder or projector needs their backward passes).  Note that the reference's
own run script ships `ENABLE_QLORA=true` (`Stage2/run_vqa_train_stage2.sh:42`,
a Qwen3-8B QLoRA run); cfg4 -- the benchmark this path is built for -- is the
unfrozen-LLM form of the same trainer (`--unfreeze_llm`, `UNFREEZE_LLM` in that
script, ignored there only because QLoRA is on).

Kept reference semantics (Stage2/trainer.py:248-488):
  * batches dealt as accelerate's prepared DataLoader deals them (even_batches),
    padded per batch by `vqa_collate_fn` on the tokenizer's padding side;
  * `accelerator.accumulate`: an optimizer step when (micro+1) % gas == 0 or at
    the end of the rank's loader; loss / gas before `backward`, which divides by
    gas again, grads summed over micro-batches;
  * clip_grad_norm_(llm, 1.0), AdamW(lr, wd) over the LLM parameters, cosine
    schedule with warmup (horizon from the unsharded loader), stepped
    num_processes times per optimizer step;
  * logging keys `train/batch_loss` (every micro-batch), `train/step_loss` (sync
    micro-batches), `train/loss` = sum of sync losses / len(train_loader) per
    epoch, `val/loss`.
`evaluate` computes the validation loss and, with a tokenizer that decodes, the reference's generated examples
(:595-700): `generate(inputs_embeds=[projected image | question], attention_mask, max_new_tokens=512,
do_sample=True, num_beams=3, top_p=0.9, top_k=50)` on libptk's stepwise KV-cache decode with beam sampling
(`Gemma3CausalLM.beam_generate`), decoded and written to `validation_examples/epoch_{n}_examples.txt` and
`all_validation_examples.txt` in the reference's format (at most 20 examples, gathered over the ranks).  `save_model` writes the fine-tuned LLM as HF-named
bf16 tensors (`language_model/model.safetensors`, accelerate's save_model
layout) plus the optimizer state of this rank (`optimizer_rank{r}.pt`).
"""
from __future__ import annotations

import logging
import math
import os

import torch

from . import dist as D
from .gemma3 import Gemma3CausalLM
from .projectors import MLPProjector
from .siglip import SiglipVisionTower
from .stage2 import Stage2Engine

logger = logging.getLogger(__name__)


def vqa_collate_fn(batch, tokenizer):
    """Stage2/trainer.py:18-61: stack pixel values; pad question and answer ids to the longest of the
    batch with tokenizer.pad_token_id on tokenizer.padding_side."""
    pad_id, side = tokenizer.pad_token_id, getattr(tokenizer, "padding_side", "right")

    def pad(seqs):
        n = max(s.shape[0] for s in seqs)
        out = []
        for s in seqs:
            p = torch.full((n - s.shape[0],), pad_id, dtype=s.dtype)
            out.append(torch.cat([p, s]) if side == "left" else torch.cat([s, p]))
        return torch.stack(out)
    return {"pixel_values": torch.stack([it["pixel_values"] for it in batch]),
            "question_input_ids": pad([it["question_input_ids"] for it in batch]),
            "answer_input_ids": pad([it["answer_input_ids"] for it in batch])}


class VQATrainerStage2:
    def __init__(self, accelerator, vision_encoder, language_model, projection_layer, tokenizer, train_dataset,
                 val_dataset, output_dir: str, batch_size: int, learning_rate: float, weight_decay: float,
                 num_epochs: int, gradient_accumulation_steps: int, warmup_ratio: float, freeze_vision_encoder: bool,
                 freeze_projection_layer: bool, freeze_llm: bool, enable_qlora: bool, train_ve_first_epoch: bool,
                 wandb_project: str, log_fn=None, seed: int = 0, generate_max_new_tokens: int = 512,
                 generate_num_beams: int = 3, generate_do_sample: bool = True, generate_top_k: int = 50,
                 generate_top_p: float = 0.9, generate_seed: int = 0):
        if enable_qlora:
            raise NotImplementedError("VQATrainerStage2 (HIP): QLoRA / 4-bit LLMs are not supported; run with the "
                                      "dense bf16 LLM and --unfreeze_llm")
        if freeze_llm or not freeze_projection_layer or not freeze_vision_encoder or train_ve_first_epoch:
            raise NotImplementedError("VQATrainerStage2 (HIP) supports the BASELINE cfg4 setting: LLM unfrozen, "
                                      "projector and vision encoder frozen")
        if accelerator is None:
            accelerator = D.DistState(gradient_accumulation_steps)
        elif not isinstance(accelerator, D.DistState):
            accelerator = D.from_accelerator(accelerator)
        self.accelerator = acc = accelerator
        self.device = acc.device
        self.tokenizer = tokenizer
        self.output_dir, self.num_epochs, self.batch_size = output_dir, num_epochs, batch_size
        self.train_dataset, self.val_dataset = train_dataset, val_dataset
        self.wandb_project, self.log_fn, self.seed = wandb_project, log_fn, seed
        self.gas = gradient_accumulation_steps
        # the validation generate of Stage2/trainer.py:603-613
        self.gen_kwargs = dict(max_new_tokens=generate_max_new_tokens, num_beams=generate_num_beams,
                               do_sample=generate_do_sample, top_k=generate_top_k, top_p=generate_top_p)
        self.generate_seed = generate_seed
        self.validation_dir = os.path.join(output_dir, "validation_examples")
        if acc.is_main_process:
            os.makedirs(self.validation_dir, exist_ok=True)

        self.vision_encoder = vision_encoder if isinstance(vision_encoder, SiglipVisionTower) \
            else SiglipVisionTower.from_hf(vision_encoder, self.device)
        self.language_model = language_model if isinstance(language_model, Gemma3CausalLM) \
            else Gemma3CausalLM.from_hf(language_model, self.device, max_pos=4096)
        if not isinstance(projection_layer, MLPProjector):
            sd = projection_layer.state_dict()
            p = MLPProjector(sd["model.0.weight"].shape[1], sd["model.2.weight"].shape[0])
            p.load_state_dict({k: v.detach().float().cpu() for k, v in sd.items()})
            projection_layer = p
        self.projection_layer = projection_layer.to(self.device)

        # schedule horizon from the UNSHARDED loader (Stage2/trainer.py:151-165)
        n_batches = math.ceil(len(train_dataset) / batch_size)
        self.max_train_steps = num_epochs * math.ceil(n_batches / gradient_accumulation_steps)
        self.num_warmup_steps = math.ceil(warmup_ratio * self.max_train_steps)
        pad = getattr(tokenizer, "pad_token_id", None)
        self.engine = Stage2Engine(self.vision_encoder, self.language_model, self.projection_layer,
                                   learning_rate=learning_rate, weight_decay=weight_decay,
                                   gradient_accumulation_steps=gradient_accumulation_steps,
                                   warmup_steps=self.num_warmup_steps, total_steps=self.max_train_steps,
                                   world_size=acc.num_processes, rank=acc.process_index,
                                   pad_token_id=-1 if pad is None else int(pad))
        self.global_step = 0

    # ------------------------------------------------------------------ data
    def _batches(self, dataset, epoch, shuffle=True):
        acc = self.accelerator
        for idx in D.shard_batches(len(dataset), self.batch_size, acc.process_index, acc.num_processes, epoch,
                                   self.seed, shuffle):
            b = vqa_collate_fn([dataset[int(i)] for i in idx], self.tokenizer)
            yield {k: v.to(self.device, non_blocking=True) for k, v in b.items()}

    def _log(self, d, step):
        if self.accelerator.is_main_process:
            if self.log_fn is not None:
                self.log_fn(d, step)
            else:
                logger.info("step %d %s", step, d)

    # ------------------------------------------------------------------ train
    def train(self):
        acc = self.accelerator
        logger.info("Process %d: Starting Stage 2 training for %d epochs on device %s", acc.process_index,
                    self.num_epochs, self.device)
        n_local = D.batches_per_rank(len(self.train_dataset), self.batch_size, acc.num_processes)
        for epoch in range(self.num_epochs):
            epoch_train_loss = 0.0
            for i, batch in enumerate(self._batches(self.train_dataset, epoch)):
                loss = self.engine.forward_backward(batch["pixel_values"], batch["question_input_ids"],
                                                    batch["answer_input_ids"])
                sync = (i + 1) % self.gas == 0 or i + 1 == n_local
                log = {}
                if sync:
                    self.engine.optimizer_step()
                    self.global_step += 1
                    avg_loss_step = float(acc.gather(loss).mean())
                    epoch_train_loss += avg_loss_step
                    log["train/step_loss"] = avg_loss_step
                log.update({"train/batch_loss": float(acc.gather(loss).mean()),
                            "train/learning_rate": self.engine.scheduler_lr, "step": self.global_step})
                self._log(log, self.global_step)
            avg = epoch_train_loss / max(1, n_local)      # len(self.train_loader) (Stage2/trainer.py:468)
            self._log({"train/loss": avg, "train/learning_rate": self.engine.scheduler_lr, "epoch": epoch + 1},
                      self.global_step)
            if self.val_dataset is not None:
                self.evaluate(epoch, self.global_step)
            # every rank: each writes its ZeRO-1 optimizer shard (the reference's save_state keeps the full
            # optimizer); the main process writes the model and tokenizer
            self.save_model(os.path.join(self.output_dir, f"checkpoint-epoch_{epoch + 1}"))
        logger.info("Process %d: Stage 2 training complete!", acc.process_index)

    def evaluate(self, epoch, global_step):
        """Validation loss (Stage2/trainer.py:490-593): forward + CE only, as under the reference's torch.no_grad
        (no grads touched); then, with a tokenizer that decodes, the generated examples (:595-700).  As the reference, the batches are
        collated with the tokenizer padding on the LEFT (restored afterwards) and a missing pad token falls
        back to eos (:499-507)."""
        tok = self.tokenizer
        side = getattr(tok, "padding_side", "right")
        pad0 = getattr(tok, "pad_token_id", None)
        tok.padding_side = "left"
        if pad0 is None:
            logger.warning("Tokenizer pad_token_id is None. Setting to eos_token_id for evaluation.")
            tok.pad_token_id = tok.eos_token_id
        eng_pad = self.engine.pad_token_id
        self.engine.pad_token_id = int(tok.pad_token_id)
        examples = []
        can_decode = hasattr(tok, "batch_decode")
        try:
            tot, n = 0.0, 0
            for bi, batch in enumerate(self._batches(self.val_dataset, 0, shuffle=False)):
                q, a = batch["question_input_ids"], batch["answer_input_ids"]
                loss = self.engine.forward_loss(batch["pixel_values"], q, a)
                tot += float(self.accelerator.gather(loss).mean())
                n += 1
                if can_decode:
                    try:   # (the reference logs a failed generation and goes on, :645-646)
                        preds = self._generate_batch(q, seed=self.generate_seed + 7919 * bi + epoch)
                        dp = tok.batch_decode(preds.cpu(), skip_special_tokens=True)
                        dq = tok.batch_decode(q.cpu(), skip_special_tokens=True)
                        da = tok.batch_decode(a.cpu(), skip_special_tokens=True)
                        examples += [{"epoch": epoch + 1, "question": dq[j], "ground_truth": da[j],
                                      "prediction": dp[j]} for j in range(len(dp))]
                    except Exception as e:  # noqa: BLE001
                        logger.error("Error during validation generation/logging: %s", e, exc_info=True)
        finally:
            tok.padding_side = side
            self.engine.pad_token_id = eng_pad
        acc = self.accelerator
        acc.wait_for_everyone()
        if can_decode:
            gathered = acc.gather_object(examples)[:min(20, len(self.val_dataset))]
            if acc.is_main_process and gathered:
                self._write_examples(epoch, gathered)
        avg = tot / max(1, n)
        self._log({"val/loss": avg, "epoch": epoch + 1}, global_step)
        return avg

    def _generate_batch(self, question_ids, seed=0):
        """The validation generate of one batch (Stage2/trainer.py:596-626): prompt = the projected image tokens
        of the batch just evaluated (the engine's LLM input rows) followed by the question embeddings, attention
        mask 1 on the image tokens and (question != pad) on the question."""
        eng = self.engine
        B, Tq = question_ids.shape
        P = eng.N - 1 + Tq
        x = eng.x.view(B, eng.Sp, -1)[:, :P].contiguous()   # forward_loss built [projected | question | answer]
        mask = torch.ones(B, P, dtype=torch.int32, device=self.device)
        mask[:, eng.N - 1:] = (question_ids.to(self.device) != int(self.tokenizer.pad_token_id)).int()
        return self.language_model.beam_generate(x, mask, eos_token_id=getattr(self.tokenizer, "eos_token_id", None),
                                                 pad_token_id=int(self.tokenizer.pad_token_id), seed=seed,
                                                 **self.gen_kwargs)

    def _write_examples(self, epoch, examples):
        """validation_examples/epoch_{n}_examples.txt and all_validation_examples.txt (Stage2/trainer.py:672-700)."""
        def body():
            out = []
            for i, ex in enumerate(examples):
                out.append(f"Example {i + 1}:\nQuestion: {ex['question']}\nGround Truth: {ex['ground_truth']}\n"
                           f"Prediction: {ex['prediction']}\n{'=' * 80}\n\n")
            return "".join(out)
        try:
            with open(os.path.join(self.validation_dir, f"epoch_{epoch + 1}_examples.txt"), "w", encoding="utf-8") as f:
                f.write(f"Validation Examples for Epoch {epoch + 1}\n{'=' * 80}\n\n" + body())
            with open(os.path.join(self.validation_dir, "all_validation_examples.txt"), "a" if epoch > 0 else "w",
                      encoding="utf-8") as f:
                f.write(f"\nValidation Examples for Epoch {epoch + 1}\n{'=' * 80}\n\n" + body())
        except OSError as e:
            logger.error("Failed to save validation examples to file: %s", e, exc_info=True)

    def save_model(self, path):
        """Called on EVERY rank.  Main process: language_model/model.safetensors (HF names, bf16) and the
        tokenizer (Stage2/trainer.py:740-742).  Every rank: optimizer_rank{r}.pt with its ZeRO-1 shard of the
        AdamW moments and the step / schedule counters, so the files of all ranks hold the complete optimizer
        state that the reference's accelerator.save_state writes (:718); load with load_optimizer_state."""
        acc = self.accelerator
        os.makedirs(path, exist_ok=True)
        torch.cuda.synchronize(self.device)
        torch.save(self.engine.optimizer_state(), os.path.join(path, f"optimizer_rank{acc.process_index}.pt"))
        if acc.is_main_process:
            from safetensors.torch import save_file
            llm_dir = os.path.join(path, "language_model")
            os.makedirs(llm_dir, exist_ok=True)
            sd = {k: v.detach().contiguous().cpu() for k, v in self.engine.state.state_dict_hf().items()}
            save_file(sd, os.path.join(llm_dir, "model.safetensors"))
            if hasattr(self.tokenizer, "save_pretrained"):
                self.tokenizer.save_pretrained(llm_dir)
            logger.info("Full language model saved to %s", llm_dir)
        acc.wait_for_everyone()

    def load_optimizer_state(self, path):
        """Restore this rank's ZeRO-1 optimizer shard written by save_model."""
        sd = torch.load(os.path.join(path, f"optimizer_rank{self.accelerator.process_index}.pt"), weights_only=True)
        self.engine.load_optimizer_state(sd)
