"""ProjectionTrainerStage1 — the reference's Stage-1 trainer API
(`Stage1/projector_trainer.py:18-521`) running its step on libptk.

Same constructor signature, `.train()` and `.save_projection(epoch, is_best)`.
What changes underneath:
  * the frozen towers run as HIP kernel sequences (`SiglipVisionTower`,
    `Gemma3CausalLM`); HF `SiglipModel` / `Gemma3ForCausalLM` instances passed
    in are converted once (weights re-laid out for the kernels);
  * one process per GPU with torch.distributed/RCCL instead of accelerate+DDP:
    batches are dealt to ranks as accelerate's prepared DataLoader deals them
    (even_batches: equal counts of full batches per rank), the projector's flat fp32 grads
    are all-reduced once per step, clip + AdamW is one fused kernel;
  * the arithmetic quirks of the reference are kept on purpose:
    loss / gas twice before backward, an optimizer step on every micro-batch,
    the scheduler advanced `num_processes` times per step with its horizon
    computed from the unsharded loader, cosine lambda without a clamp;
  * checkpoints are byte-compatible: `torch.save(state_dict)` with keys
    model.0/2.{weight,bias} + projector_config.json (`:455-521`).
Validation (`:292-448`) when val_dataset is given: the loss (forward + CE only) and, when the tokenizer can
decode (`batch_decode`), the reference's last-word accuracy of `generate` from the projected embeddings
(`:378-413`: max_new_tokens 64, do_sample=True with HF's default top-k 50 / temperature 1, pad / eos from the
tokenizer) on libptk's KV-cache decode (`Gemma3CausalLM.generate`, `ptk_gemma3_generate`).  The draws come from
a counter-based generator seeded per epoch and batch (`generate_seed`), not torch's multinomial stream.
"""
from __future__ import annotations

import json
import logging
import math
import os
import re
import time

import torch

from . import dist as D
from .gemma3 import Gemma3CausalLM
from .projectors import MLPProjector
from .siglip import SiglipVisionTower
from .stage1 import Stage1Engine, cosine_lambda

logger = logging.getLogger(__name__)


def _collate(items):
    return {k: torch.stack([it[k] for it in items]) for k in items[0]}


def get_last_word(text):
    """The reference's last-word extractor (Stage1/projector_trainer.py:132-137): the last \\w+ run, lower-cased."""
    if not text or not isinstance(text, str):
        return ""
    words = re.findall(r"\b\w+\b", text.lower())
    return words[-1] if words else ""


class ProjectionTrainerStage1:
    def __init__(self, accelerator, vision_encoder, language_model, projection_layer, processor, tokenizer,
                 train_dataset, val_dataset=None, output_dir="./trained_projection_stage1", batch_size=8,
                 learning_rate=1e-4, weight_decay=0.01, num_epochs=10, gradient_accumulation_steps=1,
                 warmup_ratio=0.0, wandb_project="xray_projection_training", save_every_n_epochs=0,
                 log_fn=None, seed=0, num_workers=8, generate_max_new_tokens=64, generate_do_sample=True,
                 generate_seed=0):
        if accelerator is None:
            accelerator = D.DistState(gradient_accumulation_steps)
        elif not isinstance(accelerator, D.DistState):
            accelerator = D.from_accelerator(accelerator)
        self.accelerator = acc = accelerator
        self.device = acc.device
        self.output_dir, self.num_epochs, self.batch_size = output_dir, num_epochs, batch_size
        self.save_every_n_epochs, self.wandb_project = save_every_n_epochs, wandb_project
        self.train_dataset, self.val_dataset = train_dataset, val_dataset
        self.processor, self.tokenizer = processor, tokenizer
        self.log_fn = log_fn
        self.seed = seed
        self.num_workers = num_workers   # decode threads for image datasets (the reference: 2 DataLoader workers, :60)
        # validation generate (projector_trainer.py:386-393): max_new_tokens 64, do_sample True
        self.generate_max_new_tokens, self.generate_do_sample = generate_max_new_tokens, generate_do_sample
        self.generate_seed = generate_seed
        self._pre = None
        if acc.is_main_process:
            os.makedirs(output_dir, exist_ok=True)

        # frozen towers on the HIP device
        self.vision_encoder = vision_encoder if isinstance(vision_encoder, SiglipVisionTower) \
            else SiglipVisionTower.from_hf(vision_encoder, self.device)
        self.language_model = language_model if isinstance(language_model, Gemma3CausalLM) \
            else Gemma3CausalLM.from_hf(language_model, self.device)
        if not isinstance(projection_layer, MLPProjector):
            sd = projection_layer.state_dict()
            p = MLPProjector(sd["model.0.weight"].shape[1], sd["model.2.weight"].shape[0])
            p.load_state_dict({k: v.detach().float().cpu() for k, v in sd.items()})
            projection_layer = p
        self.projection_layer = projection_layer.to(self.device)
        # text key mask `token_ids != tokenizer.pad_token_id`, all ones when the tokenizer has no pad
        # token (projector_trainer.py:207-209); -1 never matches a token id
        pad = getattr(tokenizer, "pad_token_id", None) if tokenizer is not None else None
        self.pad_token_id = -1 if pad is None else int(pad)

        # schedule horizon from the UNSHARDED loader (projector_trainer.py:82-95, F7)
        n_batches = math.ceil(len(train_dataset) / batch_size)
        self.max_train_steps = num_epochs * math.ceil(n_batches / gradient_accumulation_steps)
        self.num_warmup_steps = math.ceil(warmup_ratio * self.max_train_steps)
        self.engine = Stage1Engine(self.vision_encoder, self.language_model, self.projection_layer,
                                   learning_rate=learning_rate, weight_decay=weight_decay,
                                   gradient_accumulation_steps=acc.gradient_accumulation_steps,
                                   warmup_steps=self.num_warmup_steps, total_steps=self.max_train_steps,
                                   world_size=acc.num_processes)
        self.engine.pad_token_id = self.pad_token_id
        self.global_step = 0

    # ------------------------------------------------------------------ data
    def _batches(self, dataset, epoch, shuffle=True):
        acc = self.accelerator
        index_batches = [[int(i) for i in idx] for idx in
                         D.shard_batches(len(dataset), self.batch_size, acc.process_index, acc.num_processes, epoch,
                                         self.seed, shuffle)]
        if getattr(dataset, "yields_images", False):
            # decoded-image dataset (data.XrayTextPairDataset): workers decode, the GPU resizes/normalises
            yield from self._image_batches(dataset, index_batches)
            return
        for idx in index_batches:
            b = _collate([dataset[i] for i in idx])
            yield {k: v.to(self.device, non_blocking=True) for k, v in b.items()}

    def _image_batches(self, dataset, index_batches):
        from .data import ImagePreprocessor, ThreadedImageLoader
        if self._pre is None:
            self._pre = ImagePreprocessor(self.vision_encoder.cfg.image_size, self.device, processor=self.processor,
                                          dtype=torch.bfloat16)
        yield from ThreadedImageLoader(dataset, index_batches, self._pre, threads=self.num_workers)

    def _log(self, d, step):
        if self.accelerator.is_main_process:
            if self.log_fn is not None:
                self.log_fn(d, step)
            else:
                logger.info("step %d %s", step, d)

    # ------------------------------------------------------------------ train
    def train_step(self, batch):
        """One reference iteration (projector_trainer.py:152-271); returns the gathered mean loss, or None
        when the vision tower raised: the reference logs the error and skips the batch (`continue`,
        :174-176) before the projector, the LLM or the optimizer run."""
        try:
            self.engine.encode_vision(batch["pixel_values"], batch["token_ids"])
        except Exception as e:   # noqa: BLE001 -- the reference catches every exception here
            logger.error("Error getting vision embeddings: %s", e, exc_info=True)
            return None
        loss = self.engine.step(batch["pixel_values"], batch["token_ids"], batch["labels"])
        self.global_step += 1
        return self.accelerator.gather(loss).mean()

    def train(self):
        acc = self.accelerator
        logger.info("Process %d: Stage 1 training for %d epochs on %s", acc.process_index, self.num_epochs,
                    self.device)
        best_val = float("inf")
        for epoch in range(self.num_epochs):
            epoch_loss, n = 0.0, 0
            for batch in self._batches(self.train_dataset, epoch):
                avg = self.train_step(batch)
                if avg is None:
                    continue
                avg = float(avg)                              # host sync, as the reference's .item()
                epoch_loss += avg
                n += 1
                self._log({"train/batch_loss": avg, "train/learning_rate": self.engine.last_lr,
                           "step": self.global_step}, self.global_step)
            # len(self.train_loader) AFTER prepare: the per-rank batch count (projector_trainer.py:275)
            n_opt = math.ceil(D.batches_per_rank(len(self.train_dataset), self.batch_size, acc.num_processes) /
                              max(1, acc.gradient_accumulation_steps))
            self._log({"train/epoch_loss": epoch_loss / max(1, n_opt), "epoch": epoch + 1}, self.global_step)
            if acc.is_main_process and self.save_every_n_epochs > 0 and (epoch + 1) % self.save_every_n_epochs == 0:
                self.save_projection(epoch=epoch + 1)
            if self.val_dataset is not None:
                vl, acc_pct = self.validate(epoch)
                d = {"validation/loss": vl, "epoch": epoch + 1}
                if acc_pct is not None:
                    d["validation/last_word_accuracy"] = acc_pct
                self._log(d, self.global_step)
                if vl < best_val:
                    best_val = vl
                    self.save_projection(is_best=True)
        logger.info("Stage 1 Training finished.")
        self.save_projection(epoch=self.num_epochs)

    def validation_loss(self):
        """Mean LM loss over the validation set: forward + CE only (no backward, no grad exchange)."""
        return self.validate(0, generate=False)[0]

    def validate(self, epoch, generate=True):
        """The reference's validation pass (projector_trainer.py:292-421): per batch the LM loss (forward + CE), and
        when the tokenizer decodes, generate(inputs_embeds=projected_embeds) -> last-word accuracy against the
        caption (:378-413).  Returns (mean loss over all ranks' batches, accuracy in % or None)."""
        tok = self.tokenizer
        gen = generate and tok is not None and hasattr(tok, "batch_decode") and self.generate_max_new_tokens > 0
        tot, n = torch.zeros(1, device=self.device), 0
        correct, total = 0, 0
        eng = self.engine
        for bi, batch in enumerate(self._batches(self.val_dataset, 0, shuffle=False)):
            tot += eng.forward_loss(batch["pixel_values"], batch["token_ids"], batch["labels"])
            n += 1
            if not gen:
                continue
            B = batch["token_ids"].shape[0]
            # the projected embeddings are the LLM input's first N - 1 rows of each sample (eng.x, [B * Sp, H])
            ids = self.language_model.generate(
                eng.x, prompt_len=eng.N - 1, batch=B, max_new_tokens=self.generate_max_new_tokens,
                do_sample=self.generate_do_sample, pad_token_id=getattr(tok, "pad_token_id", None),
                eos_token_id=getattr(tok, "eos_token_id", None),
                seed=self.generate_seed + 1000003 * (epoch + 1) + 7919 * bi + 104729 * self.accelerator.process_index)
            generated = tok.batch_decode(ids.cpu(), skip_special_tokens=True)
            reference = tok.batch_decode(batch["token_ids"].cpu().numpy(), skip_special_tokens=True)
            for ref_text, gen_text in zip(reference, generated):
                r, g = get_last_word(ref_text), get_last_word(gen_text)
                if r and g and r == g:
                    correct += 1
                total += 1
        cnt = torch.tensor([float(n)], device=self.device)
        self.accelerator.all_reduce_sum_(tot)
        self.accelerator.all_reduce_sum_(cnt)
        acc_pct = None
        if gen:
            c = torch.tensor([float(correct), float(total)], device=self.device)
            self.accelerator.all_reduce_sum_(c)
            acc_pct = float(c[0] / c[1].clamp(min=1) * 100.0)
        return float(tot / cnt.clamp(min=1)), acc_pct

    def save_projection(self, epoch=None, is_best=False):
        """projector_{best,epoch_N,final}.bin + projector_config.json (projector_trainer.py:455-521)."""
        if not self.accelerator.is_main_process:
            return
        if is_best:
            name = "projector_best.bin"
        elif epoch is not None:
            name = f"projector_epoch_{epoch}.bin"
        else:
            name = "projector_final.bin"
        path = os.path.join(self.output_dir, name)
        sd = {k: v.detach().cpu().clone() for k, v in self.projection_layer.state_dict().items()}
        torch.save(sd, path)
        cfg = {"vision_dim": self.projection_layer.model[0].in_features,
               "llm_dim": self.projection_layer.model[2].out_features}
        with open(os.path.join(self.output_dir, "projector_config.json"), "w") as f:
            json.dump(cfg, f, indent=4)
        logger.info("Projection layer state dict saved to %s", path)
        return path
