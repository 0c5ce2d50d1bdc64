"""Generate golden fixtures by running the REFERENCE Stage-1 trainer on CPU.

Run in the build container only (needs /root/reference and HF transformers):

    python tests/golden/make_golden.py            # writes tests/golden/<name>.npz

It imports `Stage1/projector_trainer.py` (ProjectionTrainerStage1),
`Stage1/projectors.py` (MLPProjector) and `Stage1/accelerator_setup.py` from
/root/reference, builds random-init HF `SiglipModel` / `Gemma3ForCausalLM` from
tiny configs, loads the repo's deterministic weights
(`projectiontrainer_amd.weights`), and runs `trainer.train()` for two
optimizer steps.  Hooks record what the trainer actually saw and produced:
the batch (after the DataLoader's shuffle), SigLIP patch embeddings,
projector output and its gradient, loss, LR, raw / clipped projector grads
and the projector params after each AdamW step.

Fixtures:
  tiny, tiny_gqa      tiny dims, fp32 (no mixed precision)
  tiny_bf16,          tiny dims under `accelerate launch --mixed_precision bf16`
  tiny_gqa_bf16       (run_projection_train_stage1.sh:6): both towers loaded in bf16
                      (train_projection_stage1.py:169-183,204-210), the projector fp32
                      under autocast -- the precision flow of SURVEY F8
  cfg1, cfg1_bf16     BASELINE cfg1 shapes: SigLIP-B/16-224 + Gemma3-1B (26 layers,
                      vocab 262144), bs 2, T 64, fp32 / bf16 as above
  cfg2w, cfg2w_bf16   BASELINE cfg2 WIDTHS (SigLIP-L/16-384 + Gemma3-1B, vocab 262144) at 2 + 6 layers
                      (one global Gemma layer), bs 2, T 128 (S 703 > the sliding window), fp32 / bf16
  cfg5w, cfg5w_bf16   BASELINE cfg5 WIDTHS (SigLIP-L/16-384 + Gemma3-4B, vocab 262208) at 2 + 6 layers, bs 1,
                      T 256, fp32 / bf16

Large tensors are stored as a strided sub-sample `<key>@sub<sr>x<sc>` (every
sr-th row, every sc-th column of the [rows, last-dim] view) plus the exact
`@norm` and `@sum` of the whole tensor; the pixel batch of the real-size
fixtures is stored as the sample order the shuffled loader produced
(`s<i>_order`), the pixels themselves being regenerated from the seed.
Each fixture runs in its own process (accelerate's state is a singleton).

Only data (inputs and expected outputs) is written; no reference source.
"""
from __future__ import annotations

import argparse
import math
import os
import subprocess
import sys
import tempfile
import types

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)

from projectiontrainer_amd.config import PRESETS, to_hf_dicts  # noqa: E402
from projectiontrainer_amd import weights as W  # noqa: E402

REF_STAGE1 = "/root/reference/Stage1"


SUB_BUDGET = 8192   # elements kept per large tensor


def sub_strides(shape):
    """(row stride, column stride) of the stored sub-sample of a tensor viewed as [rows, last-dim]."""
    C = shape[-1] if len(shape) else 1
    R = int(np.prod(shape[:-1])) if len(shape) > 1 else 1
    sc = 1 if C <= 1024 else math.ceil(C / 512)
    kept_c = math.ceil(C / sc)
    sr = max(1, math.ceil(R / max(1, SUB_BUDGET // kept_c)))
    return sr, sc


def run(name: str, gas: int, seed_batch: int, num_epochs: int = 2, lr: float = 1e-4, precision: str = "no"):
    """precision "bf16": ACCELERATE_MIXED_PRECISION=bf16 (what `accelerate launch --mixed_precision bf16`
    exports) and both towers cast to bf16 as train_projection_stage1.py:169-183,204-210 loads them."""
    os.environ["ACCELERATE_MIXED_PRECISION"] = precision
    sys.path.insert(0, REF_STAGE1)
    import transformers
    import accelerate
    from transformers import SiglipConfig, SiglipModel, Gemma3TextConfig, Gemma3ForCausalLM
    from projectors import MLPProjector                     # reference
    from projector_trainer import ProjectionTrainerStage1   # reference
    from accelerator_setup import setup_accelerator_and_logging  # reference

    torch.manual_seed(0)
    cfg = PRESETS[name.replace("_bf16", "")]
    vis_kw, txt_kw = to_hf_dicts(cfg)
    sig = SiglipModel(SiglipConfig(
        text_config=dict(vocab_size=64, hidden_size=64, intermediate_size=128, num_hidden_layers=1,
                         num_attention_heads=1, max_position_embeddings=16,
                         bos_token_id=None, eos_token_id=None, pad_token_id=None),
        vision_config=vis_kw)).float()
    vp = W.siglip_vision_params(cfg.vision)
    missing = sig.load_state_dict({k: torch.from_numpy(v) for k, v in vp.items()}, strict=False)
    assert not [k for k in missing.missing_keys if k.startswith("vision_model.") and ".head." not in k], missing
    llm = Gemma3ForCausalLM(Gemma3TextConfig(**txt_kw)).float()
    lp = W.gemma3_params(cfg.text)
    res = llm.load_state_dict({k: torch.from_numpy(v) for k, v in lp.items()}, strict=False)
    assert set(res.missing_keys) <= {"lm_head.weight"}, res
    assert llm.lm_head.weight.data_ptr() == llm.model.embed_tokens.weight.data_ptr()
    if precision == "bf16":
        sig, llm = sig.to(torch.bfloat16), llm.to(torch.bfloat16)
        assert llm.lm_head.weight.data_ptr() == llm.model.embed_tokens.weight.data_ptr()
    proj = MLPProjector(cfg.vision.hidden_size, cfg.text.hidden_size)
    pp = W.projector_params(cfg.vision.hidden_size, cfg.text.hidden_size, cfg.expansion_factor)
    proj.load_state_dict({k: torch.from_numpy(v) for k, v in pp.items()})

    px, ids, labels = W.synthetic_batch(cfg, seed=seed_batch)
    data = [{"pixel_values": torch.from_numpy(px[i]), "token_ids": torch.from_numpy(ids[i]),
             "labels": torch.from_numpy(labels[i])} for i in range(cfg.batch_size)]

    args = types.SimpleNamespace(gradient_accumulation_steps=gas, disable_wandb=True,
                                 batch_size=cfg.batch_size, wandb_project="x", wandb_run_name=None)
    acc = setup_accelerator_and_logging(args)
    assert acc.mixed_precision == precision, (acc.mixed_precision, precision)
    tok = types.SimpleNamespace(pad_token_id=cfg.text.pad_token_id, eos_token_id=cfg.text.eos_token_id)
    out = tempfile.mkdtemp()
    trainer = ProjectionTrainerStage1(acc, sig, llm, proj, None, tok, data, None, output_dir=out,
                                      batch_size=cfg.batch_size, learning_rate=lr, weight_decay=0.01,
                                      num_epochs=num_epochs, gradient_accumulation_steps=gas,
                                      warmup_ratio=0.0, save_every_n_epochs=0)

    rec = {}
    step = {"i": 0}

    big = cfg.batch_size * cfg.vision.num_channels * cfg.vision.image_size ** 2 > 65536

    def put(k, v):
        a = v.detach().cpu().float().numpy().copy() if torch.is_tensor(v) and v.is_floating_point() else \
            (v.detach().cpu().numpy().copy() if torch.is_tensor(v) else np.asarray(v))
        key = f"s{step['i']}_{k}"
        if k == "pixel_values" and big:
            # which dataset samples (in which order) the shuffled loader put in this batch
            rec[f"s{step['i']}_order"] = np.array([int(np.argmin([np.abs(a[j] - px[i]).max() for i in range(len(px))]))
                                                    for j in range(a.shape[0])])
            return
        if a.ndim >= 2 and a.size > 16384:
            if name.startswith("tiny") and a.ndim == 2:
                # round-1 layout of the tiny fixtures: every 16th row
                rec[key + "@rows16"] = a[::16]
            else:
                sr, sc = sub_strides(a.shape)
                rec[key + f"@sub{sr}x{sc}"] = a.reshape(-1, a.shape[-1])[::sr, ::sc]
            rec[key + "@norm"] = np.array(np.linalg.norm(a.astype(np.float64)))
            rec[key + "@sum"] = np.array(a.astype(np.float64).sum())
        else:
            rec[key] = a

    vt = sig.vision_model
    vt.register_forward_pre_hook(lambda m, a, kw: put("pixel_values", kw["pixel_values"]), with_kwargs=True)
    vt.register_forward_hook(lambda m, a, kw, o: put("patch", o.last_hidden_state[:, 1:, :]), with_kwargs=True)
    llm.model.embed_tokens.register_forward_pre_hook(lambda m, a: put("token_ids", a[0]))

    def proj_hook(m, a, o):
        put("proj", o)
        o.register_hook(lambda g: put("d_proj", g))
    proj.register_forward_hook(proj_hook)

    def llm_hook(m, a, kw, o):
        put("lm_labels", kw["labels"])
        put("attention_mask", kw["attention_mask"])
        put("loss", o.loss)
    llm.register_forward_hook(llm_hook, with_kwargs=True)

    params = dict(proj.named_parameters())
    for k, p in params.items():
        p.register_hook(lambda g, k=k: put("grad." + k, g))
    opt = trainer.optimizer.optimizer

    def pre(o, a, kw):
        put("lr", o.param_groups[0]["lr"])
        for k, p in params.items():
            put("clipped." + k, p.grad)

    def post(o, a, kw):
        for k, p in params.items():
            put("param." + k, p)
        step["i"] += 1
    opt.register_step_pre_hook(pre)
    opt.register_step_post_hook(post)

    trainer.train()
    meta = dict(name=name, gas=gas, seed_batch=seed_batch, lr=lr, num_epochs=num_epochs, precision=precision,
                steps=step["i"], max_train_steps=trainer.max_train_steps,
                torch=torch.__version__, transformers=transformers.__version__,
                accelerate=accelerate.__version__)
    rec["meta"] = np.array(repr(meta))
    # fingerprint of the generated weights (detects generator drift)
    fp = np.array([float(np.sum(v.astype(np.float64))) for d in (vp, lp, pp) for v in d.values()])
    rec["weight_fingerprint"] = fp
    return rec


FIXTURES = {   # name: (gas, batch seed, precision)
    "tiny": (2, 11, "no"),
    "tiny_gqa": (1, 12, "no"),
    "tiny_bf16": (2, 11, "bf16"),     # same batch as "tiny": bf16-vs-fp32 = the reference's own bf16 noise
    "tiny_gqa_bf16": (1, 12, "bf16"),
    "cfg1": (2, 14, "no"),
    "cfg1_bf16": (2, 14, "bf16"),     # same batch as "cfg1"
    # cfg2 widths (SigLIP-L/16-384 + Gemma3-1B) at 2 + 6 layers, bs 2, T 128: pins the cfg2 per-layer shapes to the
    # reference itself, and its bf16 twin measures the reference's own mixed-precision noise at those widths
    "cfg2w": (2, 15, "no"),
    "cfg2w_bf16": (2, 15, "bf16"),   # same batch as "cfg2w"
    # cfg5 widths (SigLIP-L/16-384 + Gemma3-4B) at 2 + 6 layers, bs 1, T 256: the 4B per-layer shapes pinned to the
    # reference, and the 4B-width twin noise the cfg5 full-depth bars derive from
    "cfg5w": (2, 16, "no"),
    "cfg5w_bf16": (2, 16, "bf16"),   # same batch as "cfg5w"
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.dirname(os.path.abspath(__file__)))
    ap.add_argument("--only", default=None, help="one fixture (run in this process)")
    a = ap.parse_args()
    if a.only is None:
        for name in FIXTURES:
            subprocess.check_call([sys.executable, os.path.abspath(__file__), "--out", a.out, "--only", name])
        return
    gas, seed, precision = FIXTURES[a.only]
    torch.set_num_threads(min(8, os.cpu_count() or 8))
    rec = run(a.only, gas, seed, precision=precision)
    path = os.path.join(a.out, f"{a.only}.npz")
    np.savez_compressed(path, **rec)
    print(path, os.path.getsize(path), "bytes", rec["meta"])


if __name__ == "__main__":
    main()
