"""Stage 2 (VQA fine-tune, unfrozen Gemma3, BASELINE cfg4's flags) on the HIP path vs the reference.

`tests/golden/s2_tiny{,_bf16}.npz` come from the reference's own VQATrainerStage2.train()
(tests/golden/make_golden_stage2.py): 6 micro-batches at gradient_accumulation_steps 2 over 2 epochs,
4 optimizer steps (warmup first), with every LLM parameter's accumulated grad and post-AdamW value.
The HIP engine replays the same collated batches.  Tolerances follow tests/test_stage1_gpu.py: the
fixtures are twins (same weights and data, fp32 and `--mixed_precision bf16`), and the HIP path (bf16
parameters, grads and moments, as the reference's bf16 run) must agree with either within
max(SURVEY bar, 2 x the reference's own bf16-vs-fp32 distance) per tensor (cosine deficit x4:
1 - cos ~ rel-L2^2 / 2):
  micro-batch loss |d| <= 2e-2;  accumulated grads rel-L2 <= max(2e-2, 2 noise), cos >= min(0.999, ...);
  params after each AdamW step: max |d| <= 2.5 * sum(lr) + 1 bf16 ulp of the tensor's largest value,
  median |d| <= 0.05 * lr + half an ulp (bf16 parameters: both runs round every update).
"""
import ast
import json
import math
import os

import numpy as np
import pytest
import torch

from tests import golden_util as G

pytestmark = pytest.mark.gpu
_LOG = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpurun_out",
                    "parity_metrics.jsonl")


def record(test, key, **vals):
    if os.path.isdir(os.path.dirname(_LOG)):
        with open(_LOG, "a") as f:
            f.write(json.dumps({"test": test, "key": key, **{k: float(v) for k, v in vals.items()}}) + "\n")


def load(name):
    d = np.load(f"{G.GOLDEN}/{name}.npz", allow_pickle=False)
    return d, ast.literal_eval(str(d["meta"]))


def stored(d, key):
    if key in d.files:
        return d[key], 1, 1
    k, sr, sc = G.sub_key(d, key)
    return d[k], sr, sc


def rel_l2(a, b):
    a, b = np.asarray(a, np.float64).ravel(), np.asarray(b, np.float64).ravel()
    return np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30)


def cosine(a, b):
    a, b = np.asarray(a, np.float64).ravel(), np.asarray(b, np.float64).ravel()
    return float(a @ b / max(np.linalg.norm(a) * np.linalg.norm(b), 1e-30))


def build(name, gpu, meta):
    from projectiontrainer_amd import weights as W
    from projectiontrainer_amd.config import PRESETS
    from projectiontrainer_amd.gemma3 import Gemma3CausalLM
    from projectiontrainer_amd.projectors import MLPProjector
    from projectiontrainer_amd.siglip import SiglipVisionTower
    from projectiontrainer_amd.stage2 import Stage2Engine
    cfg = PRESETS["tiny"]
    vp, lp = W.siglip_vision_params(cfg.vision), W.gemma3_params(cfg.text)
    pp = W.projector_params(cfg.vision.hidden_size, cfg.text.hidden_size, cfg.expansion_factor)
    if meta["precision"] == "bf16":     # the reference casts the towers AND the frozen projector to bf16
        vp = {k: G.bf16_round(v) for k, v in vp.items()}
        lp = {k: G.bf16_round(v) for k, v in lp.items()}
        pp = {k: G.bf16_round(v) for k, v in pp.items()}
    proj = MLPProjector(cfg.vision.hidden_size, cfg.text.hidden_size)
    proj.load_state_dict({k: torch.from_numpy(v) for k, v in pp.items()})
    proj.to(gpu)
    total = meta["max_train_steps"]
    eng = Stage2Engine(SiglipVisionTower(cfg.vision, vp, gpu), Gemma3CausalLM(cfg.text, lp, gpu, max_pos=256), proj,
                       learning_rate=meta["lr"], weight_decay=meta["weight_decay"],
                       gradient_accumulation_steps=meta["gas"], max_grad_norm=meta["max_grad_norm"],
                       warmup_steps=math.ceil(meta["warmup_ratio"] * total), total_steps=total)
    return cfg, eng


@pytest.mark.parametrize("name", ["s2_tiny_bf16", "s2_tiny"])
def test_stage2_vs_reference_golden(gpu, name):
    from projectiontrainer_amd import weights as W
    d, meta = load(name)
    base, _ = load("s2_tiny")
    twin, _ = load("s2_tiny_bf16")
    cfg, eng = build(name, gpu, meta)
    items = W.synthetic_vqa_items(cfg, meta["n_items"], meta["seed"])
    px = torch.stack([it["pixel_values"] for it in items])
    per_epoch = math.ceil(meta["n_items"] / meta["batch_size"])
    t = f"stage2[{name}]"
    o, lr_sum = 0, 0.0
    for m in range(meta["micro_batches"]):
        i = m % per_epoch
        q = torch.from_numpy(d[f"m{m}_question_input_ids"]).to(gpu)
        a = torch.from_numpy(d[f"m{m}_answer_input_ids"]).to(gpu)
        loss = float(eng.forward_backward(px[d[f"m{m}_order"]].to(gpu), q, a))
        dl = abs(loss - float(d[f"m{m}_loss"]))
        record(t, f"m{m}_loss", abs=dl)
        assert dl <= 2e-2, (m, loss, float(d[f"m{m}_loss"]))
        if not ((i + 1) % meta["gas"] == 0 or i + 1 == per_epoch):
            continue
        torch.cuda.synchronize()
        grads = {k: v.float().cpu().numpy() for k, v in eng.state.state_dict_hf(grads=True).items()}
        for n in meta["param_names"]:
            key = f"o{o}_grad.{n}"
            ref, sr, sc = stored(d, key)
            got = grads[n] if key in d.files else G.sub_sample(grads[n], sr, sc)
            nb, _, _ = stored(base, key)
            nt, _, _ = stored(twin, key)
            tol_r = max(2e-2, 2.0 * rel_l2(nt, nb))
            tol_c = min(0.999, 1.0 - 4.0 * (1.0 - cosine(nt, nb)))   # factor 2 on the distance
            r, c = rel_l2(got, ref), cosine(got, ref)
            record(t, key, rel_l2=r, cos=c, tol_rel_l2=tol_r, tol_cos=tol_c)
            assert r <= tol_r and c >= tol_c, (key, r, tol_r, c, tol_c)
        eng.optimizer_step()
        torch.cuda.synchronize()
        assert abs(eng.last_lr - float(d[f"o{o}_lr"])) <= 1e-12, (o, eng.last_lr, float(d[f"o{o}_lr"]))
        lr_sum += eng.last_lr
        params = {k: v.float().cpu().numpy() for k, v in eng.state.state_dict_hf().items()}
        for n in meta["param_names"]:
            key = f"o{o}_param.{n}"
            ref, sr, sc = stored(d, key)
            got = G.sub_sample(params[n], sr, sc) if key not in d.files else params[n]
            ulp = 2.0 ** (np.floor(np.log2(max(np.abs(ref).max(), 1e-30))) - 7)
            mx, md = np.abs(got - ref).max(), np.median(np.abs(got - ref))
            record(t, key, max_abs=mx, median_abs=md, atol=2.5 * lr_sum + ulp)
            assert mx <= 2.5 * lr_sum + ulp, (key, mx, 2.5 * lr_sum + ulp)
            assert md <= 0.05 * meta["lr"] + ulp / 2, (key, md)
        o += 1
    assert o == meta["opt_steps"]


def test_stage2_state_roundtrip(gpu):
    """The flat bf16 store holds exactly the HF tensors it was built from (q|k|v split, gate/up
    de-interleaved), and its kernel-side copies (transposes, fp32 norms) match it."""
    from projectiontrainer_amd import weights as W
    from projectiontrainer_amd.config import PRESETS
    from projectiontrainer_amd.gemma3 import Gemma3CausalLM
    from projectiontrainer_amd.stage2 import Gemma3TrainState
    cfg = PRESETS["tiny_gqa"].text
    lp = W.gemma3_params(cfg)
    llm = Gemma3CausalLM(cfg, lp, gpu, max_pos=256)
    st = Gemma3TrainState(llm, world_size=3)
    assert st.numel % 3 == 0
    sd = st.state_dict_hf()
    for k, v in lp.items():
        np.testing.assert_array_equal(sd[k].float().cpu().numpy(), G.bf16_round(v), err_msg=k)
    lay = llm.layers[1]
    assert torch.equal(lay["wgu_t"], lay["wgu"].t().contiguous())
    assert torch.equal(lay["ln_pre_ff"], st.view("1.ln_pre_ff").float())
    assert torch.equal(llm.embed_t, llm.embed.t().contiguous())
