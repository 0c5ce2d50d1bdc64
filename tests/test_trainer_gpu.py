"""Drop-in test of the reference trainer API: HF SiglipModel / Gemma3ForCausalLM
instances and a projector go into ProjectionTrainerStage1 exactly as
Stage1/train_projection_stage1.py:338-356 passes them; two epochs of the
golden dataset must reproduce the reference's projector after two steps, and
the checkpoint files must be loadable like the reference's
(torch.load(weights_only=True) -> MLPProjector.load_state_dict)."""
import json
import os
import tempfile
import types

import numpy as np
import pytest
import torch

from tests import golden_util as G

pytestmark = pytest.mark.gpu


def hf_models(name):
    from transformers import Gemma3ForCausalLM, Gemma3TextConfig, SiglipConfig, SiglipModel
    from projectiontrainer_amd.config import to_hf_dicts
    cfg, vp, lp, pp = G.params_for(name)
    vis_kw, txt_kw = to_hf_dicts(cfg)
    sig = SiglipModel(SiglipConfig(
        text_config=dict(vocab_size=64, hidden_size=64, intermediate_size=128, num_hidden_layers=1,
                         num_attention_heads=1, max_position_embeddings=16, bos_token_id=None,
                         eos_token_id=None, pad_token_id=None),
        vision_config=vis_kw)).float()
    sig.load_state_dict({k: torch.from_numpy(v) for k, v in vp.items()}, strict=False)
    llm = Gemma3ForCausalLM(Gemma3TextConfig(**txt_kw)).float()
    llm.load_state_dict({k: torch.from_numpy(v) for k, v in lp.items()}, strict=False)
    return cfg, sig, llm, pp


def test_trainer_with_hf_models_matches_reference(gpu):
    from projectiontrainer_amd.dist import DistState
    from projectiontrainer_amd.projector_trainer import ProjectionTrainerStage1
    from projectiontrainer_amd.projectors import MLPProjector
    name = "tiny"
    d, meta = G.load(name)
    cfg, sig, llm, pp = hf_models(name)
    proj = MLPProjector(cfg.vision.hidden_size, cfg.text.hidden_size)
    proj.load_state_dict({k: torch.from_numpy(v) for k, v in pp.items()})
    px, ids, labels = G.batch(d, 0)
    data = [{"pixel_values": torch.from_numpy(px[i]), "token_ids": torch.from_numpy(ids[i]),
             "labels": torch.from_numpy(labels[i])} for i in range(cfg.batch_size)]
    tok = types.SimpleNamespace(pad_token_id=0, eos_token_id=1)
    logs = []
    with tempfile.TemporaryDirectory() as out:
        tr = ProjectionTrainerStage1(DistState(meta["gas"]), sig, llm, proj, None, tok, data, None,
                                     output_dir=out, batch_size=cfg.batch_size, learning_rate=meta["lr"],
                                     num_epochs=meta["num_epochs"], gradient_accumulation_steps=meta["gas"],
                                     log_fn=lambda dd, s: logs.append(dd))
        assert tr.max_train_steps == meta["max_train_steps"]
        tr.train()
        files = sorted(os.listdir(out))
        assert "projector_config.json" in files and f"projector_epoch_{meta['num_epochs']}.bin" in files
        sd = torch.load(os.path.join(out, f"projector_epoch_{meta['num_epochs']}.bin"), weights_only=True)
        conf = json.load(open(os.path.join(out, "projector_config.json")))
    assert conf == {"vision_dim": cfg.vision.hidden_size, "llm_dim": cfg.text.hidden_size}
    assert list(sd) == ["model.0.weight", "model.0.bias", "model.2.weight", "model.2.bias"]
    fresh = MLPProjector(cfg.vision.hidden_size, cfg.text.hidden_size)
    fresh.load_state_dict(sd)
    losses = [x["train/batch_loss"] for x in logs if "train/batch_loss" in x]
    for s in range(meta["steps"]):
        assert abs(losses[s] - float(d[f"s{s}_loss"])) <= 2e-2
    last = meta["steps"] - 1
    lr_sum = sum(float(d[f"s{s}_lr"]) for s in range(meta["steps"]))
    for k in sd:
        got = sd[k].double().numpy()
        if f"s{last}_param.{k}" in d.files:
            ref, g = d[f"s{last}_param.{k}"], got
        else:
            ref, g = d[f"s{last}_param.{k}@rows16"], got[::16]
        assert np.max(np.abs(g - ref)) <= 2.5 * lr_sum + 1e-6, k
        assert np.median(np.abs(g - ref)) <= 0.05 * meta["lr"], k
