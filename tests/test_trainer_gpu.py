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
            key, sr, sc = G.sub_key(d, f"s{last}_param.{k}")
            ref, g = d[key], G.sub_sample(got, sr, sc)
        assert np.max(np.abs(g - ref)) <= 2.5 * lr_sum + 1e-6, k
        assert np.median(np.abs(g - ref)) <= 0.05 * meta["lr"], k


def test_trainer_on_decoding_dataset_matches_pixel_dataset(gpu, tmp_path):
    """The reference's data contract end to end: JPEG files + JSON through data.XrayTextPairDataset
    (2 decode workers, GPU resize/normalise) train exactly like a dataset that yields the pixel_values
    the reference's __getitem__ makes (Pillow resize + SiglipImageProcessor, fp32)."""
    from PIL import Image
    import transformers
    from projectiontrainer_amd.data import XrayTextPairDataset
    from projectiontrainer_amd.dist import DistState
    from projectiontrainer_amd.projector_trainer import ProjectionTrainerStage1
    from projectiontrainer_amd.projectors import MLPProjector
    name = "tiny"
    d, meta = G.load(name)
    cfg, sig, llm, pp = hf_models(name)
    S, T = cfg.vision.image_size, cfg.text_len
    rng = np.random.default_rng(0)
    samples = []
    for i in range(2 * cfg.batch_size):
        h, w = int(rng.integers(S // 2, 4 * S)), int(rng.integers(S // 2, 4 * S))
        im = rng.integers(0, 256, (h, w) if i % 2 else (h, w, 3), dtype=np.uint8)
        Image.fromarray(im, "L" if i % 2 else "RGB").save(tmp_path / f"{i}.jpg", quality=90)
        samples.append({"image": f"{i}.jpg", "normal_caption": f"finding {i} " * (1 + i % 5)})
    (tmp_path / "s.json").write_text(json.dumps(samples))

    class Tok:
        pad_token_id, eos_token_id = 0, 1

        def __call__(self, text, max_length, padding, truncation, return_tensors):
            ids = [2] + [3 + (ord(ch) % 200) for ch in text][: max_length - 1]
            return types.SimpleNamespace(input_ids=torch.tensor([[0] * (max_length - len(ids)) + ids]))

    proc = transformers.SiglipImageProcessor(size={"height": S, "width": S})
    ds = XrayTextPairDataset(str(tmp_path), str(tmp_path / "s.json"), proc, Tok(), S, max_length=T)
    ref_items = []
    for i, s in enumerate(samples):
        image = Image.open(tmp_path / s["image"]).convert("RGB").resize((S, S))
        px = torch.from_numpy(proc(images=image, return_tensors="np")["pixel_values"][0])
        ids, labels = ds.tokenize(s["normal_caption"])
        ref_items.append({"pixel_values": px, "token_ids": ids, "labels": labels})

    def run(data, out):
        proj = MLPProjector(cfg.vision.hidden_size, cfg.text.hidden_size)
        proj.load_state_dict({k: torch.from_numpy(v) for k, v in pp.items()})
        logs = []
        tr = ProjectionTrainerStage1(DistState(1), sig, llm, proj, proc, Tok(), data, None, output_dir=str(out),
                                     batch_size=cfg.batch_size, learning_rate=1e-3, num_epochs=1,
                                     log_fn=lambda dd, s: logs.append(dd))
        tr.train()
        return [x["train/batch_loss"] for x in logs if "train/batch_loss" in x], tr.projection_layer

    l_img, p_img = run(ds, tmp_path / "o1")
    l_ref, p_ref = run(ref_items, tmp_path / "o2")
    assert len(l_img) == len(l_ref) == 2
    assert l_img == l_ref, (l_img, l_ref)
    for a, b in zip(p_img.state_dict().values(), p_ref.state_dict().values()):
        assert torch.equal(a, b)
