"""Load golden fixtures written by tests/golden/make_golden.py and compare."""
import ast
import os

import numpy as np
import torch

from projectiontrainer_amd.config import PRESETS
from projectiontrainer_amd import weights as W

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name):
    d = np.load(os.path.join(GOLDEN, f"{name}.npz"), allow_pickle=False)
    meta = ast.literal_eval(str(d["meta"]))
    return d, meta


def bf16_round(a):
    """float32 array rounded to the nearest bf16 value (RNE), as `.to(torch.bfloat16)` does."""
    return torch.from_numpy(np.ascontiguousarray(a)).to(torch.bfloat16).float().numpy()


def params_for(name):
    """Config and the deterministic weights the fixture was made with.  A bf16 fixture's towers were cast
    to bf16 by the reference's loader (train_projection_stage1.py:169-183,204-210): their weights are
    returned bf16-rounded; the projector stays fp32 (it is built in fp32, :252)."""
    base = name.replace("_bf16", "")
    cfg = PRESETS[base]
    vp = W.siglip_vision_params(cfg.vision)
    lp = W.gemma3_params(cfg.text)
    pp = W.projector_params(cfg.vision.hidden_size, cfg.text.hidden_size, cfg.expansion_factor)
    if name.endswith("_bf16"):
        vp = {k: bf16_round(v) for k, v in vp.items()}
        lp = {k: bf16_round(v) for k, v in lp.items()}
    return cfg, vp, lp, pp


def fingerprint(vp, lp, pp):
    return np.array([float(np.sum(v.astype(np.float64))) for d in (vp, lp, pp) for v in d.values()])


def batch(d, s):
    """(pixel_values, token_ids, labels) of step s as the reference's loader produced them; large pixel
    batches are regenerated from the fixture's seed in the recorded sample order."""
    ids = d[f"s{s}_token_ids"]
    if f"s{s}_pixel_values" in d.files:
        px = d[f"s{s}_pixel_values"]
    else:
        meta = ast.literal_eval(str(d["meta"]))
        cfg = PRESETS[meta["name"].replace("_bf16", "")]
        px = W.synthetic_batch(cfg, seed=meta["seed_batch"])[0][d[f"s{s}_order"]]
        if meta.get("precision") == "bf16":
            px = bf16_round(px)
    return px, ids, np.where(ids == 0, -100, ids)


def sub_key(d, key):
    """(stored key, row stride, column stride) of a compacted fixture entry."""
    if key + "@rows16" in d.files:
        return key + "@rows16", 16, 1
    for f in d.files:
        if f.startswith(key + "@sub"):
            sr, sc = f[len(key) + 4:].split("x")
            return f, int(sr), int(sc)
    raise KeyError(key)


def sub_sample(a, sr, sc):
    a = np.asarray(a)
    return a.reshape(-1, a.shape[-1])[::sr, ::sc]


def check_tensor(d, key, got, rtol, atol):
    """Compare `got` (full tensor) with a fixture entry stored whole or compacted."""
    got = np.asarray(got.detach().cpu().double() if torch.is_tensor(got) else got, dtype=np.float64)
    if key in d.files:
        np.testing.assert_allclose(got, d[key], rtol=rtol, atol=atol, err_msg=key)
        return
    k, sr, sc = sub_key(d, key)
    np.testing.assert_allclose(sub_sample(got, sr, sc), d[k], rtol=rtol, atol=atol, err_msg=key)
    np.testing.assert_allclose(np.linalg.norm(got), float(d[key + "@norm"]), rtol=max(rtol, 1e-6), err_msg=key)
    np.testing.assert_allclose(got.sum(), float(d[key + "@sum"]), rtol=max(rtol, 1e-4),
                               atol=atol * np.sqrt(got.size), err_msg=key)
