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


def params_for(name):
    cfg = PRESETS[name]
    vp = W.siglip_vision_params(cfg.vision)
    lp = W.gemma3_params(cfg.text)
    pp = W.projector_params(cfg.vision.hidden_size, cfg.text.hidden_size, cfg.expansion_factor)
    return cfg, vp, lp, pp


def fingerprint(vp, lp, pp):
    return np.array([float(np.sum(v.astype(np.float64))) for d in (vp, lp, pp) for v in d.values()])


def batch(d, s):
    return (d[f"s{s}_pixel_values"], d[f"s{s}_token_ids"],
            np.where(d[f"s{s}_token_ids"] == 0, -100, d[f"s{s}_token_ids"]))


def check_tensor(d, key, got, rtol, atol):
    """Compare `got` (full tensor) with a fixture entry stored whole or compacted."""
    got = np.asarray(got.detach().cpu().double() if torch.is_tensor(got) else got, dtype=np.float64)
    if key in d.files:
        np.testing.assert_allclose(got, d[key], rtol=rtol, atol=atol, err_msg=key)
        return
    np.testing.assert_allclose(got[::16], d[key + "@rows16"], rtol=rtol, atol=atol, err_msg=key)
    np.testing.assert_allclose(np.linalg.norm(got), float(d[key + "@norm"]), rtol=max(rtol, 1e-6), err_msg=key)
    np.testing.assert_allclose(got.sum(), float(d[key + "@sum"]), rtol=max(rtol, 1e-4),
                               atol=atol * np.sqrt(got.size), err_msg=key)
