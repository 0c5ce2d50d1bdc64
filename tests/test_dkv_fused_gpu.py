"""The split-slab dK/dV partials summed inside qknorm_rope_bwd (default) must give bit-identical results
to the separate attn_dkv_reduce_kernel pass (PTK_DKV_REDUCE_SPLIT=1): same piece order, same rounding."""
import os
import subprocess
import sys

import pytest
import torch

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.mark.gpu
def test_dkv_reduce_fused_is_bit_identical(tmp_path):
    outs = []
    for split in ("0", "1"):
        p = tmp_path / f"dkv_{split}.pt"
        env = dict(os.environ, PTK_DKV_REDUCE_SPLIT=split)
        subprocess.run([sys.executable, os.path.join(HERE, "dkv_fused_worker.py"), str(p)], env=env, check=True,
                       timeout=110)
        outs.append(torch.load(p, weights_only=True))
    a, b = outs
    assert torch.equal(a["loss"], b["loss"])
    assert torch.equal(a["dx"], b["dx"])
    for ga, gb in zip(a["grads"], b["grads"]):
        assert torch.equal(ga, gb)
