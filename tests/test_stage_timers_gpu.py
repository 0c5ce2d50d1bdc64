"""Per-stage HIP event timers (stages.cpp, SURVEY §5 tracing: "per-stage HIP event timers behind an env flag").

The timers only add event records: a step with them on must give bit-identical results, report every stage of
the Stage-1 step with the expected span counts, and record nothing while a HIP graph is being captured."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _engine(gpu):
    from projectiontrainer_amd.config import PRESETS
    from projectiontrainer_amd.stage1 import Stage1Engine
    from projectiontrainer_amd import weights as W
    cfg = PRESETS["cfg1"]
    cfg = cfg.replace(vision=cfg.vision.__class__(**{**cfg.vision.__dict__, "num_hidden_layers": 2}),
                      text=cfg.text.__class__(**{**cfg.text.__dict__, "num_hidden_layers": 3}))
    eng = Stage1Engine.synthetic(cfg, gpu, seed=0, total_steps=10)
    px, ids, labels = W.synthetic_batch(cfg, seed=5)
    return cfg, eng, [torch.from_numpy(t).to(gpu) for t in (px, ids, labels)]


def test_stage_timers_report_and_change_nothing(gpu):
    from projectiontrainer_amd import _lib as L
    cfg, e0, args = _engine(gpu)
    _, e1, _ = _engine(gpu)
    L.stage_timers_enable(False)
    l0 = e0.step(*args).clone()
    torch.cuda.synchronize()
    L.stage_timers_enable(True)
    try:
        L.stage_timers_read(reset=True)
        l1 = e1.step(*args).clone()
        torch.cuda.synchronize()
        rep = L.stage_timers_read(reset=True)
    finally:
        L.stage_timers_enable(False)
    assert torch.equal(l0, l1)
    assert torch.equal(e0.proj.flat, e1.proj.flat)
    assert torch.equal(e0.exp_avg_sq, e1.exp_avg_sq)
    nv, nl = cfg.vision.num_hidden_layers, cfg.text.num_hidden_layers
    want = {"vision": 1, "siglip.fwd": 1, "siglip.embed": 1, "siglip.attn": nv, "siglip.flash": nv,
            "siglip.mlp": nv, "siglip.post_norm": 1, "projector.fwd": 1, "llm": 1, "gemma.embed": 1,
            "gemma.fwd.attn": nl, "gemma.fwd.flash": nl, "gemma.fwd.mlp": nl, "gemma.lm_head_ce": 1,
            "gemma.lm_head_bwd": 1, "gemma.bwd.mlp": nl, "gemma.bwd.attn": nl, "gemma.bwd.flash": nl,
            "projector.bwd": 1, "optimizer": 1}
    assert {k: n for k, (ms, n) in rep.items()} == want
    assert all(ms > 0 for ms, n in rep.values())
    # the Gemma3 pieces are consecutive spans inside the "llm" span (event resolution slack only)
    parts = sum(rep[k][0] for k in rep if k.startswith("gemma.") and "flash" not in k)
    assert parts <= rep["llm"][0] * 1.02 + 0.05
    assert rep["gemma.fwd.flash"][0] < rep["gemma.fwd.attn"][0]
    # nothing is left behind: a second read is empty
    assert L.stage_timers_read(reset=True) == {}


def test_stage_timers_skip_graph_capture(gpu):
    from projectiontrainer_amd import _lib as L
    _, eng, args = _engine(gpu)
    eng.step(*args)
    torch.cuda.synchronize()
    L.stage_timers_enable(True)
    try:
        L.stage_timers_read(reset=True)
        eng.graph_step(*args)      # capture: the model's spans record nothing; replay runs no host code
        torch.cuda.synchronize()
        rep = L.stage_timers_read(reset=True)
    finally:
        L.stage_timers_enable(False)
    assert "siglip.fwd" not in rep and "gemma.fwd.attn" not in rep
    assert rep.get("optimizer", (0, 0))[1] == 1       # optimizer_step runs eagerly after the replay
