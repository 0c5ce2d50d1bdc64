"""Stage1Engine.graph_step (forward_backward replayed from a HIP graph) against step() (eager launches):
same kernels in the same order, so loss, projector grads and post-AdamW parameters must be bit-identical
over several steps with a new batch each step (the graph reads its inputs from static buffers)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _engine(cfg, dev):
    from projectiontrainer_amd import weights as W
    from projectiontrainer_amd.gemma3 import Gemma3CausalLM
    from projectiontrainer_amd.projectors import MLPProjector
    from projectiontrainer_amd.siglip import SiglipVisionTower
    from projectiontrainer_amd.stage1 import Stage1Engine
    vp, lp = W.siglip_vision_params(cfg.vision), W.gemma3_params(cfg.text)
    pp = W.projector_params(cfg.vision.hidden_size, cfg.text.hidden_size)
    proj = MLPProjector(cfg.vision.hidden_size, cfg.text.hidden_size)
    proj.load_state_dict({k: torch.from_numpy(v) for k, v in pp.items()})
    proj.to(dev)
    return Stage1Engine(SiglipVisionTower(cfg.vision, vp, dev),
                        Gemma3CausalLM(cfg.text, lp, dev, max_pos=Gemma3CausalLM.seq_pad(cfg.seq_len)), proj,
                        total_steps=100)


@pytest.mark.parametrize("preset", ["tiny", "tiny_gqa"])
def test_graph_step_bit_identical_to_eager(gpu, preset):
    from projectiontrainer_amd import weights as W
    from projectiontrainer_amd.config import PRESETS
    cfg = PRESETS[preset]
    batches = []
    for seed in range(4):
        px, ids, labels = W.synthetic_batch(cfg, seed=20 + seed)
        batches.append(tuple(torch.from_numpy(a).to(gpu) for a in (px, ids, labels)))
    eager, graphed = _engine(cfg, gpu), _engine(cfg, gpu)
    for k, b in enumerate(batches):
        le = float(eager.step(*b))
        lg = float(graphed.step(*b) if k == 0 else graphed.graph_step(*b))   # one eager step before capture
        torch.cuda.synchronize()
        assert le == lg, (k, le, lg)
        assert torch.equal(eager.proj.flat_grad, graphed.proj.flat_grad), k
        assert torch.equal(eager.proj.flat, graphed.proj.flat), k
    assert graphed._graph is not None


def test_graph_step_recaptures_after_reallocation(gpu):
    """A graph captured at bs 2 must not be replayed after an eager step at bs 4 reallocated the step
    buffers and workspaces (the captured pointers are freed): graph_step recaptures, and the sequence
    graph(bs 2) -> eager(bs 4) -> graph(bs 2) stays bit-identical to the all-eager sequence."""
    from projectiontrainer_amd import weights as W
    from projectiontrainer_amd.config import PRESETS
    cfg2, cfg4 = PRESETS["tiny"].replace(batch_size=2), PRESETS["tiny"].replace(batch_size=4)
    b2 = [tuple(torch.from_numpy(a).to(gpu) for a in W.synthetic_batch(cfg2, seed=40 + s)) for s in range(3)]
    b4 = tuple(torch.from_numpy(a).to(gpu) for a in W.synthetic_batch(cfg4, seed=50))
    eager, graphed = _engine(cfg2, gpu), _engine(cfg2, gpu)
    seq = [("e", b2[0]), ("g", b2[1]), ("e", b4), ("g", b2[2]), ("g", b2[0])]
    keys = []
    for mode, b in seq:
        le = float(eager.step(*b))
        lg = float(graphed.step(*b) if mode == "e" else graphed.graph_step(*b))
        torch.cuda.synchronize()
        assert le == lg, (mode, le, lg)
        assert torch.equal(eager.proj.flat, graphed.proj.flat)
        keys.append(graphed._graph_key)
    assert keys[1] is not None and keys[3] != keys[1], "bs-4 reallocation did not force a recapture"
    assert keys[4] == keys[3]


def test_graph_step_recapture_after_destroy_stays_bit_identical(gpu):
    """A forced re-capture destroys the replaced graph (graph_step keeps no retired graphs); the new graph's
    later replays must stay bit-identical to eager.  This is the sequence that gave NaN grads while the captured
    step held hipMemsetAsync nodes (tools/graph_debug.py V1/V7, profiles/r04_graph_memset_ab.txt)."""
    import gc
    from projectiontrainer_amd import weights as W
    from projectiontrainer_amd.config import PRESETS
    cfg = PRESETS["tiny"].replace(batch_size=2)
    b = [tuple(torch.from_numpy(a).to(gpu) for a in W.synthetic_batch(cfg, seed=60 + s)) for s in range(5)]
    eager, graphed = _engine(cfg, gpu), _engine(cfg, gpu)
    for k, (mode, x) in enumerate([("e", b[0]), ("g", b[1]), ("new", b[2]), ("g", b[3]), ("g", b[4])]):
        if mode == "new":              # force a re-capture: the old graph is dropped and destroyed
            graphed._graph_key = None
            gc.collect()
        le = float(eager.step(*x))
        lg = float(graphed.step(*x) if mode == "e" else graphed.graph_step(*x))
        torch.cuda.synchronize()
        assert le == lg, (k, le, lg)
        assert torch.equal(eager.proj.flat_grad, graphed.proj.flat_grad), k
