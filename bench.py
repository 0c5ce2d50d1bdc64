"""Stage-1 projector-step benchmark (BASELINE.json metric: images/sec/node).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config cfg2] [--no-cpu-baseline]

N>1 runs as one process per GPU under torch.distributed.run (RCCL); batches are
sharded (bs 32 per GPU, weak scaling) and the projector grads are all-reduced.
A step = SigLIP-L/16-384 fwd + projector fwd/bwd + Gemma3-1B fwd/loss/bwd +
grad all-reduce + clip + AdamW, on synthetic device-resident inputs and
random-init weights of the named architectures (no checkpoints offline).
Rank 0 prints one JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from projectiontrainer_amd import _lib as L  # noqa: E402
from projectiontrainer_amd import weights as W  # noqa: E402
from projectiontrainer_amd.config import PRESETS  # noqa: E402
from projectiontrainer_amd.flops import flops_per_image, geglu_step_flops  # noqa: E402
from projectiontrainer_amd.stage1 import Stage1Engine  # noqa: E402

MFMA_BF16_PEAK_TFLOPS = 2500.0   # MI355X dense bf16 (MI355X_MICROARCH.md, chip table)


def cpu_baseline(cfg_name: str, seconds_budget: float = 30.0):
    """The oracle (pure-torch fp32 CPU restatement, pinned to the reference's
    fixtures) timed on this host: one step at the workload's shapes, bs 2."""
    from oracle import stage1_ref as R
    cfg = PRESETS[cfg_name].replace(batch_size=2)
    g = torch.Generator().manual_seed(0)
    rn = lambda *s, std=0.02: torch.randn(*s, generator=g) * std
    v, t = cfg.vision, cfg.text
    D, I = v.hidden_size, v.intermediate_size
    vp = {"vision_model.embeddings.patch_embedding.weight": rn(D, 3, v.patch_size, v.patch_size),
          "vision_model.embeddings.patch_embedding.bias": torch.zeros(D),
          "vision_model.embeddings.position_embedding.weight": rn(v.num_patches, D),
          "vision_model.post_layernorm.weight": torch.ones(D), "vision_model.post_layernorm.bias": torch.zeros(D)}
    for i in range(v.num_hidden_layers):
        p = f"vision_model.encoder.layers.{i}."
        for n in ("q", "k", "v", "out"):
            vp[p + f"self_attn.{n}_proj.weight"], vp[p + f"self_attn.{n}_proj.bias"] = rn(D, D), torch.zeros(D)
        vp[p + "mlp.fc1.weight"], vp[p + "mlp.fc1.bias"] = rn(I, D), torch.zeros(I)
        vp[p + "mlp.fc2.weight"], vp[p + "mlp.fc2.bias"] = rn(D, I), torch.zeros(D)
        for n in ("layer_norm1", "layer_norm2"):
            vp[p + n + ".weight"], vp[p + n + ".bias"] = torch.ones(D), torch.zeros(D)
    H, It = t.hidden_size, t.intermediate_size
    lp = {"model.embed_tokens.weight": rn(t.vocab_size, H), "model.norm.weight": torch.zeros(H)}
    for i in range(t.num_hidden_layers):
        p = f"model.layers.{i}."
        lp[p + "self_attn.q_proj.weight"] = rn(t.q_dim, H)
        lp[p + "self_attn.k_proj.weight"] = rn(t.kv_dim, H)
        lp[p + "self_attn.v_proj.weight"] = rn(t.kv_dim, H)
        lp[p + "self_attn.o_proj.weight"] = rn(H, t.q_dim)
        lp[p + "self_attn.q_norm.weight"] = torch.zeros(t.head_dim)
        lp[p + "self_attn.k_norm.weight"] = torch.zeros(t.head_dim)
        lp[p + "mlp.gate_proj.weight"], lp[p + "mlp.up_proj.weight"] = rn(It, H), rn(It, H)
        lp[p + "mlp.down_proj.weight"] = rn(H, It)
        for n in ("input_layernorm", "post_attention_layernorm", "pre_feedforward_layernorm",
                  "post_feedforward_layernorm"):
            lp[p + n + ".weight"] = torch.zeros(H)
    pp = W.projector_params(D, H, cfg.expansion_factor)
    px, ids, labels = W.synthetic_batch(cfg, seed=99)
    st = R.init_state(pp)
    sc = R.StepConfig(gradient_accumulation_steps=1)
    times = []
    t_start = time.perf_counter()
    while True:
        t0 = time.perf_counter()
        R.stage1_step(vp, v, lp, t, st, (px, ids, labels), sc)
        times.append(time.perf_counter() - t0)
        if len(times) >= 2 or time.perf_counter() - t_start > seconds_budget:
            break
    dt = times[-1] if len(times) > 1 else times[0]
    return {"value": round(cfg.batch_size / dt, 4), "unit": "images/sec", "cores": torch.get_num_threads(),
            "kind": "port",
            "sample": f"oracle/stage1_ref.py fp32 CPU restatement, {cfg_name} shapes at bs 2 "
                      f"(T={cfg.text_len}), {len(times)} step(s), last timed: {dt:.2f} s/step"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="cfg2")
    ap.add_argument("--batch", type=int, default=None, help="per-GPU batch (default: the config's)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--prefetch", action="store_true",
                    help="overlap the next step's SigLIP forward with this step's Gemma3 on a side stream")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)
    cfg = PRESETS[args.config]
    if args.batch:
        cfg = cfg.replace(batch_size=args.batch)

    eng = Stage1Engine.synthetic(cfg, dev, seed=0, world_size=world, total_steps=10 ** 6,
                                 gradient_accumulation_steps=1)
    px, ids, labels = W.synthetic_batch(cfg, seed=1234 + rank)
    px = torch.from_numpy(px).to(dev)
    ids = torch.from_numpy(ids).to(dev)
    labels = torch.from_numpy(labels).to(dev)

    # --prefetch: every step runs the next step's (frozen) SigLIP forward on a side stream; the timed
    # window then holds exactly K vision forwards (each timed step issues the next one, the last is joined
    # before e1) and K Gemma3/projector steps.  Off by default: +0.5 % img/s measured, and the overlapped
    # SigLIP kernels share the CUs with the gate|up GEMMs the roofline times (their events read ~35 % longer)
    nxt = px if args.prefetch else None
    for _ in range(args.warmup):
        eng.step(px, ids, labels, next_pixel_values=nxt)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    L.lib().ptk_gemm_timer_enable((1 << 8) | (1 << L.ACT_GEGLU))   # events around the gate|up launches only
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(args.steps):
        loss = eng.step(px, ids, labels, next_pixel_values=nxt)
    eng.join_prefetch()
    e1.record()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = e0.elapsed_time(e1) / 1e3
    L.lib().ptk_gemm_timer_enable(0)
    import ctypes
    tot, cnt = ctypes.c_double(), ctypes.c_int()
    L.check(L.lib().ptk_gemm_timer_read(L.ACT_GEGLU, ctypes.byref(tot), ctypes.byref(cnt)), "timer")
    t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t)
    imgs = world * cfg.batch_size * args.steps
    value = imgs / elapsed
    fpi = flops_per_image(cfg)["total"]
    geglu_ms = tot.value / max(cnt.value, 1)
    traffic = None
    pmc = os.path.join(ROOT, "profiles", "r01_pmc_traffic_geglu.json")
    if os.path.exists(pmc) and args.config == "cfg2" and cfg.batch_size == 32:
        traffic = json.load(open(pmc))["traffic_bytes_per_launch"]   # rocprofv3 --pmc passes (tools/pmc_traffic.py)
    # algorithmic FLOPs of every timed gate|up launch / their summed HIP-event time
    achieved = geglu_step_flops(cfg) * args.steps / (tot.value / 1e3) / 1e12
    lm_name = {2560: "Gemma3-4B", 1152: "Gemma3-1B"}.get(cfg.text.hidden_size, f"Gemma3(h{cfg.text.hidden_size})")
    metric = ("Stage-1 images/sec/node (SigLIP-L-384 + Gemma3-1B, 576+128 tok)" if args.config == "cfg2" else
              f"Stage-1 images/sec/node ({args.config}: SigLIP + {lm_name}, {cfg.vision.num_patches}+{cfg.text_len} tok)")
    line = {
        "metric": metric,
        "value": round(value, 3), "unit": "images/sec", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "bf16", "data": "synthetic",
        "config": {"workload": f"{args.config}: SigLIP-ViT-L/16-384 frozen fwd + MLP projector fwd/bwd + "
                               f"{lm_name} frozen fwd/bwd, {cfg.num_vision_tokens} vis + {cfg.text_len} text tokens",
                   "global_batch": world * cfg.batch_size, "per_gpu_batch": cfg.batch_size,
                   "seq_len": cfg.seq_len, "parallelism": f"dp{world}"},
        "roofline": {"bound": "mfma", "kernel": "gemm_w4_kernel<ACT_GEGLU> (Gemma3 gate|up projection: 2*(B*S)*(2I)*H FLOP per launch, "
                               "last layer 2*(B*T)*(2I)*H)",
                     "achieved": round(achieved, 1), "peak": MFMA_BF16_PEAK_TFLOPS, "unit": "TFLOP/s",
                     "frac": round(achieved / MFMA_BF16_PEAK_TFLOPS, 4), "traffic": traffic,
                     "traffic_unit": "bytes/launch (PMC FETCH_SIZEx2 + WRITE_SIZE)",
                     "launches": cnt.value, "avg_ms": round(geglu_ms, 4)},
        "step_mfma_frac": round(value * fpi / (world * MFMA_BF16_PEAK_TFLOPS * 1e12), 4),
        "flop_per_image": fpi, "loss": round(float(loss), 5),
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline(args.config)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
