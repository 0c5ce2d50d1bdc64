"""Stage-1 projector-step benchmark (BASELINE.json metric: images/sec/node).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config cfg2] [--no-cpu-baseline]

N>1 runs as one process per GPU (RCCL): under `torch.distributed.run` the
launcher's WORLD_SIZE must equal N; without a launcher bench.py starts
`torch.distributed.run --nproc-per-node N` itself as a child process (before
anything touches the GPU) and exits with its status.  Batches are sharded
(bs 32 per GPU, weak scaling) and the projector grads are all-reduced.
A step = SigLIP-L/16-384 fwd + projector fwd/bwd + Gemma3-1B fwd/loss/bwd +
grad all-reduce + clip + AdamW, on synthetic device-resident inputs and
random-init weights of the named architectures (no checkpoints offline).
Rank 0 prints one JSON line.
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

MFMA_BF16_PEAK_TFLOPS = 2500.0   # MI355X dense bf16 (MI355X_MICROARCH.md, chip table)


def _args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="GPUs (one process each); default: the launcher's WORLD_SIZE, else 1")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="cfg2")
    ap.add_argument("--batch", type=int, default=None, help="per-GPU batch (default: the config's)")
    ap.add_argument("--text-len", type=int, default=None, help="text tokens T (default: the config's)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-baseline-only", action="store_true",
                    help="time only the CPU baseline (no GPU) and print it")
    ap.add_argument("--prefetch", action="store_true",
                    help="overlap the next step's SigLIP forward with this step's Gemma3 on a side stream")
    ap.add_argument("--gas", type=int, default=8,
                    help="Stage 2 (cfg4): micro-batches per optimizer step (one bench step = gas micro-batches); "
                         "default 8 = GRAD_ACCUM_STEPS of Stage2/run_vqa_train_stage2.sh and the CLI default "
                         "(train_vqa_stage2.py:106)")
    ap.add_argument("--graph", choices=("auto", "on", "off"), default="off",
                    help="replay each step's SigLIP/projector/Gemma3 launches from a HIP graph (Stage 1); auto = on "
                         "for per-GPU batches <= 4.  Off by default: measured equal at cfg1 (bs 2: 146 vs 147 img/s, "
                         "the kernels themselves, not their launches, set the step time) and at cfg2")
    ap.add_argument("--stage-timers", action="store_true",
                    help="after the timed window, run --steps more steps with the per-stage HIP event timers on "
                         "(libptk stages.cpp) and add their per-step times to the line as stages_ms_per_step")
    ap.add_argument("--launch-check", action="store_true",
                    help="launcher plumbing only: every rank joins a gloo group, rank 0 prints the world; no GPU")
    return ap.parse_args(argv)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _launch_or_check(args, argv):
    """N ranks for --gpus N.  Runs before torch is imported, so no GPU has been touched: a child
    `torch.distributed.run` is started (never exec'd over this process) and its status returned.
    Returns None when this process is itself the (only or launched) rank."""
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is not None:
        if args.gpus is not None and int(env_world) != args.gpus:
            print(f"bench.py: --gpus {args.gpus} but the launcher started WORLD_SIZE={env_world} ranks",
                  file=sys.stderr, flush=True)
            return 2
        return None
    n = 1 if args.gpus is None else args.gpus
    if n < 1:
        print("bench.py: --gpus must be >= 1", file=sys.stderr, flush=True)
        return 2
    if n == 1:
        return None
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + list(argv)
    if "--gpus" not in " ".join(argv):
        cmd += ["--gpus", str(n)]
    return subprocess.call(cmd)


def _launch_check():
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo")
    t = torch.ones(1)
    dist.all_reduce(t)
    if dist.get_rank() == 0:
        print(json.dumps({"launch_check": True, "world": dist.get_world_size(), "ranks_seen": int(t.item()),
                          "local_world": int(os.environ.get("LOCAL_WORLD_SIZE", "1"))}), flush=True)
    dist.destroy_process_group()


def _cpu_info():
    """CPU model, the CPUs this process may run on, and physical cores among them (from /proc/cpuinfo)."""
    model, cores, phys = None, set(), {}
    try:
        cpu = None
        for line in open("/proc/cpuinfo"):
            k, _, v = line.partition(":")
            k, v = k.strip(), v.strip()
            if k == "processor":
                cpu = int(v)
            elif k == "model name" and model is None:
                model = v
            elif k == "physical id":
                phys.setdefault(cpu, [None, None])[0] = v
            elif k == "core id":
                phys.setdefault(cpu, [None, None])[1] = v
    except OSError:
        pass
    aff = sorted(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else list(range(os.cpu_count() or 1))
    for c in aff:
        cores.add(tuple(phys.get(c, (None, c))))
    host_phys = len({tuple(v) for v in phys.values()}) or None
    return {"cpu_model": model, "affinity_cpus": len(aff), "affinity_physical_cores": len(cores),
            "host_physical_cores": host_phys, "host_logical_cpus": os.cpu_count()}


def _cpu_quota():
    """The cgroup CPU bandwidth limit of this process (cgroup v2 cpu.max / v1 cfs quota), in CPUs, or None."""
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        return None if q == "max" else round(int(q) / int(p), 2)
    except (OSError, ValueError):
        pass
    try:
        q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
        p = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
        return None if q <= 0 else round(q / p, 2)
    except (OSError, ValueError):
        return None


def _progress(msg):
    """One line on stderr per CPU-baseline step: the sample runs for minutes without other output."""
    print(f"bench.py: {msg}", file=sys.stderr, flush=True)


def cpu_baseline(cfg_name: str, seconds_budget: float = 45.0, min_steps: int = 3, batch_size: int = 2,
                 all_cores: bool = False, threads_override: int | None = None):
    """The oracle (pure-torch fp32 CPU restatement, pinned to the reference's fixtures) timed on this
    host: one untimed warm-up step, then >= `min_steps` timed steps (median) at the workload's shapes,
    bs 2.  Threads: the physical cores this process may use, capped by OMP_NUM_THREADS (the CPU share
    a GPU job gets on the box)."""
    import numpy as np
    import torch

    from oracle import stage1_ref as R
    from projectiontrainer_amd import weights as W
    from projectiontrainer_amd.config import PRESETS
    info = _cpu_info()
    threads = info["affinity_physical_cores"]
    limit = None
    if all_cores:
        threads = info["host_physical_cores"] or threads   # torch.set_num_threads(n_phys), SURVEY §8(d)
    elif os.environ.get("OMP_NUM_THREADS", "").isdigit() and int(os.environ["OMP_NUM_THREADS"]) < threads:
        # the GPU box gives each GPU job a CPU share and says so through OMP_NUM_THREADS (16 per GPU there);
        # more threads than that share would oversubscribe the cores the job is entitled to
        threads = int(os.environ["OMP_NUM_THREADS"])
        limit = (f"OMP_NUM_THREADS={threads}: the CPU share of this GPU job; the host has "
                 f"{info['affinity_physical_cores']} physical cores in this process's affinity")
    if threads_override:
        threads, limit = threads_override, None
    threads = max(1, threads)
    prev = torch.get_num_threads()
    torch.set_num_threads(threads)
    cfg = PRESETS[cfg_name].replace(batch_size=batch_size)
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
    R.stage1_step(vp, v, lp, t, st, (px, ids, labels), sc)       # warm-up (allocator, MKL init)
    _progress(f"cpu_baseline {cfg_name} {threads} threads: warm-up {time.perf_counter() - t_start:.1f} s")
    while len(times) < min_steps or time.perf_counter() - t_start < seconds_budget * 0.25:
        t0 = time.perf_counter()
        R.stage1_step(vp, v, lp, t, st, (px, ids, labels), sc)
        times.append(time.perf_counter() - t0)
        _progress(f"cpu_baseline {cfg_name} {threads} threads: step {len(times)} {times[-1]:.2f} s")
        if len(times) >= min_steps and time.perf_counter() - t_start > seconds_budget:
            break
    torch.set_num_threads(prev)
    med = float(np.median(times))
    return {"value": round(cfg.batch_size / med, 4), "unit": "images/sec", "cores": threads, "kind": "port",
            "sample": f"oracle/stage1_ref.py fp32 CPU restatement, {cfg_name} shapes at bs {cfg.batch_size} "
                      f"(T={cfg.text_len}): 1 warm-up + {len(times)} timed steps, median {med:.2f} s/step "
                      f"({', '.join(f'{x:.2f}' for x in times)}), {threads} threads",
            "cores_limited_by": limit, "cgroup_cpu_quota": _cpu_quota(), **info}


KERNEL_OF_PATH = {"nt128": "gemm_nt_kernel", "big": "gemm_big_kernel", "big2": "gemm_big2_kernel",
                  "w4": "gemm_w4_kernel", "p8": "gemm_p8_kernel"}


def geglu_label(census, steps):
    """The timed launches as they were dispatched (ptk_gemm_path_counts over the timed steps): the Gemma3
    gate|up projection with the GEGLU epilogue, per kernel family."""
    from projectiontrainer_amd import _lib as L
    per = {p: n for (p, a), n in census.items() if a == L.ACT_GEGLU}
    mix = " + ".join(f"{n // max(steps, 1)} x {KERNEL_OF_PATH.get(p, p)}<ACT_GEGLU>" for p, n in sorted(per.items()))
    return (f"Gemma3 gate|up projection, GEGLU epilogue, per step: {mix} (2*(B*S)*(2I)*H FLOP per launch; the last "
            f"layer's launch on the B*T loss rows, 2*(B*T)*(2I)*H); achieved = summed FLOP / summed event time")


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = _args(argv)
    rc = _launch_or_check(args, argv)
    if rc is not None:
        sys.exit(rc)
    if args.launch_check:
        _launch_check()
        return
    if args.cpu_baseline_only:
        print(json.dumps({"cpu_baseline": {c: cpu_baseline(c) for c in ("cfg1", args.config)}}), flush=True)
        return

    import numpy as np
    import torch
    import torch.distributed as dist

    from projectiontrainer_amd import _lib as L
    from projectiontrainer_amd import weights as W
    from projectiontrainer_amd.config import PRESETS
    from projectiontrainer_amd.flops import flops_per_image, geglu_algo_bytes, geglu_step_flops
    from projectiontrainer_amd.stage1 import Stage1Engine

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
    if args.text_len:
        cfg = cfg.replace(text_len=args.text_len)

    if cfg.question_len > 0:
        line = bench_stage2(args, cfg, world, rank, dev)
        if rank == 0:
            print(json.dumps(line), flush=True)
        if world > 1:
            dist.destroy_process_group()
        return

    eng = Stage1Engine.synthetic(cfg, dev, seed=0, world_size=world, total_steps=10 ** 6,
                                 gradient_accumulation_steps=1)
    px, ids, labels = W.synthetic_batch(cfg, seed=1234 + rank)
    px = torch.from_numpy(px).to(dev)
    ids = torch.from_numpy(ids).to(dev)
    labels = torch.from_numpy(labels).to(dev)

    # --prefetch: every step runs the next step's (frozen) SigLIP forward on a side stream; the timed
    # window then holds exactly K vision forwards (each timed step issues the next one, the last is joined
    # before the final event) and K Gemma3/projector steps.  Off by default: +0.5 % img/s measured, and the
    # overlapped SigLIP kernels share the CUs with the gate|up GEMMs the roofline times (their events read
    # ~35 % longer)
    nxt = px if args.prefetch else None
    graph = args.graph == "on" or (args.graph == "auto" and cfg.batch_size <= 4 and not args.prefetch)
    step = (lambda: eng.graph_step(px, ids, labels)) if graph else \
        (lambda: eng.step(px, ids, labels, next_pixel_values=nxt))
    for w in range(max(args.warmup, 2 if graph else 0)):
        # graph mode: one eager step first (lazy initialisation), then the capture + replays
        eng.step(px, ids, labels, next_pixel_values=nxt) if (w == 0 or not graph) else step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    # events around the gate|up launches only (graph mode: timed in one extra eager step after the window,
    # the replayed launches being the same kernels on the same shapes)
    if not graph:
        L.lib().ptk_gemm_timer_enable((1 << 8) | (1 << L.ACT_GEGLU))
    L.gemm_path_counts(reset=True)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)]
    t_wall = time.perf_counter()
    ev[0].record()
    for k in range(args.steps):
        loss = step()
        if k + 1 == args.steps:
            eng.join_prefetch()
        ev[k + 1].record()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t_wall = time.perf_counter() - t_wall
    if graph:
        L.lib().ptk_gemm_timer_enable((1 << 8) | (1 << L.ACT_GEGLU))
        eng.step(px, ids, labels)
        torch.cuda.synchronize()
    census = L.gemm_path_counts(reset=True)
    elapsed = ev[0].elapsed_time(ev[-1]) / 1e3
    step_ms = [ev[k].elapsed_time(ev[k + 1]) for k in range(args.steps)]
    med_ms = float(np.median(step_ms))
    L.lib().ptk_gemm_timer_enable(0)
    import ctypes
    tot, cnt = ctypes.c_double(), ctypes.c_int()
    L.check(L.lib().ptk_gemm_timer_read(L.ACT_GEGLU, ctypes.byref(tot), ctypes.byref(cnt)), "timer")
    t = torch.tensor([elapsed, med_ms], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)        # slowest rank bounds the job
    elapsed, med_ms = float(t[0]), float(t[1])
    imgs = world * cfg.batch_size * args.steps
    value = imgs / elapsed
    fpi = flops_per_image(cfg)["total"]
    geglu_ms = tot.value / max(cnt.value, 1)
    traffic, traffic_src = None, None
    # the newest profiles/rNN_pmc_traffic_geglu.json (two rocprofv3 --pmc passes, tools/pmc_traffic.py)
    pmcs = sorted(glob.glob(os.path.join(ROOT, "profiles", "r[0-9][0-9]_pmc_traffic_geglu.json")))
    if pmcs and args.config == "cfg2" and cfg.batch_size == 32 and cfg.text_len == 128:
        traffic = json.load(open(pmcs[-1]))["traffic_bytes_per_launch"]
        traffic_src = os.path.relpath(pmcs[-1], ROOT)
    # algorithmic FLOPs of every timed gate|up launch / their summed HIP-event time
    achieved = geglu_step_flops(cfg) * (1 if graph else args.steps) / (tot.value / 1e3) / 1e12
    lm_name = {2560: "Gemma3-4B", 1152: "Gemma3-1B"}.get(cfg.text.hidden_size, f"Gemma3(h{cfg.text.hidden_size})")
    headline = args.config == "cfg2" and cfg.text_len == 128
    metric = ("Stage-1 images/sec/node (SigLIP-L-384 + Gemma3-1B, 576+128 tok)" if headline else
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
        "roofline": {"bound": "mfma", "kernel": geglu_label(census, args.steps),
                     "achieved": round(achieved, 1), "peak": MFMA_BF16_PEAK_TFLOPS, "unit": "TFLOP/s",
                     "frac": round(achieved / MFMA_BF16_PEAK_TFLOPS, 4), "traffic": traffic,
                     "traffic_unit": "bytes/launch (PMC FETCH_SIZEx2 + WRITE_SIZE)", "traffic_src": traffic_src,
                     "traffic_algorithmic": geglu_algo_bytes(cfg),
                     "launches": cnt.value, "avg_ms": round(geglu_ms, 4)},
        "median_ms_per_step": round(med_ms, 3),
        "value_at_median_step": round(world * cfg.batch_size / (med_ms / 1e3), 3),
        "step_mfma_frac": round(value * fpi / (world * MFMA_BF16_PEAK_TFLOPS * 1e12), 4),
        "flop_per_image": fpi, "loss": round(float(loss), 5), "host_wall_s_timed": round(t_wall, 3),
        "hip_graph": graph,
    }
    if world > 1:
        # self-verifying multi-GPU line (outside the timed window): the world the process group sees after init,
        # a rank-sum check through the same collective, the bytes each rank exchanges per step, and the per-step
        # time of the grad exchange from the stage timers over --steps more steps
        chk = torch.ones(1, device=dev)
        dist.all_reduce(chk)
        L.stage_timers_enable(True)
        L.stage_timers_read(reset=True)
        for _ in range(args.steps):
            step()
        eng.join_prefetch()
        torch.cuda.synchronize()
        L.stage_timers_enable(False)
        st = L.stage_timers_read(reset=True)
        gx = torch.tensor([st.get("grad_exchange", (0.0, 0))[0] / args.steps], dtype=torch.float64, device=dev)
        dist.all_reduce(gx, op=dist.ReduceOp.MAX)
        line["exchange"] = {
            "backend": dist.get_backend(), "world_seen": dist.get_world_size(), "rank_sum_check": int(chk.item()),
            "overlapped_rccl": eng.comm is not None,
            "bytes_per_rank_per_step": int(eng.proj.flat_grad.numel() * eng.proj.flat_grad.element_size()),
            "grad_exchange_ms_per_step_max_over_ranks": round(float(gx.item()), 4),
            "note": "fp32 projector grads all-reduced once per step (sum, 1/W folded into clip+AdamW)"}
    if args.stage_timers and not graph:
        # outside the timed window: the event records add host work per stage
        L.stage_timers_enable(True)
        L.stage_timers_read(reset=True)
        for _ in range(args.steps):
            step()
        eng.join_prefetch()
        torch.cuda.synchronize()
        L.stage_timers_enable(False)
        line["stages_ms_per_step"] = {k: round(ms / args.steps, 4)
                                      for k, (ms, n) in L.stage_timers_read(reset=True).items()}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline(args.config)
        cb1 = cpu_baseline("cfg1", seconds_budget=20.0)
        line["cpu_baseline_cfg1"] = {k: cb1[k] for k in ("value", "unit", "cores", "kind", "sample")}
        # thread sweep (SURVEY §8(d) asks for all physical cores): 16 / 32 / 64 / 128 threads up to the host's
        # physical cores, a short sample each; the best is reported with its thread count.  More threads than the
        # job's CPU share (OMP_NUM_THREADS, the cgroup quota) time-slice on that share: OpenMP's barriers then wait
        # on descheduled threads, which is why round 5's 128-thread figure was 4.6x slower than 16 threads
        hp = line["cpu_baseline"].get("host_physical_cores") or 0
        sweep = []
        for n in (16, 32, 64, 128):
            if n > max(hp, 16):
                break
            r = cpu_baseline(args.config, seconds_budget=12.0, min_steps=2, threads_override=n)
            sweep.append({"threads": n, "value": r["value"], "sample": r["sample"]})
        line["cpu_baseline_thread_sweep"] = sweep
        if sweep:
            # the headline sample (OMP_NUM_THREADS threads, the longest) counts as one of the candidates
            main_cb = line["cpu_baseline"]
            best = max(sweep + [{"threads": main_cb["cores"], "value": main_cb["value"], "sample": main_cb["sample"]}],
                       key=lambda r: r["value"])
            line["cpu_baseline_best"] = {"value": best["value"], "unit": "images/sec", "cores": best["threads"],
                                         "kind": "port", "sample": best["sample"],
                                         "cgroup_cpu_quota": line["cpu_baseline"].get("cgroup_cpu_quota")}
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def bench_stage2(args, cfg, world, rank, dev):
    """BASELINE cfg4: Stage-2 VQA fine-tune, Gemma3-1B unfrozen (Stage2/trainer.py:299-444).  One step =
    `--gas` micro-batches (frozen SigLIP + projector forward, Gemma3 forward, manual CE, full backward with
    every weight grad) + the optimizer step (ZeRO-1 reduce-scatter over RCCL for world > 1, clip, bf16
    AdamW, all-gather)."""
    import ctypes

    import numpy as np
    import torch
    import torch.distributed as dist

    from projectiontrainer_amd import _lib as L
    from projectiontrainer_amd import weights as W
    from projectiontrainer_amd.flops import stage2_flops_per_image
    from projectiontrainer_amd.stage2 import synthetic_engine

    eng = synthetic_engine(cfg, dev, seed=0, world_size=world, rank=rank, total_steps=10 ** 6,
                           gradient_accumulation_steps=args.gas, learning_rate=1e-5)
    px, q, a = W.synthetic_vqa_batch(cfg, seed=1234 + rank)
    px, q, a = (torch.from_numpy(t).to(dev) for t in (px, q, a))

    def step():
        for _ in range(args.gas):
            loss = eng.forward_backward(px, q, a)
        eng.optimizer_step()
        return loss

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    L.lib().ptk_gemm_timer_enable((1 << 8) | (1 << L.ACT_GEGLU))
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)]
    ev[0].record()
    for k in range(args.steps):
        loss = step()
        ev[k + 1].record()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = ev[0].elapsed_time(ev[-1]) / 1e3
    med_ms = float(np.median([ev[k].elapsed_time(ev[k + 1]) for k in range(args.steps)]))
    L.lib().ptk_gemm_timer_enable(0)
    tot, cnt = ctypes.c_double(), ctypes.c_int()
    L.check(L.lib().ptk_gemm_timer_read(L.ACT_GEGLU, ctypes.byref(tot), ctypes.byref(cnt)), "timer")
    t = torch.tensor([elapsed, med_ms], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed, med_ms = float(t[0]), float(t[1])
    imgs = world * cfg.batch_size * args.gas * args.steps
    value = imgs / elapsed
    fpi = stage2_flops_per_image(cfg)["total"]
    # gate|up launches per micro-batch: layers 0..L-2 on all B*S rows, the last on the B*Ta answer rows
    tc = cfg.text
    ta = cfg.text_len - cfg.question_len
    gu = 2.0 * 2 * tc.intermediate_size * tc.hidden_size * cfg.batch_size * (cfg.seq_len * (tc.num_hidden_layers - 1) + ta)
    achieved = gu * args.gas * args.steps / (tot.value / 1e3) / 1e12
    return {
        "metric": "Stage-2 VQA fine-tune images/sec/node (SigLIP-L-384 + Gemma3-1B unfrozen, 576+64+256 tok)",
        "value": round(value, 3), "unit": "images/sec", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "bf16", "data": "synthetic",
        "config": {"workload": f"{args.config}: Stage 2 VQA, SigLIP-ViT-L/16-384 + projector frozen fwd, Gemma3-1B "
                               f"fwd + full bwd (all weight grads) + ZeRO-1 bf16 AdamW, {cfg.num_vision_tokens} vis + "
                               f"{cfg.question_len} Q + {ta} A tokens, gas {args.gas}",
                   "global_batch": world * cfg.batch_size * args.gas, "per_gpu_batch": cfg.batch_size,
                   "seq_len": cfg.seq_len, "parallelism": f"dp{world}-zero1"},
        "roofline": {"bound": "mfma", "kernel": "gemm_w4_kernel<ACT_GEGLU> (Gemma3 gate|up projection)",
                     "achieved": round(achieved, 1), "peak": MFMA_BF16_PEAK_TFLOPS, "unit": "TFLOP/s",
                     "frac": round(achieved / MFMA_BF16_PEAK_TFLOPS, 4), "traffic": None,
                     "launches": cnt.value, "avg_ms": round(tot.value / max(cnt.value, 1), 4)},
        "median_ms_per_step": round(med_ms, 3),
        "step_mfma_frac": round(value * fpi / (world * MFMA_BF16_PEAK_TFLOPS * 1e12), 4),
        "flop_per_image": fpi, "loss": round(float(loss), 5),
    }


if __name__ == "__main__":
    main()
