"""Persistent 4-wave (mode 8) vs persistent 8-wave (mode 32) vs two-group (mode 64) vs the automatic dispatch (mode 0) on the GEMM
shapes of the cfg2 / cfg4 steps: HIP-event time per launch, TFLOP/s, rounds interleaved (one process)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from projectiontrainer_amd import kernels as K, _lib as L  # noqa: E402

dev = torch.device("cuda:0")
M1, M2, MS = 32 * 704, 16 * 896, 32 * 576
SHAPES = [  # name, M, N, K, act, out dtype
    ("g_gu_geglu", M1, 13824, 1152, L.ACT_GEGLU, torch.bfloat16),
    ("g_dh_geglu_bwd", M1, 6912, 1152, L.ACT_GEGLU_BWD, torch.bfloat16),
    ("g_down", M1, 1152, 6912, L.ACT_NONE, torch.bfloat16),
    ("g_dgu_dx", M1, 1152, 13824, L.ACT_NONE, torch.bfloat16),
    ("g_qkv", M1, 1536, 1152, L.ACT_NONE, torch.bfloat16),
    ("g_o", M1, 1152, 1024, L.ACT_NONE, torch.bfloat16),
    ("g_dO", M1, 1024, 1152, L.ACT_NONE, torch.bfloat16),
    ("g_dqkv", M1, 1152, 1536, L.ACT_NONE, torch.bfloat16),
    ("lm_head", 4096, 262144, 1152, L.ACT_NONE, torch.bfloat16),
    ("sig_qkv", MS, 3072, 1024, L.ACT_NONE, torch.bfloat16),
    ("sig_fc1", MS, 4096, 1024, L.ACT_GELU_TANH, torch.bfloat16),
    ("sig_fc2", MS, 1024, 4096, L.ACT_NONE, torch.bfloat16),
    # the SigLIP calls as the model makes them (models.cpp: bias; out / fc2 with bf16(linear) + bf16 residual)
    ("sig_qkv_b", MS, 3072, 1024, L.ACT_NONE, torch.bfloat16, "bias"),
    ("sig_o_br", MS, 1024, 1024, L.ACT_NONE, torch.bfloat16, "bias_res"),
    ("sig_fc1_b", MS, 4096, 1024, L.ACT_GELU_TANH, torch.bfloat16, "bias"),
    ("sig_fc2_br", MS, 1024, 4096, L.ACT_NONE, torch.bfloat16, "bias_res"),
    ("proj_fc1", MS, 11520, 1024, L.ACT_GELU_ERF, torch.bfloat16),
    ("proj_fc2", MS, 1152, 11520, L.ACT_NONE, torch.float32),
    ("proj_dW2", 1152, 11520, 18432, L.ACT_NONE, torch.float32),
    ("proj_dW1", 11520, 1024, 18432, L.ACT_NONE, torch.float32),
    ("proj_dA", 18432, 11520, 1152, L.ACT_GELU_ERF_BWD, torch.bfloat16),
    ("sq8192", 8192, 8192, 8192, L.ACT_NONE, torch.bfloat16),
]


def setup(m, n, k, act, odt, extra=None):
    A = torch.randn(m, k, device=dev).to(torch.bfloat16)
    B = (torch.randn(n, k, device=dev) * 0.05).to(torch.bfloat16)
    kw = {}
    if extra in ("bias", "bias_res"):
        kw["bias"] = torch.randn(n, device=dev)
    if extra == "bias_res":
        kw["resid16"] = torch.randn(m, n, device=dev).to(torch.bfloat16)
        kw["bf16_linear"] = True
    if act == L.ACT_GEGLU:
        kw = dict(aux=torch.empty(m, n // 2, dtype=torch.bfloat16, device=dev),
                  aux2=torch.empty(m, n // 2, dtype=torch.bfloat16, device=dev))
    elif act == L.ACT_GEGLU_BWD:
        kw = dict(aux_in=torch.randn(m, n, device=dev).to(torch.bfloat16),
                  aux_in2=torch.randn(m, n, device=dev).to(torch.bfloat16))
    elif act == L.ACT_GELU_ERF:
        kw = dict(aux=torch.empty(m, n, dtype=torch.bfloat16, device=dev))
    elif act == L.ACT_GELU_ERF_BWD:
        kw = dict(aux_in=torch.randn(m, n, device=dev).to(torch.bfloat16))
    return A, B, kw


def timed(A, B, kw, act, odt, C, reps):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        K.gemm(A, B, C=C, out_dtype=odt, act=act, **kw)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


only = set(a for a in sys.argv[1:] if not a.startswith("-"))
TAGS = {8: "w4", 32: "p8", 64: "dual", 128: "solo", 256: "p8w", 512: "p8t224", 1024: "p8t192", 4096: "p8t160", 0: "auto"}
modes = tuple(int(x) for x in os.environ.get("MODES", "8,32,64,0").split(","))
for name, m, n, k, act, odt, *extra in SHAPES:
    if only and name not in only:
        continue
    A, B, kw = setup(m, n, k, act, odt, *extra)
    C = K.gemm(A, B, out_dtype=odt, act=act, **kw)
    reps = max(3, min(50, int(2e12 / (2.0 * m * n * k))))
    res = {m_: [] for m_ in modes}
    for rnd in range(3):
        for md in modes:
            L.lib().ptk_gemm_force_small_tiles(md)
            timed(A, B, kw, act, odt, C, 1)
            res[md].append(timed(A, B, kw, act, odt, C, reps))
    L.lib().ptk_gemm_force_small_tiles(0)
    eq = {}
    if os.environ.get("CHECK") == "1":   # each mode's output against the first mode's, bitwise
        outs = []
        for md in modes:
            L.lib().ptk_gemm_force_small_tiles(md)
            Cm = torch.full_like(C, float("nan"))
            K.gemm(A, B, C=Cm, out_dtype=odt, act=act, **kw)
            outs.append(Cm)
        L.lib().ptk_gemm_force_small_tiles(0)
        torch.cuda.synchronize()
        eq = {"eq_" + TAGS[md]: bool(torch.equal(outs[0], o)) for md, o in zip(modes[1:], outs[1:])}
    fl = 2.0 * m * n * k
    out = {"name": name, "M": m, "N": n, "K": k}
    for md in modes:
        tag = TAGS[md]
        ms = min(res[md])
        out[tag + "_us"] = round(ms * 1e3, 1)
        out[tag + "_TF"] = round(fl / ms / 1e9, 1)
    out.update(eq)
    print(json.dumps(out), flush=True)
    del A, B, C, kw
    torch.cuda.empty_cache()
