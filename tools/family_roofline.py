"""Per-kernel-family MFMA fractions of the cfg2 Stage-1 step (bs 32) from a rocprofv3 kernel-statistics CSV
(tools/rocpd_stats.py output, e.g. profiles/r04_final_kernel_stats.csv).

Each family's algorithmic FLOPs are the sum over the GEMM / attention roles the step dispatches to it (the cfg2
dispatch, as the census tests pin it: tests/test_stage1_gpu.py CENSUS_CASES), per launch on real rows (B * S,
S = 703 tokens; padded rows and the attention's masked pairs are not counted).  fraction = FLOPs / (kernel time x
2.5 PFLOP/s dense bf16).
usage: python tools/family_roofline.py STATS_CSV STEPS_IN_PROFILE [> profiles/rNN_family_roofline.md]"""
import csv
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from projectiontrainer_amd.config import PRESETS  # noqa: E402
from projectiontrainer_amd.flops import attention_pairs  # noqa: E402

PEAK = 2.5e15


def roles(cfg):
    v, t = cfg.vision, cfg.text
    B, N, S, T = cfg.batch_size, v.num_patches, cfg.seq_len, cfg.text_len
    D, Iv, Lv = v.hidden_size, v.intermediate_size, v.num_hidden_layers
    H, I, L = t.hidden_size, t.intermediate_size, t.num_hidden_layers
    q, kv = t.q_dim, t.kv_dim
    M_v, M_g = B * N, B * S
    attn_g = sum(2 * 2 * attention_pairs(S, t.sliding_window if t.is_sliding(i) else None) * t.head_dim *
                 t.num_attention_heads * B for i in range(L))
    Mp, Ip = B * cfg.num_vision_tokens, cfg.expansion_factor * D   # projector rows (575 per image), hidden
    # family -> list of (role, launches per step, FLOPs per launch); the r06 dispatch (tests/test_stage1_gpu.py
    # census): plain bf16 projections on the lean 8-wave kernel with 224- / 192- / 160-row tiles (p8_tile_height),
    # SigLIP fc2 with the stream-K tail + fixup, projector weight grads on the TN kernel, lm_head dX as K slices,
    # and the last Gemma3 layer's MLP on the B*T loss rows only (gemm_big GEGLU, 160-row p8 for down / dh /
    # d(gate|up) dX, the standalone GEGLU backward)
    R = B * T
    return {
        "gemm_p8_kernel<0, 0, false, true, 224>": [
            ("SigLIP q|k|v", Lv, 2 * M_v * D * 3 * D),
            ("Gemma o", L, 2 * M_g * q * H),
            ("Gemma d(q|k|v) dX", L, 2 * M_g * (q + 2 * kv) * H),
            ("Gemma down", L - 1, 2 * M_g * I * H),
            ("Gemma d(gate|up) dX", L - 1, 2 * M_g * 2 * I * H)],
        "gemm_p8_kernel<0, 0, false, true, 192>": [
            ("Gemma q|k|v", L, 2 * M_g * H * (q + 2 * kv)),
            ("Gemma dO", L, 2 * M_g * H * q)],
        "gemm_p8_kernel<0, 0, false, true, 160>": [("SigLIP o", Lv, 2 * M_v * D * D)],
        "gemm_w4_kernel<3, 0,": [("Gemma gate|up + GEGLU", L - 1, 2 * M_g * 2 * I * H)],
        "gemm_w4_kernel<5, 0,": [("Gemma dh + GEGLU backward", L - 1, 2 * M_g * I * H)],
        "gemm_big_kernel<3, 0>": [("last layer gate|up + GEGLU (loss rows)", 1, 2 * R * 2 * I * H)],
        "gemm_p8_kernel<0, 0, false, false, 160>": [("last layer down, dh, d(gate|up) dX (loss rows)", 3,
                                                     2 * R * I * H * 4 / 3)],
        "gemm_p8_kernel<1, 0": [("SigLIP fc1 + GELU-tanh", Lv, 2 * M_v * D * Iv)],
        "gemm_p8_kernel<0, 0, true, true|p8_fixup_kernel<0, 0>": [("SigLIP fc2 (stream-K tail + fixup)", Lv,
                                                                   2 * M_v * Iv * D)],
        "gemm_p8_kernel<2, 0": [("projector fc1 + GELU-erf", 1, 2 * Mp * D * Ip)],
        "gemm_p8_kernel<0, 2, true|p8_fixup_kernel<0, 2>": [("projector fc2", 1, 2 * Mp * Ip * H)],
        "gemm_p8_kernel<4, 0": [("projector dA + GELU-erf backward", 1, 2 * Mp * H * Ip)],
        "gemm_tn_kernel<1, false>": [("projector dW1, dW2 (TN)", 2, 2 * Mp * D * Ip)],
        "attn_fwd64_kernel": [("SigLIP attention", Lv, 2 * 2 * N * N * D * B)],
        "attn_fwd256w_kernel": [("Gemma attention forward", L, attn_g / L)],
        # the backward's four algorithmic products (dP, dV, dQ, dK) over both kernels' time (dQ recomputes S, dP)
        "attn_bwd_dkv256b_kernel|attn_bwd_dq256w_kernel": [("Gemma attention backward (dK / dV + dQ)", 2 * L,
                                                            attn_g / L)],
        "gemm_big_kernel<0, 0>": [("lm_head forward (+ softmax statistics)", 1, 2 * B * T * H * t.vocab_size)],
        "gemm_p8_kernel<0, 1, false, false, 256>": [("lm_head dX (16 K slices)", 1, 2 * B * T * H * t.vocab_size)],
    }


def main():
    path, steps = sys.argv[1], int(sys.argv[2])
    rows = list(csv.DictReader(open(path)))
    cfg = PRESETS["cfg2"]
    print(f"# Per-family MFMA fractions, cfg2 step (bs 32), from `{os.path.relpath(path, ROOT)}` ({steps} profiled "
          "steps; kernel time = rocprofv3 total / steps)\n")
    print("| kernel family | roles | launches / step (expected) | ms / step | algorithmic TFLOP | TFLOP/s | "
          "fraction of 2.5 PF |")
    print("|---|---|---|---|---|---|---|")
    tot_ms = tot_fl = 0.0
    for fam, rl in roles(cfg).items():
        ks = [r for r in rows if any(f in r["Name"] for f in fam.split("|"))]
        if not ks:
            continue
        calls = sum(int(r["Calls"]) for r in ks) / steps
        ms = sum(float(r["TotalDurationNs"]) for r in ks) / steps / 1e6
        exp = sum(n for _, n, _ in rl)
        fl = sum(n * f for _, n, f in rl)
        tot_ms += ms
        tot_fl += fl
        name = " + ".join(f"`{f}{'>' if '<' in f and not f.endswith('>') else ''}`" for f in fam.split("|"))
        role_names = ", ".join(r.replace("|", "\\|") for r, _, _ in rl)
        print(f"| {name} | {role_names} | {calls:.0f} ({exp}) | {ms:.2f} | {fl / 1e12:.2f} | "
              f"{fl / (ms / 1e3) / 1e12:.0f} | {fl / (ms / 1e3) / PEAK:.3f} |")
    print(f"| all of the above | | | {tot_ms:.2f} | {tot_fl / 1e12:.2f} | {tot_fl / (tot_ms / 1e3) / 1e12:.0f} | "
          f"{tot_fl / (tot_ms / 1e3) / PEAK:.3f} |")
    print("\nLaunch counts that differ from the expected ones include launches of other roles on the same family "
          "(their FLOPs are not counted, so the family's fraction is a lower bound).")


if __name__ == "__main__":
    main()
