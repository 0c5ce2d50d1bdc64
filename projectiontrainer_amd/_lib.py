"""ctypes binding of libptk.so (include/ptk.h).  Fails loudly if the library
is missing: there is no CPU fallback on the product path."""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libptk.so")
if os.environ.get("PTK_LIB"):   # A/B timing of a diagnostic build (tools/); never set by tests or the driver
    LIB_PATH = os.path.join(os.path.dirname(_HERE), os.environ["PTK_LIB"])

c_void_p, c_int, c_int64, c_float, c_size_t, c_uint64 = C.c_void_p, C.c_int, C.c_int64, C.c_float, C.c_size_t, C.c_uint64
c_float_p = C.POINTER(C.c_float)

ACT_NONE, ACT_GELU_TANH, ACT_GELU_ERF, ACT_GEGLU, ACT_GELU_ERF_BWD, ACT_GEGLU_BWD = range(6)
OUT_BF16, OUT_F32, OUT_F32_BF16ROUND = range(3)


class RowMap(C.Structure):
    _fields_ = [("g", c_int), ("skip", c_int), ("gs", c_int64), ("off", c_int64)]


class GemmDesc(C.Structure):
    _fields_ = [("A", c_void_p), ("B", c_void_p), ("C", c_void_p),
                ("M", c_int), ("N", c_int), ("K", c_int),
                ("lda", c_int64), ("ldb", c_int64), ("ldc", c_int64),
                ("batch", c_int), ("batch_inner", c_int),
                ("sA0", c_int64), ("sA1", c_int64), ("sB0", c_int64), ("sB1", c_int64),
                ("sC0", c_int64), ("sC1", c_int64),
                ("alpha", c_float), ("act", c_int), ("out", c_int),
                ("bias", c_void_p), ("rowadd", c_void_p), ("rowadd_period", c_int),
                ("ld_rowadd", c_int64), ("resid", c_void_p), ("ld_resid", c_int64),
                ("aux", c_void_p), ("aux2", c_void_p), ("ld_aux", c_int64),
                ("aux_in", c_void_p), ("aux_in2", c_void_p), ("ld_aux_in", c_int64),
                ("amap", RowMap), ("cmap", RowMap), ("resid16", c_void_p), ("ld_resid16", c_int64),
                ("bf16_linear", c_int), ("tail_ws", c_void_p)]


class FlashDesc(C.Structure):
    _fields_ = [("Q", c_void_p), ("K", c_void_p), ("V", c_void_p), ("O", c_void_p), ("lse", c_void_p),
                ("rows", c_int), ("nkeys", c_int), ("head_dim", c_int),
                ("ldq", c_int64), ("ldk", c_int64), ("ldo", c_int64),
                ("batch", c_int), ("batch_inner", c_int), ("zdiv", c_int),
                ("sQ0", c_int64), ("sQ1", c_int64), ("sK0", c_int64), ("sK1", c_int64),
                ("sO0", c_int64), ("sO1", c_int64), ("qmap", RowMap), ("omap", RowMap),
                ("qdiv", c_int), ("causal", c_int), ("window", c_int), ("key_valid", c_void_p),
                ("scale", c_float)]


class FlashBwdDesc(C.Structure):
    _fields_ = [("Q", c_void_p), ("K", c_void_p), ("V", c_void_p), ("O", c_void_p), ("dO", c_void_p),
                ("lse", c_void_p), ("delta", c_void_p), ("dQ", c_void_p), ("dK", c_void_p), ("dV", c_void_p),
                ("rows", c_int), ("nkeys", c_int), ("head_dim", c_int),
                ("batch", c_int), ("batch_inner", c_int), ("zdiv", c_int),
                ("ldo", c_int64), ("sO0", c_int64), ("sO1", c_int64), ("omap", RowMap),
                ("qdiv", c_int), ("causal", c_int), ("window", c_int), ("key_valid", c_void_p),
                ("scale", c_float), ("workspace", c_void_p), ("workspace_bytes", c_int64)]


class SiglipConfigC(C.Structure):
    _fields_ = [("image_size", c_int), ("patch_size", c_int), ("channels", c_int), ("hidden", c_int),
                ("heads", c_int), ("intermediate", c_int), ("layers", c_int), ("eps", c_float)]


class SiglipLayerC(C.Structure):
    _fields_ = [("wqkv", c_void_p), ("bqkv", c_void_p), ("wo", c_void_p), ("bo", c_void_p),
                ("w1", c_void_p), ("b1", c_void_p), ("w2", c_void_p), ("b2", c_void_p),
                ("ln1_w", c_void_p), ("ln1_b", c_void_p), ("ln2_w", c_void_p), ("ln2_b", c_void_p)]


class SiglipWeightsC(C.Structure):
    _fields_ = [("patch_w", c_void_p), ("patch_b", c_void_p), ("pos", c_void_p),
                ("post_w", c_void_p), ("post_b", c_void_p), ("layers", C.POINTER(SiglipLayerC))]


class ProjectorC(C.Structure):
    _fields_ = [("vision_dim", c_int), ("inter_dim", c_int), ("llm_dim", c_int),
                ("w1", c_void_p), ("b1", c_void_p), ("w2", c_void_p), ("b2", c_void_p), ("w2t", c_void_p),
                ("tail_ws", c_void_p)]


class Gemma3ConfigC(C.Structure):
    _fields_ = [("vocab", c_int), ("hidden", c_int), ("inter", c_int), ("layers", c_int), ("heads", c_int),
                ("kv_heads", c_int), ("head_dim", c_int), ("sliding_window", c_int),
                ("sliding_pattern", c_int), ("pad_token_id", c_int),
                ("query_pre_attn_scalar", c_float), ("eps", c_float)]


class Gemma3LayerC(C.Structure):
    _fields_ = [("wqkv", c_void_p), ("wqkv_t", c_void_p), ("wo", c_void_p), ("wo_t", c_void_p),
                ("wgu", c_void_p), ("wgu_t", c_void_p), ("wd", c_void_p), ("wd_t", c_void_p),
                ("ln_in", c_void_p), ("ln_post_attn", c_void_p), ("ln_pre_ff", c_void_p),
                ("ln_post_ff", c_void_p), ("q_norm", c_void_p), ("k_norm", c_void_p)]


class Gemma3WeightsC(C.Structure):
    _fields_ = [("embed", c_void_p), ("embed_t", c_void_p), ("final_norm", c_void_p),
                ("rope_cos_local", c_void_p), ("rope_sin_local", c_void_p),
                ("rope_cos_global", c_void_p), ("rope_sin_global", c_void_p),
                ("rope_max_pos", c_int), ("layers", C.POINTER(Gemma3LayerC))]


class Gemma3BatchC(C.Structure):
    _fields_ = [("batch", c_int), ("text_len", c_int), ("num_vision", c_int), ("seq_pad", c_int),
                ("token_ids", c_void_p), ("labels", c_void_p), ("x", c_void_p), ("dx", c_void_p),
                ("loss_scale", c_float), ("loss", c_void_p), ("label_offset", c_int)]


class Gemma3GenerateC(C.Structure):
    _fields_ = [("batch", c_int), ("prompt_len", c_int), ("max_new_tokens", c_int), ("do_sample", c_int),
                ("top_k", c_int), ("temperature", c_float), ("seed", C.c_uint64), ("eos_token_id", c_int64),
                ("pad_token_id", c_int64), ("prompt_batch_stride", c_int64), ("top_p", c_float)]


class Gemma3DecodeC(C.Structure):
    _fields_ = [("rows", c_int), ("prompt_len", c_int), ("max_new_tokens", c_int), ("prompt_repeat", c_int),
                ("prompt_batch_stride", c_int64)]


class Gemma3LayerGradsC(C.Structure):
    _fields_ = [(n, c_void_p) for n in ("wqkv", "wo", "wgu", "wd", "ln_in", "ln_post_attn", "ln_pre_ff",
                                        "ln_post_ff", "q_norm", "k_norm")]


class Gemma3GradsC(C.Structure):
    _fields_ = [("embed", c_void_p), ("final_norm", c_void_p), ("layers", C.POINTER(Gemma3LayerGradsC))]


class ImageDesc(C.Structure):
    _fields_ = [("src_off", c_int64), ("h", C.c_int32), ("w", C.c_int32), ("c", C.c_int32),
                ("kh", C.c_int32), ("kv", C.c_int32), ("pad_", C.c_int32),
                ("coef_off", c_int64), ("tmp_off", c_int64)]


ABI_VERSION = 8      # include/ptk.h PTK_ABI_VERSION

# exported symbol -> (restype, argtypes)
SIGNATURES = {
    "ptk_abi_version": (c_int, []),
    "ptk_last_error": (C.c_char_p, []),
    "ptk_gemm": (c_int, [C.POINTER(GemmDesc), c_void_p]),
    "ptk_gemm_tail_scratch_bytes": (c_size_t, []),
    "ptk_gemm_tail_split": (c_int, [C.POINTER(GemmDesc)]),
    "ptk_layernorm": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_float, c_void_p]),
    "ptk_rmsnorm": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_float, c_void_p]),
    "ptk_rmsnorm_bwd": (c_int, [c_void_p] * 6 + [c_int, c_int, c_void_p]),
    "ptk_qknorm_rope_fwd": (c_int, [c_void_p] * 5 + [c_int] * 5 + [c_float] + [c_void_p] * 6),
    "ptk_qknorm_rope_bwd": (c_int, [c_void_p] * 5 + [c_int] * 5 + [c_void_p] * 7),
    "ptk_softmax": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_int64, c_int, c_int, c_int, c_int,
                            c_int, c_void_p, c_int, c_void_p]),
    "ptk_cross_entropy": (c_int, [c_void_p, c_int64, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p]),
    "ptk_transpose_bf16": (c_int, [c_void_p, c_int64, c_void_p, c_int64, c_int, c_int64, c_int64, c_int,
                                   c_int, c_int, c_void_p]),
    "ptk_transpose_rows_bf16": (c_int, [c_void_p, c_int64, c_int, c_int64, c_int64, c_int, c_int, c_void_p, c_int64,
                                        c_int, c_void_p]),
    "ptk_weight_grad_bf16": (c_int, [c_void_p, c_int64, c_int, c_int64, c_int64, c_int,
                                     c_void_p, c_int64, c_int, c_int64, c_int64, c_int, c_int,
                                     c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_int, c_void_p]),
    "ptk_cast_f32_bf16": (c_int, [c_void_p, c_void_p, c_int64, c_void_p]),
    "ptk_fill_normal_bf16": (c_int, [c_void_p, c_int64, c_uint64, c_float, c_float, c_void_p]),
    "ptk_gemm_timer_enable": (c_int, [c_int]),
    "ptk_gemm_force_small_tiles": (c_int, [c_int]),
    "ptk_gemm_timer_read": (c_int, [c_int, C.POINTER(C.c_double), C.POINTER(c_int)]),
    "ptk_gemm_path_counts": (c_int, [c_void_p, c_int]),
    "ptk_stage_timers_enable": (c_int, [c_int]),
    "ptk_stage_begin": (c_int, [C.c_char_p, c_void_p]),
    "ptk_stage_end": (c_int, [c_void_p]),
    "ptk_stage_timers_read": (c_int64, [C.c_char_p, c_size_t, c_int]),
    "ptk_flash_attn_fwd": (c_int, [C.POINTER(FlashDesc), c_void_p]),
    "ptk_flash_attn_bwd": (c_int, [C.POINTER(FlashBwdDesc), c_void_p]),
    "ptk_flash_bwd_workspace_bytes": (c_size_t, [C.POINTER(FlashBwdDesc)]),
    "ptk_siglip_workspace_bytes": (c_size_t, [C.POINTER(SiglipConfigC), c_int]),
    "ptk_siglip_fwd": (c_int, [C.POINTER(SiglipConfigC), C.POINTER(SiglipWeightsC), c_int, c_void_p, c_void_p,
                               c_void_p, c_size_t, c_void_p]),
    "ptk_projector_fwd": (c_int, [C.POINTER(ProjectorC), c_int, c_void_p, c_void_p, c_void_p, c_void_p, RowMap,
                                  c_int64, c_int, c_void_p]),
    "ptk_projector_workspace_bytes": (c_size_t, [C.POINTER(ProjectorC), c_int]),
    "ptk_projector_bwd": (c_int, [C.POINTER(ProjectorC), c_int] + [c_void_p] * 8 + [c_void_p, c_size_t, c_void_p]),
    "ptk_gather_vision_grad": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_void_p]),
    "ptk_gemma3_workspace_bytes": (c_size_t, [C.POINTER(Gemma3ConfigC), c_int, c_int, c_int]),
    "ptk_gemma3_loss_fwd_bwd": (c_int, [C.POINTER(Gemma3ConfigC), C.POINTER(Gemma3WeightsC),
                                        C.POINTER(Gemma3BatchC), c_void_p, c_size_t, c_void_p]),
    "ptk_gemma3_loss_fwd": (c_int, [C.POINTER(Gemma3ConfigC), C.POINTER(Gemma3WeightsC),
                                    C.POINTER(Gemma3BatchC), c_void_p, c_size_t, c_void_p]),
    "ptk_gemma3_train_workspace_bytes": (c_size_t, [C.POINTER(Gemma3ConfigC), c_int, c_int, c_int]),
    "ptk_gemma3_train_fwd_bwd": (c_int, [C.POINTER(Gemma3ConfigC), C.POINTER(Gemma3WeightsC),
                                         C.POINTER(Gemma3BatchC), C.POINTER(Gemma3GradsC), c_void_p, c_size_t,
                                         c_void_p]),
    "ptk_gemma3_generate_workspace_bytes": (c_size_t, [C.POINTER(Gemma3ConfigC), c_int, c_int, c_int]),
    "ptk_gemma3_generate": (c_int, [C.POINTER(Gemma3ConfigC), C.POINTER(Gemma3WeightsC), C.POINTER(Gemma3GenerateC),
                                    c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_size_t, c_void_p]),
    "ptk_gemma3_decode_workspace_bytes": (c_size_t, [C.POINTER(Gemma3ConfigC), C.POINTER(Gemma3DecodeC)]),
    "ptk_gemma3_decode_prefill": (c_int, [C.POINTER(Gemma3ConfigC), C.POINTER(Gemma3WeightsC),
                                          C.POINTER(Gemma3DecodeC), c_void_p, c_void_p, c_int64, c_void_p, c_void_p,
                                          c_size_t, c_void_p]),
    "ptk_gemma3_decode_step": (c_int, [C.POINTER(Gemma3ConfigC), C.POINTER(Gemma3WeightsC), C.POINTER(Gemma3DecodeC),
                                       c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_size_t, c_void_p]),
    "ptk_beam_candidates_workspace_bytes": (c_size_t, [c_int, c_int, c_int]),
    "ptk_beam_candidates": (c_int, [c_void_p, c_int64, c_void_p, c_int, c_int, c_int, c_int, c_int, c_float, c_float,
                                    c_int, c_uint64, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_size_t,
                                    c_void_p]),
    "ptk_gemm_skinny_part_bytes": (c_size_t, [c_int, c_int, c_int]),
    "ptk_gemm_skinny": (c_int, [c_void_p, c_int64, c_void_p, c_int64, c_void_p, c_int64, c_int, c_int, c_int, c_int,
                                c_void_p, c_size_t, c_void_p]),
    "ptk_bf16_sumsq_partial_floats": (c_int, []),
    "ptk_bf16_grad_scale_sumsq": (c_int, [c_void_p, c_int64, c_float, c_void_p, c_void_p, c_void_p]),
    "ptk_adamw_bf16": (c_int, [c_void_p] * 4 + [c_int64, c_void_p, c_float] + [C.c_double] * 5 +
                       [c_int, c_void_p, c_void_p]),
    "ptk_resize_ksize": (c_int, [c_int, c_int]),
    "ptk_resize_coeffs": (c_int, [c_int, c_int, c_void_p, c_void_p]),
    "ptk_image_preprocess": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_int,
                                     c_void_p, c_void_p, c_void_p]),
    "ptk_comm_unique_id_bytes": (c_int, []),
    "ptk_comm_get_unique_id": (c_int, [c_void_p]),
    "ptk_comm_init": (c_int, [C.POINTER(c_void_p), c_void_p, c_int, c_int]),
    "ptk_comm_destroy": (c_int, [c_void_p]),
    "ptk_comm_world": (c_int, [c_void_p]),
    "ptk_comm_allreduce_sum": (c_int, [c_void_p, c_void_p, c_int64, c_void_p]),
    "ptk_comm_allreduce_avg": (c_int, [c_void_p, c_void_p, c_int64, c_void_p]),
    "ptk_projector_bwd_allreduce": (c_int, [C.POINTER(ProjectorC), c_int] + [c_void_p] * 5 +
                                    [c_void_p, c_size_t, c_void_p, c_void_p, c_void_p]),
    "ptk_clip_adamw": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_float, c_float, c_float,
                               c_float, c_float, c_float, c_float, c_int, c_void_p, c_void_p, c_void_p]),
}

_lib = None


class PtkError(RuntimeError):
    pass


def lib():
    """Load libptk.so once; raise if it is absent (build with __graft_entry__.build())."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise PtkError(f"libptk.so not found at {LIB_PATH}: run `python -c 'import __graft_entry__ as g; g.build()'`")
        L = C.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            if os.environ.get("PTK_LIB") and not hasattr(L, name):
                continue   # an older diagnostic build may predate an entry point
            f = getattr(L, name)
            f.restype, f.argtypes = res, args
        if L.ptk_abi_version() != ABI_VERSION:
            raise PtkError("libptk ABI version mismatch")
        _lib = L
    return _lib


def check(rc: int, what: str = ""):
    if rc != 0:
        raise PtkError(f"{what}: {lib().ptk_last_error().decode()}")


def ptr(t) -> int | None:
    """Device pointer of a torch tensor (None for None)."""
    return None if t is None else t.data_ptr()


# nt128b: batched / split-K slices of the 128x128 kernel; p8sk: the persistent 8-wave kernel with a stream-K tail
GEMM_PATHS = ("nt128", "big", "big2", "w4", "nt128b", "p8sk", "p8", "tn", "unused8")


def gemm_path_counts(reset=False):
    """{(path name, act class): launches} since the last reset (host-side census of launch_gemm)."""
    buf = (C.c_int64 * (8 * len(GEMM_PATHS)))()
    check(lib().ptk_gemm_path_counts(buf, int(reset)), "gemm_path_counts")
    return {(GEMM_PATHS[i // 8], i % 8): int(v) for i, v in enumerate(buf) if v}


_stages_on = os.environ.get("PTK_STAGE_TIMERS", "0") not in ("", "0")


def stage_timers_enable(on=True):
    """Per-stage device timers (stages.cpp; SURVEY §5 tracing) on or off for this process."""
    global _stages_on
    _stages_on = bool(on)
    check(lib().ptk_stage_timers_enable(int(bool(on))), "stage_timers_enable")


class stage:
    """`with stage("projector.bwd", device):` brackets the enclosed launches on the current stream as one
    stage (nothing is recorded unless the timers are on)."""

    def __init__(self, name, device=None):
        self.name, self.device, self.on = name, device, False

    def __enter__(self):
        self.on = _stages_on
        if self.on:
            self.st = stream_ptr(self.device)
            check(lib().ptk_stage_begin(self.name.encode(), self.st), "stage_begin")
        return self

    def __exit__(self, *exc):
        if self.on:
            check(lib().ptk_stage_end(self.st), "stage_end")
        return False


def stage_timers_read(reset=False):
    """{stage name: (total ms, spans)} recorded since the last reset (waits for the recorded spans)."""
    n = lib().ptk_stage_timers_read(None, 0, 0)
    if n < 0:
        check(-1, "stage_timers_read")
    buf = C.create_string_buffer(int(n) + 64)
    n = lib().ptk_stage_timers_read(buf, len(buf), int(reset))
    if n < 0:
        check(-1, "stage_timers_read")
    out = {}
    for line in buf.value.decode().splitlines():
        name, ms, cnt = line.split("\t")
        out[name] = (float(ms), int(cnt))
    return out


def stream_ptr(device=None) -> int:
    import torch
    return torch.cuda.current_stream(device).cuda_stream
