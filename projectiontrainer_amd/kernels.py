"""Tensor-level wrappers over libptk primitive ops (device tensors in, device
tensors out, launched on torch's current HIP stream).  Used by the model
classes and by the kernel parity tests."""
from __future__ import annotations

import torch

from . import _lib as L
from ._lib import check, ptr


def _require_cuda(*ts):
    for t in ts:
        if t is not None and not t.is_cuda:
            raise L.PtkError("libptk ops need HIP device tensors (no CPU fallback)")


def _bits(t):
    """bf16 tensors are passed as raw 16-bit storage."""
    return ptr(t)


def gemm(A, B, *, C=None, out_dtype=torch.bfloat16, act=L.ACT_NONE, alpha=1.0, bias=None, rowadd=None,
         resid=None, aux=None, aux2=None, aux_in=None, aux_in2=None, M=None, N=None, K=None,
         lda=None, ldb=None, ldc=None, batch=1, batch_inner=1, strides=(0, 0, 0, 0, 0, 0),
         amap=(0, 0, 0, 0), cmap=(0, 0, 0, 0), out_mode=None, resid16=None, bf16_linear=False, tail_ws=None):
    """C = epi(alpha * A . B^T) with A [M,K], B [N,K] bf16 (K-contiguous).  tail_ws: stream-K tail scratch
    (uint8 [ptk_gemm_tail_scratch_bytes], its counters zero)."""
    _require_cuda(A, B)
    M = A.shape[-2] if M is None else M
    K = A.shape[-1] if K is None else K
    N = B.shape[-2] if N is None else N
    n_out = N // 2 if act == L.ACT_GEGLU else (2 * N if act == L.ACT_GEGLU_BWD else N)
    if C is None:
        C = torch.empty((M, n_out), dtype=out_dtype, device=A.device)
    if out_mode is None:
        out_mode = L.OUT_BF16 if C.dtype == torch.bfloat16 else L.OUT_F32
    d = L.GemmDesc()
    d.A, d.B, d.C = ptr(A), ptr(B), ptr(C)
    d.M, d.N, d.K = M, N, K
    d.lda = A.stride(-2) if lda is None else lda
    d.ldb = B.stride(-2) if ldb is None else ldb
    d.ldc = C.stride(-2) if ldc is None else ldc
    d.batch, d.batch_inner = batch, batch_inner
    d.sA0, d.sA1, d.sB0, d.sB1, d.sC0, d.sC1 = strides
    d.alpha, d.act, d.out = alpha, act, out_mode
    d.bias = ptr(bias)
    if rowadd is not None:
        d.rowadd, d.rowadd_period, d.ld_rowadd = ptr(rowadd), rowadd.shape[0], rowadd.stride(0)
    if resid is not None:
        d.resid, d.ld_resid = ptr(resid), resid.stride(-2)
    if aux is not None:
        d.aux, d.ld_aux = ptr(aux), aux.stride(-2)
    d.aux2 = ptr(aux2)
    if aux_in is not None:
        d.aux_in, d.ld_aux_in = ptr(aux_in), aux_in.stride(-2)
    d.aux_in2 = ptr(aux_in2)
    d.amap = L.RowMap(*amap)
    d.cmap = L.RowMap(*cmap)
    if resid16 is not None:
        d.resid16, d.ld_resid16 = ptr(resid16), resid16.stride(-2)
    d.bf16_linear = int(bool(bf16_linear))
    d.tail_ws = ptr(tail_ws)
    check(L.lib().ptk_gemm(d, L.stream_ptr(A.device)), "ptk_gemm")
    return C


def layernorm(x, w, b, eps):
    _require_cuda(x)
    y = torch.empty(x.shape, dtype=torch.bfloat16, device=x.device)
    rows, cols = x.numel() // x.shape[-1], x.shape[-1]
    check(L.lib().ptk_layernorm(ptr(x), ptr(w), ptr(b), ptr(y), rows, cols, eps, L.stream_ptr(x.device)), "layernorm")
    return y


def rmsnorm(x, w, eps):
    _require_cuda(x)
    rows, cols = x.numel() // x.shape[-1], x.shape[-1]
    y = torch.empty(x.shape, dtype=torch.bfloat16, device=x.device)
    rstd = torch.empty(rows, dtype=torch.float32, device=x.device)
    check(L.lib().ptk_rmsnorm(ptr(x), ptr(w), ptr(y), ptr(rstd), rows, cols, eps, L.stream_ptr(x.device)), "rmsnorm")
    return y, rstd


def rmsnorm_bwd(x, w, rstd, dn, dacc=None):
    rows, cols = x.numel() // x.shape[-1], x.shape[-1]
    dx = torch.empty_like(x)
    check(L.lib().ptk_rmsnorm_bwd(ptr(x), ptr(w), ptr(rstd), ptr(dn), ptr(dacc), ptr(dx), rows, cols,
                                  L.stream_ptr(x.device)), "rmsnorm_bwd")
    return dx


def qknorm_rope(qkv, q_w, k_w, cos_t, sin_t, *, batch, seq, heads, kv_heads, head_dim, eps):
    """Gemma3 q/k RMSNorm + RoPE (ptk_qknorm_rope_fwd) -> Q [B,Hkv,S,G,D], K, V [B,Hkv,S,D], rstd_q, rstd_k."""
    _require_cuda(qkv)
    dev, G = qkv.device, heads // kv_heads
    Q = torch.empty(batch, kv_heads, seq, G, head_dim, dtype=torch.bfloat16, device=dev)
    K = torch.empty(batch, kv_heads, seq, head_dim, dtype=torch.bfloat16, device=dev)
    V = torch.empty_like(K)
    rq = torch.empty(batch * seq, heads, dtype=torch.float32, device=dev)
    rk = torch.empty(batch * seq, kv_heads, dtype=torch.float32, device=dev)
    check(L.lib().ptk_qknorm_rope_fwd(ptr(qkv), ptr(q_w), ptr(k_w), ptr(cos_t), ptr(sin_t), batch, seq, heads, kv_heads,
                                      head_dim, eps, ptr(Q), ptr(K), ptr(V), ptr(rq), ptr(rk), L.stream_ptr(dev)),
          "qknorm_rope_fwd")
    return Q, K, V, rq, rk


def qknorm_rope_bwd(qkv, q_w, k_w, cos_t, sin_t, rq, rk, dQ, dK, dV, *, batch, seq, heads, kv_heads, head_dim):
    """Backward of qknorm_rope (ptk_qknorm_rope_bwd) -> d(qkv) bf16 [B*S, (Hq+2Hkv)*D]."""
    _require_cuda(qkv)
    dqkv = torch.empty_like(qkv)
    check(L.lib().ptk_qknorm_rope_bwd(ptr(qkv), ptr(q_w), ptr(k_w), ptr(cos_t), ptr(sin_t), batch, seq, heads,
                                      kv_heads, head_dim, ptr(rq), ptr(rk), ptr(dQ), ptr(dK), ptr(dV), ptr(dqkv),
                                      L.stream_ptr(qkv.device)), "qknorm_rope_bwd")
    return dqkv


def softmax(S, *, nz, rows, cols, rows_per_batch=0, qdiv=1, zdiv=1, causal=False, window=0, key_valid=None,
            key_len=None):
    P = torch.empty(S.shape, dtype=torch.bfloat16, device=S.device)
    check(L.lib().ptk_softmax(ptr(S), ptr(P), nz, rows, cols, S.stride(-2), rows_per_batch, qdiv, zdiv, int(causal),
                              window, ptr(key_valid), cols if key_len is None else key_len,
                              L.stream_ptr(S.device)), "softmax")
    return P


def cross_entropy_(logits, targets, gscale):
    """In-place fused CE fwd/bwd on bf16 logits [R, V]; returns per-row loss."""
    R, V = logits.shape
    row_loss = torch.empty(R, dtype=torch.float32, device=logits.device)
    check(L.lib().ptk_cross_entropy(ptr(logits), logits.stride(0), R, V, ptr(targets), ptr(row_loss), ptr(gscale),
                                    L.stream_ptr(logits.device)), "cross_entropy")
    return row_loss


def transpose_rows(x, rows, rows_pad, map_g=0, map_gs=0, map_off=0, ld_out=None):
    """Stage-2 weight-grad operand transpose (ptk_transpose_rows_bf16): out[c][r] = x[map(r)][c] for r < rows,
    0 up to rows_pad; map(r) = (r // g) * gs + r % g + off (g = 0: r + off).  x: 2-D bf16, row stride x.stride(0)."""
    if x.dtype != torch.bfloat16 or x.dim() != 2 or x.stride(1) != 1:
        raise L.PtkError("transpose_rows: x must be a 2-D bf16 tensor with unit column stride")
    cols = x.shape[1]
    ld = rows_pad if ld_out is None else ld_out
    out = torch.empty((cols, ld), dtype=torch.bfloat16, device=x.device)
    check(L.lib().ptk_transpose_rows_bf16(ptr(x), x.stride(0), map_g, map_gs, map_off, rows, cols, ptr(out), ld,
                                          rows_pad, L.stream_ptr(x.device)), "transpose_rows")
    return out


def weight_grad(dy, x, grad, rows=None, ymap=(0, 0, 0), xmap=(0, 0, 0), part=None, mode=0):
    """Stage-2 weight grad of one nn.Linear into its bf16 .grad (ptk_weight_grad_bf16): grad [Ny, Nx] =
    bf16(grad + bf16(dY^T X)) over `rows` token rows of dy [.., Ny] / x [.., Nx] (row maps (g, gs, off) as
    transpose_rows').  part: fp32 scratch for K-slice partials (None: one slice); mode 0 auto, 1 the transpose path,
    2 the TN path only.  Returns grad."""
    for t in (dy, x, grad):
        if t.dtype != torch.bfloat16 or t.dim() != 2 or t.stride(1) != 1:
            raise L.PtkError("weight_grad: dy, x, grad must be 2-D bf16 tensors with unit column stride")
    Ny, Nx = dy.shape[1], x.shape[1]
    if tuple(grad.shape) != (Ny, Nx) or grad.stride(0) != Nx:
        raise L.PtkError("weight_grad: grad must be a contiguous [Ny, Nx] tensor")
    rows = dy.shape[0] if rows is None else rows
    kp = (rows + 63) // 64 * 64
    ta = tb = None
    if mode != 2:   # the TN path is not guaranteed (shape, alignment, maps): the transpose fallback's scratch
        ta = torch.empty((Ny, kp), dtype=torch.bfloat16, device=dy.device)
        tb = torch.empty((Nx, kp), dtype=torch.bfloat16, device=dy.device)
    pf = 0 if part is None else part.numel()
    check(L.lib().ptk_weight_grad_bf16(ptr(dy), dy.stride(0), ymap[0], ymap[1], ymap[2], Ny, ptr(x), x.stride(0),
                                       xmap[0], xmap[1], xmap[2], Nx, rows, ptr(grad), ptr(ta), ptr(tb), ptr(part),
                                       pf, mode, L.stream_ptr(dy.device)), "weight_grad")
    return grad


def transpose(x, rows_pad=None, out=None):
    """[Z, rows, cols] or [rows, cols] bf16 -> [.., cols, rows_pad] (zero-padded); out: preallocated result."""
    squeeze = x.dim() == 2
    x3 = x.unsqueeze(0) if squeeze else x
    Z, rows, cols = x3.shape
    rp = rows if rows_pad is None else rows_pad
    if out is None:
        out = torch.empty((Z, cols, rp), dtype=x.dtype, device=x.device)
    else:
        if tuple(out.shape[-2:]) != (cols, rp) or out.numel() != Z * cols * rp or not out.is_contiguous():
            raise L.PtkError(f"transpose: out {tuple(out.shape)} does not hold [{Z}, {cols}, {rp}]")
        out = out.view(Z, cols, rp)
    check(L.lib().ptk_transpose_bf16(ptr(x3), x3.stride(1), ptr(out), rp, Z, x3.stride(0), cols * rp, rows, cols, rp,
                                     L.stream_ptr(x.device)), "transpose")
    return out[0] if squeeze else out


def cast_bf16(x, out=None):
    out = torch.empty(x.shape, dtype=torch.bfloat16, device=x.device) if out is None else out
    check(L.lib().ptk_cast_f32_bf16(ptr(x), ptr(out), x.numel(), L.stream_ptr(x.device)), "cast")
    return out


def fill_normal_(t, seed, std=0.02, mean=0.0):
    assert t.dtype == torch.bfloat16 and t.is_contiguous()
    check(L.lib().ptk_fill_normal_bf16(ptr(t), t.numel(), seed & (2**64 - 1), std, mean, L.stream_ptr(t.device)),
          "fill_normal")
    return t


def flash_attn(Q, K, V, O, *, rows, nkeys, head_dim, ldq, ldk, ldo, batch, batch_inner=1, zdiv=1,
               strides=(0, 0, 0, 0, 0, 0), qmap=(0, 0, 0, 0), omap=(0, 0, 0, 0), qdiv=1, causal=False,
               window=0, key_valid=None, scale=1.0, lse=None):
    """Flash attention forward (ptk_flash_attn_fwd); O written in place."""
    _require_cuda(Q, K, V, O)
    d = L.FlashDesc()
    d.Q, d.K, d.V, d.O, d.lse = ptr(Q), ptr(K), ptr(V), ptr(O), ptr(lse)
    d.rows, d.nkeys, d.head_dim = rows, nkeys, head_dim
    d.ldq, d.ldk, d.ldo = ldq, ldk, ldo
    d.batch, d.batch_inner, d.zdiv = batch, batch_inner, zdiv
    d.sQ0, d.sQ1, d.sK0, d.sK1, d.sO0, d.sO1 = strides
    d.qmap, d.omap = L.RowMap(*qmap), L.RowMap(*omap)
    d.qdiv, d.causal, d.window = qdiv, int(causal), window
    d.key_valid, d.scale = ptr(key_valid), scale
    check(L.lib().ptk_flash_attn_fwd(d, L.stream_ptr(Q.device)), "flash_attn_fwd")
    return O


def flash_attn_bwd(Q, K, V, O, dO, lse, *, rows, nkeys, head_dim, batch, batch_inner=1, zdiv=1, ldo=None,
                   sO=(0, 0), omap=(0, 0, 0, 0), qdiv=1, causal=False, window=0, key_valid=None, scale=1.0,
                   split=True):
    """Flash attention backward (ptk_flash_attn_bwd) -> (dQ, dK, dV) in the Q / K layouts.
    split=False passes no workspace (every key slab in one piece)."""
    _require_cuda(Q, K, V, O, dO, lse)
    dQ, dK, dV = torch.empty_like(Q), torch.empty_like(K), torch.empty_like(V)
    delta = torch.empty(batch * rows, dtype=torch.float32, device=Q.device)
    d = L.FlashBwdDesc()
    d.Q, d.K, d.V, d.O, d.dO, d.lse, d.delta = ptr(Q), ptr(K), ptr(V), ptr(O), ptr(dO), ptr(lse), ptr(delta)
    d.dQ, d.dK, d.dV = ptr(dQ), ptr(dK), ptr(dV)
    d.rows, d.nkeys, d.head_dim = rows, nkeys, head_dim
    d.batch, d.batch_inner, d.zdiv = batch, batch_inner, zdiv
    d.ldo = head_dim if ldo is None else ldo
    d.sO0, d.sO1 = sO
    d.omap = L.RowMap(*omap)
    d.qdiv, d.causal, d.window = qdiv, int(causal), window
    d.key_valid, d.scale = ptr(key_valid), scale
    ws = None
    if split:
        nb = L.lib().ptk_flash_bwd_workspace_bytes(d)
        if nb:
            ws = torch.empty(nb, dtype=torch.uint8, device=Q.device)
            d.workspace, d.workspace_bytes = ptr(ws), nb
    check(L.lib().ptk_flash_attn_bwd(d, L.stream_ptr(Q.device)), "flash_attn_bwd")
    return dQ, dK, dV
