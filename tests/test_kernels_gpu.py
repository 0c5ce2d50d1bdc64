"""Per-kernel parity: libptk HIP kernels vs a plain PyTorch fp32 reference of
the same op (on the same bf16-valued inputs).  Tolerances are stated per test:
bf16 outputs are compared at ~1 bf16 ulp relative scale (rtol 1e-2), fp32
outputs of bf16-input GEMMs at rtol 2e-3 (fp32 accumulate, order differs)."""
import math

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _k():
    from projectiontrainer_amd import kernels as K, _lib as L
    return K, L


def rnd(*shape, dev, dtype=torch.bfloat16, scale=1.0, seed=0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    return (torch.randn(*shape, generator=g) * scale).to(dev).to(dtype)


def close(got, ref, rtol, atol_scale=1e-2):
    got, ref = got.float(), ref.float()
    atol = atol_scale * ref.abs().max().item() * rtol / 1e-2 if ref.numel() else 0
    torch.testing.assert_close(got, ref, rtol=rtol, atol=max(atol, 1e-6))


@pytest.mark.parametrize("M,N,K", [(128, 128, 64), (256, 384, 1024), (200, 130, 192), (1000, 1152, 1152),
                                   (77, 64, 64)])
def test_gemm_plain_f32_and_bf16(gpu, M, N, K):
    Kn, L = _k()
    A, B = rnd(M, K, dev=gpu, seed=1), rnd(N, K, dev=gpu, seed=2)
    ref = A.float() @ B.float().T
    C = Kn.gemm(A, B, out_dtype=torch.float32)
    torch.testing.assert_close(C, ref, rtol=2e-3, atol=2e-3 * math.sqrt(K))
    Cb = Kn.gemm(A, B, out_dtype=torch.bfloat16)
    torch.testing.assert_close(Cb.float(), ref, rtol=1e-2, atol=1e-2 * math.sqrt(K))


def test_gemm_asymmetric_identity(gpu):
    """A = I with an asymmetric B catches a transposed C write."""
    Kn, L = _k()
    n = 128
    A = torch.eye(n, device=gpu, dtype=torch.bfloat16)
    B = (torch.arange(n * n, device=gpu, dtype=torch.float32).view(n, n) % 97).to(torch.bfloat16)
    C = Kn.gemm(A, B, out_dtype=torch.float32)
    torch.testing.assert_close(C, B.float().T)


def test_gemm_epilogues(gpu):
    Kn, L = _k()
    M, N, K = 300, 256, 128
    A, B = rnd(M, K, dev=gpu, seed=3), rnd(N, K, dev=gpu, seed=4, scale=0.1)
    bias = rnd(N, dev=gpu, dtype=torch.float32, seed=5)
    pos = rnd(7, N, dev=gpu, dtype=torch.float32, seed=6)
    res = rnd(M, N, dev=gpu, dtype=torch.float32, seed=7)
    base = A.float() @ B.float().T + bias
    # bias + periodic row add + residual (SigLIP patch embed / out_proj)
    C = res.clone()
    Kn.gemm(A, B, C=C, bias=bias, rowadd=pos, resid=C, alpha=1.0)
    ref = base + pos[torch.arange(M, device=gpu) % 7] + res
    torch.testing.assert_close(C, ref, rtol=2e-3, atol=2e-2)
    # gelu tanh
    C = Kn.gemm(A, B, bias=bias, act=L.ACT_GELU_TANH)
    torch.testing.assert_close(C.float(), F.gelu(base, approximate="tanh"), rtol=2e-2, atol=2e-2)
    # gelu erf with pre-activation aux
    aux = torch.empty(M, N, dtype=torch.bfloat16, device=gpu)
    C = Kn.gemm(A, B, bias=bias, act=L.ACT_GELU_ERF, aux=aux)
    torch.testing.assert_close(aux.float(), base, rtol=1e-2, atol=2e-2)
    torch.testing.assert_close(C.float(), F.gelu(aux.float()), rtol=1e-2, atol=1e-2)
    # gelu erf backward: C = (A B^T) * gelu'(aux)
    C = Kn.gemm(A, B, act=L.ACT_GELU_ERF_BWD, aux_in=aux)
    x = aux.float().requires_grad_(True)
    F.gelu(x).backward((A.float() @ B.float().T).to(torch.bfloat16).float())
    torch.testing.assert_close(C.float(), x.grad, rtol=2e-2, atol=2e-2)
    # alpha + row remap (scatter into padded layout, skipping the first row of each group)
    out = torch.zeros(4 * 80, N, device=gpu)
    Kn.gemm(A[:240], B, C=out, M=240, alpha=0.5, out_mode=L.OUT_F32, cmap=(60, 1, 80, -1))
    ref = 0.5 * (A[:240].float() @ B.float().T)
    for g in range(4):
        torch.testing.assert_close(out[g * 80: g * 80 + 59], ref[g * 60 + 1: g * 60 + 60], rtol=2e-3, atol=2e-3)
        assert out[g * 80 + 59:(g + 1) * 80].abs().sum() == 0


def _geglu_ref(gr, ur, dh):
    """The reference's GEGLU and its autograd (TF gemma3 :131-133, bf16 tensors under autocast) from the fp32 gate
    / up projections: g, u rounded to bf16; the forward's saved factors a = bf16(gelu(g)), b = bf16(gelu'(g) u) and
    h = bf16(a u); the backward of h on a bf16 dh as autograd computes it (dg = gelu'(g) bf16(dh u), du = dh a)."""
    b16 = lambda t: t.to(torch.bfloat16).float()
    g, u = b16(gr), b16(ur)
    gg = g.clone().requires_grad_(True)
    f = F.gelu(gg, approximate="tanh")
    (df,) = torch.autograd.grad(f.sum(), gg)
    a, b = b16(f.detach()), b16(df * u)
    gg2 = g.clone().requires_grad_(True)
    uu = u.clone().requires_grad_(True)
    (b16(F.gelu(gg2, approximate="tanh")) * uu).backward(dh)
    return a, b, b16(a * u), gg2.grad, uu.grad


def _check_geglu(Kn, L, x, Wg, Wu, y, Wd, M, I, tol_fwd=1e-2):
    from projectiontrainer_amd.gemma3 import interleave_gate_up
    Wgu = interleave_gate_up(Wg, Wu)
    ga = torch.empty(M, I, dtype=torch.bfloat16, device=x.device)
    gb = torch.empty_like(ga)
    L.gemm_path_counts(reset=True)
    h = Kn.gemm(x, Wgu, act=L.ACT_GEGLU, aux=ga, aux2=gb)
    torch.cuda.synchronize()
    fwd_paths = L.gemm_path_counts(reset=True)
    gr, ur = (x.float() @ Wg.float().T), (x.float() @ Wu.float().T)
    dh = (y.float() @ Wd.float()).to(torch.bfloat16).float()
    a, b, href, dg_ref, du_ref = _geglu_ref(gr, ur, dh)
    # the saved factors and h: one bf16 rounding of the same functions (g, u from another fp32 summation order)
    torch.testing.assert_close(ga.float(), a, rtol=tol_fwd, atol=tol_fwd)
    torch.testing.assert_close(gb.float(), b, rtol=2 * tol_fwd, atol=2 * tol_fwd)
    torch.testing.assert_close(h.float(), href, rtol=2e-2, atol=2e-2)
    # backward: dh . Wd^T... here dh = y . Wd_t^T with Wd_t [I, H]; dg = bf16(dh) * b, du = bf16(dh) * a
    Wd_t = Wd.T.contiguous()
    dgu = Kn.gemm(y, Wd_t, act=L.ACT_GEGLU_BWD, aux_in=ga, aux_in2=gb)
    torch.cuda.synchronize()
    bwd_paths = L.gemm_path_counts(reset=True)
    dg = dgu.view(M, I // 16, 2, 16)[:, :, 0].reshape(M, I)
    du = dgu.view(M, I // 16, 2, 16)[:, :, 1].reshape(M, I)
    torch.testing.assert_close(dg.float(), dg_ref, rtol=3e-2, atol=3e-2)
    torch.testing.assert_close(du.float(), du_ref, rtol=3e-2, atol=3e-2)
    # exactly the two products of the saved factors (what the epilogue computes, rounded once)
    dhb = (y.float() @ Wd.float()).to(torch.bfloat16).float()
    torch.testing.assert_close(du.float(), (dhb * ga.float()).to(torch.bfloat16).float(), rtol=1e-2, atol=1e-2)
    torch.testing.assert_close(dg.float(), (dhb * gb.float()).to(torch.bfloat16).float(), rtol=1e-2, atol=1e-2)
    return fwd_paths, bwd_paths


def test_gemm_geglu_and_bwd(gpu):
    Kn, L = _k()
    M, H, I = 200, 128, 256
    x = rnd(M, H, dev=gpu, seed=8)
    Wg, Wu = rnd(I, H, dev=gpu, seed=9, scale=0.1), rnd(I, H, dev=gpu, seed=10, scale=0.1)
    y = rnd(M, H, dev=gpu, seed=11)
    Wd = rnd(H, I, dev=gpu, seed=12, scale=0.1)
    _check_geglu(Kn, L, x, Wg, Wu, y, Wd, M, I)


@pytest.mark.parametrize("M", [4608, 5632])
def test_gemm_geglu_and_bwd_persistent_vs_fp32(gpu, M):
    """The GEGLU gate|up and dh + GEGLU-backward epilogues at the row counts where launch_gemm selects the
    persistent kernels (M >= 4096, Gemma3-1B widths H 1152, I 2304 / 6912 cut to fit), vs torch fp32 of the
    same math (modeling_gemma3.py:131-133: down(gelu_tanh(gate(x)) * up(x)) and its autograd); the census
    asserts which kernel family ran."""
    Kn, L = _k()
    H, I = 1152, 2304
    x = rnd(M, H, dev=gpu, seed=81)
    Wg, Wu = rnd(I, H, dev=gpu, seed=82, scale=0.03), rnd(I, H, dev=gpu, seed=83, scale=0.03)
    y = rnd(M, H, dev=gpu, seed=84)
    Wd = rnd(H, I, dev=gpu, seed=85, scale=0.03)
    fwd_paths, bwd_paths = _check_geglu(Kn, L, x, Wg, Wu, y, Wd, M, I)
    persistent = {"w4", "p8"}
    assert any(p in persistent and a == L.ACT_GEGLU for p, a in fwd_paths), fwd_paths
    assert any(p in persistent and a == L.ACT_GEGLU_BWD for p, a in bwd_paths), bwd_paths


def test_gemm_batched_strided(gpu):
    Kn, L = _k()
    Bz, H, S, D = 3, 2, 96, 64
    q = rnd(Bz, S, H * D, dev=gpu, seed=13)
    k = rnd(Bz, S, H * D, dev=gpu, seed=14)
    Np = 128
    C = torch.full((Bz, H, S, Np), float("nan"), device=gpu)
    Kn.gemm(q, k, C=C, M=S, N=S, K=D, lda=H * D, ldb=H * D, ldc=Np, batch=Bz * H, batch_inner=H,
            strides=(S * H * D, D, S * H * D, D, H * S * Np, S * Np), alpha=0.125, out_mode=L.OUT_F32)
    qh = q.float().view(Bz, S, H, D).transpose(1, 2)
    kh = k.float().view(Bz, S, H, D).transpose(1, 2)
    ref = (qh @ kh.transpose(-1, -2)) * 0.125
    torch.testing.assert_close(C[..., :S], ref, rtol=2e-3, atol=2e-3)


def test_layernorm_rmsnorm(gpu):
    Kn, L = _k()
    for cols in (128, 1152, 1024):
        x = rnd(37, cols, dev=gpu, dtype=torch.float32, seed=15) * 3 + 1
        w = rnd(cols, dev=gpu, dtype=torch.float32, seed=16)
        b = rnd(cols, dev=gpu, dtype=torch.float32, seed=17)
        y = Kn.layernorm(x, w, b, 1e-6)
        torch.testing.assert_close(y.float(), F.layer_norm(x, (cols,), w, b, 1e-6), rtol=1e-2, atol=1e-2)
        y, rstd = Kn.rmsnorm(x, w, 1e-6)
        xr = x.clone().requires_grad_(True)
        ref = xr * torch.rsqrt(xr.pow(2).mean(-1, keepdim=True) + 1e-6) * (1 + w)
        torch.testing.assert_close(y.float(), ref.detach(), rtol=1e-2, atol=1e-2)
        dn = rnd(37, cols, dev=gpu, dtype=torch.float32, seed=18)
        dacc = rnd(37, cols, dev=gpu, dtype=torch.float32, seed=19)
        dx = Kn.rmsnorm_bwd(x, w, rstd, dn, dacc)
        ref.backward(dn)
        torch.testing.assert_close(dx, xr.grad + dacc, rtol=1e-4, atol=1e-5)


def test_softmax_masks(gpu):
    Kn, L = _k()
    B, Hkv, G, S = 2, 1, 4, 128
    SG = S * G
    Sc = rnd(B * Hkv, SG, S, dev=gpu, dtype=torch.float32, seed=20) * 4
    kv = torch.ones(B, S, dtype=torch.int32, device=gpu)
    kv[0, 70:75] = 0
    kv[1, 100:] = 0
    for window in (0, 16):
        P = Kn.softmax(Sc, nz=B * Hkv, rows=SG, cols=S, rows_per_batch=SG, qdiv=G, zdiv=Hkv, causal=True,
                       window=window, key_valid=kv)
        q = torch.arange(SG, device=gpu)[:, None] // G
        kk = torch.arange(S, device=gpu)[None, :]
        m = (kk <= q)
        if window:
            m = m & (kk > q - window)
        m = m[None] & kv.bool()[:, None, :]
        ref = torch.softmax(Sc.masked_fill(~m, float("-inf")), -1)
        ref = torch.nan_to_num(ref, nan=0.0)     # fully masked rows -> all-zero P (kernel convention)
        torch.testing.assert_close(P.float(), ref, rtol=1e-2, atol=4e-3)


def test_transpose(gpu):
    Kn, L = _k()
    x = rnd(3, 100, 70, dev=gpu, seed=21)
    t = Kn.transpose(x, rows_pad=128)
    torch.testing.assert_close(t[..., :100], x.transpose(1, 2))
    assert t[..., 100:].abs().sum() == 0


@pytest.mark.parametrize("rows,cols,rows_pad,map_g,map_gs,map_off,ld_extra", [
    (14336, 1152, 14336, 0, 0, 0, 8),        # Stage-2 weight-grad operand (16-B path), padded input rows
    (1000, 200, 1024, 0, 0, 24, 0),          # rows not a tile multiple, zero padding, row offset
    (700, 64, 768, 175, 224, 0, 0),          # gathered rows (per-sample groups)
    (130, 36, 192, 0, 0, 0, 0),              # cols % 8 != 0: the 8-B fallback kernel
])
def test_transpose_rows_gathered(gpu, rows, cols, rows_pad, map_g, map_gs, map_off, ld_extra):
    """Bit-exact: out[c][r] = x[map(r)][c] for r < rows, zeros to rows_pad (train.hip transpose_rows)."""
    Kn, L = _k()
    n_src = (rows // map_g) * map_gs + map_g if map_g else rows + map_off
    x = rnd(n_src, cols + ld_extra, dev=gpu, seed=23)[:, :cols]
    t = Kn.transpose_rows(x, rows, rows_pad, map_g, map_gs, map_off)
    r = torch.arange(rows, device=gpu)
    src = (r // map_g) * map_gs + r % map_g if map_g else r + map_off
    assert torch.equal(t[:, :rows], x[src].t())
    assert t[:, rows:].abs().sum() == 0


def test_cross_entropy(gpu):
    Kn, L = _k()
    R, V = 33, 4096
    logits = rnd(R, V, dev=gpu, seed=22, scale=3)
    tgt = torch.randint(0, V, (R,), device=gpu)
    tgt[5] = -100
    cnt = (tgt != -100).sum().float()
    gscale = (0.25 / cnt).reshape(1).float()
    x = logits.float().requires_grad_(True)
    loss = F.cross_entropy(x, tgt, ignore_index=-100) * 0.25
    loss.backward()
    lg = logits.clone()
    rl = Kn.cross_entropy_(lg, tgt, gscale)
    torch.testing.assert_close(rl.sum() / cnt * 0.25, loss.detach(), rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(lg.float(), x.grad, rtol=1e-2, atol=1e-6)


@pytest.mark.parametrize("mode", [2, 4, 8, 32])
@pytest.mark.parametrize("M,N,K", [(1024, 512, 64), (1024, 512, 128), (1100, 700, 192), (2048, 1152, 1152),
                                   (4096, 1536, 256), (300, 200, 64), (4096, 4096, 576), (8448, 2304, 1152),
                                   (9000, 8200, 128), (4096, 4608, 1152), (4200, 4700, 320), (22528, 1152, 1024),
                                   (18432, 1024, 4096)])
def test_gemm_big_tile_path(gpu, M, N, K, mode):
    """256x256 8-wave kernel (mode 2), its barrier-staggered variant (mode 4), the persistent 4-wave
    kernel (mode 8) and the persistent 8-wave kernel (mode 32; several tiles per workgroup), forced: ragged
    M/N, 1..64 K-tiles, vs fp32."""
    Kn, L = _k()
    A, B = rnd(M, K, dev=gpu, seed=31), rnd(N, K, dev=gpu, seed=32)
    ref = A.float() @ B.float().T
    L.lib().ptk_gemm_force_small_tiles(mode)
    try:
        C = Kn.gemm(A, B, out_dtype=torch.float32)
        C2 = Kn.gemm(A, B, out_dtype=torch.float32)
    finally:
        L.lib().ptk_gemm_force_small_tiles(0)
    torch.testing.assert_close(C, ref, rtol=2e-3, atol=2e-3 * math.sqrt(K))
    assert torch.equal(C, C2)   # fixed accumulation order: deterministic


@pytest.mark.parametrize("mode", [2, 4, 8, 32])
def test_gemm_big_vs_small_all_epilogues(gpu, mode):
    """Every epilogue through the 256x256 (mode 2) / staggered 256x256 (mode 4) / persistent 4-wave (mode 8)
    path matches the 128x128 path
    (fp32 accumulation order differs, so compare at bf16-level tolerance)."""
    Kn, L = _k()
    from projectiontrainer_amd.gemma3 import interleave_gate_up
    M, N, K = 1300, 768, 320
    A, B = rnd(M, K, dev=gpu, seed=33), rnd(N, K, dev=gpu, seed=34, scale=0.1)
    bias = rnd(N, dev=gpu, dtype=torch.float32, seed=35)
    res = rnd(M, N, dev=gpu, dtype=torch.float32, seed=36)
    aux_in = rnd(M, N, dev=gpu, seed=37)
    outs = []
    for md in (mode, 1):
        L.lib().ptk_gemm_force_small_tiles(md)
        try:
            o = {}
            C = res.clone()
            Kn.gemm(A, B, C=C, bias=bias, resid=C)
            o["resid"] = C
            o["gelu_tanh"] = Kn.gemm(A, B, bias=bias, act=L.ACT_GELU_TANH)
            # SigLIP's linear: bf16(acc + bias) + bf16 residual, in place (the lean epilogue's residual path)
            C16 = res.to(torch.bfloat16)
            Kn.gemm(A, B, C=C16, bias=bias, resid16=C16, bf16_linear=True)
            o["resid16"] = C16
            # a group row map that is the identity (the Gemma dO GEMM's at one kv head): the lean path's affine case
            o["gmap"] = Kn.gemm(A, B, C=torch.zeros(M, N, dtype=torch.bfloat16, device=gpu), cmap=(128, 0, 128, 0))
            aux = torch.empty(M, N, dtype=torch.bfloat16, device=gpu)
            o["gelu_erf"] = Kn.gemm(A, B, bias=bias, act=L.ACT_GELU_ERF, aux=aux)
            o["aux"] = aux
            o["erf_bwd"] = Kn.gemm(A, B, act=L.ACT_GELU_ERF_BWD, aux_in=aux_in)
            g = torch.empty(M, N // 2, dtype=torch.bfloat16, device=gpu)
            u = torch.empty_like(g)
            o["geglu"] = Kn.gemm(A, B, act=L.ACT_GEGLU, aux=g, aux2=u)
            o["g"], o["u"] = g, u
            o["geglu_bwd"] = Kn.gemm(A, B, act=L.ACT_GEGLU_BWD, aux_in=aux_in, aux_in2=aux_in)
            cm = torch.zeros(M + 64, N, device=gpu)
            Kn.gemm(A, B, C=cm, out_mode=L.OUT_F32_BF16ROUND, cmap=(100, 1, 104, -1), M=1300)
            o["cmap"] = cm
            outs.append(o)
        finally:
            L.lib().ptk_gemm_force_small_tiles(0)
    for k in outs[0]:
        a, b = outs[0][k].float(), outs[1][k].float()
        bad = ~torch.isclose(a, b, rtol=1e-2, atol=1e-3)
        if mode in (8, 32) and k == "erf_bwd":
            # the 4-wave kernel accumulates with the MFMA operands swapped (C^T tiles): fp32 sums differ in
            # the last bits, and bf16(v) * gelu'(aux) rounds twice, so isolated elements move by 1-2 bf16 ulps
            assert bad.float().mean() < 1e-3, (k, bad.sum().item())
            torch.testing.assert_close(a, b, rtol=3e-2, atol=1e-3, msg=k)
            continue
        torch.testing.assert_close(a, b, rtol=1e-2, atol=1e-3, msg=lambda m: f"{k}: {bad.sum().item()} bad; {m}")


def _attn_ref(q, k, v, mask, scale):
    s = (q.float() @ k.float().transpose(-1, -2)) * scale
    s = s.masked_fill(~mask, float("-inf"))
    m = s.amax(-1, keepdim=True)
    p = torch.exp(s - m)
    l = p.sum(-1, keepdim=True)
    return (p / l) @ v.float(), (m + torch.log(l)).squeeze(-1)


@pytest.mark.parametrize("N", [576, 288, 196, 16])
def test_flash_fwd_siglip_layout(gpu, N):
    """Non-causal, head_dim 64, Q/K/V read in place from the fused [B*N, 3D] qkv buffer."""
    Kn, L = _k()
    B, H, hd = 2, 4, 64
    D = H * hd
    qkv = rnd(B * N, 3 * D, dev=gpu, seed=40)
    O = torch.zeros(B * N, D, dtype=torch.bfloat16, device=gpu)
    Kn.flash_attn(qkv, qkv[:, D:], qkv[:, 2 * D:], O, rows=N, nkeys=N, head_dim=hd, ldq=3 * D, ldk=3 * D, ldo=D,
                  batch=B * H, batch_inner=H, zdiv=H, strides=(N * 3 * D, hd, N * 3 * D, hd, N * D, hd),
                  scale=hd ** -0.5)
    x = qkv.float().view(B, N, 3, H, hd)
    q, k, v = (x[:, :, i].transpose(1, 2) for i in range(3))
    ref, _ = _attn_ref(q, k, v, torch.ones(N, N, dtype=torch.bool, device=gpu), hd ** -0.5)
    ref = ref.transpose(1, 2).reshape(B * N, D)
    torch.testing.assert_close(O.float(), ref, rtol=2e-2, atol=2e-2)


@pytest.mark.parametrize("Hkv,G,window,S", [(1, 4, 0, 320), (1, 4, 100, 320), (2, 2, 64, 320), (1, 4, 512, 704),
                                            (1, 3, 0, 300), (1, 1, 0, 100), (1, 1, 0, 36)])
def test_flash_fwd_gemma_layout(gpu, Hkv, G, window, S):
    """Causal GQA, head_dim 256, key padding, sliding window, token-major O via row map, LSE.  S 704 with
    window 512 = the cfg2 step's sliding layers; G 3 / S 300 and S 100 / 36: query rows that are not a
    multiple of the 128-row block (idle waves, partial tiles)."""
    Kn, L = _k()
    B, hd = 2, 256
    Hq = Hkv * G
    Q = rnd(B, Hkv, S, G, hd, dev=gpu, seed=41)
    Kt = rnd(B, Hkv, S, hd, dev=gpu, seed=42)
    Vt = rnd(B, Hkv, S, hd, dev=gpu, seed=43)
    kv = torch.ones(B, S, dtype=torch.int32, device=gpu)
    kv[0, 200:215] = 0
    kv[1, S - 30:] = 0
    O = torch.zeros(B * S, Hq * hd, dtype=torch.bfloat16, device=gpu)
    lse = torch.zeros(B * Hkv, S * G, dtype=torch.float32, device=gpu)
    scale = 256 ** -0.5
    Kn.flash_attn(Q, Kt, Vt, O, lse=lse, rows=S * G, nkeys=S, head_dim=hd, ldq=hd, ldk=hd, ldo=hd,
                  batch=B * Hkv, batch_inner=Hkv, zdiv=Hkv,
                  strides=(Hkv * S * G * hd, S * G * hd, Hkv * S * hd, S * hd, S * Hq * hd, G * hd),
                  omap=(G, 0, Hq, 0), qdiv=G, causal=True, window=window, key_valid=kv, scale=scale)
    q = Q.float().permute(0, 1, 3, 2, 4).reshape(B, Hq, S, hd)          # head h = kvh*G + j
    k = Kt.float().repeat_interleave(G, dim=1)
    v = Vt.float().repeat_interleave(G, dim=1)
    i = torch.arange(S, device=gpu)
    m = i[None, :] <= i[:, None]
    if window:
        m = m & (i[None, :] > i[:, None] - window)
    m = m[None, None] & kv.bool()[:, None, None, :]
    ref, lref = _attn_ref(q, k, v, m, scale)
    ref = ref.transpose(1, 2).reshape(B * S, Hq * hd)
    torch.testing.assert_close(O.float(), ref, rtol=2e-2, atol=2e-2)
    lg = lse.view(B, Hkv, S, G).permute(0, 1, 3, 2).reshape(B, Hq, S)
    torch.testing.assert_close(lg, lref, rtol=1e-3, atol=1e-3)


@pytest.mark.parametrize("D,Hkv,G,window,S,split,B", [(256, 1, 4, 0, 320, True, 2), (256, 1, 4, 0, 320, False, 2),
                                                       (256, 1, 4, 100, 320, True, 2), (256, 2, 2, 64, 320, True, 2),
                                                       (256, 1, 4, 0, 704, True, 2), (64, 1, 2, 8, 320, True, 2),
                                                       (256, 1, 4, 512, 1088, True, 1), (256, 1, 4, 0, 1088, True, 1),
                                                       (256, 1, 3, 0, 320, True, 1), (256, 1, 1, 0, 4160, False, 1),
                                                       (64, 1, 1, 0, 4160, False, 1)])
def test_flash_bwd_vs_autograd(gpu, D, Hkv, G, window, S, split, B):
    """dQ/dK/dV of softmax(scale QK^T + causal/window/key-pad mask) V vs torch autograd (fp32 math on the
    same bf16 inputs).  Uses the forward kernel's O and LSE as the backward does.  split: heavy key slabs
    cut into query pieces (fp32 partials + ordered reduce) vs one piece per slab; S 704 = the cfg2 length;
    S 1088 at batch 1 = the reference's default T 512 (few z: the split plan must stay within its
    128-entry work table).  The shape fallbacks: a GQA group of 3 (not a power of two: the generic dK/dV
    kernel) and 4160 keys (past the 4096-key mask table: the generic forward, delta and dQ kernels)."""
    Kn, L = _k()
    Hq = Hkv * G
    Q = rnd(B * Hkv, S * G, D, dev=gpu, seed=51)
    Kt = rnd(B * Hkv, S, D, dev=gpu, seed=52)
    Vt = rnd(B * Hkv, S, D, dev=gpu, seed=53)
    dO = rnd(B * Hkv, S * G, D, dev=gpu, seed=54)
    kv = torch.ones(B, S, dtype=torch.int32, device=gpu)
    kv[0, 200:215] = 0
    kv[B - 1, S - 30:] = 0
    scale = D ** -0.5
    O = torch.zeros(B * Hkv, S * G, D, dtype=torch.bfloat16, device=gpu)
    lse = torch.zeros(B * Hkv, S * G, dtype=torch.float32, device=gpu)
    common = dict(rows=S * G, nkeys=S, head_dim=D, batch=B * Hkv, batch_inner=Hkv, zdiv=Hkv, qdiv=G, causal=True,
                  window=window, key_valid=kv, scale=scale)
    Kn.flash_attn(Q, Kt, Vt, O, lse=lse, ldq=D, ldk=D, ldo=D,
                  strides=(Hkv * S * G * D, S * G * D, Hkv * S * D, S * D, Hkv * S * G * D, S * G * D), **common)
    dQ, dK, dV = Kn.flash_attn_bwd(Q, Kt, Vt, O, dO, lse, sO=(Hkv * S * G * D, S * G * D), split=split, **common)
    # reference: rows (s, j) of each z, position s = r // G
    q = Q.float().requires_grad_(True)
    k = Kt.float().requires_grad_(True)
    v = Vt.float().requires_grad_(True)
    sc = (q @ k.transpose(-1, -2)) * scale
    pos = torch.arange(S * G, device=gpu)[:, None] // G
    kk = torch.arange(S, device=gpu)[None, :]
    m = kk <= pos
    if window:
        m = m & (kk > pos - window)
    m = m[None] & kv.bool().repeat_interleave(Hkv, 0)[:, None, :]
    p = torch.softmax(sc.masked_fill(~m, float("-inf")), -1)
    p = torch.where(m.any(-1, keepdim=True), p, torch.zeros_like(p))   # fully masked rows: P = 0 (kernel convention)
    out = p @ v
    out.backward(dO.float())
    for got, ref, nm in ((dQ, q.grad, "dQ"), (dK, k.grad, "dK"), (dV, v.grad, "dV")):
        err = (got.float() - ref).norm() / ref.norm()
        assert err < 2e-2, (nm, float(err))


def _qknorm_rope_ref(qkv, qw, kw, cos_h, sin_h, B, S, Hq, Hkv, D, eps):
    """fp32 restatement of Gemma3 q_norm / k_norm (RMSNorm, scale 1+w) + rotate-half RoPE
    (TF/models/gemma3/modeling_gemma3.py:136-150, :356-360)."""
    x = qkv.float().view(B, S, Hq + 2 * Hkv, D)
    q, k, v = x[:, :, :Hq], x[:, :, Hq:Hq + Hkv], x[:, :, Hq + Hkv:]
    rms = lambda t, w: t * torch.rsqrt(t.pow(2).mean(-1, keepdim=True) + eps) * (1 + w)
    cos = torch.cat([cos_h, cos_h], -1)[None, :, None, :]
    sin = torch.cat([sin_h, sin_h], -1)[None, :, None, :]
    rot = lambda t: torch.cat([-t[..., D // 2:], t[..., :D // 2]], -1)
    q, k = rms(q, qw), rms(k, kw)
    return q * cos + rot(q) * sin, k * cos + rot(k) * sin, v


@pytest.mark.parametrize("Hq,Hkv,D", [(4, 1, 256), (8, 4, 256), (2, 1, 64)])
def test_qknorm_rope_fwd_bwd(gpu, Hq, Hkv, D):
    """q/k RMSNorm + RoPE forward (layout scatter) and backward vs torch fp32 autograd."""
    Kn, L = _k()
    B, S, eps, G = 2, 96, 1e-6, Hq // Hkv
    qkv = rnd(B * S, (Hq + 2 * Hkv) * D, dev=gpu, seed=41, scale=2.0)
    qw = rnd(D, dev=gpu, dtype=torch.float32, seed=42, scale=0.3)
    kw = rnd(D, dev=gpu, dtype=torch.float32, seed=43, scale=0.3)
    inv = 1.0 / (10000.0 ** (torch.arange(0, D, 2, device=gpu, dtype=torch.float32) / D))
    ang = torch.arange(S, device=gpu, dtype=torch.float32)[:, None] * inv[None]
    cos_h, sin_h = ang.cos().contiguous(), ang.sin().contiguous()
    Q, K, V, rq, rk = Kn.qknorm_rope(qkv, qw, kw, cos_h, sin_h, batch=B, seq=S, heads=Hq, kv_heads=Hkv,
                                     head_dim=D, eps=eps)
    x = qkv.float().requires_grad_(True)
    qr, kr, vr = _qknorm_rope_ref(x, qw, kw, cos_h, sin_h, B, S, Hq, Hkv, D, eps)
    # kernel layouts: Q [B,Hkv,S,G,D], K/V [B,Hkv,S,D]
    Qr = qr.view(B, S, Hkv, G, D).permute(0, 2, 1, 3, 4)
    Kr, Vr = kr.permute(0, 2, 1, 3), vr.permute(0, 2, 1, 3)
    torch.testing.assert_close(Q.float(), Qr, rtol=2e-2, atol=2e-2)
    torch.testing.assert_close(K.float(), Kr, rtol=2e-2, atol=2e-2)
    torch.testing.assert_close(V.float(), Vr, rtol=0, atol=0)
    dQ, dK, dV = rnd(*Q.shape, dev=gpu, seed=44), rnd(*K.shape, dev=gpu, seed=45), rnd(*V.shape, dev=gpu, seed=46)
    (Qr * dQ.float()).sum().add((Kr * dK.float()).sum()).add((Vr * dV.float()).sum()).backward()
    dqkv = Kn.qknorm_rope_bwd(qkv, qw, kw, cos_h, sin_h, rq, rk, dQ, dK, dV, batch=B, seq=S, heads=Hq,
                              kv_heads=Hkv, head_dim=D)
    ref = x.grad
    cos = torch.nn.functional.cosine_similarity(dqkv.float().flatten(), ref.flatten(), dim=0)
    assert cos > 0.999, cos
    torch.testing.assert_close(dqkv.float(), ref, rtol=3e-2, atol=3e-2)


@pytest.mark.parametrize("M,N,K", [(1000, 1024, 1152), (4096, 2304, 640), (2304, 3072, 1024), (513, 896, 1280),
                                   (22528, 1152, 1152), (300, 256, 128), (4608, 13824, 1152), (256, 128, 128),
                                   (18432, 1024, 4096)])
def test_gemm_p8_matches_w4(gpu, M, N, K):
    """Persistent 8-wave kernel (forced mode 32: two waves per SIMD, 128x64 per wave, several tiles per
    workgroup, ragged M/N) against the persistent 4-wave kernel (mode 8):
    the same k-step order per output element, so every epilogue -- plain bf16 / fp32 / fp32-rounded, bias +
    residual, bias + bf16(linear) + bf16 residual in place, an identity group row map, GELU-tanh, GELU-erf with its
    pre-activation, GELU-erf backward, GEGLU with g, u side outputs, GEGLU backward into the interleaved dg|du
    layout -- is bit-identical (both take the lean bf16 epilogue where it applies); plain fp32 also against torch
    fp32."""
    Kn, L = _k()
    A, B = rnd(M, K, dev=gpu, seed=11), rnd(N, K, dev=gpu, seed=12, scale=0.05)
    gin, uin = rnd(M, N, dev=gpu, seed=13), rnd(M, N, dev=gpu, seed=14)
    bias = rnd(N, dev=gpu, dtype=torch.float32, seed=15)
    res = rnd(M, N, dev=gpu, dtype=torch.float32, seed=16)
    outs = []
    modes = {8: "w4", 32: "p8"}
    for md in modes:
        L.lib().ptk_gemm_force_small_tiles(md)
        L.gemm_path_counts(reset=True)
        try:
            o = {"f32": Kn.gemm(A, B, out_dtype=torch.float32), "bf16": Kn.gemm(A, B),
                 "f32r": Kn.gemm(A, B, C=torch.empty(M, N, device=gpu), out_mode=L.OUT_F32_BF16ROUND)}
            C = res.clone()
            Kn.gemm(A, B, C=C, bias=bias, resid=C)
            o["resid"] = C
            o["gelu_tanh"] = Kn.gemm(A, B, bias=bias, act=L.ACT_GELU_TANH)
            # SigLIP's linear: bf16(acc + bias) + bf16 residual, in place (the lean epilogue's residual path)
            C16 = res.to(torch.bfloat16)
            Kn.gemm(A, B, C=C16, bias=bias, resid16=C16, bf16_linear=True)
            o["resid16"] = C16
            # a group row map that is the identity (the Gemma dO GEMM's at one kv head): the lean path's affine case
            o["gmap"] = Kn.gemm(A, B, C=torch.zeros(M, N, dtype=torch.bfloat16, device=gpu), cmap=(128, 0, 128, 0))
            aux = torch.empty(M, N, dtype=torch.bfloat16, device=gpu)
            o["gelu_erf"] = Kn.gemm(A, B, bias=bias, act=L.ACT_GELU_ERF, aux=aux)
            o["aux"] = aux
            o["erf_bwd"] = Kn.gemm(A, B, act=L.ACT_GELU_ERF_BWD, aux_in=gin)
            if N % 32 == 0:
                g = torch.zeros(M, N // 2, dtype=torch.bfloat16, device=gpu)
                u = torch.zeros_like(g)
                o["h"] = Kn.gemm(A, B, act=L.ACT_GEGLU, aux=g, aux2=u)
                o["g"], o["u"] = g, u
            o["dgdu"] = Kn.gemm(A, B, act=L.ACT_GEGLU_BWD, aux_in=gin, aux_in2=uin)
            torch.cuda.synchronize()
            paths = {p for p, _ in L.gemm_path_counts(reset=True)}
            assert paths == {modes[md]}, paths
            outs.append(o)
        finally:
            L.lib().ptk_gemm_force_small_tiles(0)
    for other in outs[1:]:
        for k in outs[0]:
            assert torch.equal(outs[0][k], other[k]), (k, (outs[0][k].float() - other[k].float()).abs().max())
    ref = A.float() @ B.float().T
    torch.testing.assert_close(outs[1]["f32"], ref, rtol=2e-3, atol=2e-3 * math.sqrt(K))


@pytest.mark.parametrize("M,N,K", [(22528, 1152, 1152), (1000, 1024, 1152), (4500, 1536, 640), (18432, 3072, 1024),
                                   (224, 256, 128), (230, 320, 192)])
def test_gemm_p8_tm224_matches_p8(gpu, M, N, K):
    """The 8-wave kernel's 224-, 192- and 160-row tiles (forced modes 512 / 1024 / 4096: 7 / 6 / 5 row blocks per wave, the waves
    past them staging only B, ragged M) against its 256-row tiles (mode 32): the same k-step order per output element, so the plain bf16 / fp32 /
    fp32-rounded, bias + residual, bias + bf16(linear) + bf16 residual in place, identity group row map and
    GELU-tanh epilogues are bit-identical; the census shows the p8 family ran."""
    Kn, L = _k()
    A, B = rnd(M, K, dev=gpu, seed=21), rnd(N, K, dev=gpu, seed=22, scale=0.05)
    bias = rnd(N, dev=gpu, dtype=torch.float32, seed=25)
    res = rnd(M, N, dev=gpu, dtype=torch.float32, seed=26)
    outs = []
    for md in (32, 512, 1024, 4096):
        L.lib().ptk_gemm_force_small_tiles(md)
        L.gemm_path_counts(reset=True)
        try:
            o = {"f32": Kn.gemm(A, B, out_dtype=torch.float32), "bf16": Kn.gemm(A, B),
                 "f32r": Kn.gemm(A, B, C=torch.empty(M, N, device=gpu), out_mode=L.OUT_F32_BF16ROUND)}
            C = res.clone()
            Kn.gemm(A, B, C=C, bias=bias, resid=C)
            o["resid"] = C
            o["gelu_tanh"] = Kn.gemm(A, B, bias=bias, act=L.ACT_GELU_TANH)
            C16 = res.to(torch.bfloat16)
            Kn.gemm(A, B, C=C16, bias=bias, resid16=C16, bf16_linear=True)
            o["resid16"] = C16
            o["gmap"] = Kn.gemm(A, B, C=torch.zeros(M, N, dtype=torch.bfloat16, device=gpu), cmap=(112, 0, 112, 0))
            torch.cuda.synchronize()
            paths = {p for p, _ in L.gemm_path_counts(reset=True)}
            assert paths == {"p8"}, paths
            outs.append(o)
        finally:
            L.lib().ptk_gemm_force_small_tiles(0)
    for other in outs[1:]:
        for k in outs[0]:
            assert torch.equal(outs[0][k], other[k]), (k, (outs[0][k].float() - other[k].float()).abs().max())
    ref = A.float() @ B.float().T
    torch.testing.assert_close(outs[1]["f32"], ref, rtol=2e-3, atol=2e-3 * math.sqrt(K))


def test_projector_module_autograd(gpu):
    """MLPProjector as an nn.Module under autograd (the public API, Stage1/projectors.py:22-29): output,
    parameter grads and the INPUT grad vs torch fp32 autograd of the same Sequential(Linear, GELU, Linear);
    bf16 GEMM operands (autocast semantics) bound the difference."""
    from projectiontrainer_amd.projectors import MLPProjector
    torch.manual_seed(0)
    Dv, Dl = 64, 128
    proj = MLPProjector(Dv, Dl, expansion_factor=4)
    ref = torch.nn.Sequential(torch.nn.Linear(Dv, 4 * Dv), torch.nn.GELU(), torch.nn.Linear(4 * Dv, Dl))
    ref.load_state_dict(proj.model.state_dict())
    proj.to(gpu)
    x = rnd(3, 40, Dv, dev=gpu, dtype=torch.float32, seed=91)
    xr = x.detach().clone().requires_grad_(True)
    x = x.detach().clone().requires_grad_(True)
    out = proj(x)
    w = rnd(3, 40, Dl, dev=gpu, dtype=torch.float32, seed=92)
    (out * w).sum().backward()
    ref = ref.to(gpu)
    outr = ref(xr)
    (outr * w).sum().backward()
    torch.testing.assert_close(out, outr, rtol=3e-2, atol=3e-2)
    assert x.grad is not None and x.grad.shape == x.shape
    cos = F.cosine_similarity(x.grad.flatten(), xr.grad.flatten(), dim=0)
    assert cos > 0.999, cos
    torch.testing.assert_close(x.grad, xr.grad, rtol=5e-2, atol=5e-2 * xr.grad.abs().max().item())
    for g, p in zip(proj.grads(), [ref[0].weight, ref[0].bias, ref[2].weight, ref[2].bias]):
        assert F.cosine_similarity(g.flatten(), p.grad.flatten(), dim=0) > 0.999


@pytest.mark.parametrize("rows", [2 * 575, 3 * 64])
def test_projector_weight_grads_tn_vs_fp32(gpu, rows):
    """The projector's weight grads at cfg2 widths (Stage1/projectors.py:16-20: 1024 -> 10240 -> 1152) on the TN GEMM
    (token-major dY / h / dA / x read in place, K = rows padded to a multiple of 64 with the pad rows read as zero:
    2 x 575 = 1150 tokens, and an exact multiple) against torch fp32 autograd of the same Sequential; the census
    asserts the TN path ran.  bf16 operands (autocast semantics) bound the difference."""
    from projectiontrainer_amd import _lib as L
    from projectiontrainer_amd.projectors import MLPProjector
    torch.manual_seed(0)
    Dv, Dl = 1024, 1152
    proj = MLPProjector(Dv, Dl)
    ref = torch.nn.Sequential(torch.nn.Linear(Dv, 10 * Dv), torch.nn.GELU(), torch.nn.Linear(10 * Dv, Dl))
    ref.load_state_dict(proj.model.state_dict())
    proj.to(gpu)
    ref = ref.to(gpu)
    x = rnd(1, rows, Dv, dev=gpu, dtype=torch.float32, seed=95).requires_grad_(True)
    w = rnd(1, rows, Dl, dev=gpu, dtype=torch.float32, seed=96)
    L.gemm_path_counts(reset=True)
    (proj(x) * w).sum().backward()
    torch.cuda.synchronize()
    paths = {p for p, _ in L.gemm_path_counts(reset=True)}
    assert "tn" in paths, paths
    (ref(x) * w).sum().backward()
    for g, p in zip(proj.grads(), [ref[0].weight, ref[0].bias, ref[2].weight, ref[2].bias]):
        g, r = g.float().reshape(p.shape), p.grad.float()
        rel = float((g - r).norm() / r.norm())
        assert rel < 1.5e-2, rel
        assert F.cosine_similarity(g.flatten(), r.flatten(), dim=0) > 0.9999


def test_projector_module_device_move(gpu):
    """Moving the module drops every device-resident cache (bf16 shadows, W1^T, backward workspace, grad scratch,
    tail scratch): autograd backward, a move to the CPU and back, and the same backward again give the same grads
    (a one-GPU box cannot move between GPUs; the CPU round trip re-homes the caches the same way)."""
    from projectiontrainer_amd.projectors import MLPProjector
    torch.manual_seed(0)
    proj = MLPProjector(64, 128, expansion_factor=4).to(gpu)
    x = rnd(2, 40, 64, dev=gpu, dtype=torch.float32, seed=93).requires_grad_(True)
    w = rnd(2, 40, 128, dev=gpu, dtype=torch.float32, seed=94)
    (proj(x) * w).sum().backward()
    g1, dx1 = proj.flat_grad.clone(), x.grad.clone()
    proj.cpu()
    for name in ("_w1b", "_w1t", "_tail", "_bwd_ws", "_grad_tmp"):
        assert getattr(proj, name) is None, name
    proj.to(gpu)
    x.grad = None
    (proj(x) * w).sum().backward()
    assert proj.flat_grad.device == x.device
    assert torch.equal(proj.flat_grad, g1) and torch.equal(x.grad, dx1)


# the stream-K tail of the persistent 8-wave GEMM (gemm_w4.hip P8Tail): (M, N, K, epilogue) at shapes its plan
# splits (a grid of <= 64 tiles, or one full round + <= 24: where it measured faster, profiles/r04_sk_ab.txt) --
# Stage 2's M = 14 336 down projection and d(gate|up) dX (cut to K 4608), its q|k|v weight grad with the bf16
# .grad accumulate (bf16(grad + bf16(dY^T X))), an fp32-out weight grad of N 1024, and a projector-fc2-like
# fp32 output rounded to bf16 and row-scattered
SK_CASES = [(14336, 1152, 6912, "plain"), (14336, 1152, 4608, "plain"), (1536, 1152, 14336, "acc"),
            (1152, 1024, 14336, "f32"), (13824, 1152, 4096, "proj_fc2")]


@pytest.mark.parametrize("M,N,K,kind", SK_CASES)
def test_gemm_stream_k_tail_vs_fp32(gpu, M, N, K, kind):
    """The stream-K tail against torch fp32 of the same GEMM and epilogue, against the same GEMM without the
    tail split (every output element the sum of the same products; only the K-split summation order differs),
    and bit for bit against itself (a second launch: the K-order sum of the pieces is deterministic whichever
    piece arrives last); the census shows the p8sk path ran, the arrival counters are left zero."""
    Kn, L = _k()
    tail = torch.zeros(L.lib().ptk_gemm_tail_scratch_bytes(), dtype=torch.uint8, device=gpu)
    A, B = rnd(M, K, dev=gpu, seed=91), rnd(N, K, dev=gpu, seed=92, scale=0.03)
    kw, ref = {}, A.float() @ B.float().T
    out_dtype = torch.bfloat16
    if kind == "acc":   # the weight-grad accumulate: grad = bf16(grad + bf16(dY^T X))
        res = rnd(M, N, dev=gpu, seed=93)
        kw = dict(resid16=res, bf16_linear=True)
        ref = ref.to(torch.bfloat16).float() + res.float()
    elif kind == "f32":
        out_dtype = torch.float32
    elif kind == "proj_fc2":   # fp32 out rounded to bf16, rows (b, i >= 1) scattered as in the projector's fc2
        out_dtype = torch.float32
        bias = torch.randn(N, device=gpu) * 0.1
        kw = dict(bias=bias, out_mode=L.OUT_F32_BF16ROUND, cmap=(576, 1, 704, -1))
        ref = (ref + bias).to(torch.bfloat16).float()
    rows_out = M if kind != "proj_fc2" else (M // 576) * 704
    mk = lambda: torch.zeros(rows_out, N, dtype=out_dtype, device=gpu)
    C1, C2, C0 = mk(), mk(), mk()
    d = L.GemmDesc()
    d.M, d.N, d.K, d.act, d.out = M, N, K, L.ACT_NONE, kw.get("out_mode", L.OUT_BF16 if out_dtype == torch.bfloat16 else L.OUT_F32)
    d.tail_ws = tail.data_ptr()
    assert L.lib().ptk_gemm_tail_split(d) > 0, "the plan does not split this shape"
    L.gemm_path_counts(reset=True)
    Kn.gemm(A, B, C=C1, tail_ws=tail, **{k: (v.clone() if k == "resid16" else v) for k, v in kw.items()})
    paths = L.gemm_path_counts(reset=True)
    kw2 = {k: (v.clone() if k == "resid16" else v) for k, v in kw.items()}
    Kn.gemm(A, B, C=C2, tail_ws=tail, **kw2)
    Kn.gemm(A, B, C=C0, **{k: (v.clone() if k == "resid16" else v) for k, v in kw.items()})   # no tail split
    torch.cuda.synchronize()
    assert ("p8sk", L.ACT_NONE) in paths, paths
    assert not tail[:16384].any(), "arrival counters not left zero"
    assert torch.equal(C1, C2)
    got = C1 if kind != "proj_fc2" else C1.view(M // 576, 704, N)[:, :575].reshape(-1, N)
    if kind == "proj_fc2":
        ref = ref.view(M // 576, 576, N)[:, 1:].reshape(-1, N)
    torch.testing.assert_close(got.float(), ref, rtol=2e-2, atol=2e-2 if out_dtype == torch.bfloat16 else 1e-2)
    # against the unsplit kernel: equal up to the fp32 summation order of the K pieces (and one bf16 rounding)
    d0 = (C1.float() - C0.float()).abs().max().item()
    assert d0 <= 2e-2 * max(1.0, C0.float().abs().max().item()), d0


# Stage-2 weight grads on the token-major TN path (gemm_tn.hip): the cfg4 dW shapes (K = 14 336 token rows) with the
# stream-K tail over a slab (dW_qkv 30 tiles, dW_o 20, dW_down 135: all tail; dW_gate|up 270 = one round + 14),
# with equal K slices (no slab: partials summed by splitk_reduce) and unsplit, a partial last M tile (Ny 1000),
# padded row strides, the minimum K (128)
WG_CASES = [(1536, 1152, 14336, 0, "slab"), (1152, 1024, 14336, 0, "slab"), (1152, 6912, 14336, 0, "slab"),
            (13824, 1152, 14336, 0, "slab"), (1536, 1152, 14336, 0, "slices"), (1152, 6912, 4096, 0, "slices"),
            (13824, 1152, 2048, 0, "none"), (1000, 320, 640, 8, "slab"), (1000, 320, 640, 8, "slices"),
            (256, 128, 128, 0, "none"), (2304, 1152, 1024, 24, "slices"),
            (262144, 1152, 4096, 0, "slab"),   # the tied lm_head's dW: a 2 GiB d(logits) operand (32-bit offsets)
            # ragged token counts: K padded to a multiple of 64, the pad rows read as zero
            (1152, 1024, 1150, 0, "none"), (1000, 320, 650, 8, "slices"), (1536, 1152, 7150, 0, "slab")]


@pytest.mark.parametrize("Ny,Nx,rows,ld_extra,split", WG_CASES)
def test_weight_grad_tn_vs_fp32(gpu, Ny, Nx, rows, ld_extra, split):
    """grad = bf16(grad + bf16(dY^T X)) on the TN path against torch fp32 of the same products (one bf16 rounding
    of the product, one of the sum: rtol 1e-2 at the product's scale), against the transposed-operand path (same
    products, another fp32 summation order), bit for bit against itself (stream-K pieces and K slices summed in K
    order); the census shows the TN kernel ran and nothing else."""
    Kn, L = _k()
    dy = rnd(rows, Ny + ld_extra, dev=gpu, seed=101)[:, :Ny]
    x = rnd(rows, Nx + ld_extra, dev=gpu, seed=102, scale=0.05)[:, :Nx]
    g0 = rnd(Ny, Nx, dev=gpu, seed=103)
    slab = torch.cuda.get_device_properties(gpu).multi_processor_count * 2 * 8 * 128 * 64
    part = {"slab": torch.empty(max(slab, 8 * Ny * Nx), dtype=torch.float32, device=gpu),
            "slices": torch.empty(min(8 * Ny * Nx, slab - 4), dtype=torch.float32, device=gpu),
            "none": None}[split]
    L.gemm_path_counts(reset=True)
    g1 = Kn.weight_grad(dy, x, g0.clone(), part=part, mode=2)
    paths = L.gemm_path_counts(reset=True)
    g2 = Kn.weight_grad(dy, x, g0.clone(), part=part, mode=2)
    gt = Kn.weight_grad(dy, x, g0.clone(), part=part, mode=1)
    torch.cuda.synchronize()
    assert set(paths) == {("tn", L.ACT_NONE)}, paths
    assert torch.equal(g1, g2)
    prod = dy.float().t() @ x.float()
    ref = (g0.float() + prod.to(torch.bfloat16).float()).to(torch.bfloat16).float()
    scale = max(prod.abs().max().item(), g0.float().abs().max().item())
    torch.testing.assert_close(g1.float(), ref, rtol=1e-2, atol=1e-2 * scale)
    # against the transposed-operand path: the same products, another fp32 summation order
    d = (g1.float() - gt.float()).abs().max().item()
    assert d <= 1e-2 * scale, d
    # the bulk of the elements equal to the fp32 reference after its two roundings
    assert (g1.float() == ref).float().mean().item() > 0.9


def test_weight_grad_tn_gated_shapes(gpu):
    """Shapes the TN path does not take run the transpose path in auto mode and fail loudly in TN-only mode:
    fewer than 65 token rows (K padded to 64 is below the kernel's two K-tiles), gathered rows, N % 64 != 0."""
    Kn, L = _k()
    dy, x = rnd(40, 256, dev=gpu, seed=104), rnd(40, 128, dev=gpu, seed=105)
    g0 = torch.zeros(256, 128, dtype=torch.bfloat16, device=gpu)
    L.gemm_path_counts(reset=True)
    g = Kn.weight_grad(dy, x, g0.clone(), mode=0)
    paths = L.gemm_path_counts(reset=True)
    assert ("tn", L.ACT_NONE) not in paths, paths
    torch.testing.assert_close(g.float(), (dy.float().t() @ x.float()).to(torch.bfloat16).float(), rtol=1e-2,
                               atol=1e-2)
    with pytest.raises(L.PtkError):
        Kn.weight_grad(dy, x, g0.clone(), mode=2)
    dy2, x2 = rnd(256, 256, dev=gpu, seed=106), rnd(256, 96, dev=gpu, seed=107)
    with pytest.raises(L.PtkError):
        Kn.weight_grad(dy2, x2, torch.zeros(256, 96, dtype=torch.bfloat16, device=gpu), mode=2)
    # auto mode on identity maps whose shape the TN kernel rejects (N % 64, exactly 64 rows: ADVICE r05) takes the
    # transpose path with the scratch kernels.weight_grad now always passes
    for a, b in ((dy2, x2), (rnd(64, 256, dev=gpu, seed=108), rnd(64, 128, dev=gpu, seed=109))):
        L.gemm_path_counts(reset=True)
        g = Kn.weight_grad(a, b, torch.zeros(a.shape[1], b.shape[1], dtype=torch.bfloat16, device=gpu), mode=0)
        assert ("tn", L.ACT_NONE) not in L.gemm_path_counts(reset=True)
        torch.testing.assert_close(g.float(), (a.float().t() @ b.float()).to(torch.bfloat16).float(), rtol=1e-2,
                                   atol=1e-2)
    # without that scratch the C ABI refuses on the host (no launch: the transpose kernels once got NULL and faulted)
    gz = torch.zeros(256, 96, dtype=torch.bfloat16, device=gpu)
    rc = L.lib().ptk_weight_grad_bf16(dy2.data_ptr(), dy2.stride(0), 0, 0, 0, 256, x2.data_ptr(), x2.stride(0), 0, 0, 0,
                                      96, 256, gz.data_ptr(), None, None, None, 0, 0, L.stream_ptr(gpu))
    assert rc != 0 and b"transpose path" in L.lib().ptk_last_error()
    torch.cuda.synchronize()
    assert not gz.any()


@pytest.mark.parametrize("M,N,K,act", [(1, 128, 64, 0), (5, 1152, 1152, 0), (16, 1536, 1152, 0), (33, 1152, 6912, 0),
                                       (48, 262144, 1152, 0), (64, 1152, 1024, 0), (48, 13824, 1152, 3),
                                       (7, 256, 128, 3)])
def test_gemm_skinny_vs_fp32(gpu, M, N, K, act):
    """The decode steps' skinny GEMM (gemm_skinny.hip: one workgroup per 64 columns and K slice, fragments straight
    from global memory, K-split partials summed in split order): against torch fp32 on the same bf16 operands,
    plain (C rounded to bf16 once) and GEGLU on interleaved gate|up columns (h = bf16(bf16(gelu(g)) * u))."""
    from projectiontrainer_amd import _lib as L
    g = torch.Generator(device=gpu).manual_seed(M * 7 + N)
    A = (torch.randn(M, K, device=gpu, generator=g) * 0.5).to(torch.bfloat16)
    B = (torch.randn(N, K, device=gpu, generator=g) * 0.05).to(torch.bfloat16)
    NO = N // 2 if act == 3 else N
    C = torch.empty(M, NO, dtype=torch.bfloat16, device=gpu)
    n = L.lib().ptk_gemm_skinny_part_bytes(M, N, K)
    part = torch.empty(max(n, 16), dtype=torch.uint8, device=gpu)
    L.check(L.lib().ptk_gemm_skinny(A.data_ptr(), K, B.data_ptr(), K, C.data_ptr(), NO, M, N, K, act, part.data_ptr(),
                                    n, L.stream_ptr(gpu)), "ptk_gemm_skinny")
    ref = A.float() @ B.float().t()
    if act == 3:
        q = torch.arange(NO, device=gpu)
        gate = ref[:, 32 * (q // 16) + q % 16].to(torch.bfloat16).float()
        up = ref[:, 32 * (q // 16) + 16 + q % 16].to(torch.bfloat16).float()
        a = torch.nn.functional.gelu(gate, approximate="tanh").to(torch.bfloat16).float()
        ref = a * up
    torch.testing.assert_close(C.float(), ref, rtol=2e-2, atol=2e-2 * float(ref.abs().max()))
