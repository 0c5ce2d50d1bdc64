"""fp32-accumulate check of the product kernels at <= 1e-4 (SURVEY.md:297 "fp32-accumulate debug mode").

The product path computes with bf16 operands and fp32 accumulation everywhere (SURVEY F8 flow).  Its distance
to the reference's fp32 run therefore has two parts: (1) the rounding of operands to bf16, which the
reference's own `--mixed_precision bf16` run shares and which the twin-fixture tolerances of
test_stage1_gpu.py / test_stage2_gpu.py bound; (2) the accumulation itself.  This module isolates (2): every
kernel family is fed bf16-EXACT operands and compared with a float64 evaluation of the same values, so any
difference is the kernel's own arithmetic (fp32 partial sums, their order, split-K reduction, the output cast).

Bars (all stated per test):
  fp32 outputs: rel-L2 <= 1e-5 and max |d| <= 1e-4 * max |ref| (fp32 sums of K <= 262144 bf16 products);
  bf16 outputs: equal to bf16(float64 result) except where the fp32 sum straddles a rounding boundary: <= 1 bf16
  ulp (+ 1e-4 * max |ref|) on every element and <= 1 % of elements off;
  attention LSE (fp32): |d| <= 1e-4 (log-domain), softmax statistics in fp32.
Every GEMM dispatch path of `launch_gemm` is exercised: the automatic rule (mode 0), the 128x128 kernel
(mode 1), the 256x256 8-wave kernel (2), its staggered variant (4), the persistent 4-wave kernel (8), the
persistent 8-wave kernel (32), and the batched split-K form the lm_head dX uses.
"""

import pytest
import torch

pytestmark = pytest.mark.gpu

F32_RL2, F32_MAX = 1e-5, 1e-4


def _k():
    from projectiontrainer_amd import kernels as K, _lib as L
    return K, L


def rnd(*shape, dev, scale=1.0, seed=0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    return (torch.randn(*shape, generator=g) * scale).to(torch.bfloat16).to(dev)


def ref64(A, B):
    return A.double() @ B.double().T


def check_f32(got, ref, what):
    got, ref = got.double(), ref.double()
    rl2 = ((got - ref).norm() / ref.norm()).item()
    mx = (got - ref).abs().max().item() / ref.abs().max().item()
    assert rl2 <= F32_RL2 and mx <= F32_MAX, (what, rl2, mx)


def check_bf16(got, ref, what):
    """bf16 output vs the float64 result: within one bf16 ulp (+ the fp32 accumulation bar) of it everywhere,
    and equal to bf16(ref) at >= 99 % of elements (the rest: fp32 sums that straddle a rounding boundary)."""
    exact = ref.to(torch.bfloat16)
    g = got.to(torch.bfloat16)
    off = g != exact
    ulp = torch.finfo(torch.bfloat16).eps * ref.abs() + F32_MAX * ref.abs().max()   # 2^-7 relative = one ulp
    assert ((g.double() - ref).abs() <= ulp).all(), what
    assert off.double().mean().item() <= 1e-2, (what, off.double().mean().item())


SHAPES = [(22528, 1152, 13824), (22528, 13824, 1152), (4096, 1536, 1152), (1100, 700, 192), (2048, 1152, 6912)]


@pytest.mark.parametrize("mode", [0, 1, 2, 4, 8, 32])
@pytest.mark.parametrize("M,N,K", SHAPES)
def test_gemm_fp32_accumulate(gpu, M, N, K, mode):
    Kn, L = _k()
    A, B = rnd(M, K, dev=gpu, seed=1), rnd(N, K, dev=gpu, seed=2, scale=0.05)
    ref = ref64(A, B)
    L.lib().ptk_gemm_force_small_tiles(mode)
    try:
        C = Kn.gemm(A, B, out_dtype=torch.float32)
        Cb = Kn.gemm(A, B, out_dtype=torch.bfloat16)
    finally:
        L.lib().ptk_gemm_force_small_tiles(0)
    check_f32(C, ref, (M, N, K, mode, "f32"))
    check_bf16(Cb, ref, (M, N, K, mode, "bf16"))


def test_gemm_split_k_fp32_accumulate(gpu):
    """The lm_head dX form: K = vocab split into 8 slices, batched fp32 partials, summed in slice order."""
    Kn, L = _k()
    M, N, K, S = 512, 1152, 262144, 8
    A, B = rnd(M, K, dev=gpu, seed=3, scale=0.01), rnd(N, K, dev=gpu, seed=4, scale=0.05)
    kc = K // S
    P = torch.empty(S, M, N, dtype=torch.float32, device=gpu)
    Kn.gemm(A, B, C=P, M=M, N=N, K=kc, lda=K, ldb=K, ldc=N, batch=S, strides=(kc, 0, kc, 0, M * N, 0))
    got = P.double().sum(0)
    check_f32(got, ref64(A, B), "split-K")


@pytest.mark.parametrize("window", [0, 512])
def test_attention_lse_fp32(gpu, window):
    """Flash forward at the Gemma3-1B shape (GQA 4:1, head_dim 256, S 704): the fp32 log-sum-exp."""
    Kn, L = _k()
    B, S, hd, Hkv, G = 2, 704, 256, 1, 4
    Q = rnd(B, Hkv, S, G, hd, dev=gpu, seed=41)
    Kt = rnd(B, Hkv, S, hd, dev=gpu, seed=42)
    Vt = rnd(B, Hkv, S, hd, dev=gpu, seed=43)
    kv = torch.ones(B, S, dtype=torch.int32, device=gpu)
    kv[1, :37] = 0                                            # left padding
    O = torch.zeros(B * S, G * hd, dtype=torch.bfloat16, device=gpu)
    lse = torch.zeros(B * Hkv, S * G, dtype=torch.float32, device=gpu)
    scale = hd ** -0.5
    Kn.flash_attn(Q, Kt, Vt, O, lse=lse, rows=S * G, nkeys=S, head_dim=hd, ldq=hd, ldk=hd, ldo=hd,
                  batch=B * Hkv, batch_inner=Hkv, zdiv=Hkv,
                  strides=(Hkv * S * G * hd, S * G * hd, Hkv * S * hd, S * hd, S * G * hd, G * hd),
                  omap=(G, 0, G, 0), qdiv=G, causal=True, window=window, key_valid=kv, scale=scale)
    q = Q.double().permute(0, 1, 3, 2, 4).reshape(B, G, S, hd)
    k = Kt.double()
    s = (q @ k.transpose(-1, -2)) * scale
    i = torch.arange(S, device=gpu)
    m = i[None, :] <= i[:, None]
    if window:
        m = m & (i[None, :] > i[:, None] - window)
    m = m[None, None] & kv.bool()[:, None, None, :]
    s = s.masked_fill(~m, float("-inf"))
    lref = torch.logsumexp(s, -1)                              # [B, G, S]
    lg = lse.view(B, S, G).permute(0, 2, 1).double()
    ok = torch.isfinite(lref)
    err = (lg[ok] - lref[ok]).abs().max().item()
    assert err <= 1e-4, err


def test_cross_entropy_fp32(gpu):
    """Fused CE over a vocab-262144 row block: per-row loss (fp32 max / sum-exp) vs float64."""
    Kn, L = _k()
    R, V = 64, 262144
    logits = rnd(R, V, dev=gpu, seed=5, scale=2.0)
    tgt = torch.randint(0, V, (R,), generator=torch.Generator().manual_seed(6)).to(gpu)
    tgt[::7] = -100
    ref = torch.logsumexp(logits.double(), -1) - logits.double().gather(1, tgt.clamp_min(0)[:, None])[:, 0]
    gscale = torch.ones(1, dtype=torch.float32, device=gpu)
    row = Kn.cross_entropy_(logits.clone(), tgt, gscale)
    keep = tgt >= 0
    err = (row.double()[keep] - ref[keep]).abs().max().item()
    assert err <= 1e-4 * max(1.0, ref[keep].abs().max().item()), err
    assert (row[~keep] == 0).all()
