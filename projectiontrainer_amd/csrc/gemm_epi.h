// Shared GEMM epilogue helpers (bias, row-add, activations, GEGLU fwd/bwd, residual, row maps,
// bf16/f32 stores) used by the GEMM kernels of gemm.hip and gemm_w4.hip.
#pragma once
#include "common.h"
#include "ptk_internal.h"

namespace ptk {

// ---------------------------------------------------------------- epilogue
// The wave's 64x64 fp32 accumulator tile is staged through LDS ([64][68] f32,
// 17 KiB per wave) and re-read row-contiguously, so every global access of the
// epilogue (bias, row-add, residual, aux in/out, C) is a 8/16-byte vector and
// consecutive lanes touch consecutive addresses.
constexpr int EPI_LD = 68;                       // floats per staged row (64 + 4 pad)
constexpr int EPI_WAVE_BYTES = 64 * EPI_LD * 4;  // 17408

PTK_DEV float4 ldf4(const float* p) { return *reinterpret_cast<const float4*>(p); }
PTK_DEV float4 ldbf4(const bf16_t* p) {
  u16x4_t u = *reinterpret_cast<const u16x4_t*>(p);
  return make_float4(bf2f(u[0]), bf2f(u[1]), bf2f(u[2]), bf2f(u[3]));
}
PTK_DEV void stbf4(bf16_t* p, float4 v) {
  u16x4_t u;
  u[0] = f2bf(v.x); u[1] = f2bf(v.y); u[2] = f2bf(v.z); u[3] = f2bf(v.w);
  *reinterpret_cast<u16x4_t*>(p) = u;
}
PTK_DEV float& el(float4& v, int e) { return reinterpret_cast<float*>(&v)[e]; }
PTK_DEV float el(const float4& v, int e) { return reinterpret_cast<const float*>(&v)[e]; }

template <int ACT, int OUT>
PTK_DEV void epi_vec4(const GemmArgs& p, char* Cz, long r, long c, float4 v) {
  // r < M; c..c+3 < N (checked by caller); c % 4 == 0
  if (p.bias) { float4 b = ldf4(p.bias + c); v.x += b.x; v.y += b.y; v.z += b.z; v.w += b.w; }
  if (p.bf16_linear) v = make_float4(bfround(v.x), bfround(v.y), bfround(v.z), bfround(v.w));
  if (p.rowadd) {
    float4 b = ldf4(p.rowadd + (r % p.rowadd_period) * p.ld_rowadd + c);
    v.x += b.x; v.y += b.y; v.z += b.z; v.w += b.w;
  }
  if constexpr (ACT == ACT_GELU_TANH) {
#pragma unroll
    for (int e = 0; e < 4; ++e) el(v, e) = gelu_tanh(bfround(el(v, e)));
  } else if constexpr (ACT == ACT_GELU_ERF) {
    // pre-activation kept (bf16) for the backward: Stage1/projectors.py:17-18
#pragma unroll
    for (int e = 0; e < 4; ++e) el(v, e) = bfround(el(v, e));
    if (p.aux) stbf4(p.aux + r * p.ld_aux + c, v);
#pragma unroll
    for (int e = 0; e < 4; ++e) el(v, e) = gelu_erf(el(v, e));
  } else if constexpr (ACT == ACT_GELU_ERF_BWD) {
    float4 a = ldbf4(p.aux_in + r * p.ld_aux_in + c);
#pragma unroll
    for (int e = 0; e < 4; ++e) el(v, e) = bfround(el(v, e)) * gelu_erf_grad(el(a, e));
  }
  const long cr = map_row(p.cmap, r);
  if (cr < 0) return;
  if (p.resid) {
    float4 b = ldf4(p.resid + cr * p.ld_resid + c);
    v.x += b.x; v.y += b.y; v.z += b.z; v.w += b.w;
  }
  if (p.resid16) {
    float4 b = ldbf4(p.resid16 + cr * p.ld_resid16 + c);
    v.x += b.x; v.y += b.y; v.z += b.z; v.w += b.w;
  }
  if constexpr (OUT == OUT_BF16) {
    stbf4(reinterpret_cast<bf16_t*>(Cz) + cr * p.ldc + c, v);
  } else {
    if constexpr (OUT == OUT_F32_BFR) v = make_float4(bfround(v.x), bfround(v.y), bfround(v.z), bfround(v.w));
    *reinterpret_cast<float4*>(reinterpret_cast<float*>(Cz) + cr * p.ldc + c) = v;
  }
}

// 8 columns per lane, one 16-B store (bf16 output): the epilogue is store-issue bound
// (one wave store instruction per ~140 cycles per CU regardless of width), so every
// bf16 store moves 16 B.
typedef __attribute__((ext_vector_type(8))) unsigned short u16x8_t;
PTK_DEV void ldbf8(const bf16_t* p, float* v) {
  const u16x8_t u = *reinterpret_cast<const u16x8_t*>(p);
#pragma unroll
  for (int e = 0; e < 8; ++e) v[e] = bf2f(u[e]);
}
PTK_DEV void stbf8(bf16_t* p, const float* v) {
  u16x8_t u;
#pragma unroll
  for (int e = 0; e < 8; ++e) u[e] = f2bf(v[e]);
  *reinterpret_cast<u16x8_t*>(p) = u;
}

template <int ACT>
PTK_DEV void epi_vec8_bf16(const GemmArgs& p, char* Cz, long r, long c, float4 v0, float4 v1) {
  // r < M; c..c+7 < N; c % 8 == 0; all leading dims multiples of 8
  float v[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
  if (p.bias) {
    const float4 b0 = ldf4(p.bias + c), b1 = ldf4(p.bias + c + 4);
    v[0] += b0.x; v[1] += b0.y; v[2] += b0.z; v[3] += b0.w; v[4] += b1.x; v[5] += b1.y; v[6] += b1.z; v[7] += b1.w;
  }
  if (p.bf16_linear) {
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = bfround(v[e]);
  }
  if (p.rowadd) {
    const float* ra = p.rowadd + (r % p.rowadd_period) * p.ld_rowadd + c;
    const float4 b0 = ldf4(ra), b1 = ldf4(ra + 4);
    v[0] += b0.x; v[1] += b0.y; v[2] += b0.z; v[3] += b0.w; v[4] += b1.x; v[5] += b1.y; v[6] += b1.z; v[7] += b1.w;
  }
  if constexpr (ACT == ACT_GELU_TANH) {
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = gelu_tanh(bfround(v[e]));
  } else if constexpr (ACT == ACT_GELU_ERF) {
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = bfround(v[e]);
    if (p.aux) stbf8(p.aux + r * p.ld_aux + c, v);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = gelu_erf(v[e]);
  } else if constexpr (ACT == ACT_GELU_ERF_BWD) {
    float a[8];
    ldbf8(p.aux_in + r * p.ld_aux_in + c, a);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = bfround(v[e]) * gelu_erf_grad(a[e]);
  }
  const long cr = map_row(p.cmap, r);
  if (cr < 0) return;
  if (p.resid) {
    const float* rp = p.resid + cr * p.ld_resid + c;
    const float4 b0 = ldf4(rp), b1 = ldf4(rp + 4);
    v[0] += b0.x; v[1] += b0.y; v[2] += b0.z; v[3] += b0.w; v[4] += b1.x; v[5] += b1.y; v[6] += b1.z; v[7] += b1.w;
  }
  if (p.resid16) {
    float rr[8];
    ldbf8(p.resid16 + cr * p.ld_resid16 + c, rr);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] += rr[e];
  }
  stbf8(reinterpret_cast<bf16_t*>(Cz) + cr * p.ldc + c, v);
}

// scalar fallback for ragged column tails / unaligned leading dims
template <int ACT, int OUT>
PTK_DEV void epi_scalar(const GemmArgs& p, char* Cz, long r, long c, float v) {
  if (p.bias) v += p.bias[c];
  if (p.bf16_linear) v = bfround(v);
  if (p.rowadd) v += p.rowadd[(r % p.rowadd_period) * p.ld_rowadd + c];
  if constexpr (ACT == ACT_GELU_TANH) {
    v = gelu_tanh(bfround(v));
  } else if constexpr (ACT == ACT_GELU_ERF) {
    float a = bfround(v);
    if (p.aux) p.aux[r * p.ld_aux + c] = f2bf(a);
    v = gelu_erf(a);
  } else if constexpr (ACT == ACT_GELU_ERF_BWD) {
    v = bfround(v) * gelu_erf_grad(bf2f(p.aux_in[r * p.ld_aux_in + c]));
  }
  const long cr = map_row(p.cmap, r);
  if (cr < 0) return;
  if (p.resid) v += p.resid[cr * p.ld_resid + c];
  if (p.resid16) v += bf2f(p.resid16[cr * p.ld_resid16 + c]);
  if constexpr (OUT == OUT_BF16) {
    reinterpret_cast<bf16_t*>(Cz)[cr * p.ldc + c] = f2bf(v);
  } else if constexpr (OUT == OUT_F32) {
    reinterpret_cast<float*>(Cz)[cr * p.ldc + c] = v;
  } else {
    reinterpret_cast<float*>(Cz)[cr * p.ldc + c] = bfround(v);
  }
}

// GEGLU: GEMM cols [32q, 32q+16) = gate[16q..], [32q+16, 32q+32) = up[16q..] (interleaved
// weights); writes h = bf16(bf16(gelu_tanh(g)) * u) and the backward's bf16 factors a = gelu(g) (aux) and
// b = gelu'(g) * u (aux2) (common.h geglu_fwd2; TF gemma3 :131-133)
PTK_DEV void geglu_vec4(const GemmArgs& p, char* Cz, long r, long hc, float4 g, float4 u) {
  uint32_t a[2], b[2], h[2];
#pragma unroll
  for (int e = 0; e < 4; e += 2)
    geglu_fwd2(bfround2(f32x2_t{el(g, e), el(g, e + 1)}), bfround2(f32x2_t{el(u, e), el(u, e + 1)}), a[e / 2],
               b[e / 2], h[e / 2]);
  if (p.aux) *reinterpret_cast<uint2*>(p.aux + r * p.ld_aux + hc) = uint2{a[0], a[1]};
  if (p.aux2) *reinterpret_cast<uint2*>(p.aux2 + r * p.ld_aux + hc) = uint2{b[0], b[1]};
  const long cr = map_row(p.cmap, r);
  if (cr >= 0) *reinterpret_cast<uint2*>(reinterpret_cast<bf16_t*>(Cz) + cr * p.ldc + hc) = uint2{h[0], h[1]};
}

PTK_DEV void geglu_vec8(const GemmArgs& p, char* Cz, long r, long hc, const float* g, const float* u) {
  uint32_t a[4], b[4], h[4];
#pragma unroll
  for (int e = 0; e < 8; e += 2)
    geglu_fwd2(bfround2(f32x2_t{g[e], g[e + 1]}), bfround2(f32x2_t{u[e], u[e + 1]}), a[e / 2], b[e / 2], h[e / 2]);
  if (p.aux) *reinterpret_cast<uint4*>(p.aux + r * p.ld_aux + hc) = uint4{a[0], a[1], a[2], a[3]};
  if (p.aux2) *reinterpret_cast<uint4*>(p.aux2 + r * p.ld_aux + hc) = uint4{b[0], b[1], b[2], b[3]};
  const long cr = map_row(p.cmap, r);
  if (cr >= 0) *reinterpret_cast<uint4*>(reinterpret_cast<bf16_t*>(Cz) + cr * p.ldc + hc) = uint4{h[0], h[1], h[2], h[3]};
}

// GEGLU backward: GEMM output = dh [M, I]; the forward's factors a (aux_in), b (aux_in2); writes dg = dh * b,
// du = dh * a into the interleaved [M, 2I] layout
PTK_DEV void geglu_bwd_vec4(const GemmArgs& p, char* Cz, long r, long c, float4 dh) {
  const uint2 a = *reinterpret_cast<const uint2*>(p.aux_in + r * p.ld_aux_in + c);
  const uint2 b = *reinterpret_cast<const uint2*>(p.aux_in2 + r * p.ld_aux_in + c);
  float4 dg, du;
  f32x2_t g0, g1, u0, u1;
  geglu_bwd2(bfround2(f32x2_t{dh.x, dh.y}), a.x, b.x, g0, u0);
  geglu_bwd2(bfround2(f32x2_t{dh.z, dh.w}), a.y, b.y, g1, u1);
  dg = make_float4(g0.x, g0.y, g1.x, g1.y);
  du = make_float4(u0.x, u0.y, u1.x, u1.y);
  const long cr = map_row(p.cmap, r);
  if (cr < 0) return;
  bf16_t* C = reinterpret_cast<bf16_t*>(Cz) + cr * p.ldc + (c >> 4) * 32 + (c & 15);
  stbf4(C, dg);
  stbf4(C + 16, du);
}

// 8-wide GEGLU backward: 16-B loads of g, u and 16-B stores of dg, du (8 columns stay inside one
// 16-column interleave group)
PTK_DEV void geglu_bwd_vec8(const GemmArgs& p, char* Cz, long r, long c, const float* dh) {
  const uint4 a = *reinterpret_cast<const uint4*>(p.aux_in + r * p.ld_aux_in + c);
  const uint4 b = *reinterpret_cast<const uint4*>(p.aux_in2 + r * p.ld_aux_in + c);
  const uint32_t av[4] = {a.x, a.y, a.z, a.w}, bv[4] = {b.x, b.y, b.z, b.w};
  float dg[8], du[8];
#pragma unroll
  for (int e = 0; e < 8; e += 2) {
    f32x2_t x, y;
    geglu_bwd2(bfround2(f32x2_t{dh[e], dh[e + 1]}), av[e / 2], bv[e / 2], x, y);
    dg[e] = x.x;
    dg[e + 1] = x.y;
    du[e] = y.x;
    du[e + 1] = y.y;
  }
  const long cr = map_row(p.cmap, r);
  if (cr < 0) return;
  bf16_t* C = reinterpret_cast<bf16_t*>(Cz) + cr * p.ldc + (c >> 4) * 32 + (c & 15);
  stbf8(C, dg);
  stbf8(C + 16, du);
}


// exchange rows 1,3 of x with rows 0,2 of y (rows of 16 lanes): for two 16-column C^T MFMA tiles of
// the same C rows, lane row q then holds 8 consecutive columns 16(q&1) + 8(q>>1) + 0..7 (x: the
// first four, y: the last four)
PTK_DEV void swap16(f32x4_t& x, f32x4_t& y) {
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(x[e]), __float_as_uint(y[e]), false, false);
    x[e] = __uint_as_float(r[0]);
    y[e] = __uint_as_float(r[1]);
  }
}

}  // namespace ptk
