// Shared device helpers for libptk (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef uint16_t bf16_t;                                         // raw bf16 bits
typedef __attribute__((ext_vector_type(8))) short bf16x8_t;      // MFMA A/B fragment
typedef __attribute__((ext_vector_type(4))) float f32x4_t;       // 16x16 accumulator
typedef __attribute__((ext_vector_type(4))) unsigned short u16x4_t;
typedef __attribute__((ext_vector_type(8))) unsigned short u16x8_t;

#define PTK_DEV __device__ __forceinline__

PTK_DEV float bf2f(bf16_t h) { return __uint_as_float(((uint32_t)h) << 16); }

// round-to-nearest-even f32 -> bf16 (NaN stays NaN): one v_cvt_pk_bf16_f32 (adjacent pairs pack)
PTK_DEV bf16_t f2bf(float f) { return __builtin_bit_cast(bf16_t, (__bf16)f); }
PTK_DEV float bfround(float f) { return bf2f(f2bf(f)); }

// lane ^ 32 / lane ^ 16 exchanges without the LDS crossbar (__shfl_xor lowers to ds_bpermute for
// these): v_permlane32_swap / v_permlane16_swap of a register with itself returns the partner's value
// in one of the two results and the lane's own in the other, so op(r0, r1) is the butterfly step
PTK_DEV float xor32_sum(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
PTK_DEV float xor16_sum(float v) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
PTK_DEV float xor32_max(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
PTK_DEV float xor16_max(float v) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}

// the value of lane ^ 32 (ds_bpermute; only used by HBM-bound kernels)
PTK_DEV float xor32_get(float v) { return __shfl_xor(v, 32, 64); }

// within a 16-lane row: DPP butterflies (quad_perm [1,0,3,2], [2,3,0,1], row_half_mirror, row_mirror);
// after each step every lane of the group holds the group's result
template <int CTRL>
PTK_DEV float dpp(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, false));
}
PTK_DEV float row_sum16(float v) {
  v += dpp<0xB1>(v);
  v += dpp<0x4E>(v);
  v += dpp<0x141>(v);
  v += dpp<0x140>(v);
  return v;
}
PTK_DEV float row_max16(float v) {
  v = fmaxf(v, dpp<0xB1>(v));
  v = fmaxf(v, dpp<0x4E>(v));
  v = fmaxf(v, dpp<0x141>(v));
  v = fmaxf(v, dpp<0x140>(v));
  return v;
}
PTK_DEV float warp_sum(float v) { return xor32_sum(xor16_sum(row_sum16(v))); }
PTK_DEV float warp_max(float v) { return xor32_max(xor16_max(row_max16(v))); }

// block-wide sum for blockDim.x == NT (multiple of 64); `red` holds NT/64 floats
template <int NT>
PTK_DEV float block_sum(float v, float* red) {
  v = warp_sum(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  __syncthreads();
  if (l == 0) red[w] = v;
  __syncthreads();
  float t = 0.f;
#pragma unroll
  for (int i = 0; i < NT / 64; ++i) t += red[i];
  return t;
}
template <int NT>
PTK_DEV float block_max(float v, float* red) {
  v = warp_max(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  __syncthreads();
  if (l == 0) red[w] = v;
  __syncthreads();
  float t = -INFINITY;
#pragma unroll
  for (int i = 0; i < NT / 64; ++i) t = fmaxf(t, red[i]);
  return t;
}

// GELU variants (TF/activations.py: gelu_pytorch_tanh; torch nn.GELU default = erf)
// 0.5 * (1 + tanh(u)) == sigmoid(2u): one exp + one reciprocal instead of tanhf
// x * sigmoid(2u) = 0.5 x (1 + tanh(u)) with one v_exp_f32 and one v_rcp_f32 (hipcc lowers
// __fdividef to the IEEE division sequence, 8 instructions: the GEGLU epilogue's largest cost)
PTK_DEV float fast_sigmoid2(float u) {   // 1 / (1 + e^(-2u)); e^(-2u) -> inf gives 0, -> 0 gives 1
  return __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(u * -2.8853900817779268f));
}
PTK_DEV float gelu_tanh_arg(float x, float x2) {   // u = k0 (x + k1 x^3), one evaluation order everywhere
  return 0.7978845608028654f * (x + 0.044715f * x2 * x);
}
PTK_DEV float gelu_tanh(float x) { return x * fast_sigmoid2(gelu_tanh_arg(x, x * x)); }
// two lanes of gelu_tanh with packed f32 math (v_pk_mul / v_pk_fma: half the VALU issue of the scalar
// form; for epilogues, where no MFMA of the wave runs beside them)
typedef __attribute__((ext_vector_type(2))) float f32x2_t;
PTK_DEV f32x2_t gelu_tanh2(f32x2_t x) {   // e^(-2u) = exp2(x (c1 + c2 x^2)), factored as in gelu_tanh_fg2
  constexpr float k0 = 0.7978845608028654f, k1 = 0.044715f, l2e2 = -2.8853900817779268f;
  const f32x2_t a = x * ((x * x) * (k0 * k1 * l2e2) + k0 * l2e2);
  const f32x2_t e = f32x2_t{__builtin_amdgcn_exp2f(a.x), __builtin_amdgcn_exp2f(a.y)} + 1.f;
  return x * f32x2_t{__builtin_amdgcn_rcpf(e.x), __builtin_amdgcn_rcpf(e.y)};
}
// gelu_tanh and its derivative from one exp / rcp pair (the GEGLU backward needs both)
PTK_DEV void gelu_tanh_fg(float x, float& f, float& df) {
  const float k0 = 0.7978845608028654f, k1 = 0.044715f;
  const float x2 = x * x;
  const float s = fast_sigmoid2(gelu_tanh_arg(x, x2));
  f = x * s;
  df = s + 2.f * x * s * (1.f - s) * k0 * (1.f + 3.f * k1 * x2);
}
// gelu_tanh_fg on two lanes with packed f32 math (v_pk_mul / v_pk_fma for everything but the exp / rcp),
// the polynomial factored for the fewest packed operations:
//   e^(-2u) = exp2(x (c1 + c2 x^2)),  f = x s,  f' = s + f (1 - s) (2 k0 + 6 k0 k1 x^2)
// (the same function as gelu_tanh_fg up to fp32 rounding; epilogues only: beside MFMAs packed f32 is an
// anti-lever, MI355X_MICROARCH.md)
PTK_DEV void gelu_tanh_fg2(f32x2_t x, f32x2_t& f, f32x2_t& df) {
  constexpr float k0 = 0.7978845608028654f, k1 = 0.044715f, l2e2 = -2.8853900817779268f;
  const f32x2_t x2 = x * x;
  const f32x2_t a = x * (x2 * (k0 * k1 * l2e2) + k0 * l2e2);
  const f32x2_t e = f32x2_t{__builtin_amdgcn_exp2f(a.x), __builtin_amdgcn_exp2f(a.y)} + 1.f;
  const f32x2_t s = f32x2_t{__builtin_amdgcn_rcpf(e.x), __builtin_amdgcn_rcpf(e.y)};
  f = x * s;
  const f32x2_t q = f - f * s;                              // f (1 - s)
  df = q * (x2 * (6.f * k0 * k1) + 2.f * k0) + s;
}
// bf16 round trip of two lanes: one v_cvt_pk_bf16_f32 and two unpacks
typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2_t;
// IEEE 754-2019 maximum (NaN-propagating): v_maximum3_f32 / v_maximum_f32 on gfx950, without the operand
// canonicalisation fmaxf (maxNum) costs in IEEE mode
PTK_DEV float fmaxe(float a, float b) { return __builtin_elementwise_maximum(a, b); }
PTK_DEV float fmax3e(float a, float b, float c) { return fmaxe(fmaxe(a, b), c); }
PTK_DEV f32x2_t bfround2(f32x2_t v) {
  const uint32_t u = __builtin_bit_cast(uint32_t, __builtin_convertvector(v, bf16x2_t));
  return f32x2_t{__uint_as_float(u << 16), __uint_as_float(u & 0xffff0000u)};
}
// two bf16 packed in a dword (element 0 in the low half) -> two f32
PTK_DEV f32x2_t bf2x2(uint32_t w) { return f32x2_t{__uint_as_float(w << 16), __uint_as_float(w & 0xffff0000u)}; }
PTK_DEV uint32_t pkbf2(f32x2_t v) { return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, bf16x2_t)); }

// GEGLU (TF gemma3 :131-133: h = gelu_tanh(gate) * up, bf16 ops) from the bf16-rounded g, u of two lanes, with the
// two bf16 factors its backward needs saved instead of g and u:
//   a = bf16(gelu(g))            (du = bf16(dh * a): the reference's MulBackward on the bf16 act output)
//   b = bf16(gelu'(g) * u)       (dg = bf16(dh * b); the reference rounds bf16(dh * u) before gelu', so dg differs
//                                 from it by which of the two products is rounded -- one bf16 rounding either way)
//   h = bf16(a * u)
// so the backward epilogue is two multiplies per element, no transcendental (the tanh-GELU value and derivative
// come from the forward's one exp / rcp pair, gelu_tanh_fg2).  Packed dwords, element 0 in the low half.
PTK_DEV void geglu_fwd2(f32x2_t g, f32x2_t u, uint32_t& a, uint32_t& b, uint32_t& h) {
  f32x2_t f, df;
  gelu_tanh_fg2(g, f, df);
  a = pkbf2(f);
  h = pkbf2(bf2x2(a) * u);
  b = pkbf2(df * u);
}
// the backward from the saved factors: dg = dh * b, du = dh * a (dh already bf16-rounded; stored rounded)
PTK_DEV void geglu_bwd2(f32x2_t d, uint32_t a, uint32_t b, f32x2_t& dg, f32x2_t& du) {
  dg = d * bf2x2(b);
  du = d * bf2x2(a);
}
PTK_DEV float gelu_tanh_grad(float x) {
  float f, df;
  gelu_tanh_fg(x, f, df);
  return df;
}
PTK_DEV float gelu_erf(float x) { return 0.5f * x * (1.f + erff(x * 0.7071067811865476f)); }
PTK_DEV float gelu_erf_grad(float x) {
  return 0.5f * (1.f + erff(x * 0.7071067811865476f)) + x * 0.3989422804014327f * __expf(-0.5f * x * x);
}

// Row remap r -> (r / g) * gs + (r % g) + off   (g == 0: identity)
struct RowMap {
  int g;
  int skip;      // rows with (r % g) < skip map to -1 (not stored)
  long gs;
  long off;
};
PTK_DEV long map_row(const RowMap& m, long r) {
  if (m.g == 0) return r + m.off;
  long q = r / m.g, s = r - q * m.g;
  if (s < m.skip) return -1;
  return q * m.gs + s + m.off;
}
