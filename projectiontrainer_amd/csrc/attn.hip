// Attention side kernels: fused q/k RMSNorm + RoPE (fwd/bwd) and masked row
// softmax (fwd/bwd).  The QK^T and PV contractions run on the MFMA GEMM.
//
// Gemma3Attention.forward (TF/models/gemma3/modeling_gemma3.py:341-383):
//   q,k = RMSNorm_hd(q,k) (scale 1+w, bf16 out) -> RoPE (rotate_half, fp32 cos/sin)
// masks: causal, key padding, sliding window kv > q - W (TF/masking_utils.py:92-101).
#include "common.h"
#include "ptk_internal.h"

namespace ptk {

// One wave per token m: every head of its fused qkv row (q heads, k heads, v heads), four heads'
// loads in flight at a time, the token's cos/sin and the q/k norm weights loaded once.  EPL =
// head_dim / 64 contiguous elements per lane; the RoPE partner i +- D/2 sits in lane ^ 32.
constexpr int QKR_HB = 4;   // heads per load batch

template <int EPL>
__global__ void __launch_bounds__(256) qknorm_rope_fwd_kernel(const bf16_t* __restrict__ qkv,
                                                              const float* __restrict__ qw,
                                                              const float* __restrict__ kw,
                                                              const float* __restrict__ cos_t,
                                                              const float* __restrict__ sin_t, AttnShape sh,
                                                              float eps, bf16_t* __restrict__ Q,
                                                              bf16_t* __restrict__ K, bf16_t* __restrict__ V,
                                                              float* __restrict__ rstd_q, float* __restrict__ rstd_k) {
  constexpr int D = EPL * 64;
  const int lane = threadIdx.x & 63;
  const int nh = sh.Hq + 2 * sh.Hkv;
  const long m = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (m >= (long)sh.B * sh.S) return;
  const int b = (int)(m / sh.S), s = (int)(m - (long)b * sh.S);
  const int G = sh.Hq / sh.Hkv;
  const int fi = (lane & 31) * EPL;   // frequency index (cos[i] == cos[i + D/2])
  const long ps = sh.pos ? (long)sh.pos[m] : (long)s;   // the generate path's position ids
  float cs[EPL], sn[EPL], wq[EPL], wk[EPL];
#pragma unroll
  for (int e = 0; e < EPL; ++e) {
    cs[e] = cos_t[ps * (D / 2) + fi + e];
    sn[e] = sin_t[ps * (D / 2) + fi + e];
    wq[e] = 1.f + qw[lane * EPL + e];
    wk[e] = 1.f + kw[lane * EPL + e];
  }
  const float sgn = lane < 32 ? -1.f : 1.f;
  const bf16_t* row = qkv + m * (long)nh * D + lane * EPL;
  for (int h0 = 0; h0 < nh; h0 += QKR_HB) {
    bf16_t raw[QKR_HB][EPL];
#pragma unroll
    for (int i = 0; i < QKR_HB; ++i)
      if (h0 + i < nh)
#pragma unroll
        for (int e = 0; e < EPL; ++e) raw[i][e] = row[(long)(h0 + i) * D + e];
#pragma unroll
    for (int i = 0; i < QKR_HB; ++i) {
      const int h = h0 + i;
      if (h >= nh) break;
      if (h >= sh.Hq + sh.Hkv) {   // v head: relayout only
        bf16_t* dst = V + (((long)b * sh.Hkv + (h - sh.Hq - sh.Hkv)) * sh.S + s) * D + lane * EPL;
#pragma unroll
        for (int e = 0; e < EPL; ++e) dst[e] = raw[i][e];
        continue;
      }
      const bool isq = h < sh.Hq;
      float x[EPL], ss = 0.f;
#pragma unroll
      for (int e = 0; e < EPL; ++e) {
        x[e] = bf2f(raw[i][e]);
        ss += x[e] * x[e];
      }
      const float rs = rsqrtf(warp_sum(ss) / D + eps);
      float xn[EPL], part[EPL];
#pragma unroll
      for (int e = 0; e < EPL; ++e) xn[e] = bfround(x[e] * rs * (isq ? wq[e] : wk[e]));
#pragma unroll
      for (int e = 0; e < EPL; ++e) part[e] = xor32_get(xn[e]);
      bf16_t* dst;
      if (isq) {
        const int kvh = h / G, j = h - kvh * G;
        dst = Q + ((((long)b * sh.Hkv + kvh) * sh.S + s) * G + j) * D + lane * EPL;
        if (lane == 0) rstd_q[m * sh.Hq + h] = rs;
      } else {
        const int kvh = h - sh.Hq;
        dst = K + (((long)b * sh.Hkv + kvh) * sh.S + s) * D + lane * EPL;
        if (lane == 0) rstd_k[m * sh.Hkv + kvh] = rs;
      }
#pragma unroll
      for (int e = 0; e < EPL; ++e) dst[e] = f2bf(xn[e] * cs[e] + sgn * part[e] * sn[e]);
    }
  }
}

template <int EPL>
__global__ void __launch_bounds__(256) qknorm_rope_bwd_kernel(
    const bf16_t* __restrict__ qkv, const float* __restrict__ qw, const float* __restrict__ kw,
    const float* __restrict__ cos_t, const float* __restrict__ sin_t, AttnShape sh, const float* __restrict__ rstd_q,
    const float* __restrict__ rstd_k, const bf16_t* __restrict__ dQ, const bf16_t* __restrict__ dK,
    const bf16_t* __restrict__ dV, bf16_t* __restrict__ dqkv, FlashBwdArgs fb) {
  constexpr int D = EPL * 64;
  const int lane = threadIdx.x & 63;
  const int nh = sh.Hq + 2 * sh.Hkv;
  const long m = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (m >= (long)sh.B * sh.S) return;
  const int b = (int)(m / sh.S), s = (int)(m - (long)b * sh.S);
  const int G = sh.Hq / sh.Hkv;
  // deferred dK/dV reduce (D = 256 split slabs): this token's key row still lives as fp32 partials;
  // sum them in piece order and round exactly like attn_dkv_reduce_kernel (bit-identical)
  const float* dkv_src = nullptr;
  int dkv_np = 0;
  if (D == 256 && fb.dkv_deferred) {
    const int slab = s / DKV_KEYS;
    const int P = dkv_pieces(fb, slab);
    if (P > 1) {
      dkv_np = P;
      dkv_src = fb.dkv_part + (long)dkv_part_base(fb, slab) * fb.nz * (2L * DKV_KEYS * D) +
                (long)(s - slab * DKV_KEYS) * D + lane * EPL;
    }
  }
  const int fi = (lane & 31) * EPL;
  float cs[EPL], sn[EPL], wq[EPL], wk[EPL];
#pragma unroll
  for (int e = 0; e < EPL; ++e) {
    cs[e] = cos_t[(long)s * (D / 2) + fi + e];
    sn[e] = sin_t[(long)s * (D / 2) + fi + e];
    wq[e] = 1.f + qw[lane * EPL + e];
    wk[e] = 1.f + kw[lane * EPL + e];
  }
  // rot^T(v)_i = v_{i+D/2} (i < D/2), -v_{i-D/2} (i >= D/2)
  const float sgn = lane < 32 ? 1.f : -1.f;
  const bf16_t* xrow = qkv + m * (long)nh * D + lane * EPL;
  bf16_t* orow = dqkv + m * (long)nh * D + lane * EPL;
  for (int h0 = 0; h0 < nh; h0 += QKR_HB) {
    bf16_t gy[QKR_HB][EPL], xr[QKR_HB][EPL];
    float rsv[QKR_HB];
#pragma unroll
    for (int i = 0; i < QKR_HB; ++i) {
      const int h = h0 + i;
      if (h >= nh) break;
      const bf16_t* dy;
      if (h < sh.Hq) {
        const int kvh = h / G, j = h - kvh * G;
        dy = dQ + ((((long)b * sh.Hkv + kvh) * sh.S + s) * G + j) * D + lane * EPL;
        rsv[i] = rstd_q[m * sh.Hq + h];
      } else if (h < sh.Hq + sh.Hkv) {
        const int kvh = h - sh.Hq;
        dy = dK + (((long)b * sh.Hkv + kvh) * sh.S + s) * D + lane * EPL;
        rsv[i] = rstd_k[m * sh.Hkv + kvh];
      } else {
        dy = dV + (((long)b * sh.Hkv + (h - sh.Hq - sh.Hkv)) * sh.S + s) * D + lane * EPL;
        rsv[i] = 0.f;
      }
      if (dkv_np > 0 && h >= sh.Hq) {
        const int which = h < sh.Hq + sh.Hkv ? 0 : 1;   // 0 = dK, 1 = dV
        const int kvh = which == 0 ? h - sh.Hq : h - sh.Hq - sh.Hkv;
        const long z = (long)b * sh.Hkv + kvh;
        const float* src = dkv_src + z * (2L * DKV_KEYS * D) + (long)which * DKV_KEYS * D;
        const long pstride = (long)fb.nz * (2L * DKV_KEYS * D);
        float acc[EPL];
#pragma unroll
        for (int e = 0; e < EPL; ++e) acc[e] = 0.f;
        for (int pc = 0; pc < dkv_np; ++pc) {
#pragma unroll
          for (int e = 0; e < EPL; ++e) acc[e] += src[pc * pstride + e];
        }
        const float mul = which == 0 ? fb.scale : 1.f;
#pragma unroll
        for (int e = 0; e < EPL; ++e) gy[i][e] = f2bf(acc[e] * mul);
      } else {
#pragma unroll
        for (int e = 0; e < EPL; ++e) gy[i][e] = dy[e];
      }
      if (h < sh.Hq + sh.Hkv)
#pragma unroll
        for (int e = 0; e < EPL; ++e) xr[i][e] = xrow[(long)h * D + e];
    }
#pragma unroll
    for (int i = 0; i < QKR_HB; ++i) {
      const int h = h0 + i;
      if (h >= nh) break;
      bf16_t* out = orow + (long)h * D;
      if (h >= sh.Hq + sh.Hkv) {
#pragma unroll
        for (int e = 0; e < EPL; ++e) out[e] = gy[i][e];
        continue;
      }
      const bool isq = h < sh.Hq;
      const float rs = rsv[i];
      float ds[EPL], dc[EPL], part[EPL];
#pragma unroll
      for (int e = 0; e < EPL; ++e) {
        const float g = bf2f(gy[i][e]);
        dc[e] = g * cs[e];
        ds[e] = g * sn[e];
      }
#pragma unroll
      for (int e = 0; e < EPL; ++e) part[e] = xor32_get(ds[e]);
      float x[EPL], dxn[EPL];
      float sdot = 0.f;
#pragma unroll
      for (int e = 0; e < EPL; ++e) {
        x[e] = bf2f(xr[i][e]);
        dxn[e] = bfround(dc[e] + sgn * part[e]) * (isq ? wq[e] : wk[e]);
        sdot += dxn[e] * x[e];
      }
      sdot = warp_sum(sdot);
      const float c3 = rs * rs * rs * sdot / D;
#pragma unroll
      for (int e = 0; e < EPL; ++e) out[e] = f2bf(rs * dxn[e] - c3 * x[e]);
    }
  }
}

constexpr int SMAXV = 8;   // float4 per lane -> cols <= 2048

__global__ void __launch_bounds__(256) softmax_fwd_kernel(const float* __restrict__ S, bf16_t* __restrict__ P,
                                                          long nrows, int rows, int cols, long ld, MaskSpec mk) {
  const int lane = threadIdx.x & 63;
  const long gr = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (gr >= nrows) return;
  const long z = gr / rows;
  const int r = (int)(gr - z * rows);
  const int q = (r % mk.rows_per_batch) / mk.qdiv;
  const long b = z / mk.zdiv;
  const float* srow = S + gr * ld;
  bf16_t* prow = P + gr * ld;
  float4 v[SMAXV];
  float mx = -INFINITY;
#pragma unroll
  for (int i = 0; i < SMAXV; ++i) {
    const int c0 = lane * 4 + i * 256;
    if (c0 >= cols) break;
    float4 t = *reinterpret_cast<const float4*>(srow + c0);
    float tv[4] = {t.x, t.y, t.z, t.w};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int k = c0 + e;
      bool ok = mk.key_valid ? (mk.key_valid[b * cols + k] != 0) : (k < mk.key_len);
      if (mk.causal) ok = ok && (k <= q);
      if (mk.window) ok = ok && (k > q - mk.window);
      tv[e] = ok ? tv[e] : -INFINITY;
      mx = fmaxf(mx, tv[e]);
    }
    v[i] = make_float4(tv[0], tv[1], tv[2], tv[3]);
  }
  mx = warp_max(mx);
  float sum = 0.f;
#pragma unroll
  for (int i = 0; i < SMAXV; ++i) {
    const int c0 = lane * 4 + i * 256;
    if (c0 >= cols) break;
    float4 t = v[i];
    t.x = t.x == -INFINITY ? 0.f : __expf(t.x - mx);
    t.y = t.y == -INFINITY ? 0.f : __expf(t.y - mx);
    t.z = t.z == -INFINITY ? 0.f : __expf(t.z - mx);
    t.w = t.w == -INFINITY ? 0.f : __expf(t.w - mx);
    v[i] = t;
    sum += t.x + t.y + t.z + t.w;
  }
  sum = warp_sum(sum);
  const float inv = sum > 0.f ? 1.f / sum : 0.f;
#pragma unroll
  for (int i = 0; i < SMAXV; ++i) {
    const int c0 = lane * 4 + i * 256;
    if (c0 >= cols) break;
    u16x4_t o;
    o[0] = f2bf(v[i].x * inv); o[1] = f2bf(v[i].y * inv); o[2] = f2bf(v[i].z * inv); o[3] = f2bf(v[i].w * inv);
    *reinterpret_cast<u16x4_t*>(prow + c0) = o;
  }
}

__global__ void __launch_bounds__(256) softmax_bwd_kernel(const bf16_t* __restrict__ P, const float* __restrict__ dP,
                                                          bf16_t* __restrict__ dS, long nrows, int cols, long ld,
                                                          float scale) {
  const int lane = threadIdx.x & 63;
  const long gr = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (gr >= nrows) return;
  float4 pv[SMAXV], gv[SMAXV];
  float dot = 0.f;
#pragma unroll
  for (int i = 0; i < SMAXV; ++i) {
    const int c0 = lane * 4 + i * 256;
    if (c0 >= cols) break;
    u16x4_t u = *reinterpret_cast<const u16x4_t*>(P + gr * ld + c0);
    pv[i] = make_float4(bf2f(u[0]), bf2f(u[1]), bf2f(u[2]), bf2f(u[3]));
    gv[i] = *reinterpret_cast<const float4*>(dP + gr * ld + c0);
    dot += pv[i].x * gv[i].x + pv[i].y * gv[i].y + pv[i].z * gv[i].z + pv[i].w * gv[i].w;
  }
  dot = warp_sum(dot);
#pragma unroll
  for (int i = 0; i < SMAXV; ++i) {
    const int c0 = lane * 4 + i * 256;
    if (c0 >= cols) break;
    u16x4_t o;
    o[0] = f2bf(pv[i].x * (gv[i].x - dot) * scale);
    o[1] = f2bf(pv[i].y * (gv[i].y - dot) * scale);
    o[2] = f2bf(pv[i].z * (gv[i].z - dot) * scale);
    o[3] = f2bf(pv[i].w * (gv[i].w - dot) * scale);
    *reinterpret_cast<u16x4_t*>(dS + gr * ld + c0) = o;
  }
}

#define QKR_DISPATCH(KERNEL, ...)                                                                     \
  switch (s.D) {                                                                                      \
    case 64: hipLaunchKernelGGL(KERNEL<1>, grid, dim3(256), 0, st, __VA_ARGS__); break;              \
    case 128: hipLaunchKernelGGL(KERNEL<2>, grid, dim3(256), 0, st, __VA_ARGS__); break;             \
    case 256: hipLaunchKernelGGL(KERNEL<4>, grid, dim3(256), 0, st, __VA_ARGS__); break;             \
    default: return set_error("qknorm_rope: head_dim %d unsupported", s.D);                          \
  }

int launch_qknorm_rope_fwd(const bf16_t* qkv, const float* qw, const float* kw, const float* cos_t,
                           const float* sin_t, AttnShape s, float eps, bf16_t* Q, bf16_t* K, bf16_t* V,
                           float* rstd_q, float* rstd_k, hipStream_t st) {
  if (s.Hq % s.Hkv) return set_error("qknorm_rope: Hq %% Hkv != 0");
  const long waves = (long)s.B * s.S;   // one wave per token
  dim3 grid((unsigned)((waves + 3) / 4));
  QKR_DISPATCH(qknorm_rope_fwd_kernel, qkv, qw, kw, cos_t, sin_t, s, eps, Q, K, V, rstd_q, rstd_k)
  return hipGetLastError() == hipSuccess ? 0 : set_error("qknorm_rope_fwd launch failed");
}
int launch_qknorm_rope_bwd(const bf16_t* qkv, const float* qw, const float* kw, const float* cos_t,
                           const float* sin_t, AttnShape s, const float* rstd_q, const float* rstd_k,
                           const bf16_t* dQ, const bf16_t* dK, const bf16_t* dV, bf16_t* dqkv, hipStream_t st,
                           const FlashBwdArgs* dkv) {
  if (s.Hq % s.Hkv) return set_error("qknorm_rope: Hq %% Hkv != 0");
  FlashBwdArgs fb;
  fb.dkv_deferred = 0;
  if (dkv && dkv->dkv_deferred) {
    if (s.D != 256 || dkv->D != 256 || dkv->nkeys != s.S || dkv->nz != s.B * s.Hkv || !dkv->dkv_part)
      return set_error("qknorm_rope_bwd: deferred dK/dV plan does not match the shape");
    fb = *dkv;
  }
  const long waves = (long)s.B * s.S;   // one wave per token
  dim3 grid((unsigned)((waves + 3) / 4));
  QKR_DISPATCH(qknorm_rope_bwd_kernel, qkv, qw, kw, cos_t, sin_t, s, rstd_q, rstd_k, dQ, dK, dV, dqkv, fb)
  return hipGetLastError() == hipSuccess ? 0 : set_error("qknorm_rope_bwd launch failed");
}
int launch_softmax_fwd(const float* S, bf16_t* P, int nz, int rows, int cols, long ld, MaskSpec m, hipStream_t st) {
  if (cols % 4 || cols > SMAXV * 256 || ld % 4) return set_error("softmax: cols=%d unsupported", cols);
  const long nrows = (long)nz * rows;
  if (nrows <= 0) return 0;
  hipLaunchKernelGGL(softmax_fwd_kernel, dim3((unsigned)((nrows + 3) / 4)), dim3(256), 0, st, S, P, nrows, rows,
                     cols, ld, m);
  return hipGetLastError() == hipSuccess ? 0 : set_error("softmax_fwd launch failed");
}
int launch_softmax_bwd(const bf16_t* P, const float* dP, bf16_t* dS, int nrows, int cols, long ld, float scale,
                       hipStream_t st) {
  if (cols % 4 || cols > SMAXV * 256 || ld % 4) return set_error("softmax_bwd: cols=%d unsupported", cols);
  if (nrows <= 0) return 0;
  hipLaunchKernelGGL(softmax_bwd_kernel, dim3((unsigned)((nrows + 3) / 4)), dim3(256), 0, st, P, dP, dS,
                     (long)nrows, cols, ld, scale);
  return hipGetLastError() == hipSuccess ? 0 : set_error("softmax_bwd launch failed");
}

}  // namespace ptk
