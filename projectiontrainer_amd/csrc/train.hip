// Kernels of the unfrozen-LLM step (Stage 2, BASELINE cfg4): the weight-gradient plumbing around the
// MFMA GEMMs and the bf16 optimizer.  All HBM-bound.
//
//   transpose_rows     token-major activations / output grads -> feature-major operands of dW = dY^T X
//                      (the GEMM contracts K-contiguous rows; K is the token axis here)
//   rms_wgrad          Gemma3RMSNorm weight grads: dw[c] = sum_r dy[r,c] * x[r,c] * rstd[r]
//                      (modeling_gemma3.py:136-150, output (x * rstd) * (1 + w))
//   qknorm_wgrad       q_norm / k_norm weight grads through the rotate-half RoPE (:356-360, :208-258)
//   embed_grad         input-embedding grads of the question / answer tokens
//                      (Stage2/trainer.py:351-360: weight[ids] * embed_scale), summed per token id
//   scale_sumsq / adamw_bf16
//                      clip_grad_norm_(1.0) + torch.optim.AdamW over bf16 parameters, every tensor op
//                      rounded to bf16 as torch's single-tensor AdamW does on bf16 params
//                      (Stage2/trainer.py:145-149, :426-443; the LLM is loaded in bf16 under
//                      --mixed_precision bf16, train_vqa_stage2.py:141-147,180-187)
#include <math.h>

#include "common.h"
#include "ptk_internal.h"

namespace ptk {

#define RET_OK(name) return hipGetLastError() == hipSuccess ? 0 : set_error(name " launch failed")

// ---------------------------------------------------------------- transpose with a row gather
// out [cols][rows_pad] = in[map(r)][c] for r < rows, 0 for rows <= r < rows_pad.  64x64 LDS tiles.
__global__ void __launch_bounds__(256) transpose_rows_kernel(const bf16_t* __restrict__ in, long ld_in, RowMap map,
                                                             int rows, int cols, bf16_t* __restrict__ out,
                                                             long ld_out, int rows_pad) {
  __shared__ bf16_t tile[64][66];
  const int r0 = blockIdx.y * 64, c0 = blockIdx.x * 64;
  const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int r = r0 + ty + 16 * k;
    const int c = c0 + tx * 4;
    u16x4_t v = {0, 0, 0, 0};
    if (r < rows) {
      const long sr = map_row(map, r);
      const bf16_t* src = in + sr * ld_in;
      if (c + 3 < cols && ((ld_in & 3) == 0)) {
        v = *reinterpret_cast<const u16x4_t*>(src + c);
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = (c + e < cols) ? src[c + e] : 0;
      }
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) tile[ty + 16 * k][tx * 4 + e] = v[e];
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int oc = c0 + ty + 16 * k;
    const int orr = r0 + tx * 4;
    if (oc >= cols || orr >= rows_pad) continue;
    u16x4_t v;
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = tile[tx * 4 + e][ty + 16 * k];
    if (orr + 3 < rows_pad && ((ld_out & 3) == 0)) {
      *reinterpret_cast<u16x4_t*>(out + (long)oc * ld_out + orr) = v;
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (orr + e < rows_pad) out[(long)oc * ld_out + orr + e] = v[e];
    }
  }
}

int launch_transpose_rows(const bf16_t* in, long ld_in, RowMap map, int rows, int cols, bf16_t* out, long ld_out,
                          int rows_pad, hipStream_t st) {
  if (cols <= 0 || rows_pad <= 0) return 0;
  if (rows_pad < rows) return set_error("transpose_rows: rows_pad < rows");
  dim3 grid((unsigned)((cols + 63) / 64), (unsigned)((rows_pad + 63) / 64));
  hipLaunchKernelGGL(transpose_rows_kernel, grid, dim3(256), 0, st, in, ld_in, map, rows, cols, out, ld_out, rows_pad);
  RET_OK("transpose_rows");
}

// ---------------------------------------------------------------- RMSNorm weight grads
// partial[blk][c] = sum over the block's rows of dy[r,c] * x[xmap(r),c] * rstd[r]; dy optionally rounded to
// bf16 first (the post-norms' output grads arrive as bf16 in the reference's autocast graph).
// 256 threads own float4 column groups c = 4 t + 1024 j; WG_ROWS rows per block, split over WG_GROUPS row groups.
// One group of 256 threads per 32-row block (448 blocks at cfg4's 14 336 rows, 7 waves per CU) streamed at
// ~2.6 TB/s; 8-row blocks (4x the waves) took cfg4 161.3 -> 163.4 img/s, and 4 row groups per 32-row block (the
// same waves, a quarter of the partial rows, one colsum level less) +0.4 % more (profiles/r05_wgrad_rows_ab.txt)
#ifndef PTK_WG_ROWS
#define PTK_WG_ROWS 32
#endif
#ifndef PTK_WG_GROUPS
#define PTK_WG_GROUPS 4
#endif
constexpr int WG_GROUPS = PTK_WG_GROUPS;
constexpr int WG_ROWS = PTK_WG_ROWS;
PTK_DEV float4 ldv4(const float* p) { return *reinterpret_cast<const float4*>(p); }
PTK_DEV float4 ldv4(const bf16_t* p) {
  u16x4_t u = *reinterpret_cast<const u16x4_t*>(p);
  return make_float4(bf2f(u[0]), bf2f(u[1]), bf2f(u[2]), bf2f(u[3]));
}

template <typename TX, typename TD, int NJ>
__global__ void __launch_bounds__(256 * WG_GROUPS) rms_wgrad_partial_kernel(const TX* __restrict__ x, long ldx,
                                                                            RowMap xmap, const float* __restrict__ rstd,
                                                                            const TD* __restrict__ dy, long lddy,
                                                                            int dy_round, int rows, int cols,
                                                                            float* __restrict__ partial) {
  // WG_GROUPS row groups of 256 threads: group g sums rows r0 + g, r0 + g + WG_GROUPS, ... of the block's WG_ROWS
  // (more waves per CU on the memory stream without more partial rows), then the groups' sums are added in group
  // order through LDS
  __shared__ float4 red[WG_GROUPS > 1 ? WG_GROUPS - 1 : 1][NJ][256];
  const int t = threadIdx.x & 255, grp = threadIdx.x >> 8;
  float4 acc[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) acc[j] = make_float4(0.f, 0.f, 0.f, 0.f);
  const int r0 = blockIdx.x * WG_ROWS, r1 = min(rows, r0 + WG_ROWS);
  for (int r = r0 + grp; r < r1; r += WG_GROUPS) {
    const float rs = rstd[r];
    const TX* xr = x + map_row(xmap, r) * ldx;
    const TD* dr = dy + (long)r * lddy;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int c = t * 4 + 1024 * j;
      if (c < cols) {
        float4 xv = ldv4(xr + c), dv = ldv4(dr + c);
        if (dy_round) dv = make_float4(bfround(dv.x), bfround(dv.y), bfround(dv.z), bfround(dv.w));
        acc[j].x += dv.x * xv.x * rs;
        acc[j].y += dv.y * xv.y * rs;
        acc[j].z += dv.z * xv.z * rs;
        acc[j].w += dv.w * xv.w * rs;
      }
    }
  }
  if constexpr (WG_GROUPS > 1) {
    if (grp > 0)
#pragma unroll
      for (int j = 0; j < NJ; ++j) red[grp - 1][j][t] = acc[j];
    __syncthreads();
    if (grp > 0) return;
#pragma unroll
    for (int g = 0; g < WG_GROUPS - 1; ++g)
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const float4 v = red[g][j][t];
        acc[j].x += v.x; acc[j].y += v.y; acc[j].z += v.z; acc[j].w += v.w;
      }
  }
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int c = t * 4 + 1024 * j;
    if (c < cols) *reinterpret_cast<float4*>(partial + (long)blockIdx.x * cols + c) = acc[j];
  }
}

// grad[c] = bf16(grad[c] + bf16(sum_b partial[b][c]))   (autograd accumulation into a bf16 .grad).
// Two stages, fixed order: colsum16 folds groups of 16 partial rows (64 columns x 4 row-groups per block,
// coalesced), repeated until at most 16 rows remain; wgrad_finish sums those and accumulates.
__global__ void __launch_bounds__(256) colsum16_kernel(const float* __restrict__ in, int rows, int cols,
                                                       float* __restrict__ out) {
  __shared__ float red[4][64];
  const int cl = threadIdx.x & 63, grp = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cl, r0 = blockIdx.y * 16;
  float s = 0.f;
  if (c < cols)
    for (int r = r0 + grp; r < min(rows, r0 + 16); r += 4) s += in[(long)r * cols + c];
  red[grp][cl] = s;
  __syncthreads();
  if (grp == 0 && c < cols) out[(long)blockIdx.y * cols + c] = (red[0][cl] + red[1][cl]) + (red[2][cl] + red[3][cl]);
}

__global__ void __launch_bounds__(256) wgrad_finish_kernel(const float* __restrict__ partial, int nblk, int cols,
                                                           bf16_t* __restrict__ grad) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= cols) return;
  float s = 0.f;
  for (int b = 0; b < nblk; ++b) s += partial[(long)b * cols + c];
  grad[c] = f2bf(bf2f(grad[c]) + bfround(s));
}

// nblk <= 256 in one launch: 16 row groups x 64 columns per 1024-thread block, group g sums rows g, g + 16, ...
// (all its loads in flight at once), the groups added in order through LDS, then the bf16 accumulate.  Replaces
// the last colsum16 fold + wgrad_finish (two latency-bound launches of ~5 us each on cfg4's 4-row norm partials)
__global__ void __launch_bounds__(1024) wgrad_finish16_kernel(const float* __restrict__ partial, int nblk, int cols,
                                                              bf16_t* __restrict__ grad) {
  __shared__ float red[16][64];
  const int cl = threadIdx.x & 63, grp = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cl;
  float v[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int r = grp + 16 * i;
    v[i] = (c < cols && r < nblk) ? partial[(long)r * cols + c] : 0.f;
  }
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 16; ++i) s += v[i];
  red[grp][cl] = s;
  __syncthreads();
  if (grp == 0 && c < cols) {
    float t = red[0][cl];
#pragma unroll
    for (int g = 1; g < 16; ++g) t += red[g][cl];
    grad[c] = f2bf(bf2f(grad[c]) + bfround(t));
  }
}

#ifndef PTK_FINISH16
#define PTK_FINISH16 1
#endif
// partial [nblk][cols] -> grad; `scratch` holds ceil(nblk/16) * cols floats (the folded rows ping-pong in
// partial's own head and scratch)
static void wgrad_finish(float* partial, int nblk, int cols, bf16_t* grad, float* scratch, hipStream_t st) {
  float* src = partial;
  float* dst = scratch;
  if (PTK_FINISH16) {
    while (nblk > 256) {
      const int n2 = (nblk + 15) / 16;
      hipLaunchKernelGGL(colsum16_kernel, dim3((unsigned)((cols + 63) / 64), (unsigned)n2), dim3(256), 0, st, src,
                         nblk, cols, dst);
      std::swap(src, dst);
      nblk = n2;
    }
    hipLaunchKernelGGL(wgrad_finish16_kernel, dim3((unsigned)((cols + 63) / 64)), dim3(1024), 0, st, src, nblk, cols,
                       grad);
    return;
  }
  while (nblk > 16) {
    const int n2 = (nblk + 15) / 16;
    hipLaunchKernelGGL(colsum16_kernel, dim3((unsigned)((cols + 63) / 64), (unsigned)n2), dim3(256), 0, st, src, nblk,
                       cols, dst);
    std::swap(src, dst);
    nblk = n2;
  }
  hipLaunchKernelGGL(wgrad_finish_kernel, dim3((unsigned)((cols + 255) / 256)), dim3(256), 0, st, src, nblk, cols,
                     grad);
}

template <typename TX, typename TD>
static int rms_wgrad_t(const TX* x, long ldx, RowMap xmap, const float* rstd, const TD* dy, long lddy, int dy_round,
                       int rows, int cols, bf16_t* grad, float* partial, hipStream_t st) {
  if (rows <= 0) return 0;
  if (cols % 4 || cols > 4096) return set_error("rms_wgrad: cols %d (multiple of 4, <= 4096)", cols);
  const int nblk = (rows + WG_ROWS - 1) / WG_ROWS;
  const int nj = (cols + 1023) / 1024;
  const dim3 g((unsigned)nblk);
  switch (nj) {
    case 1: hipLaunchKernelGGL((rms_wgrad_partial_kernel<TX, TD, 1>), g, dim3(256 * WG_GROUPS), 0, st, x, ldx, xmap, rstd, dy, lddy, dy_round, rows, cols, partial); break;
    case 2: hipLaunchKernelGGL((rms_wgrad_partial_kernel<TX, TD, 2>), g, dim3(256 * WG_GROUPS), 0, st, x, ldx, xmap, rstd, dy, lddy, dy_round, rows, cols, partial); break;
    case 3: hipLaunchKernelGGL((rms_wgrad_partial_kernel<TX, TD, 3>), g, dim3(256 * WG_GROUPS), 0, st, x, ldx, xmap, rstd, dy, lddy, dy_round, rows, cols, partial); break;
    default: hipLaunchKernelGGL((rms_wgrad_partial_kernel<TX, TD, 4>), g, dim3(256 * WG_GROUPS), 0, st, x, ldx, xmap, rstd, dy, lddy, dy_round, rows, cols, partial); break;
  }
  wgrad_finish(partial, nblk, cols, grad, partial + (long)nblk * cols, st);
  RET_OK("rms_wgrad");
}

int rms_wgrad_finish_floats(int nblk, int cols) { return (nblk + (nblk + 15) / 16) * cols; }
int launch_rms_wgrad_finish(float* partial, int nblk, int cols, bf16_t* grad, hipStream_t st) {
  if (nblk <= 0) return 0;
  wgrad_finish(partial, nblk, cols, grad, partial + (long)nblk * cols, st);
  RET_OK("rms_wgrad_finish");
}

int rms_wgrad_partial_floats(int rows, int cols) {
  const int nblk = (rows + WG_ROWS - 1) / WG_ROWS;
  return (nblk + (nblk + 15) / 16) * cols;   // partials + the first fold
}

int launch_rms_wgrad(const float* x, long ldx, RowMap xmap, const float* rstd, const float* dy, long lddy,
                     int dy_round, int rows, int cols, bf16_t* grad, float* partial, hipStream_t st) {
  return rms_wgrad_t<float, float>(x, ldx, xmap, rstd, dy, lddy, dy_round, rows, cols, grad, partial, st);
}
int launch_rms_wgrad_bx(const bf16_t* x, long ldx, RowMap xmap, const float* rstd, const float* dy, long lddy,
                        int dy_round, int rows, int cols, bf16_t* grad, float* partial, hipStream_t st) {
  return rms_wgrad_t<bf16_t, float>(x, ldx, xmap, rstd, dy, lddy, dy_round, rows, cols, grad, partial, st);
}
int launch_rms_wgrad_bdy(const float* x, long ldx, RowMap xmap, const float* rstd, const bf16_t* dy, long lddy,
                         int rows, int cols, bf16_t* grad, float* partial, hipStream_t st) {
  return rms_wgrad_t<float, bf16_t>(x, ldx, xmap, rstd, dy, lddy, 0, rows, cols, grad, partial, st);
}

// ---------------------------------------------------------------- q_norm / k_norm weight grads
// For every (token row, head): dn = RoPE^T(dr) (dr = grad of the rotated, normed head), x_hat = x * rstd;
// dw[d] += dn[d] * x_hat[d].  RoPE (rotate-half, cos/sin tables of D/2): rot[d] = n[d] c[d] - n[d+h] s[d]
// (d < h), rot[d] = n[d] c[d-h] + n[d-h] s[d-h] (d >= h), so dn[d] = dr[d] c[d] + dr[d+h] s[d] (d < h),
// dn[d] = dr[d] c[d-h] - dr[d-h] s[d-h] (d >= h).
// dQ is in the attention layout [B, Hkv, S, G, D], dK in [B, Hkv, S, D]; qkv rows are token-major.
// D = 256: one wave per token (4 lanes-elements each: lane l owns d = 4l..4l+3, its RoPE partner d +- 128 is
// lane l +- 32, loaded directly), QK_ROWS tokens per block; per-block partials [blk][D], fixed-order finish.
#ifndef PTK_QK_ROWS
#define PTK_QK_ROWS 8
#endif
constexpr int QK_ROWS = PTK_QK_ROWS;   // tokens per block of the partial sums (8 measured +0.25 % on cfg4 when the RMSNorm
                                       // partials ran 8-row blocks; kept, not re-measured, with their final 32-row x 4-group form)
PTK_DEV float4 ldb4(const bf16_t* p) {
  u16x4_t u = *reinterpret_cast<const u16x4_t*>(p);
  return make_float4(bf2f(u[0]), bf2f(u[1]), bf2f(u[2]), bf2f(u[3]));
}
__global__ void __launch_bounds__(256) qknorm_wgrad_partial_kernel(const bf16_t* __restrict__ qkv,
                                                                   const float* __restrict__ cos_t,
                                                                   const float* __restrict__ sin_t,
                                                                   const float* __restrict__ rstd_q,
                                                                   const float* __restrict__ rstd_k,
                                                                   const bf16_t* __restrict__ dQ,
                                                                   const bf16_t* __restrict__ dK, AttnShape s,
                                                                   float* __restrict__ part_q,
                                                                   float* __restrict__ part_k) {
  __shared__ float4 red_q[4][64], red_k[4][64];
  const int D = 256, h = 128;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int d = 4 * lane, dp = d < h ? d + h : d - h, dc = d < h ? d : d - h;
  const float sg = d < h ? 1.f : -1.f;
  const int G = s.Hq / s.Hkv, Dqkv = (s.Hq + 2 * s.Hkv) * D;
  const long M = (long)s.B * s.S;
  float4 aq = make_float4(0.f, 0.f, 0.f, 0.f), ak = aq;
  for (long r = (long)blockIdx.x * QK_ROWS + wv; r < min(M, (long)(blockIdx.x + 1) * QK_ROWS); r += 4) {
    const int b = (int)(r / s.S), pos = (int)(r - (long)b * s.S);
    const float4 c = *reinterpret_cast<const float4*>(cos_t + (long)pos * h + dc);
    const float4 sn = *reinterpret_cast<const float4*>(sin_t + (long)pos * h + dc);
    const bf16_t* qrow = qkv + r * Dqkv;
    for (int hq = 0; hq < s.Hq; ++hq) {
      const int kvh = hq / G, j = hq - kvh * G;
      const bf16_t* g = dQ + ((((long)b * s.Hkv + kvh) * s.S + pos) * G + j) * D;
      const float4 g0 = ldb4(g + d), g1 = ldb4(g + dp), x = ldb4(qrow + hq * D + d);
      const float rs = rstd_q[r * s.Hq + hq];
      aq.x += (g0.x * c.x + sg * g1.x * sn.x) * x.x * rs;
      aq.y += (g0.y * c.y + sg * g1.y * sn.y) * x.y * rs;
      aq.z += (g0.z * c.z + sg * g1.z * sn.z) * x.z * rs;
      aq.w += (g0.w * c.w + sg * g1.w * sn.w) * x.w * rs;
    }
    for (int kvh = 0; kvh < s.Hkv; ++kvh) {
      const bf16_t* g = dK + (((long)b * s.Hkv + kvh) * s.S + pos) * D;
      const float4 g0 = ldb4(g + d), g1 = ldb4(g + dp), x = ldb4(qrow + (s.Hq + kvh) * D + d);
      const float rs = rstd_k[r * s.Hkv + kvh];
      ak.x += (g0.x * c.x + sg * g1.x * sn.x) * x.x * rs;
      ak.y += (g0.y * c.y + sg * g1.y * sn.y) * x.y * rs;
      ak.z += (g0.z * c.z + sg * g1.z * sn.z) * x.z * rs;
      ak.w += (g0.w * c.w + sg * g1.w * sn.w) * x.w * rs;
    }
  }
  red_q[wv][lane] = aq;
  red_k[wv][lane] = ak;
  __syncthreads();
  if (wv == 0) {
    float4 tq = red_q[0][lane], tk = red_k[0][lane];
    for (int w = 1; w < 4; ++w) {
      const float4 a = red_q[w][lane], bk = red_k[w][lane];
      tq.x += a.x; tq.y += a.y; tq.z += a.z; tq.w += a.w;
      tk.x += bk.x; tk.y += bk.y; tk.z += bk.z; tk.w += bk.w;
    }
    *reinterpret_cast<float4*>(part_q + (long)blockIdx.x * D + d) = tq;
    *reinterpret_cast<float4*>(part_k + (long)blockIdx.x * D + d) = tk;
  }
}

// generic head_dim (tests, tiny models): one thread per element d, QK_ROWS tokens per block
__global__ void __launch_bounds__(256) qknorm_wgrad_partial_any_kernel(const bf16_t* __restrict__ qkv,
                                                                       const float* __restrict__ cos_t,
                                                                       const float* __restrict__ sin_t,
                                                                       const float* __restrict__ rstd_q,
                                                                       const float* __restrict__ rstd_k,
                                                                       const bf16_t* __restrict__ dQ,
                                                                       const bf16_t* __restrict__ dK, AttnShape s,
                                                                       float* __restrict__ part_q,
                                                                       float* __restrict__ part_k) {
  const int D = s.D, h = D / 2, d = threadIdx.x;
  const int G = s.Hq / s.Hkv, Dqkv = (s.Hq + 2 * s.Hkv) * D;
  const long M = (long)s.B * s.S;
  const long r0 = (long)blockIdx.x * QK_ROWS, r1 = min(M, r0 + QK_ROWS);
  if (d >= D) return;
  float aq = 0.f, ak = 0.f;
  const int dp = d < h ? d + h : d - h, dc = d < h ? d : d - h;
  const float sg = d < h ? 1.f : -1.f;
  for (long r = r0; r < r1; ++r) {
    const int b = (int)(r / s.S), pos = (int)(r - (long)b * s.S);
    const float c = cos_t[(long)pos * h + dc], sn = sin_t[(long)pos * h + dc];
    const bf16_t* qrow = qkv + r * Dqkv;
    for (int hq = 0; hq < s.Hq; ++hq) {
      const int kvh = hq / G, j = hq - kvh * G;
      const bf16_t* g = dQ + ((((long)b * s.Hkv + kvh) * s.S + pos) * G + j) * D;
      aq += (bf2f(g[d]) * c + sg * bf2f(g[dp]) * sn) * bf2f(qrow[hq * D + d]) * rstd_q[r * s.Hq + hq];
    }
    for (int kvh = 0; kvh < s.Hkv; ++kvh) {
      const bf16_t* g = dK + (((long)b * s.Hkv + kvh) * s.S + pos) * D;
      ak += (bf2f(g[d]) * c + sg * bf2f(g[dp]) * sn) * bf2f(qrow[(s.Hq + kvh) * D + d]) * rstd_k[r * s.Hkv + kvh];
    }
  }
  part_q[(long)blockIdx.x * D + d] = aq;
  part_k[(long)blockIdx.x * D + d] = ak;
}

int launch_qknorm_wgrad(const bf16_t* qkv, const float* cos_t, const float* sin_t, AttnShape s, const float* rstd_q,
                        const float* rstd_k, const bf16_t* dQ, const bf16_t* dK, bf16_t* gq, bf16_t* gk,
                        float* partial, hipStream_t st) {
  if (s.D > 256 || s.D % 8) return set_error("qknorm_wgrad: head_dim %d", s.D);
  const long M = (long)s.B * s.S;
  const int nblk = (int)((M + QK_ROWS - 1) / QK_ROWS);
  float* pq = partial;
  float* pk = partial + (long)nblk * s.D;
  if (s.D == 256)
    hipLaunchKernelGGL(qknorm_wgrad_partial_kernel, dim3((unsigned)nblk), dim3(256), 0, st, qkv, cos_t, sin_t, rstd_q,
                       rstd_k, dQ, dK, s, pq, pk);
  else
    hipLaunchKernelGGL(qknorm_wgrad_partial_any_kernel, dim3((unsigned)nblk), dim3(256), 0, st, qkv, cos_t, sin_t,
                       rstd_q, rstd_k, dQ, dK, s, pq, pk);
  float* scratch = pk + (long)nblk * s.D;
  wgrad_finish(pq, nblk, s.D, gq, scratch, st);
  wgrad_finish(pk, nblk, s.D, gk, scratch, st);
  RET_OK("qknorm_wgrad");
}

int qknorm_wgrad_partial_floats(long M, int D) {
  const long nblk = (M + QK_ROWS - 1) / QK_ROWS;
  return (int)((2 * nblk + (nblk + 15) / 16) * D);
}

// ---------------------------------------------------------------- split-K reduce
// C = sum_s part[s] (fp32 out) or C = bf16(resid + bf16(sum_s part[s])) (bf16 out, resid may alias C or be
// null); part [S][M][N] packed, C [M][ldc].  Fixed summation order.
__global__ void __launch_bounds__(256) splitk_reduce_kernel(const float* __restrict__ part, int S, int M, int N,
                                                            void* C, long ldc, int out_bf16,
                                                            const bf16_t* resid, long ldr) {
  const long i = ((long)blockIdx.x * 256 + threadIdx.x) * 4;
  const long MN = (long)M * N;
  if (i >= MN) return;
  const int m = (int)(i / N), n = (int)(i - (long)m * N);
  float4 acc = *reinterpret_cast<const float4*>(part + i);
  for (int z = 1; z < S; ++z) {
    const float4 v = *reinterpret_cast<const float4*>(part + (long)z * MN + i);
    acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
  }
  if (!out_bf16) {
    *reinterpret_cast<float4*>((float*)C + (long)m * ldc + n) = acc;
    return;
  }
  float4 r = make_float4(0.f, 0.f, 0.f, 0.f);
  if (resid) r = ldb4(resid + (long)m * ldr + n);
  u16x4_t o;
  o[0] = f2bf(r.x + bfround(acc.x)); o[1] = f2bf(r.y + bfround(acc.y));
  o[2] = f2bf(r.z + bfround(acc.z)); o[3] = f2bf(r.w + bfround(acc.w));
  *reinterpret_cast<u16x4_t*>((bf16_t*)C + (long)m * ldc + n) = o;
}

int launch_splitk_reduce(const float* part, int S, int M, int N, void* C, long ldc, int out_bf16, const bf16_t* resid,
                         long ldr, hipStream_t st) {
  if (N % 4 || ldc % 4 || (resid && ldr % 4)) return set_error("splitk_reduce: N / ld must be multiples of 4");
  const long n4 = (long)M * N / 4;
  hipLaunchKernelGGL(splitk_reduce_kernel, dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0, st, part, S, M, N, C, ldc,
                     out_bf16, resid, ldr);
  RET_OK("splitk_reduce");
}

// ---------------------------------------------------------------- input-embedding grads
// Text position t of sample b sits at LLM row b*Spad + Nv + t and embeds token ids[b*T + t] as
// bf16(E[id] * escale).  Its grad into E[id] is bf16(bf16(dx_row) * escale) (the bf16 mul's backward on the
// fp32 grad cast to bf16); rows sharing an id are summed in position order (deterministic, no atomics), then
// added to the tied weight's bf16 grad.  Two launches: the (id, position) keys sorted by rank (positions
// ascending within an id), then one workgroup per sorted key whose id starts a run sums that run.  The round-5
// form (every workgroup compacting its id's positions out of all B*T ids, and the pad id's run summed with one
// guarded load -- one memory round trip -- per row and column) took 828 us per cfg4 micro-batch.
constexpr int EG_MAX = 16384;   // text tokens per batch (EG_POS_BITS of position in a key)
constexpr int EG_POS_BITS = 14;
// key = id << 14 | position (all distinct): each key's rank among all keys is its place in the sorted order.
// 64 keys per workgroup, each wave counting one quarter of every LDS tile of the keys (a one-workgroup bitonic
// sort in LDS took 117 us at cfg4's 5 120 keys, one key per thread over all of them 80 us)
__global__ void __launch_bounds__(256) embed_rank_kernel(const int64_t* __restrict__ ids, int n,
                                                         uint64_t* __restrict__ sorted) {
  __shared__ uint64_t tile[1024];
  __shared__ int part[4][64];
  const int kl = threadIdx.x & 63, qtr = threadIdx.x >> 6;
  const int i = blockIdx.x * 64 + kl;
  const uint64_t key = i < n ? ((uint64_t)ids[i] << EG_POS_BITS) | (uint64_t)i : ~0ull;
  int rank = 0;
  for (int t0 = 0; t0 < n; t0 += 1024) {
    __syncthreads();
    for (int u = threadIdx.x; u < 1024; u += 256) {
      const int j = t0 + u;
      tile[u] = j < n ? ((uint64_t)ids[j] << EG_POS_BITS) | (uint64_t)j : ~0ull;
    }
    __syncthreads();
    // the whole quarter, LDS reads unrolled (past n the tile holds ~0, never below a key)
    const uint64_t* tq = tile + qtr * 256;
#pragma unroll 32
    for (int u = 0; u < 256; ++u) rank += tq[u] < key ? 1 : 0;
  }
  part[qtr][kl] = rank;
  __syncthreads();
  if (qtr == 0 && i < n) sorted[part[0][kl] + part[1][kl] + part[2][kl] + part[3][kl]] = key;
}

__global__ void __launch_bounds__(256) embed_grad_kernel(const uint64_t* __restrict__ sorted, int n, int T, int Nv,
                                                         int Spad, int H, float escale, const float* __restrict__ dx,
                                                         bf16_t* __restrict__ dE) {
  const int k = blockIdx.x;
  const uint64_t id = sorted[k] >> EG_POS_BITS;
  if (k > 0 && (sorted[k - 1] >> EG_POS_BITS) == id) return;   // not the first position of its id
  int cnt = 0;   // the run's length (contiguous in the sorted keys)
  for (int base = k; base < n; base += 256) {
    const int idx = base + threadIdx.x;
    const int c = __syncthreads_count(idx < n && (sorted[idx] >> EG_POS_BITS) == id);
    cnt += c;
    if (c < 256) break;
  }
  // the run's rows staged in LDS, EG_COLS column sets of 256 per pass and EG_UNROLL rows' loads in flight
  // before their adds: the sum per column stays in position order, but the pad id's run (hundreds of rows at
  // cfg4) no longer waits one memory round trip per row and column set
  constexpr int EG_COLS = 5, EG_UNROLL = 8, EG_CHUNK = 2048;
  __shared__ int rows_s[EG_CHUNK];
  const uint64_t pmask = (1ull << EG_POS_BITS) - 1;
  for (int c0 = 0; c0 < H; c0 += 256 * EG_COLS) {
    float acc[EG_COLS];
#pragma unroll
    for (int q = 0; q < EG_COLS; ++q) acc[q] = 0.f;
    for (int u0 = 0; u0 < cnt; u0 += EG_CHUNK) {
      const int m = min(EG_CHUNK, cnt - u0);
      __syncthreads();
      for (int u = threadIdx.x; u < m; u += 256) {
        const int j = (int)(sorted[k + u0 + u] & pmask), b = j / T, t = j - b * T;
        rows_s[u] = b * Spad + Nv + t;
      }
      __syncthreads();
      int u = 0;
      for (; u + EG_UNROLL <= m; u += EG_UNROLL) {
        float v[EG_UNROLL][EG_COLS];
#pragma unroll
        for (int uu = 0; uu < EG_UNROLL; ++uu) {
          const float* row = dx + (long)rows_s[u + uu] * H;
#pragma unroll   // unguarded loads (clamped column; the value is dropped below): a guarded load is a branch
          for (int q = 0; q < EG_COLS; ++q) v[uu][q] = row[min(c0 + q * 256 + (int)threadIdx.x, H - 1)];
        }
#pragma unroll
        for (int uu = 0; uu < EG_UNROLL; ++uu)
#pragma unroll
          for (int q = 0; q < EG_COLS; ++q) acc[q] += bfround(bfround(v[uu][q]) * escale);
      }
      for (; u < m; ++u) {
        const float* row = dx + (long)rows_s[u] * H;
#pragma unroll
        for (int q = 0; q < EG_COLS; ++q) {
          const int c = c0 + q * 256 + threadIdx.x;
          if (c < H) acc[q] += bfround(bfround(row[c]) * escale);
        }
      }
    }
#pragma unroll
    for (int q = 0; q < EG_COLS; ++q) {
      const int c = c0 + q * 256 + threadIdx.x;
      if (c < H) {
        bf16_t* g = dE + (long)id * H + c;
        *g = f2bf(bf2f(*g) + bfround(acc[q]));
      }
    }
  }
}

size_t embed_grad_ws_bytes(int B, int T) { return (size_t)(B * T > 0 ? B * T : 1) * sizeof(uint64_t); }
int launch_embed_grad(const int64_t* ids, int B, int T, int Nv, int Spad, int H, float escale, const float* dx,
                      bf16_t* dE, void* ws, hipStream_t st) {
  const int n = B * T;
  if (n <= 0) return 0;
  if (n > EG_MAX) return set_error("embed_grad: %d text tokens per batch (max %d)", n, EG_MAX);
  uint64_t* sorted = static_cast<uint64_t*>(ws);
  hipLaunchKernelGGL(embed_rank_kernel, dim3((unsigned)((n + 63) / 64)), dim3(256), 0, st, ids, n, sorted);
  hipLaunchKernelGGL(embed_grad_kernel, dim3((unsigned)n), dim3(256), 0, st, sorted, n, T, Nv, Spad, H, escale, dx,
                     dE);
  RET_OK("embed_grad");
}

// ---------------------------------------------------------------- bf16 grad scale + sum of squares
// g = bf16(g * scale) in place when scale != 1 (DDP's 1/world average of a summed gradient), and
// out[0] = sum g^2 in fp32: SS_BLOCKS fixed block partials summed in block order by one block (the same
// grid for a given n, so the result is bit-reproducible).
constexpr int SS_BLOCKS = 1024;
__global__ void __launch_bounds__(256) scale_sumsq_kernel(bf16_t* __restrict__ g, long n, float scale,
                                                          float* __restrict__ partial) {
  __shared__ float red[4];
  float s = 0.f;
  for (long i = ((long)blockIdx.x * 256 + threadIdx.x) * 8; i < n; i += (long)gridDim.x * 2048) {
    if (i + 7 < n) {
      u16x8_t u = *reinterpret_cast<const u16x8_t*>(g + i);
      if (scale != 1.f) {
#pragma unroll
        for (int e = 0; e < 8; ++e) u[e] = f2bf(bf2f(u[e]) * scale);
        *reinterpret_cast<u16x8_t*>(g + i) = u;
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float v = bf2f(u[e]);
        s += v * v;
      }
    } else {
      for (long j = i; j < n; ++j) {
        float v = bf2f(g[j]);
        if (scale != 1.f) {
          v = bfround(v * scale);
          g[j] = f2bf(v);
        }
        s += v * v;
      }
    }
  }
  s = block_sum<256>(s, red);
  if (threadIdx.x == 0) partial[blockIdx.x] = s;
}
__global__ void __launch_bounds__(256) sum_blocks_kernel(const float* __restrict__ partial, int nb,
                                                         float* __restrict__ out) {
  __shared__ float red[4];
  float s = 0.f;
  for (int i = threadIdx.x; i < nb; i += 256) s += partial[i];
  s = block_sum<256>(s, red);
  if (threadIdx.x == 0) out[0] = s;
}

int scale_sumsq_partial_floats() { return SS_BLOCKS; }

int launch_scale_sumsq_bf16(bf16_t* g, long n, float scale, float* partial, float* out, hipStream_t st) {
  if (n <= 0) {
    hipLaunchKernelGGL(sum_blocks_kernel, dim3(1), dim3(256), 0, st, partial, 0, out);
    RET_OK("scale_sumsq");
  }
  hipLaunchKernelGGL(scale_sumsq_kernel, dim3(SS_BLOCKS), dim3(256), 0, st, g, n, scale, partial);
  hipLaunchKernelGGL(sum_blocks_kernel, dim3(1), dim3(256), 0, st, partial, SS_BLOCKS, out);
  RET_OK("scale_sumsq");
}

// ---------------------------------------------------------------- clip + AdamW on bf16 parameters
// clip_grad_norm_(max_norm) on bf16 grads: total = ||g|| (fp32 sum of squares, rounded to bf16 as the
// reference's bf16 norm tensor), coef = bf16(max_norm / bf16(total + 1e-6)) clamped to 1, g = bf16(g coef).
// Then torch's _single_tensor_adamw on bf16 tensors, each in-place op rounded to bf16:
//   p = bf16(p (1 - lr wd)); m = bf16(m + (1-b1)(g - m)); v = bf16(v b2); v = bf16(v + (1-b2) g g);
//   den = bf16(sqrt(v)); den = bf16(den / bc2s); den = bf16(den + eps); p = bf16(p - step_size m / den).
__global__ void __launch_bounds__(256) adamw_bf16_kernel(bf16_t* __restrict__ p, bf16_t* __restrict__ g,
                                                         bf16_t* __restrict__ m, bf16_t* __restrict__ v, long n,
                                                         const float* __restrict__ sumsq, float max_norm,
                                                         float decay, float b1c, float b2, float b2c, float step_size,
                                                         float bc2s, float eps, float* norm_out) {
  float coef = 1.f;
  if (max_norm > 0.f) {
    const float total = bfround(sqrtf(sumsq[0]));
    coef = fminf(bfround(max_norm / bfround(total + 1e-6f)), 1.f);
    if (blockIdx.x == 0 && threadIdx.x == 0 && norm_out) norm_out[0] = total;
  }
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    float gi = bf2f(g[i]);
    if (coef != 1.f) {
      gi = bfround(gi * coef);
      g[i] = f2bf(gi);
    }
    float pi = bfround(bf2f(p[i]) * decay);
    const float mo = bf2f(m[i]);
    const float mi = bfround(mo + b1c * (gi - mo));
    float vi = bfround(bf2f(v[i]) * b2);
    vi = bfround(vi + b2c * gi * gi);
    float den = bfround(sqrtf(vi));
    den = bfround(den / bc2s);
    den = bfround(den + eps);
    pi = bfround(pi - step_size * mi / den);
    p[i] = f2bf(pi);
    m[i] = f2bf(mi);
    v[i] = f2bf(vi);
  }
}

int launch_adamw_bf16(bf16_t* p, bf16_t* g, bf16_t* m, bf16_t* v, long n, const float* sumsq, float max_norm,
                      double lr, double b1, double b2, double eps, double wd, int step, float* norm_out,
                      hipStream_t st) {
  if (n <= 0) return 0;
  if (step < 1) return set_error("adamw_bf16: step must be >= 1");
  const double bc1 = 1.0 - pow(b1, step), bc2 = 1.0 - pow(b2, step);
  const long blocks = std::min<long>(4096, (n + 255) / 256);
  hipLaunchKernelGGL(adamw_bf16_kernel, dim3((unsigned)blocks), dim3(256), 0, st, p, g, m, v, n, sumsq, max_norm,
                     (float)(1.0 - lr * wd), (float)(1.0 - b1), (float)b2, (float)(1.0 - b2), (float)(lr / bc1),
                     (float)sqrt(bc2), (float)eps, norm_out);
  RET_OK("adamw_bf16");
}

}  // namespace ptk
