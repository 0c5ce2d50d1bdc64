// Row-wise normalisation kernels (HBM-bound).  One wave64 per row, 4 rows per
// 256-thread block, 16-B vector loads; the row stays in registers between the
// statistics pass and the output pass (cols <= 64*4*MAXV).
//
// SigLIP LayerNorm: TF/models/siglip/modeling_siglip.py:329,331,567 (eps 1e-6).
// Gemma3 RMSNorm (fp32 math, scale 1+w, cast to input dtype):
// TF/models/gemma3/modeling_gemma3.py:136-150; sandwich placement :412-429.
#include "common.h"
#include "ptk_internal.h"

namespace ptk {

constexpr int MAXV = 12;   // float4 per lane -> cols <= 3072

PTK_DEV float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }
PTK_DEV void st4(float* p, float4 v) { *reinterpret_cast<float4*>(p) = v; }
PTK_DEV float4 ld4bf(const bf16_t* p) {
  u16x4_t u = *reinterpret_cast<const u16x4_t*>(p);
  return make_float4(bf2f(u[0]), bf2f(u[1]), bf2f(u[2]), bf2f(u[3]));
}
PTK_DEV void st4bf(bf16_t* p, float4 v) {
  u16x4_t u;
  u[0] = f2bf(v.x); u[1] = f2bf(v.y); u[2] = f2bf(v.z); u[3] = f2bf(v.w);
  *reinterpret_cast<u16x4_t*>(p) = u;
}
PTK_DEV float dot4(float4 a, float4 b) { return a.x * b.x + a.y * b.y + a.z * b.z + a.w * b.w; }
PTK_DEV float4 bfr4(float4 v) { return make_float4(bfround(v.x), bfround(v.y), bfround(v.z), bfround(v.w)); }
PTK_DEV float4 onep(float4 w) { return make_float4(1.f + w.x, 1.f + w.y, 1.f + w.z, 1.f + w.w); }
PTK_DEV float4 mul4(float4 a, float4 b) { return make_float4(a.x * b.x, a.y * b.y, a.z * b.z, a.w * b.w); }
PTK_DEV float4 add4(float4 a, float4 b) { return make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w); }
PTK_DEV float4 scl4(float4 a, float s) { return make_float4(a.x * s, a.y * s, a.z * s, a.w * s); }

#define ROW_SETUP                                          \
  const int lane = threadIdx.x & 63;                       \
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6); \
  if (row >= rows) return;

// NV = ceil(cols / 256) exactly (NORM_DISPATCH), so only the last float4 column group can run past cols: the
// others go unguarded -- a guarded load is a branch whose wait serialises the row's loads
#define FOR_V for (int v = 0; v < NV; ++v) if (v < NV - 1 || lane * 4 + v * 256 < cols)
#define COL (lane * 4 + v * 256)

PTK_DEV float4 ldx4(const float* p) { return ld4(p); }
PTK_DEV float4 ldx4(const bf16_t* p) { return ld4bf(p); }

template <typename T, int NV>
PTK_DEV void layernorm_body(const T* __restrict__ x, const float* __restrict__ w, const float* __restrict__ b,
                            bf16_t* __restrict__ y, long rows, int cols, float eps) {
  ROW_SETUP
  float4 r[NV];
  float s = 0.f;
#pragma unroll
  FOR_V { r[v] = ldx4(x + row * cols + COL); s += r[v].x + r[v].y + r[v].z + r[v].w; }
  const float mean = warp_sum(s) / cols;
  float q = 0.f;
#pragma unroll
  FOR_V {
    float4 d = make_float4(r[v].x - mean, r[v].y - mean, r[v].z - mean, r[v].w - mean);
    r[v] = d;
    q += dot4(d, d);
  }
  const float rstd = rsqrtf(warp_sum(q) / cols + eps);
#pragma unroll
  FOR_V { st4bf(y + row * cols + COL, add4(mul4(scl4(r[v], rstd), ld4(w + COL)), ld4(b + COL))); }
}

template <int NV>
__global__ void __launch_bounds__(256) layernorm_f32(const float* __restrict__ x, const float* __restrict__ w,
                                                     const float* __restrict__ b, bf16_t* __restrict__ y, long rows,
                                                     int cols, float eps) {
  layernorm_body<float, NV>(x, w, b, y, rows, cols, eps);
}
template <int NV>
__global__ void __launch_bounds__(256) layernorm_b16(const bf16_t* __restrict__ x, const float* __restrict__ w,
                                                     const float* __restrict__ b, bf16_t* __restrict__ y, long rows,
                                                     int cols, float eps) {
  layernorm_body<bf16_t, NV>(x, w, b, y, rows, cols, eps);
}

template <int NV>
__global__ void __launch_bounds__(256) rmsnorm_fwd_kernel(const float* __restrict__ x, long ldx, RowMap xmap,
                                                          const float* __restrict__ w, bf16_t* __restrict__ y,
                                                          float* __restrict__ rstd_out, long rows, int cols,
                                                          float eps) {
  ROW_SETUP
  const float* xr = x + map_row(xmap, row) * ldx;
  float4 r[NV];
  float q = 0.f;
#pragma unroll
  FOR_V { r[v] = ld4(xr + COL); q += dot4(r[v], r[v]); }
  const float rs = rsqrtf(warp_sum(q) / cols + eps);
  if (lane == 0 && rstd_out) rstd_out[row] = rs;
#pragma unroll
  FOR_V { st4bf(y + row * cols + COL, mul4(scl4(r[v], rs), onep(ld4(w + COL)))); }
}

template <int NV>
__global__ void __launch_bounds__(256) residual_norm_fwd_kernel(
    const bf16_t* __restrict__ t, const float* __restrict__ xi, const float* __restrict__ w_post,
    const float* __restrict__ w_next, float* __restrict__ xo, bf16_t* __restrict__ n,
    float* __restrict__ rstd_t, float* __restrict__ rstd_x, long rows, int cols, float eps) {
  ROW_SETUP
  float4 r[NV];
  float q = 0.f;
#pragma unroll
  FOR_V { r[v] = ld4bf(t + row * cols + COL); q += dot4(r[v], r[v]); }
  const float rs = rsqrtf(warp_sum(q) / cols + eps);
  if (lane == 0) rstd_t[row] = rs;
  float q2 = 0.f;
#pragma unroll
  FOR_V {
    float4 yv = bfr4(mul4(scl4(r[v], rs), onep(ld4(w_post + COL))));   // post-norm output is bf16
    float4 xv = add4(ld4(xi + row * cols + COL), yv);                   // fp32 residual stream
    st4(xo + row * cols + COL, xv);
    r[v] = xv;
    q2 += dot4(xv, xv);
  }
  if (!w_next) return;
  const float rs2 = rsqrtf(warp_sum(q2) / cols + eps);
  if (lane == 0) rstd_x[row] = rs2;
#pragma unroll
  FOR_V { st4bf(n + row * cols + COL, mul4(scl4(r[v], rs2), onep(ld4(w_next + COL)))); }
}

// rms backward helper: returns dx given x row, (1+w), rstd, dn (all in regs)
#define RMS_BWD_BODY(XV, DNV, RS, OUTEXPR)                                   \
  {                                                                           \
    float sdot = 0.f;                                                         \
    _Pragma("unroll") FOR_V { sdot += dot4(mul4(DNV[v], onep(ld4(w + COL))), XV[v]); } \
    sdot = warp_sum(sdot);                                                    \
    const float c3 = RS * RS * RS * sdot / cols;                              \
    _Pragma("unroll") FOR_V {                                                 \
      float4 dxv = add4(scl4(mul4(DNV[v], onep(ld4(w + COL))), RS), scl4(XV[v], -c3)); \
      OUTEXPR;                                                                \
    }                                                                         \
  }

template <typename TD, int NV>
PTK_DEV void rmsnorm_bwd_body(const float* __restrict__ x, const float* __restrict__ w, const float* __restrict__ rstd,
                              const TD* __restrict__ dn, const float* dacc, float* dx, long rows, int cols) {
  ROW_SETUP
  float4 xv[NV], dv[NV];
#pragma unroll
  FOR_V { xv[v] = ld4(x + row * cols + COL); dv[v] = ldx4(dn + row * cols + COL); }
  const float rs = rstd[row];
  RMS_BWD_BODY(xv, dv, rs, {
    float4 o = dacc ? add4(ld4(dacc + row * cols + COL), dxv) : dxv;
    st4(dx + row * cols + COL, o);
  })
}
template <int NV>
__global__ void __launch_bounds__(256) rmsnorm_bwd_f32_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                                              const float* __restrict__ rstd, const float* __restrict__ dn,
                                                              const float* dacc, float* dx, long rows, int cols) {
  rmsnorm_bwd_body<float, NV>(x, w, rstd, dn, dacc, dx, rows, cols);
}
// dn in bf16: the output grad of a bf16 linear (the reference's autocast linear backward returns bf16)
template <int NV>
__global__ void __launch_bounds__(256) rmsnorm_bwd_bdn_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                                              const float* __restrict__ rstd, const bf16_t* __restrict__ dn,
                                                              const float* dacc, float* dx, long rows, int cols) {
  rmsnorm_bwd_body<bf16_t, NV>(x, w, rstd, dn, dacc, dx, rows, cols);
}

template <int NV>
__global__ void __launch_bounds__(256) rmsnorm_bwd_scatter_kernel(const float* __restrict__ x, RowMap xmap,
                                                                  const float* __restrict__ w,
                                                                  const float* __restrict__ rstd,
                                                                  const float* __restrict__ dn, float* dR,
                                                                  long rows, int cols) {
  ROW_SETUP
  const long xr = map_row(xmap, row);
  float4 xv[NV], dv[NV];
#pragma unroll
  FOR_V { xv[v] = ld4(x + xr * cols + COL); dv[v] = ld4(dn + row * cols + COL); }
  const float rs = rstd[row];
  RMS_BWD_BODY(xv, dv, rs, { st4(dR + xr * cols + COL, add4(ld4(dR + xr * cols + COL), dxv)); })
}

// grad through a post-norm whose output (bf16) was added to the residual:
// dy = bf16(dR); dt = bf16(rms_bwd(t, w, rstd_t, dy))
template <int NV>
PTK_DEV void post_norm_bwd_row(const float* dR, const bf16_t* t, const float* w, float rs, bf16_t* dt, int lane,
                               int cols) {
  float4 xv[NV], dv[NV];
#pragma unroll
  FOR_V { xv[v] = ld4bf(t + COL); dv[v] = bfr4(ld4(dR + COL)); }
  RMS_BWD_BODY(xv, dv, rs, { st4bf(dt + COL, dxv); })
}

template <typename TD, int NV>
PTK_DEV void residual_norm_bwd_body(
    const float* __restrict__ x2, const float* __restrict__ w_pre, const float* __restrict__ rstd_pre,
    const TD* __restrict__ dn, float* __restrict__ dR, const bf16_t* __restrict__ t,
    const float* __restrict__ w_post, const float* __restrict__ rstd_t, bf16_t* __restrict__ dt, long rows,
    int cols) {
  ROW_SETUP
  float4 nd[NV];   // the updated dR row stays in registers for the post-norm pass
  {
    const float* w = w_pre;
    float4 xv[NV], dv[NV];
#pragma unroll
    FOR_V { xv[v] = ld4(x2 + row * cols + COL); dv[v] = ldx4(dn + row * cols + COL); }
    const float rs = rstd_pre[row];
    RMS_BWD_BODY(xv, dv, rs, {
      nd[v] = add4(ld4(dR + row * cols + COL), dxv);
      st4(dR + row * cols + COL, nd[v]);
    })
  }
  {
    const float* w = w_post;
    const float rs = rstd_t[row];
    float4 xv[NV], dv[NV];
#pragma unroll
    FOR_V { xv[v] = ld4bf(t + row * cols + COL); dv[v] = bfr4(nd[v]); }
    RMS_BWD_BODY(xv, dv, rs, { st4bf(dt + row * cols + COL, dxv); })
  }
}
template <int NV>
__global__ void __launch_bounds__(256) residual_norm_bwd_kernel(
    const float* __restrict__ x2, const float* __restrict__ w_pre, const float* __restrict__ rstd_pre,
    const float* __restrict__ dn, float* __restrict__ dR, const bf16_t* __restrict__ t,
    const float* __restrict__ w_post, const float* __restrict__ rstd_t, bf16_t* __restrict__ dt, long rows,
    int cols) {
  residual_norm_bwd_body<float, NV>(x2, w_pre, rstd_pre, dn, dR, t, w_post, rstd_t, dt, rows, cols);
}
template <int NV>
__global__ void __launch_bounds__(256) residual_norm_bwd_bdn_kernel(
    const float* __restrict__ x2, const float* __restrict__ w_pre, const float* __restrict__ rstd_pre,
    const bf16_t* __restrict__ dn, float* __restrict__ dR, const bf16_t* __restrict__ t,
    const float* __restrict__ w_post, const float* __restrict__ rstd_t, bf16_t* __restrict__ dt, long rows,
    int cols) {
  residual_norm_bwd_body<bf16_t, NV>(x2, w_pre, rstd_pre, dn, dR, t, w_post, rstd_t, dt, rows, cols);
}

// residual_norm_bwd_bdn with both norms' weight-grad partials folded in (Stage 2, unfrozen LM): the rows of
// x2 / dn / t and the updated dR are already in registers, so the two separate rms_wgrad passes that re-read
// them from HBM (2 x 6.9 KB per token at H = 1152) go away.  partial[blk][c] = sum over the block's 4 rows of
// dy[r, c] * x[r, c] * rstd[r] -- pre norm: dy = dn, x = x2; post norm: dy = bf16(dR_new), x = t.
// Same grid as residual_norm_bwd_bdn (one wave per row, 4 rows per block: the occupancy this HBM-bound pass
// needs: a 32-row block looping 8 rows per wave, 1.75 waves per SIMD, left the cfg4 step slower than the two
// separate passes did).  Each wave parks its product row in LDS, one norm at a time; wave 0 sums the 4 rows in
// row order and writes the block's partial row (1.15 KB per token per norm, folded by rms_wgrad_finish).
#ifndef PTK_NWG_WAVES
#define PTK_NWG_WAVES 4
#endif
constexpr int NWG = PTK_NWG_WAVES;   // rows (waves) per block
template <int NV>
__global__ void __launch_bounds__(64 * NWG) residual_norm_bwd_wg_kernel(
    const float* __restrict__ x2, const float* __restrict__ w_pre, const float* __restrict__ rstd_pre,
    const bf16_t* __restrict__ dn, float* __restrict__ dR, const bf16_t* __restrict__ t,
    const float* __restrict__ w_post, const float* __restrict__ rstd_t, bf16_t* __restrict__ dt, long rows,
    int cols, float* __restrict__ part_pre, float* __restrict__ part_post) {
  __shared__ float4 red[NWG][NV][64];   // one norm at a time: 20 KB at H = 1152 keeps 7 waves per SIMD
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const long row = (long)blockIdx.x * NWG + wv;
  const bool ok = row < rows;
  // the block's 4 product rows -> one partial row, summed in row order by wave 0
#define NWG_SUM(PART)                                                                    \
  __syncthreads();                                                                       \
  if (wv == 0) {                                                                         \
    float* part = PART + (long)blockIdx.x * cols;                                        \
    _Pragma("unroll") FOR_V {                                                            \
      float4 a = red[0][v][lane];                                                        \
      _Pragma("unroll") for (int g = 1; g < NWG; ++g) a = add4(a, red[g][v][lane]);      \
      st4(part + COL, a);                                                                \
    }                                                                                    \
  }                                                                                      \
  __syncthreads();
  float4 nd[NV];
  if (ok) {
    const float* w = w_pre;
    float4 xv[NV], dv[NV];
#pragma unroll
    FOR_V { xv[v] = ld4(x2 + row * cols + COL); dv[v] = ld4bf(dn + row * cols + COL); }
    const float rs = rstd_pre[row];
#pragma unroll
    FOR_V { red[wv][v][lane] = scl4(mul4(dv[v], xv[v]), rs); }
    RMS_BWD_BODY(xv, dv, rs, {
      nd[v] = add4(ld4(dR + row * cols + COL), dxv);
      st4(dR + row * cols + COL, nd[v]);
    })
  } else {
#pragma unroll
    for (int v = 0; v < NV; ++v) red[wv][v][lane] = make_float4(0.f, 0.f, 0.f, 0.f);
  }
  NWG_SUM(part_pre)
  if (ok) {
    const float* w = w_post;
    const float rs = rstd_t[row];
    float4 xv[NV], dv[NV];
#pragma unroll
    FOR_V { xv[v] = ld4bf(t + row * cols + COL); dv[v] = bfr4(nd[v]); }
#pragma unroll
    FOR_V { red[wv][v][lane] = scl4(mul4(dv[v], xv[v]), rs); }
    RMS_BWD_BODY(xv, dv, rs, { st4bf(dt + row * cols + COL, dxv); })
  } else {
#pragma unroll
    for (int v = 0; v < NV; ++v) red[wv][v][lane] = make_float4(0.f, 0.f, 0.f, 0.f);
  }
  NWG_SUM(part_post)
#undef NWG_SUM
}

template <int NV>
__global__ void __launch_bounds__(256) post_norm_bwd_kernel(const float* __restrict__ dR, const bf16_t* __restrict__ t,
                                                            const float* __restrict__ w, const float* __restrict__ rstd_t,
                                                            bf16_t* __restrict__ dt, long rows, int cols) {
  ROW_SETUP
  post_norm_bwd_row<NV>(dR + row * cols, t + row * cols, w, rstd_t[row], dt + row * cols, lane, cols);
}

// float4 registers per lane for a row of `cols` (one wave per row): kernels are instantiated per exact count
// (FOR_V relies on it) so the row arrays take only the registers they need (occupancy of these HBM-bound kernels)
#define NORM_DISPATCH(KERNEL, ...)                                                                  \
  do {                                                                                              \
    switch ((cols + 255) / 256) {                                                                   \
      case 1: hipLaunchKernelGGL(KERNEL<1>, NORM_GRID, __VA_ARGS__); break;                         \
      case 2: hipLaunchKernelGGL(KERNEL<2>, NORM_GRID, __VA_ARGS__); break;                         \
      case 3: hipLaunchKernelGGL(KERNEL<3>, NORM_GRID, __VA_ARGS__); break;                         \
      case 4: hipLaunchKernelGGL(KERNEL<4>, NORM_GRID, __VA_ARGS__); break;                         \
      case 5: hipLaunchKernelGGL(KERNEL<5>, NORM_GRID, __VA_ARGS__); break;                         \
      case 6: hipLaunchKernelGGL(KERNEL<6>, NORM_GRID, __VA_ARGS__); break;                         \
      case 7: hipLaunchKernelGGL(KERNEL<7>, NORM_GRID, __VA_ARGS__); break;                         \
      case 8: hipLaunchKernelGGL(KERNEL<8>, NORM_GRID, __VA_ARGS__); break;                         \
      case 9: hipLaunchKernelGGL(KERNEL<9>, NORM_GRID, __VA_ARGS__); break;                         \
      case 10: hipLaunchKernelGGL(KERNEL<10>, NORM_GRID, __VA_ARGS__); break;                       \
      case 11: hipLaunchKernelGGL(KERNEL<11>, NORM_GRID, __VA_ARGS__); break;                       \
      default: hipLaunchKernelGGL(KERNEL<MAXV>, NORM_GRID, __VA_ARGS__); break;                     \
    }                                                                                               \
  } while (0)

static int check_cols(int cols) {
  if (cols <= 0 || cols % 4 || cols > 256 * MAXV) return set_error("norm: cols=%d unsupported", cols);
  return 0;
}
#define NORM_GRID dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, st
#define RET_LAUNCH(name) return hipGetLastError() == hipSuccess ? 0 : set_error(name " launch failed")

int launch_layernorm(const float* x, const float* w, const float* b, bf16_t* y, int rows, int cols, float eps,
                     hipStream_t st) {
  if (check_cols(cols)) return -1;
  if (rows <= 0) return 0;
  NORM_DISPATCH(layernorm_f32, x, w, b, y, (long)rows, cols, eps);
  RET_LAUNCH("layernorm");
}
int launch_layernorm_bf16(const bf16_t* x, const float* w, const float* b, bf16_t* y, int rows, int cols, float eps,
                          hipStream_t st) {
  if (check_cols(cols)) return -1;
  if (rows <= 0) return 0;
  NORM_DISPATCH(layernorm_b16, x, w, b, y, (long)rows, cols, eps);
  RET_LAUNCH("layernorm_bf16");
}
int launch_rmsnorm_fwd(const float* x, long ldx, RowMap xmap, const float* w, bf16_t* y, float* rstd, int rows,
                       int cols, float eps, hipStream_t st) {
  if (check_cols(cols)) return -1;
  if (rows <= 0) return 0;
  NORM_DISPATCH(rmsnorm_fwd_kernel, x, ldx, xmap, w, y, rstd, (long)rows, cols, eps);
  RET_LAUNCH("rmsnorm_fwd");
}
int launch_residual_norm_fwd(const bf16_t* t, const float* xi, const float* w_post, const float* w_next, float* xo,
                             bf16_t* n, float* rstd_t, float* rstd_x, int rows, int cols, float eps,
                             hipStream_t st) {
  if (check_cols(cols)) return -1;
  if (rows <= 0) return 0;
  NORM_DISPATCH(residual_norm_fwd_kernel, t, xi, w_post, w_next, xo, n, rstd_t, rstd_x,
                     (long)rows, cols, eps);
  RET_LAUNCH("residual_norm_fwd");
}
int launch_rmsnorm_bwd_f32(const float* x, const float* w, const float* rstd, const float* dn, const float* dacc,
                           float* dx, int rows, int cols, hipStream_t st) {
  if (check_cols(cols)) return -1;
  if (rows <= 0) return 0;
  NORM_DISPATCH(rmsnorm_bwd_f32_kernel, x, w, rstd, dn, dacc, dx, (long)rows, cols);
  RET_LAUNCH("rmsnorm_bwd");
}
int launch_rmsnorm_bwd_bdn(const float* x, const float* w, const float* rstd, const bf16_t* dn, const float* dacc,
                           float* dx, int rows, int cols, hipStream_t st) {
  if (check_cols(cols)) return -1;
  if (rows <= 0) return 0;
  NORM_DISPATCH(rmsnorm_bwd_bdn_kernel, x, w, rstd, dn, dacc, dx, (long)rows, cols);
  RET_LAUNCH("rmsnorm_bwd_bdn");
}
int launch_residual_norm_bwd_bdn(const float* x2, const float* w_pre, const float* rstd_pre, const bf16_t* dn,
                                 float* dR, const bf16_t* t, const float* w_post, const float* rstd_t, bf16_t* dt,
                                 int rows, int cols, hipStream_t st) {
  if (check_cols(cols)) return -1;
  if (rows <= 0) return 0;
  NORM_DISPATCH(residual_norm_bwd_bdn_kernel, x2, w_pre, rstd_pre, dn, dR, t, w_post, rstd_t, dt, (long)rows, cols);
  RET_LAUNCH("residual_norm_bwd_bdn");
}
int residual_norm_bwd_wg_blocks(int rows) { return (rows + NWG - 1) / NWG; }
int launch_residual_norm_bwd_wg(const float* x2, const float* w_pre, const float* rstd_pre, const bf16_t* dn,
                                float* dR, const bf16_t* t, const float* w_post, const float* rstd_t, bf16_t* dt,
                                int rows, int cols, float* part_pre, float* part_post, hipStream_t st) {
  if (check_cols(cols)) return -1;
  if (rows <= 0) return 0;
#undef NORM_GRID
#define NORM_GRID dim3((unsigned)residual_norm_bwd_wg_blocks(rows)), dim3(64 * NWG), 0, st
  NORM_DISPATCH(residual_norm_bwd_wg_kernel, x2, w_pre, rstd_pre, dn, dR, t, w_post, rstd_t, dt, (long)rows, cols,
                part_pre, part_post);
#undef NORM_GRID
#define NORM_GRID dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, st
  RET_LAUNCH("residual_norm_bwd_wg");
}
int launch_rmsnorm_bwd_scatter(const float* x, RowMap xmap, const float* w, const float* rstd, const float* dn,
                               float* dR, int rows, int cols, hipStream_t st) {
  if (check_cols(cols)) return -1;
  if (rows <= 0) return 0;
  NORM_DISPATCH(rmsnorm_bwd_scatter_kernel, x, xmap, w, rstd, dn, dR, (long)rows, cols);
  RET_LAUNCH("rmsnorm_bwd_scatter");
}
int launch_residual_norm_bwd(const float* x2, const float* w_pre, const float* rstd_pre, const float* dn, float* dR,
                             const bf16_t* t, const float* w_post, const float* rstd_t, bf16_t* dt, int rows,
                             int cols, hipStream_t st) {
  if (check_cols(cols)) return -1;
  if (rows <= 0) return 0;
  NORM_DISPATCH(residual_norm_bwd_kernel, x2, w_pre, rstd_pre, dn, dR, t, w_post, rstd_t, dt,
                     (long)rows, cols);
  RET_LAUNCH("residual_norm_bwd");
}
int launch_post_norm_bwd(const float* dR, const bf16_t* t, const float* w, const float* rstd_t, bf16_t* dt,
                         int rows, int cols, hipStream_t st) {
  if (check_cols(cols)) return -1;
  if (rows <= 0) return 0;
  NORM_DISPATCH(post_norm_bwd_kernel, dR, t, w, rstd_t, dt, (long)rows, cols);
  RET_LAUNCH("post_norm_bwd");
}

}  // namespace ptk
