// Byte-moving and reduction kernels of the Stage-1 step (all HBM-bound):
// transpose, im2col, LLM input assembly, fused cross-entropy fwd/bwd,
// projector-grad gather, column sums, grad-norm + clip + AdamW, synthetic init.
#include "common.h"

#include <algorithm>
#include <cstdlib>
#include "ptk_internal.h"

namespace ptk {

#define RET_OK(name) return hipGetLastError() == hipSuccess ? 0 : set_error(name " launch failed")

// ---------------------------------------------------------------- transpose
// in[z] [rows][cols] (ld_in) -> out[z] [cols][rows_pad] (ld_out), 64x64 tiles via LDS.
__global__ void __launch_bounds__(256) transpose_kernel(const bf16_t* __restrict__ in, long ld_in, long sin0, long sin1,
                                                        int zin, bf16_t* __restrict__ out, long ld_out, long sout0,
                                                        long sout1, int rows, int cols, int rows_pad) {
  __shared__ bf16_t tile[64][66];
  const int z = blockIdx.z, z0 = z / zin, z1 = z - z0 * zin;
  const bf16_t* src = in + z0 * sin0 + z1 * sin1;
  bf16_t* dst = out + z0 * sout0 + z1 * sout1;
  const int r0 = blockIdx.y * 64, c0 = blockIdx.x * 64;
  const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int r = r0 + ty + 16 * k;
    const int c = c0 + tx * 4;
    u16x4_t v = {0, 0, 0, 0};
    if (r < rows) {
      if (c + 3 < cols && ((ld_in & 3) == 0)) {
        v = *reinterpret_cast<const u16x4_t*>(src + (long)r * ld_in + c);
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = (c + e < cols) ? src[(long)r * ld_in + c + e] : 0;
      }
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) tile[ty + 16 * k][tx * 4 + e] = v[e];
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int oc = c0 + ty + 16 * k;      // output row = input col
    const int orr = r0 + tx * 4;          // output col = input row
    if (oc >= cols) continue;
    u16x4_t v;
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = tile[tx * 4 + e][ty + 16 * k];
    if (orr + 3 < rows_pad && ((ld_out & 3) == 0)) {
      *reinterpret_cast<u16x4_t*>(dst + (long)oc * ld_out + orr) = v;
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (orr + e < rows_pad) dst[(long)oc * ld_out + orr + e] = v[e];
    }
  }
}

int launch_transpose(const bf16_t* in, long ld_in, long sin0, long sin1, int zin, bf16_t* out, long ld_out,
                     long sout0, long sout1, int nz, int rows, int cols, int rows_pad, hipStream_t st) {
  if (rows <= 0 || cols <= 0 || nz <= 0) return 0;
  if (rows_pad < rows) return set_error("transpose: rows_pad < rows");
  dim3 grid((unsigned)((cols + 63) / 64), (unsigned)((rows_pad + 63) / 64), (unsigned)nz);
  hipLaunchKernelGGL(transpose_kernel, grid, dim3(256), 0, st, in, ld_in, sin0, sin1, zin, out, ld_out, sout0,
                     sout1, rows, cols, rows_pad);
  RET_OK("transpose");
}

// ---------------------------------------------------------------- im2col (Conv2d k=P, stride=P)
// px [B][C][H][W] bf16 -> out [B*N][C*P*P], column order (c, ky, kx) = conv weight flatten order.
__global__ void __launch_bounds__(256) im2col_kernel(const bf16_t* __restrict__ px, bf16_t* __restrict__ out, int B,
                                                     int C, int H, int W, int P) {
  const int gx = W / P, gy = H / P;
  const int oct = P / 8;                                      // 8-wide kx groups per kernel row
  const long total = (long)B * gy * gx * C * P * oct;
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= total) return;
  long t = i;
  const int o = t % oct; t /= oct;
  const int ky = t % P; t /= P;
  const int c = t % C; t /= C;
  const int px_ = t % gx; t /= gx;
  const int py = t % gy; t /= gy;
  const int b = (int)t;
  const bf16_t* s = px + (((long)b * C + c) * H + (py * P + ky)) * W + px_ * P + o * 8;
  const long row = ((long)b * gy + py) * gx + px_;
  bf16_t* d = out + row * (C * P * P) + (long)c * P * P + ky * P + o * 8;
  *reinterpret_cast<u16x8_t*>(d) = *reinterpret_cast<const u16x8_t*>(s);
}

int launch_im2col(const bf16_t* px, bf16_t* out, int B, int C, int H, int W, int P, hipStream_t st) {
  if (P % 8 || H % P || W % P) return set_error("im2col: patch %d must be a multiple of 8 dividing %dx%d", P, H, W);
  const long total = (long)B * (H / P) * (W / P) * C * P * (P / 8);
  if (total <= 0) return 0;
  hipLaunchKernelGGL(im2col_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, px, out, B, C, H, W, P);
  RET_OK("im2col");
}

__global__ void cast_f32_bf16_kernel(const float* __restrict__ in, bf16_t* __restrict__ out, long n) {
  const long i = ((long)blockIdx.x * 256 + threadIdx.x) * 4;
  if (i + 3 < n) {
    float4 v = *reinterpret_cast<const float4*>(in + i);
    u16x4_t o;
    o[0] = f2bf(v.x); o[1] = f2bf(v.y); o[2] = f2bf(v.z); o[3] = f2bf(v.w);
    *reinterpret_cast<u16x4_t*>(out + i) = o;
  } else {
    for (long j = i; j < n; ++j) out[j] = f2bf(in[j]);
  }
}
int launch_cast_f32_bf16(const float* in, bf16_t* out, long n, hipStream_t st) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(cast_f32_bf16_kernel, dim3((unsigned)((n / 4 + 256) / 256)), dim3(256), 0, st, in, out, n);
  RET_OK("cast");
}

// ---------------------------------------------------------------- LLM input assembly
// Stage1/projector_trainer.py:183-212: text rows = E[ids] * bf16(sqrt(H)) (bf16 math,
// TF gemma3 :116-117), padded rows zeroed, key_valid = [1]*Nv ++ (ids != pad) ++ [0]*(Spad-S).
// Vision rows (s < Nv) are written by the projector GEMM epilogue and left alone.
__global__ void __launch_bounds__(256) build_llm_inputs_kernel(const bf16_t* __restrict__ E,
                                                               const int64_t* __restrict__ ids, int T, int Nv,
                                                               int S, int Spad, int H, float scale, int pad_id,
                                                               float* __restrict__ x, int32_t* __restrict__ kv) {
  const long row = blockIdx.x;
  const int b = (int)(row / Spad), s = (int)(row - (long)b * Spad);
  if (threadIdx.x == 0) {
    int valid = 0;
    if (s < Nv) valid = 1;
    else if (s < S) valid = ids[(long)b * T + (s - Nv)] != pad_id;
    kv[row] = valid;
  }
  if (s < Nv) return;
  float* xr = x + row * H;
  if (s >= S) {
    for (int c = threadIdx.x * 4; c < H; c += 1024) *reinterpret_cast<float4*>(xr + c) = make_float4(0, 0, 0, 0);
    return;
  }
  const long id = ids[(long)b * T + (s - Nv)];
  const bf16_t* er = E + id * H;
  for (int c = threadIdx.x * 4; c < H; c += 1024) {
    u16x4_t u = *reinterpret_cast<const u16x4_t*>(er + c);
    *reinterpret_cast<float4*>(xr + c) = make_float4(bfround(bf2f(u[0]) * scale), bfround(bf2f(u[1]) * scale),
                                                     bfround(bf2f(u[2]) * scale), bfround(bf2f(u[3]) * scale));
  }
}
int launch_build_llm_inputs(const bf16_t* embed, const int64_t* ids, int B, int T, int Nv, int S, int Spad, int H,
                            float scale_bf16, int pad_id, float* x, int32_t* key_valid, hipStream_t st) {
  if (H % 4) return set_error("build_llm_inputs: hidden %% 4");
  hipLaunchKernelGGL(build_llm_inputs_kernel, dim3((unsigned)((long)B * Spad)), dim3(256), 0, st, embed, ids, T, Nv,
                     S, Spad, H, scale_bf16, pad_id, x, key_valid);
  RET_OK("build_llm_inputs");
}

// ---------------------------------------------------------------- cross entropy
// dlogits = (softmax - onehot) * g in place over one row, 256 threads x 8 columns per 16-B access.  The
// loads of a group of 8 accesses go out before its stores (the compiler cannot move a load of the row above
// a store to it), so each thread keeps 8 loads in flight instead of 1.
PTK_DEV void ce_write_dlogits(bf16_t* __restrict__ lr, int V, float lse, long tgt, float g) {
  auto one = [&](int c, const u16x8_t& u) {
    u16x8_t o;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float p = __expf(bf2f(u[e]) - lse);
      if (c + e == tgt) p -= 1.f;
      o[e] = f2bf(p * g);
    }
    *reinterpret_cast<u16x8_t*>(lr + c) = o;
  };
  int c = threadIdx.x * 8;
  for (; c + 7 * 2048 < V; c += 8 * 2048) {
    u16x8_t u[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) u[j] = *reinterpret_cast<const u16x8_t*>(lr + c + j * 2048);
#pragma unroll
    for (int j = 0; j < 8; ++j) one(c + j * 2048, u[j]);
  }
  for (; c < V; c += 2048) one(c, *reinterpret_cast<const u16x8_t*>(lr + c));
}

// ForCausalLMLoss (TF/loss/loss_utils.py:49-67): logits (bf16, as the reference's
// autocast lm_head produces) upcast to fp32, CE mean over valid targets.
// One block per row: pass 1 online max/sum-exp, pass 2 writes
// dlogits = (softmax - onehot) * gscale in place (bf16).
__global__ void __launch_bounds__(256) ce_kernel(bf16_t* __restrict__ logits, long ld, int V,
                                                 const int64_t* __restrict__ targets, float* __restrict__ row_loss,
                                                 const float* __restrict__ gscale) {
  __shared__ float red[8];
  const long r = blockIdx.x;
  bf16_t* lr = logits + r * ld;
  const long tgt = targets[r];
  float m = -INFINITY, s = 0.f;
  for (int c = threadIdx.x * 8; c < V; c += 2048) {
    u16x8_t u = *reinterpret_cast<const u16x8_t*>(lr + c);
    float v[8], vm = -INFINITY;
#pragma unroll
    for (int e = 0; e < 8; ++e) { v[e] = bf2f(u[e]); vm = fmaxf(vm, v[e]); }
    const float mn = fmaxf(m, vm);
    float acc = s * __expf(m - mn);
#pragma unroll
    for (int e = 0; e < 8; ++e) acc += __expf(v[e] - mn);
    m = mn;
    s = acc;
  }
  const float M = block_max<256>(m, red);
  const float Ssum = block_sum<256>(m == -INFINITY ? 0.f : s * __expf(m - M), red);
  const float lse = M + __logf(Ssum);
  const bool valid = tgt >= 0;
  if (threadIdx.x == 0) row_loss[r] = valid ? lse - bf2f(lr[tgt]) : 0.f;
  __syncthreads();   // target logit read before it is overwritten
  ce_write_dlogits(lr, V, lse, tgt, valid ? gscale[0] : 0.f);
}
// The same loss and d(logits) from the lm_head GEMM's softmax statistics (GemmArgs::row_stats: per row and
// 64-column chunk the max and sum exp(x - max) of the bf16 logits): the row's log-sum-exp is combined from
// its V / 64 chunk statistics, so the logits are read once (and d(logits) written in place) instead of
// twice.  Same arithmetic per element as ce_kernel; the sum over the row is taken in a different order.
__global__ void __launch_bounds__(256) ce_stats_kernel(bf16_t* __restrict__ logits, long ld, int V,
                                                       const float* __restrict__ stats, long ld_stats,
                                                       const int64_t* __restrict__ targets,
                                                       float* __restrict__ row_loss, const float* __restrict__ gscale) {
  __shared__ float red[8];
  const long r = blockIdx.x;
  bf16_t* lr = logits + r * ld;
  const float* st = stats + r * ld_stats;
  const int nch = V >> 6;
  const long tgt = targets[r];
  float m = -INFINITY, s = 0.f;
  for (int k = threadIdx.x; k < nch; k += 256) {
    const float2 ms = *reinterpret_cast<const float2*>(st + 2 * k);
    const float mn = fmaxe(m, ms.x);   // NaN-propagating: a NaN chunk max makes the row NaN (fmaxf would drop it)
    s = (m == -INFINITY ? 0.f : s * __expf(m - mn)) + (ms.x == -INFINITY ? 0.f : ms.y * __expf(ms.x - mn));
    m = mn;
  }
  const float M = block_max<256>(m, red);
  const float Ssum = block_sum<256>(m == -INFINITY ? 0.f : s * __expf(m - M), red);
  const float lse = M + __logf(Ssum);
  const bool valid = tgt >= 0;
  if (threadIdx.x == 0) row_loss[r] = valid ? lse - bf2f(lr[tgt]) : 0.f;
  __syncthreads();   // target logit read before it is overwritten
  ce_write_dlogits(lr, V, lse, tgt, valid ? gscale[0] : 0.f);
}
int launch_ce_stats_fwd_bwd(bf16_t* logits, long ld, int R, int V, const float* stats, long ld_stats,
                            const int64_t* targets, float* row_loss, const float* gscale, hipStream_t st) {
  if (V % 64 || ld % 8) return set_error("ce_stats: vocab %% 64");
  if (R <= 0) return 0;
  hipLaunchKernelGGL(ce_stats_kernel, dim3(R), dim3(256), 0, st, logits, ld, V, stats, ld_stats, targets, row_loss,
                     gscale);
  RET_OK("ce_stats");
}
int launch_ce_fwd_bwd(bf16_t* logits, long ld, int R, int V, const int64_t* targets, float* row_loss,
                      const float* gscale, hipStream_t st) {
  if (V % 8 || ld % 8) return set_error("ce: vocab %% 8");
  if (R <= 0) return 0;
  hipLaunchKernelGGL(ce_kernel, dim3(R), dim3(256), 0, st, logits, ld, V, targets, row_loss, gscale);
  RET_OK("ce");
}

// zero-fill of a 16-B aligned buffer (bytes % 16 == 0) by 16-B stores.  Used instead of hipMemsetAsync so
// that a captured step is kernel nodes only (graph_step); grid-stride over at most 4 blocks per CU.
__global__ void __launch_bounds__(256) zero16_kernel(uint4* __restrict__ p, long n16) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n16; i += (long)gridDim.x * 256) p[i] = uint4{0, 0, 0, 0};
}
// PTK_HIP_MEMSET=1 (diagnostic builds only, -DPTK_DIAG): hipMemsetAsync instead, the form graph_step's
// retired-graph corruption was traced to (tools/graph_debug.py DESTROY=1: NaN grads with memset nodes in the
// captured step, none without).  The product library always zero-fills by kernel.
static bool hip_memset_ab() {
#ifdef PTK_DIAG
  static const bool v = [] { const char* e = getenv("PTK_HIP_MEMSET"); return e && e[0] == '1'; }();
  return v;
#else
  return false;
#endif
}
int launch_zero(void* p, size_t bytes, hipStream_t st) {
  if (((uintptr_t)p | bytes) & 15) return set_error("zero: pointer / size not 16-B aligned");
  if (hip_memset_ab())
    return hipMemsetAsync(p, 0, bytes, st) == hipSuccess ? 0 : set_error("zero: hipMemsetAsync failed");
  const long n16 = (long)(bytes / 16);
  if (n16 == 0) return 0;
  const long blocks = std::min<long>((n16 + 255) / 256, 1024);
  hipLaunchKernelGGL(zero16_kernel, dim3((unsigned)blocks), dim3(256), 0, st, (uint4*)p, n16);
  RET_OK("zero");
}

__global__ void __launch_bounds__(256) count_valid_kernel(const int64_t* __restrict__ labels, int n, float loss_scale,
                                                          float* gscale, float* count) {
  __shared__ float red[4];
  float c = 0.f;
  for (int i = threadIdx.x; i < n; i += 256) c += labels[i] != -100 ? 1.f : 0.f;
  c = block_sum<256>(c, red);
  if (threadIdx.x == 0) {
    count[0] = c;
    gscale[0] = c > 0.f ? loss_scale / c : 0.f;
  }
}
int launch_count_valid(const int64_t* labels, int n, float loss_scale, float* gscale, float* count, hipStream_t st) {
  hipLaunchKernelGGL(count_valid_kernel, dim3(1), dim3(256), 0, st, labels, n, loss_scale, gscale, count);
  RET_OK("count_valid");
}

__global__ void __launch_bounds__(256) loss_reduce_kernel(const float* __restrict__ rl, int R, const float* count,
                                                          float* loss) {
  __shared__ float red[4];
  float s = 0.f;
  for (int i = threadIdx.x; i < R; i += 256) s += rl[i];
  s = block_sum<256>(s, red);
  if (threadIdx.x == 0) loss[0] = count[0] > 0.f ? s / count[0] : NAN;
}
int launch_loss_reduce(const float* row_loss, int R, const float* count, float* loss, hipStream_t st) {
  hipLaunchKernelGGL(loss_reduce_kernel, dim3(1), dim3(256), 0, st, row_loss, R, count, loss);
  RET_OK("loss_reduce");
}

// ---------------------------------------------------------------- projector grad plumbing
// dy[(b,i)] = bf16(dX_llm[b*Spad + i - 1]) for i >= 1, 0 for the dropped patch 0
// (Stage1/projector_trainer.py:173 slices [:,1:,:] before the projector).
__global__ void __launch_bounds__(256) gather_dy_kernel(const float* __restrict__ dx, int N, int Spad, int H,
                                                        bf16_t* __restrict__ dy) {
  const long row = blockIdx.x;
  const int b = (int)(row / N), i = (int)(row - (long)b * N);
  bf16_t* o = dy + row * H;
  for (int c = threadIdx.x * 4; c < H; c += 1024) {
    u16x4_t u = {0, 0, 0, 0};
    if (i > 0) {
      float4 v = *reinterpret_cast<const float4*>(dx + ((long)b * Spad + i - 1) * H + c);
      u[0] = f2bf(v.x); u[1] = f2bf(v.y); u[2] = f2bf(v.z); u[3] = f2bf(v.w);
    }
    *reinterpret_cast<u16x4_t*>(o + c) = u;
  }
}
int launch_gather_dy(const float* dx, int B, int N, int Spad, int H, bf16_t* dy, hipStream_t st) {
  if (H % 4) return set_error("gather_dy: hidden %% 4");
  hipLaunchKernelGGL(gather_dy_kernel, dim3((unsigned)((long)B * N)), dim3(256), 0, st, dx, N, Spad, H, dy);
  RET_OK("gather_dy");
}

// column sums of bf16 [rows][cols] -> f32 [cols] (the projector's bias grads): stage 1 over row chunks, stage 2
// over chunks in chunk order.  A lane owns 8 adjacent columns (16-B loads) and keeps 8 rows' loads in flight,
// adding them in row order; the chunk count is chosen so the grid holds >= 4096 waves where the partial buffer
// allows it (1152 columns: 144 lanes per row, so 64 chunks left the chip latency-bound at 0.6 TB/s).
__global__ void __launch_bounds__(64) colsum_partial_kernel(const bf16_t* __restrict__ x, int rows, int cols,
                                                            int per, float* __restrict__ partial) {
  const int cg = blockIdx.x * 64 + threadIdx.x;
  if (cg * 8 >= cols) return;
  const int r0 = blockIdx.y * per, r1 = min(rows, r0 + per);
  const bf16_t* xp = x + (long)cg * 8;
  float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  int r = r0;
  for (; r + 8 <= r1; r += 8) {
    u16x8_t u[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) u[j] = *reinterpret_cast<const u16x8_t*>(xp + (long)(r + j) * cols);
#pragma unroll
    for (int j = 0; j < 8; ++j)
#pragma unroll
      for (int e = 0; e < 8; ++e) s[e] += bf2f(u[j][e]);
  }
  for (; r < r1; ++r) {
    const u16x8_t u = *reinterpret_cast<const u16x8_t*>(xp + (long)r * cols);
#pragma unroll
    for (int e = 0; e < 8; ++e) s[e] += bf2f(u[e]);
  }
  float* pp = partial + (long)blockIdx.y * cols + cg * 8;
  *reinterpret_cast<float4*>(pp) = make_float4(s[0], s[1], s[2], s[3]);
  *reinterpret_cast<float4*>(pp + 4) = make_float4(s[4], s[5], s[6], s[7]);
}
// stage 2: 8 threads per column, thread g summing chunks g, g + 8, ... (8 loads in flight), then the 8 sums in
// g order through LDS
__global__ void __launch_bounds__(256) colsum_final_kernel(const float* __restrict__ partial, int cols, int chunks,
                                                           float* __restrict__ out) {
  __shared__ float red[8][33];
  const int cl = threadIdx.x & 31, g = threadIdx.x >> 5;
  const int c = blockIdx.x * 32 + cl;
  float s = 0.f;
  if (c < cols) {
    int k = g;
    for (; k + 56 < chunks; k += 64) {
      float v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = partial[(long)(k + 8 * j) * cols + c];
#pragma unroll
      for (int j = 0; j < 8; ++j) s += v[j];
    }
    for (; k < chunks; k += 8) s += partial[(long)k * cols + c];
  }
  red[g][cl] = s;
  __syncthreads();
  if (g == 0 && c < cols) {
    float t = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) t += red[j][cl];
    out[c] = t;
  }
}
int launch_colsum_bf16(const bf16_t* x, int rows, int cols, float* out, float* partial, long part_floats,
                       hipStream_t st) {
  if (cols % 8 || ((uintptr_t)x & 15) || ((uintptr_t)partial & 15)) return set_error("colsum: cols %% 8 / alignment");
  if (rows <= 0 || cols <= 0) return 0;
  const int lanes = cols / 8, blocks_x = (lanes + 63) / 64;
  long chunks = std::max<long>(1, std::min<long>(4096 / blocks_x, (rows + 15) / 16));
  chunks = std::max<long>(1, std::min<long>(chunks, part_floats / cols));
  const int per = (int)((rows + chunks - 1) / chunks);
  chunks = (rows + per - 1) / per;
  hipLaunchKernelGGL(colsum_partial_kernel, dim3((unsigned)blocks_x, (unsigned)chunks), dim3(64), 0, st, x, rows, cols,
                     per, partial);
  hipLaunchKernelGGL(colsum_final_kernel, dim3((cols + 31) / 32), dim3(256), 0, st, partial, cols, (int)chunks, out);
  RET_OK("colsum");
}

// ---------------------------------------------------------------- grad norm + clip + AdamW
// clip_grad_norm_(5.0) then torch.optim.AdamW (Stage1/projector_trainer.py:75-79, :240-242)
// over the projector's flat fp32 parameter buffer.  grad_scale folds DDP's 1/W.
__global__ void __launch_bounds__(256) sumsq_kernel(const float* __restrict__ x, long n, float* __restrict__ partial) {
  __shared__ float red[4];
  float s = 0.f;
  for (long i = ((long)blockIdx.x * 256 + threadIdx.x) * 4; i < n; i += (long)gridDim.x * 1024) {
    if (i + 3 < n) {
      float4 v = *reinterpret_cast<const float4*>(x + i);
      s += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
    } else {
      for (long j = i; j < n; ++j) s += x[j] * x[j];
    }
  }
  s = block_sum<256>(s, red);
  if (threadIdx.x == 0) partial[blockIdx.x] = s;
}
int launch_sumsq_partial(const float* x, long n, float* partial, int nparts, hipStream_t st) {
  hipLaunchKernelGGL(sumsq_kernel, dim3(nparts), dim3(256), 0, st, x, n, partial);
  RET_OK("sumsq");
}

__global__ void __launch_bounds__(256) clip_adamw_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                         float* __restrict__ m, float* __restrict__ v, long n,
                                                         const float* __restrict__ partial, int nparts,
                                                         float grad_scale, float max_norm, float lr, float b1,
                                                         float b2, float eps, float wd, float bc1, float bc2s,
                                                         float* norm_out) {
  __shared__ float red[4];
  __shared__ float coef_s;
  float s = 0.f;
  for (int i = threadIdx.x; i < nparts; i += 256) s += partial[i];
  s = block_sum<256>(s, red);
  if (threadIdx.x == 0) {
    const float norm = sqrtf(s) * grad_scale;
    coef_s = fminf(max_norm / (norm + 1e-6f), 1.f) * grad_scale;
    if (blockIdx.x == 0 && norm_out) norm_out[0] = norm;
  }
  __syncthreads();
  const float coef = coef_s;
  const float step_size = lr / bc1;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    const float gi = g[i] * coef;
    float pi = p[i] * (1.f - lr * wd);
    const float mi = m[i] + (1.f - b1) * (gi - m[i]);
    const float vi = v[i] * b2 + (1.f - b2) * gi * gi;
    pi -= step_size * mi / (sqrtf(vi) / bc2s + eps);
    p[i] = pi;
    m[i] = mi;
    v[i] = vi;
  }
}
int launch_clip_adamw(float* p, const float* g, float* m, float* v, long n, const float* partial, int nparts,
                      float grad_scale, float max_norm, float lr, float b1, float b2, float eps, float wd, int step,
                      float* norm_out, hipStream_t st) {
  const float bc1 = 1.f - powf(b1, (float)step);
  const float bc2s = sqrtf(1.f - powf(b2, (float)step));
  hipLaunchKernelGGL(clip_adamw_kernel, dim3(1024), dim3(256), 0, st, p, g, m, v, n, partial, nparts, grad_scale,
                     max_norm, lr, b1, b2, eps, wd, bc1, bc2s, norm_out);
  RET_OK("clip_adamw");
}

// ---------------------------------------------------------------- synthetic init (bench weights)
PTK_DEV uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}
__global__ void fill_normal_kernel(bf16_t* __restrict__ out, long n, uint64_t seed, float std, float mean) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const uint64_t h = splitmix64(seed ^ splitmix64((uint64_t)i));
  const float u1 = ((h >> 40) + 1) * (1.0f / 16777217.0f);
  const float u2 = ((h & 0xFFFFFF) + 0.5f) * (1.0f / 16777216.0f);
  const float z = sqrtf(-2.f * __logf(u1)) * __cosf(6.283185307f * u2);
  out[i] = f2bf(mean + std * z);
}
int launch_fill_normal_bf16(bf16_t* out, long n, uint64_t seed, float std, float mean, hipStream_t st) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(fill_normal_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, out, n, seed, std,
                     mean);
  RET_OK("fill_normal");
}

}  // namespace ptk

namespace ptk {
// out[i] = sum_s part[s][i]  (split-K partial reduction, fixed order: deterministic)
__global__ void __launch_bounds__(256) sum_partials_kernel(const float* __restrict__ part, int nsplit, long n,
                                                           float* __restrict__ out) {
  const long i = ((long)blockIdx.x * 256 + threadIdx.x) * 4;
  if (i >= n) return;
  float4 acc = *reinterpret_cast<const float4*>(part + i);
  for (int s = 1; s < nsplit; ++s) {
    const float4 v = *reinterpret_cast<const float4*>(part + (long)s * n + i);
    acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
  }
  *reinterpret_cast<float4*>(out + i) = acc;
}
int launch_sum_partials(const float* part, int nsplit, long n, float* out, hipStream_t st) {
  if (n % 4) return set_error("sum_partials: n %% 4");
  hipLaunchKernelGGL(sum_partials_kernel, dim3((unsigned)((n / 4 + 255) / 256)), dim3(256), 0, st, part, nsplit, n,
                     out);
  return hipGetLastError() == hipSuccess ? 0 : set_error("sum_partials launch failed");
}
}  // namespace ptk

namespace ptk {
// GEGLU backward as a streaming pass (TF gemma3 :131-133 autograd, bf16 ops) from the forward's saved factors
// (common.h geglu_fwd2: a = bf16(gelu_tanh(g)), b = bf16(gelu_tanh'(g) * u)):
//   dg = bf16(dh * b),  du = bf16(dh * a)
// dh, a, b [M, I] bf16 -> dgu [M, 2I] bf16 in the interleaved gate/up layout (16-column groups).
__global__ void __launch_bounds__(256) geglu_bwd_kernel(const bf16_t* __restrict__ dh, const bf16_t* __restrict__ g,
                                                        const bf16_t* __restrict__ u, bf16_t* __restrict__ dgu,
                                                        long n8, int I) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;   // one 8-element group
  if (i >= n8) return;
  const long e0 = i * 8;
  const long r = e0 / I;
  const int c = (int)(e0 - r * I);
  const u16x8_t vd = *reinterpret_cast<const u16x8_t*>(dh + e0);
  const u16x8_t vg = *reinterpret_cast<const u16x8_t*>(g + e0);
  const u16x8_t vu = *reinterpret_cast<const u16x8_t*>(u + e0);
  u16x8_t og, ou;   // (vg: the factor a, vu: the factor b)
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const float d = bf2f(vd[k]);
    og[k] = f2bf(d * bf2f(vu[k]));
    ou[k] = f2bf(d * bf2f(vg[k]));
  }
  bf16_t* o = dgu + r * 2L * I + (c >> 4) * 32 + (c & 15);
  *reinterpret_cast<u16x8_t*>(o) = og;
  *reinterpret_cast<u16x8_t*>(o + 16) = ou;
}
int launch_geglu_bwd(const bf16_t* dh, const bf16_t* g, const bf16_t* u, bf16_t* dgu, long M, int I, hipStream_t st) {
  if (I % 16) return set_error("geglu_bwd: intermediate %% 16");
  const long n8 = M * I / 8;
  hipLaunchKernelGGL(geglu_bwd_kernel, dim3((unsigned)((n8 + 255) / 256)), dim3(256), 0, st, dh, g, u, dgu, n8, I);
  return hipGetLastError() == hipSuccess ? 0 : set_error("geglu_bwd launch failed");
}
}  // namespace ptk
