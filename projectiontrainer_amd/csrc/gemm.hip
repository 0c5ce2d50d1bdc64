// bf16 MFMA GEMM for gfx950 with fused epilogues.
//
//   C[z][M,N] = epi( alpha * A[z][M,K] . B[z][N,K]^T )
//
// Both operands K-contiguous ("NT"): A is an activation [tokens, K], B is a
// weight stored like nn.Linear ([out, in]) or a pre-transposed copy of one.
// Every dense contraction of the Stage-1 step maps onto this one kernel:
// Linear forwards (x . W^T), frozen-weight dX (dY . (W^T)^T with W^T stored),
// attention scores (Q . K^T) and P.V (P . (V^T)^T), projector weight grads
// (dY^T . (H^T)^T).
//
// Tile 128x128x64, 256 threads = 4 waves (2x2), each wave 64x64 as 4x4
// v_mfma_f32_16x16x32_bf16 tiles (fp32 accumulate).  Operands are staged
// global->LDS with global_load_lds_dwordx4 (LDS-DMA, 1 KiB per wave
// instruction = 8 rows x 128 B), double-buffered so the next K-tile's DMA
// overlaps the current tile's MFMAs.  LDS rows are 128 B; the 16-B chunk of
// logical k-chunk c in row r sits at c ^ ((r>>1)&7), applied on the DMA
// *source* address (LDS stays lane-linear) and on the ds_read_b128 address,
// which makes every 16-lane ds_read_b128 group conflict-free.
// Block ids are remapped so each XCD walks a contiguous range of tiles in
// GROUP_M-row groups (L2 reuse of A row-panels and B column-panels).
#include <stdlib.h>

#include "common.h"
#include "ptk_internal.h"
#include "gemm_epi.h"

#include <algorithm>
#include <vector>

namespace ptk {

constexpr int BM = 128, BN = 128, BK = 64, GROUP_M = 8;
constexpr int STAGE_BYTES = (BM + BN) * BK * 2;   // 32 KiB
static_assert(4 * 64 * 68 * 4 >= 2 * STAGE_BYTES, "epilogue staging must cover the pipeline buffers");

typedef const __attribute__((address_space(1))) void* gptr_t;
typedef __attribute__((address_space(3))) void* lptr_t;

// diagnostic: PTK_NO_SRC_SWZ builds stage the 256x256 kernels' tiles without the XOR source swizzle
// (wrong results, timing only: does a lane-permuted DMA source cost issue time?)
#ifdef PTK_NO_SRC_SWZ
#define PTK_SRC_SWZ(c, r) (c)
#else
#define PTK_SRC_SWZ(c, r) ((c) ^ (((r) >> 1) & 7))
#endif

#ifndef PTK_GLDS_AUX
#define PTK_GLDS_AUX 0   // cache-policy bits of the LDS-DMA staging loads (diagnostic builds vary it)
#endif
PTK_DEV void glds16(const void* src, void* lds) {
  __builtin_amdgcn_global_load_lds((gptr_t)src, (lptr_t)lds, 16, 0, PTK_GLDS_AUX);
}

template <int ACT, int OUT>
PTK_DEV void epilogue(const GemmArgs& p, char* smem, int wave, int lane, f32x4_t (&acc)[4][4], long row0,
                      long col0, char* Cz) {
  // stage: lane holds C[16i + 4fq + j][16k + fr]
  float* T = reinterpret_cast<float*>(smem + wave * EPI_WAVE_BYTES);
  const int fr = lane & 15, fq = lane >> 4;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int k = 0; k < 4; ++k)
#pragma unroll
      for (int j = 0; j < 4; ++j) T[(16 * i + 4 * fq + j) * EPI_LD + 16 * k + fr] = p.alpha * acc[i][k][j];
  __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0): own LDS writes done (wave-private region)
  __builtin_amdgcn_wave_barrier();
  const bool vec_ok = ((p.ldc & 3) == 0) && (!p.resid || (p.ld_resid & 3) == 0) &&
                      (!p.resid16 || (p.ld_resid16 & 7) == 0) &&
                      (!p.rowadd || (p.ld_rowadd & 3) == 0) && (!p.aux || (p.ld_aux & 3) == 0) &&
                      (!p.aux_in || (p.ld_aux_in & 3) == 0);
  if constexpr (ACT == ACT_GEGLU) {
    const bool v8 = ((p.ldc | p.ld_aux) & 7) == 0;
    if (v8) {
      // 4 lanes per row, each 8 h-columns (one 16-B store per output); 16 rows per pass
      const int rr = lane >> 2, cg = lane & 3, q = cg >> 1, cc = (cg & 1) * 8;
      const long hc = col0 / 2 + q * 16 + cc;
#pragma unroll
      for (int it = 0; it < 4; ++it) {
        const int lr = it * 16 + rr;
        const long r = row0 + lr;
        if (r >= p.M || 2 * hc >= p.N) continue;
        const float* tg = T + lr * EPI_LD + q * 32 + cc;
        float g[8], u[8];
        *reinterpret_cast<float4*>(g) = *reinterpret_cast<const float4*>(tg);
        *reinterpret_cast<float4*>(g + 4) = *reinterpret_cast<const float4*>(tg + 4);
        *reinterpret_cast<float4*>(u) = *reinterpret_cast<const float4*>(tg + 16);
        *reinterpret_cast<float4*>(u + 4) = *reinterpret_cast<const float4*>(tg + 20);
        geglu_vec8(p, Cz, r, hc, g, u);
      }
    } else {
      // 8 lanes per row, each 4 h-columns; 8 rows per pass
      const int rr = lane >> 3, cg = lane & 7, q = cg >> 2, cc = (cg & 3) * 4;
      const long hc = col0 / 2 + q * 16 + cc;
#pragma unroll
      for (int it = 0; it < 8; ++it) {
        const int lr = it * 8 + rr;
        const long r = row0 + lr;
        if (r >= p.M || 2 * hc >= p.N) continue;
        const float4 g = *reinterpret_cast<const float4*>(T + lr * EPI_LD + q * 32 + cc);
        const float4 u = *reinterpret_cast<const float4*>(T + lr * EPI_LD + q * 32 + 16 + cc);
        geglu_vec4(p, Cz, r, hc, g, u);
      }
    }
  } else if (ACT == ACT_GEGLU_BWD && ((p.ldc | p.ld_aux_in) & 7) == 0 && col0 + 63 < p.N) {
    // 8 lanes per row, each 8 columns; 8 rows per pass
    const int rr = lane >> 3, c8 = (lane & 7) * 8;
    const long c = col0 + c8;
#pragma unroll
    for (int it = 0; it < 8; ++it) {
      const int lr = it * 8 + rr;
      const long r = row0 + lr;
      if (r >= p.M) continue;
      float v[8];
      *reinterpret_cast<float4*>(v) = *reinterpret_cast<const float4*>(T + lr * EPI_LD + c8);
      *reinterpret_cast<float4*>(v + 4) = *reinterpret_cast<const float4*>(T + lr * EPI_LD + c8 + 4);
      geglu_bwd_vec8(p, Cz, r, c, v);
    }
  } else if (OUT == OUT_BF16 && ACT != ACT_GEGLU_BWD && vec_ok && ((p.ldc & 7) == 0) &&
             (!p.aux || (p.ld_aux & 7) == 0) && (!p.aux_in || (p.ld_aux_in & 7) == 0) && col0 + 63 < p.N) {
    // 8 lanes per row, each 8 columns (16-B stores); 8 rows per pass
    const int rr = lane >> 3, c8 = (lane & 7) * 8;
    const long c = col0 + c8;
    if (ACT == ACT_NONE && p.row_stats) {
      // softmax statistics (max, sum exp(x - max)) of each row's 64 columns, from the bf16-rounded values the
      // logits store holds.  This runs with the MFMAs idle (one workgroup per CU, lock-step epilogue), so it is
      // written for VALU issue slots: NaN-propagating v_maximum3 (no operand canonicalisation), packed f32 FMAs
      // and adds, the 8 rows' max all-reduced over the row's 8 lanes by DPP, the 8 rows' sums reduce-scattered
      // (partners 7 - j, j ^ 1, j ^ 2: 7 DPP adds instead of 24), after which lane j holds the row
      // 4 (j >= 4) + 2 (j & 1) + ((j >> 1) & 1) of its row group and stores that row's pair: one 8-B store per lane.
      constexpr float L2E = 1.4426950408889634f;
      const f32x2_t l2e = {L2E, L2E};
      float mx[8], sm[8];
#pragma unroll
      for (int it = 0; it < 8; ++it) {
        const float* tr = T + (it * 8 + rr) * EPI_LD + c8;
        const float4 v0 = *reinterpret_cast<const float4*>(tr);
        const float4 v1 = *reinterpret_cast<const float4*>(tr + 4);
        const f32x2_t x0 = bfround2(f32x2_t{v0.x, v0.y}), x1 = bfround2(f32x2_t{v0.z, v0.w});
        const f32x2_t x2 = bfround2(f32x2_t{v1.x, v1.y}), x3 = bfround2(f32x2_t{v1.z, v1.w});
        float m = fmax3e(fmax3e(x0[0], x0[1], x1[0]), fmax3e(x1[1], x2[0], x2[1]), fmaxe(x3[0], x3[1]));
        m = fmaxe(m, dpp<0xB1>(m));
        m = fmaxe(m, dpp<0x4E>(m));
        m = fmaxe(m, dpp<0x141>(m));
        const float nm = -m * L2E;
        const f32x2_t nm2 = {nm, nm};
        const f32x2_t a0 = x0 * l2e + nm2, a1 = x1 * l2e + nm2, a2 = x2 * l2e + nm2, a3 = x3 * l2e + nm2;
        const f32x2_t e0 = {__builtin_amdgcn_exp2f(a0[0]), __builtin_amdgcn_exp2f(a0[1])};
        const f32x2_t e1 = {__builtin_amdgcn_exp2f(a1[0]), __builtin_amdgcn_exp2f(a1[1])};
        const f32x2_t e2 = {__builtin_amdgcn_exp2f(a2[0]), __builtin_amdgcn_exp2f(a2[1])};
        const f32x2_t e3 = {__builtin_amdgcn_exp2f(a3[0]), __builtin_amdgcn_exp2f(a3[1])};
        const f32x2_t s2 = (e0 + e1) + (e2 + e3);
        mx[it] = m;
        sm[it] = s2[0] + s2[1];
      }
      const int j = lane & 7;
      const bool b1 = j >= 4, b2 = j & 1, b3 = (j >> 1) & 1;
      float s4[4], m4[4], s2[2], m2[2];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        s4[i] = (b1 ? sm[i + 4] : sm[i]) + dpp<0x141>(b1 ? sm[i] : sm[i + 4]);
        m4[i] = b1 ? mx[i + 4] : mx[i];
      }
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        s2[i] = (b2 ? s4[i + 2] : s4[i]) + dpp<0xB1>(b2 ? s4[i] : s4[i + 2]);
        m2[i] = b2 ? m4[i + 2] : m4[i];
      }
      const float ss = (b3 ? s2[1] : s2[0]) + dpp<0x4E>(b3 ? s2[0] : s2[1]);
      const float ms = b3 ? m2[1] : m2[0];
      const long rs = row0 + (4 * b1 + 2 * b2 + b3) * 8 + rr;
      if (rs < p.M) *reinterpret_cast<float2*>(p.row_stats + rs * p.ld_stats + 2 * (col0 >> 6)) = make_float2(ms, ss);
      if (p.stats_only) return;   // diagnostic: what the lm_head costs without writing its logits
    }
#pragma unroll
    for (int it = 0; it < 8; ++it) {
      const int lr = it * 8 + rr;
      const long r = row0 + lr;
      const float4 v0 = *reinterpret_cast<const float4*>(T + lr * EPI_LD + c8);
      const float4 v1 = *reinterpret_cast<const float4*>(T + lr * EPI_LD + c8 + 4);
      if (r >= p.M) continue;
      epi_vec8_bf16<ACT>(p, Cz, r, c, v0, v1);
    }
  } else {
    // 16 lanes per row, each 4 columns; 4 rows per pass
    const int rr = lane >> 4, c4 = (lane & 15) * 4;
    const long c = col0 + c4;
#pragma unroll 8
    for (int it = 0; it < 16; ++it) {
      const int lr = it * 4 + rr;
      const long r = row0 + lr;
      if (r >= p.M) continue;
      const float4 v = *reinterpret_cast<const float4*>(T + lr * EPI_LD + c4);
      if constexpr (ACT == ACT_GEGLU_BWD) {
        if (c + 3 < p.N) geglu_bwd_vec4(p, Cz, r, c, v);
      } else {
        if (vec_ok && c + 3 < p.N) {
          epi_vec4<ACT, OUT>(p, Cz, r, c, v);
        } else {
          float vv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
          for (int e = 0; e < 4; ++e)
            if (c + e < p.N) epi_scalar<ACT, OUT>(p, Cz, r, c + e, vv[e]);
        }
      }
    }
  }
}

template <int ACT, int OUT>
__global__ void __launch_bounds__(256, 2) gemm_nt_kernel(GemmArgs p) {
  __shared__ __attribute__((aligned(16))) char smem[4 * EPI_WAVE_BYTES];   // >= 2 * STAGE_BYTES
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 1, wc = wave & 1;

  const int nbm = (p.M + BM - 1) / BM, nbn = (p.N + BN - 1) / BN;
  const int ntile = nbm * nbn;
  int bid = blockIdx.x;
  {  // XCD remap (bijective): blocks b, b+8, ... share an XCD -> give them consecutive tiles
    const int q = ntile >> 3, rr = ntile & 7, x = bid & 7;
    bid = (x < rr ? x * (q + 1) : rr * (q + 1) + (x - rr) * q) + (bid >> 3);
  }
  const int per_group = GROUP_M * nbn;
  const int first_m = (bid / per_group) * GROUP_M;
  const int gsz = min(nbm - first_m, GROUP_M);
  const int bm = first_m + (bid % per_group) % gsz;
  const int bn = (bid % per_group) / gsz;

  const int z = blockIdx.z;
  const int z0 = z / p.zin, z1 = z - z0 * p.zin;
  const bf16_t* A = p.A + z0 * p.sA0 + z1 * p.sA1;
  const bf16_t* B = p.B + z0 * p.sB0 + z1 * p.sB1;

  // staging: lane i of a wave instruction writes LDS row (i>>3) chunk (i&7) of an 8-row group
  const int sr = lane >> 3, sc = lane & 7;
  const bf16_t* asrc[4];
  const bf16_t* bsrc[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int lr = wave * 32 + j * 8 + sr;
    const int lc = sc ^ ((lr >> 1) & 7);
    const long gm = min(bm * BM + lr, p.M - 1);
    const long am = map_row(p.amap, gm);
    asrc[j] = A + am * p.lda + lc * 8;
    const long gn = min(bn * BN + lr, p.N - 1);
    bsrc[j] = B + gn * p.ldb + lc * 8;
  }
  auto stage = [&](int t, int s) {
    char* base = smem + s * STAGE_BYTES + wave * 32 * 128;
#pragma unroll
    for (int j = 0; j < 4; ++j) glds16(asrc[j] + t * BK, base + j * 8 * 128);
#pragma unroll
    for (int j = 0; j < 4; ++j) glds16(bsrc[j] + t * BK, base + BM * 128 + j * 8 * 128);
  };

  f32x4_t acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4_t){0.f, 0.f, 0.f, 0.f};

  // per-lane fragment offset: row (lane&15), logical chunk (lane>>4), swizzled by (row>>1)&7
  const int frag_off = (lane & 15) * 128 + (((lane >> 4) ^ ((lane >> 1) & 7)) << 4);

  const int nt = p.K / BK;
  stage(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int t = 0; t < nt; ++t) {
    const int s = t & 1;
    if (t + 1 < nt) stage(t + 1, s ^ 1);
    const char* As = smem + s * STAGE_BYTES + wr * 64 * 128;
    const char* Bs = smem + s * STAGE_BYTES + BM * 128 + wc * 64 * 128;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8_t a[4], b[4];
#pragma unroll
      for (int i = 0; i < 4; ++i)
        a[i] = *reinterpret_cast<const bf16x8_t*>(As + i * 16 * 128 + (frag_off ^ (ks << 6)));
#pragma unroll
      for (int i = 0; i < 4; ++i)
        b[i] = *reinterpret_cast<const bf16x8_t*>(Bs + i * 16 * 128 + (frag_off ^ (ks << 6)));
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  // epilogue (LDS free after the loop's final barrier)
  char* Cz = reinterpret_cast<char*>(p.C) + (z0 * p.sC0 + z1 * p.sC1) * (OUT == OUT_BF16 ? 2 : 4);
  epilogue<ACT, OUT>(p, smem, wave, lane, acc, (long)bm * BM + wr * 64, (long)bn * BN + wc * 64, Cz);
}

// ---------------------------------------------------------------- 256x256 tile, 8 waves
// For the large projection GEMMs (M >= 1024, N >= 512).  Tile 256x256x64,
// 512 threads = 8 waves (2 along M x 4 along N), each wave 128x64 = 8x4
// MFMA 16x16x32 tiles (128 fp32 accumulators/lane).  LDS holds two K-tile
// buffers of four 16 KiB half-tiles (A rows 0-127 | A 128-255 | B 0-127 |
// B 128-255, same swizzle as above).  Each K-tile is four phases of 16 MFMAs
// (m-half x n-half of the wave tile); every phase issues exactly one half-tile
// of LDS-DMA for a later K-tile:
//   phase 0: A0(t+1)  1: A1(t+1)  2: B0(t+2)  3: B1(t+2)
// A half-tile is restaged only after the barrier that follows the phase that
// last read it (A: phase 2, B: phase 1), and the single counted wait per
// K-tile (vmcnt(4) at phase 3, B(t+2) still in flight) retires K-tile t+1
// one phase before it is read.  Raw s_barrier keeps the DMA in flight across
// barriers (a __syncthreads would drain vmcnt to 0).
constexpr int BIG = 256;
constexpr int HALF_BYTES = 128 * BK * 2;   // 16 KiB
constexpr int BUF_BYTES = 4 * HALF_BYTES;   // 64 KiB

#ifdef PTK_STAMPS
// diagnostic build only (make stamps): per-block s_memtime / s_memrealtime stamps of the 256x256 kernel
__device__ unsigned long long g_stamps[1 << 15][6];
__device__ int g_epi_mode;   // 0 normal, 1 no global stores, 2 no epilogue
#define PTK_STAMP(i)                                                                  \
  if (threadIdx.x == 0 && blockIdx.x < (1 << 15)) {                                   \
    g_stamps[blockIdx.x][i] = __builtin_amdgcn_s_memtime();                           \
    if (i == 0) g_stamps[blockIdx.x][5] = __builtin_amdgcn_s_memrealtime();           \
    if (i == 3) g_stamps[blockIdx.x][4] = __builtin_amdgcn_s_memrealtime();           \
  }
#else
#define PTK_STAMP(i)
#endif

#define PTK_BIG_BAR() __builtin_amdgcn_s_barrier()
#define PTK_BIG_STAGE(h, t) stage(h, t)

template <int ACT, int OUT>
__global__ void __launch_bounds__(512, 1) gemm_big_kernel(GemmArgs p) {
  __shared__ __attribute__((aligned(16))) char smem[8 * EPI_WAVE_BYTES];   // 136 KiB >= 2 * BUF_BYTES
  PTK_STAMP(0);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 2, wc = wave & 3;

  const int nbm = (p.M + BIG - 1) / BIG, nbn = (p.N + BIG - 1) / BIG;
  const int ntile = nbm * nbn;
  int bid = blockIdx.x;
  {
    const int q = ntile >> 3, rr = ntile & 7, x = bid & 7;
    bid = (x < rr ? x * (q + 1) : rr * (q + 1) + (x - rr) * q) + (bid >> 3);
  }
  const int per_group = GROUP_M * nbn;
  const int first_m = (bid / per_group) * GROUP_M;
  const int gsz = min(nbm - first_m, GROUP_M);
  const int bm = first_m + (bid % per_group) % gsz;
  const int bn = (bid % per_group) / gsz;

  const bf16_t* A = p.A;
  const bf16_t* B = p.B;
  // staging sources: half-tile h (0,1 = A halves, 2,3 = B halves), instruction j (0,1):
  // lane writes LDS row (wave*16 + j*8 + (lane>>3)) of the half, chunk (lane&7)
  const int sr = lane >> 3, sc = lane & 7;
  const bf16_t* src[4][2];
#pragma unroll
  for (int h = 0; h < 4; ++h)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int lr = wave * 16 + j * 8 + sr;               // row within the half-tile
      const int lc = PTK_SRC_SWZ(sc, lr);
      if (h < 2) {
        const long gm = min((long)bm * BIG + h * 128 + lr, (long)p.M - 1);
        src[h][j] = A + map_row(p.amap, gm) * p.lda + lc * 8;
      } else {
        const long gn = min((long)bn * BIG + (h - 2) * 128 + lr, (long)p.N - 1);
        src[h][j] = B + gn * p.ldb + lc * 8;
      }
    }
  auto stage = [&](int h, int t) {
    char* dst = smem + (t & 1) * BUF_BYTES + h * HALF_BYTES + wave * 16 * 128;
    glds16(src[h][0] + (long)t * BK, dst);
    glds16(src[h][1] + (long)t * BK, dst + 8 * 128);
  };

  f32x4_t acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4_t){0.f, 0.f, 0.f, 0.f};

  const int frag_off = (lane & 15) * 128 + (((lane >> 4) ^ ((lane >> 1) & 7)) << 4);
  const int nt = p.K / BK;
  // prologue: K-tile 0 complete, B halves of K-tile 1 in flight
  stage(0, 0); stage(1, 0); stage(2, 0); stage(3, 0);
  if (nt > 1) {
    stage(2, 1); stage(3, 1);
    asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __builtin_amdgcn_s_barrier();
  PTK_STAMP(1);

  bf16x8_t a[4][2], b0[2][2], b1[2][2];
  for (int t = 0; t < nt; ++t) {
    const char* buf = smem + (t & 1) * BUF_BYTES;
    const char* As = buf + wr * HALF_BYTES;                                  // this wave's 128 A rows
    const char* Bs = buf + (2 + (wc >> 1)) * HALF_BYTES + (wc & 1) * 64 * 128;   // this wave's 64 B rows
    // ---- phase 0: fragments A(mh0), B(nh0) and, one phase early, B(nh1)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
        a[i][ks] = *reinterpret_cast<const bf16x8_t*>(As + (i * 16) * 128 + (frag_off ^ (ks << 6)));
#pragma unroll
    for (int n = 0; n < 2; ++n)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
        b0[n][ks] = *reinterpret_cast<const bf16x8_t*>(Bs + (n * 16) * 128 + (frag_off ^ (ks << 6)));
#pragma unroll
    for (int n = 0; n < 2; ++n)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
        b1[n][ks] = *reinterpret_cast<const bf16x8_t*>(Bs + (32 + n * 16) * 128 + (frag_off ^ (ks << 6)));
    if (t + 1 < nt) PTK_BIG_STAGE(0, t + 1);
    asm volatile("s_waitcnt lgkmcnt(4)" ::: "memory");   // A(mh0), B(nh0) landed; B(nh1) may be in flight
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int n = 0; n < 2; ++n)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
          acc[i][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i][ks], b0[n][ks], acc[i][n], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    PTK_BIG_BAR();
    // ---- phase 1: A(mh0) x B(nh1); A(mh1) is re-read into a[i] as soon as a[i] is consumed
    if (t + 1 < nt) PTK_BIG_STAGE(1, t + 1);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
#pragma unroll
      for (int n = 0; n < 2; ++n)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
          acc[i][2 + n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i][ks], b1[n][ks], acc[i][2 + n], 0, 0, 0);
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
        a[i][ks] = *reinterpret_cast<const bf16x8_t*>(As + (64 + i * 16) * 128 + (frag_off ^ (ks << 6)));
    }
    __builtin_amdgcn_s_setprio(0);
    PTK_BIG_BAR();
    // ---- phase 2: A(mh1) x B(nh0)
    if (t + 2 < nt) PTK_BIG_STAGE(2, t + 2);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int n = 0; n < 2; ++n)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
          acc[4 + i][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i][ks], b0[n][ks], acc[4 + i][n], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    PTK_BIG_BAR();
    // ---- phase 3: A(mh1) x B(nh1); retire K-tile t+1 (B(t+2) stays in flight)
    if (t + 2 < nt) {
      PTK_BIG_STAGE(3, t + 2);
      asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int n = 0; n < 2; ++n)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
          acc[4 + i][2 + n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i][ks], b1[n][ks], acc[4 + i][2 + n], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    PTK_BIG_BAR();
  }
  PTK_STAMP(2);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  char* Cz = reinterpret_cast<char*>(p.C);
  // the wave's 128x64 tile as two 64x64 halves through its private LDS region
  f32x4_t (&top)[4][4] = *reinterpret_cast<f32x4_t(*)[4][4]>(&acc[0][0]);
  f32x4_t (&bot)[4][4] = *reinterpret_cast<f32x4_t(*)[4][4]>(&acc[4][0]);
  const long r0 = (long)bm * BIG + wr * 128, c0 = (long)bn * BIG + wc * 64;
#ifdef PTK_STAMPS
  const int em = g_epi_mode;
  GemmArgs pe = p;
  if (em == 1) pe.M = 0;   // every row skipped after staging
  if (em != 2) {
    epilogue<ACT, OUT>(pe, smem, wave, lane, top, r0, c0, Cz);
    __builtin_amdgcn_wave_barrier();
    epilogue<ACT, OUT>(pe, smem, wave, lane, bot, r0 + 64, c0, Cz);
  }
#else
  epilogue<ACT, OUT>(p, smem, wave, lane, top, r0, c0, Cz);
  __builtin_amdgcn_wave_barrier();
  epilogue<ACT, OUT>(p, smem, wave, lane, bot, r0 + 64, c0, Cz);
#endif
#ifdef PTK_STAMPS
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
#endif
  PTK_STAMP(3);
}



// K-tiles [k0, k1) of the 256x256 tile (bm, bn) into acc (zeroed by the caller), wave groups wr = 0 / 1
// one barrier apart (half a phase): on every SIMD one wave of the pair issues its LDS reads while the
// other runs its MFMA cluster.  Each phase: reads + DMA issue, barrier, MFMA cluster, barrier.  Ends with
// every DMA retired and a workgroup barrier (the LDS is free for the epilogue).
PTK_DEV void big2_kloop(const GemmArgs& p, char* smem, int bm, int bn, int k0, int k1, f32x4_t (&acc)[8][4],
                        int tid) {
  const int lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 2, wc = wave & 3;
  const bf16_t* A = p.A;
  const bf16_t* B = p.B;
  // staging sources: half-tile h (0,1 = A halves, 2,3 = B halves), instruction j (0,1):
  // lane writes LDS row (wave*16 + j*8 + (lane>>3)) of the half, chunk (lane&7)
  const int sr = lane >> 3, sc = lane & 7;
  const bf16_t* src[4][2];
#pragma unroll
  for (int h = 0; h < 4; ++h)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int lr = wave * 16 + j * 8 + sr;               // row within the half-tile
      const int lc = PTK_SRC_SWZ(sc, lr);
      if (h < 2) {
        const long gm = min((long)bm * BIG + h * 128 + lr, (long)p.M - 1);
        src[h][j] = A + map_row(p.amap, gm) * p.lda + lc * 8;
      } else {
        const long gn = min((long)bn * BIG + (h - 2) * 128 + lr, (long)p.N - 1);
        src[h][j] = B + gn * p.ldb + lc * 8;
      }
    }
  auto stage = [&](int h, int t) {
    char* dst = smem + ((t - k0) & 1) * BUF_BYTES + h * HALF_BYTES + wave * 16 * 128;
    glds16(src[h][0] + (long)t * BK, dst);
    glds16(src[h][1] + (long)t * BK, dst + 8 * 128);
  };

  const int frag_off = (lane & 15) * 128 + (((lane >> 4) ^ ((lane >> 1) & 7)) << 4);
  // prologue: K-tile k0 complete, B halves of K-tile k0+1 in flight
  stage(0, k0); stage(1, k0); stage(2, k0); stage(3, k0);
  if (k1 - k0 > 1) {
    stage(2, k0 + 1); stage(3, k0 + 1);
    asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __builtin_amdgcn_s_barrier();

  if (__builtin_amdgcn_readfirstlane(wr) == 1) __builtin_amdgcn_s_barrier();
  bf16x8_t a[4][2], b0[2][2], b1[2][2];
  for (int t = k0; t < k1; ++t) {
    const char* buf = smem + ((t - k0) & 1) * BUF_BYTES;
    const char* As = buf + wr * HALF_BYTES;
    const char* Bs = buf + (2 + (wc >> 1)) * HALF_BYTES + (wc & 1) * 64 * 128;
    // ---- phase 0: A(mh0), B(nh0), B(nh1) fragments; DMA A0(t+1)
#pragma unroll
    for (int n = 0; n < 2; ++n)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
        b0[n][ks] = *reinterpret_cast<const bf16x8_t*>(Bs + (n * 16) * 128 + (frag_off ^ (ks << 6)));
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
        a[i][ks] = *reinterpret_cast<const bf16x8_t*>(As + (i * 16) * 128 + (frag_off ^ (ks << 6)));
#pragma unroll
    for (int n = 0; n < 2; ++n)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
        b1[n][ks] = *reinterpret_cast<const bf16x8_t*>(Bs + (32 + n * 16) * 128 + (frag_off ^ (ks << 6)));
    if (t + 1 < k1) stage(0, t + 1);
    __builtin_amdgcn_s_barrier();
    asm volatile("s_waitcnt lgkmcnt(4)" ::: "memory");   // A(mh0), B(nh0) landed
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int n = 0; n < 2; ++n)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
          acc[i][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i][ks], b0[n][ks], acc[i][n], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    // every read of tile t's B region is complete before any wave can reach phase 2's DMA into it
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    // ---- phase 1: DMA A1(t+1); A(mh0) x B(nh1), A(mh1) re-read into a[i] as a[i] is consumed
    if (t + 1 < k1) stage(1, t + 1);
    __builtin_amdgcn_s_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
#pragma unroll
      for (int n = 0; n < 2; ++n)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
          acc[i][2 + n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i][ks], b1[n][ks], acc[i][2 + n], 0, 0, 0);
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
        a[i][ks] = *reinterpret_cast<const bf16x8_t*>(As + (64 + i * 16) * 128 + (frag_off ^ (ks << 6)));
    }
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_s_barrier();
    // ---- phase 2: DMA B0(t+2) (B of tile t is in registers since phase 0); A(mh1) x B(nh0)
    if (t + 2 < k1) stage(2, t + 2);
    __builtin_amdgcn_s_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int n = 0; n < 2; ++n)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
          acc[4 + i][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i][ks], b0[n][ks], acc[4 + i][n], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_s_barrier();
    // ---- phase 3: DMA B1(t+2); retire K-tile t+1 (B(t+2) stays in flight); A(mh1) x B(nh1)
    if (t + 2 < k1) {
      stage(3, t + 2);
      asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int n = 0; n < 2; ++n)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
          acc[4 + i][2 + n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i][ks], b1[n][ks], acc[4 + i][2 + n], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_s_barrier();
  }
  if (__builtin_amdgcn_readfirstlane(wr) == 0) __builtin_amdgcn_s_barrier();
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
}

// tile index -> (bm, bn): GROUP_M-row groups (A row-panels and B column-panels reused through L2)
PTK_DEV void big_tile_coords(const GemmArgs& p, int tile, int& bm, int& bn) {
  const int nbm = (p.M + BIG - 1) / BIG, nbn = (p.N + BIG - 1) / BIG;
  const int per_group = GROUP_M * nbn;
  const int first_m = (tile / per_group) * GROUP_M;
  const int gsz = min(nbm - first_m, GROUP_M);
  bm = first_m + (tile % per_group) % gsz;
  bn = (tile % per_group) / gsz;
}

// blocks b, b+8, ... share an XCD: give them consecutive indices (bijective over n)
PTK_DEV int xcd_remap(int b, int n) {
  const int q = n >> 3, rr = n & 7, x = b & 7;
  return (x < rr ? x * (q + 1) : rr * (q + 1) + (x - rr) * q) + (b >> 3);
}

template <int ACT, int OUT>
PTK_DEV void big_epilogue(const GemmArgs& p, char* smem, int bm, int bn, f32x4_t (&acc)[8][4], int tid) {
  const int lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 2, wc = wave & 3;
  char* Cz = reinterpret_cast<char*>(p.C);
  // the wave's 128x64 tile as two 64x64 halves through its private LDS region
  f32x4_t (&top)[4][4] = *reinterpret_cast<f32x4_t(*)[4][4]>(&acc[0][0]);
  f32x4_t (&bot)[4][4] = *reinterpret_cast<f32x4_t(*)[4][4]>(&acc[4][0]);
  const long r0 = (long)bm * BIG + wr * 128, c0 = (long)bn * BIG + wc * 64;
  epilogue<ACT, OUT>(p, smem, wave, lane, top, r0, c0, Cz);
  __builtin_amdgcn_wave_barrier();
  epilogue<ACT, OUT>(p, smem, wave, lane, bot, r0 + 64, c0, Cz);
}

template <int ACT, int OUT>
__global__ void __launch_bounds__(512, 1) gemm_big2_kernel(GemmArgs p) {
  __shared__ __attribute__((aligned(16))) char smem[8 * EPI_WAVE_BYTES];   // 136 KiB >= 2 * BUF_BYTES
  const int nbm = (p.M + BIG - 1) / BIG, nbn = (p.N + BIG - 1) / BIG;
  int bm, bn;
  big_tile_coords(p, xcd_remap(blockIdx.x, nbm * nbn), bm, bn);
  f32x4_t acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
  big2_kloop(p, smem, bm, bn, 0, p.K / BK, acc, threadIdx.x);
  big_epilogue<ACT, OUT>(p, smem, bm, bn, acc, threadIdx.x);
}

static int g_num_cu = 0;
static int num_cus() {
  if (!g_num_cu) {
    int dev = 0;
    hipDeviceProp_t prop;
    if (hipGetDevice(&dev) != hipSuccess || hipGetDeviceProperties(&prop, dev) != hipSuccess) return 256;
    g_num_cu = prop.multiProcessorCount;
  }
  return g_num_cu;
}

// ---- optional live per-class timing (HIP events around launches; bench.py roofline)
static bool g_timing = false;
static int g_timing_mask = 0;   // activation classes whose launches are timed
static int g_force_tiles = 0;   // tests: 1 = every GEMM on 128x128, 2 / 4 = single-batch GEMMs on 256x256 / staggered 256x256,
                                // 8 = persistent 4-wave kernel, 32 = persistent 8-wave kernel, 64 = persistent two-group kernel
                                // wherever they are supported
void force_small_tiles(int mode) { g_force_tiles = mode; }
static std::vector<hipEvent_t> g_ev[8];
static size_t g_ev_used[8];

void timer_enable(int on) {
  // on: 0 = off, 1 = every class, otherwise (1 << 8) | mask of classes (only those launches get events)
  g_timing = on != 0;
  g_timing_mask = on == 1 ? 0xff : (on & 0xff);
  if (g_timing)
    for (int c = 0; c < 8; ++c) g_ev_used[c] = 0;   // a new measurement window starts
}
static hipEvent_t next_event(int cls) {
  auto& v = g_ev[cls];
  if (g_ev_used[cls] == v.size()) {
    hipEvent_t e;
    if (hipEventCreate(&e) != hipSuccess) return nullptr;
    v.push_back(e);
  }
  return v[g_ev_used[cls]++];
}
int timer_read(int cls, double* total_ms, int* count) {
  *total_ms = 0;
  *count = 0;
  if (cls < 0 || cls >= 8) return set_error("timer: class out of range");
  for (size_t i = 0; i + 1 < g_ev_used[cls]; i += 2) {
    float ms = 0;
    if (hipEventSynchronize(g_ev[cls][i + 1]) != hipSuccess) return set_error("timer: sync failed");
    if (hipEventElapsedTime(&ms, g_ev[cls][i], g_ev[cls][i + 1]) != hipSuccess) return set_error("timer: elapsed");
    *total_ms += ms;
    *count += 1;
  }
  return 0;
}

#define PTK_GEMM_CASE(ACT_, OUT_)                                                              \
  if (act == ACT_ && out == OUT_) {                                                            \
    hipEvent_t e0 = nullptr, e1 = nullptr;                                                     \
    if (g_timing && ((g_timing_mask >> act) & 1)) { e0 = next_event(act); e1 = next_event(act); }                              \
    if (e0) (void)hipEventRecord(e0, st);                                                          \
    count_path(batch > 1 ? GEMM_PATH_NTB : GEMM_PATH_NT, act);                                 \
    hipLaunchKernelGGL((gemm_nt_kernel<ACT_, OUT_>), grid, dim3(256), 0, st, a);              \
    if (e1) (void)hipEventRecord(e1, st);                                                          \
    return hipGetLastError() == hipSuccess ? 0 : set_error("gemm launch failed");             \
  }

// Dispatch census (tests assert which kernel family a model-level call ran): launches per (path, act)
static long g_path_count[GEMM_NPATH][8];
int path_counts(int64_t* out, int reset) {
  for (int p = 0; p < GEMM_NPATH; ++p)
    for (int c = 0; c < 8; ++c) {
      if (out) out[p * 8 + c] = g_path_count[p][c];
      if (reset) g_path_count[p][c] = 0;
    }
  return 0;
}
static inline void count_path(int path, int act) { ++g_path_count[path][act & 7]; }

int launch_gemm(const GemmArgs& a, int act, int out, int batch, hipStream_t st) {
  if (a.M <= 0 || a.N <= 0 || batch <= 0) return 0;
  if (a.K <= 0 || a.K % BK) return set_error("gemm: K=%d must be a positive multiple of 64", a.K);
  if ((a.lda % 8) || (a.ldb % 8)) return set_error("gemm: lda/ldb must be multiples of 8 (16-B rows)");
  if (((uintptr_t)a.A | (uintptr_t)a.B) & 15) return set_error("gemm: A/B must be 16-B aligned");
  if (a.zin <= 0) return set_error("gemm: zin must be >= 1");
  const long ntile = (long)((a.M + BM - 1) / BM) * ((a.N + BN - 1) / BN);
  if (ntile > 0x7fffffffL) return set_error("gemm: too many tiles");
  // 256x256 (one block per CU) only where the K loop amortises its lock-step epilogue: long K or
  // wide N at K >= 1152.  Elsewhere two co-resident 128x128 blocks per CU overlap one block's
  // epilogue with the other's MFMA and quantise better (tools/gemm_bench.py --all, r01).
  // long K: the barrier-staggered 256x256 variant (+6-7 % at K >= 4096, tools/gemm_bench.py --all)
  const bool big_shape = a.M >= 1024 && a.N >= 512 && (a.K >= 6144 || (a.N >= 6144 && a.K >= 1152));
  // persistent 4-wave 256x256 kernel (gemm_w4.hip) where it measured ahead of the 8-wave and
  // 128x128 kernels (tools/gemm_bench.py --all, same box, r01): the GEGLU gate|up projection, and
  // plain projections (bf16 or fp32 out, K <= 8192) whose 256x256 tiles fill >= 80 % of the
  // persistent grid's rounds (SigLIP qkv +4 %, Gemma o +6 %, dh +17 %, down +3 %, dqkv +2 %).  Not the
  // N = 1024 / 1536 shapes (352 / 528 tiles: 69 % round fill, the 128x128 kernel wins), the
  // vocab-wide lm_head, the K = 11520 / 13824 projections or the GELU epilogues
  // (r02: + the GELU-tanh epilogue with packed f32 math, SigLIP fc1 887 -> 936 TFLOP/s, tools/gemm_bench.py --all)
  const bool w4_auto = g_force_tiles == 0 && a.M >= 4096 && a.N <= 16384 &&
                       (act == ACT_GEGLU || act == ACT_GEGLU_BWD ||
                        (((act == ACT_NONE && (out == OUT_BF16 || out == OUT_F32)) ||
                          (act == ACT_GELU_TANH && out == OUT_BF16)) &&
                         a.K <= 8192 && w4_round_fill(a.M, a.N) >= 0.8));
  // persistent 8-wave kernel (two waves per SIMD, gemm_w4.hip) where it measured ahead of the 4-wave one
  // (tools/p8_probe.py, same box, interleaved, r03): the w4 plain / GELU-tanh shapes at K <= 2048 (Gemma q|k|v
  // 90 -> 87 us, o 58 -> 56, SigLIP q|k|v 111 -> 109, fc1 157 -> 151), the projector fc1 with the GELU-erf
  // epilogue (674 -> 583 us) and its backward (dA, 858 -> 703 us) and the long-K d(gate|up) dX (K 13 824, N <= 2048: 700 -> 672 us); w4 keeps the
  // GEGLU / GEGLU-backward epilogues and the K 6 912 down projection (697 / 486 / 330 us vs 723 / 500 / 342).
  // PTK_P8=1 (A/B builds, PTK_AB) puts every w4 shape on it
  const bool p8_env = PTK_AB("PTK_P8", 0) == 1;
  const bool p8_auto = g_force_tiles == 0 && a.M >= 4096 && a.N <= 16384 &&
                       ((w4_auto && (p8_env || (act != ACT_GEGLU && act != ACT_GEGLU_BWD && a.K <= 2048))) ||
                        ((act == ACT_GELU_ERF || act == ACT_GELU_ERF_BWD) && out == OUT_BF16 && a.K <= 2048 &&
                         w4_round_fill(a.M, a.N) >= 0.8) ||
                        (act == ACT_NONE && (out == OUT_BF16 || out == OUT_F32) && a.K >= 12288 && a.N <= 2048) ||
                        // r05: with the lean bf16 epilogue the 8-wave kernel also beats the 128x128 one on the N 1536
                        // projection at 69 % round fill (Gemma q|k|v 90.7 vs 95.3 us, profiles/r05_dual_solo_probe.txt);
                        // the N 1024 ones stay on 128x128 (dO 66.0 vs 63.2, SigLIP fc2 187 vs 171)
                        (act == ACT_NONE && out == OUT_BF16 && a.N >= 1536 && a.K <= 2048 &&
                         w4_round_fill(a.M, a.N) >= 0.65 && lean_epilogue_candidate(a)) ||
                        // r05: a plain bf16 grid of one partial round of 256x256 tiles beats the 128x128 kernel's
                        // ~1.1 rounds of two blocks per CU (tools/sk_ab.py, Stage 2's SigLIP at M = 9 216: o 31.3 vs
                        // 41.8 us, fc2 85.1 vs 109.1; its down projection at bs 8 133.6 vs 177.8)
                        (act == ACT_NONE && out == OUT_BF16 && a.K <= 8192 &&
                         (long)((a.M + 255) / 256) * ((a.N + 255) / 256) <= device_cus() && lean_epilogue_candidate(a)));
  // the stream-K tail (gemm_w4.hip P8Tail): a plain GEMM whose last tile round fills the CUs badly, with tail
  // scratch lent by the model-level call (or in the descriptor), runs on the persistent 8-wave kernel with that
  // round's K-tiles spread over the CUs (r04: the N = 1024 / 1152 / 1536 projections, the long-K d(gate|up) dX
  // and down projection, the projector's fc2 and weight grads)
  const int sk = (g_force_tiles == 0 || g_force_tiles == 32) && batch == 1 && act == ACT_NONE && a.M >= 1024 &&
                 a.N >= 256 && a.N <= 16384 && p8_supported(a, act, out) ? p8_tail_split(a, act, out) : 0;
  // (the two-group persistent kernel on 256x128 tiles, gemm_dual.hip, measured 17-44 % slower than the 8-wave
  // kernel in round 5, profiles/r05_dual_probe.txt, and was removed from the tree in round 6)
  // 224- / 192-row tiles on the 8-wave kernel where their rounds undercut the 256-row ones (p8_tile_height:
  // Gemma3's N 1152 / 1536 / 1024 projections at M 22 528, SigLIP's q|k|v, o and fc1 at M 18 432), ahead of the
  // 4-wave and 128x128 kernels; force modes 512 / 1024 put every plain / GELU-tanh single GEMM on 224 / 192 rows
  // (tests).  PTK_TM224=0 (A/B builds, PTK_AB): 256-row tiles only
  const bool tm_env = PTK_AB("PTK_TM224", 1) != 0;
  const bool short_ok = batch == 1 && !sk && p8_supported(a, act, out) &&
                        (act == ACT_NONE || (act == ACT_GELU_TANH && out == OUT_BF16));
  int tm = 256;
  if (short_ok && g_force_tiles == 0 && tm_env && a.M >= 4096) tm = p8_tile_height(a, act, out);
  else if (short_ok && g_force_tiles == 512) tm = 224;
  else if (short_ok && g_force_tiles == 1024) tm = 192;
  else if (short_ok && g_force_tiles == 4096) tm = 160;
  if (batch == 1 && (g_force_tiles == 32 || p8_auto || sk || tm != 256) && p8_supported(a, act, out)) {
    hipEvent_t e0 = nullptr, e1 = nullptr;
    if (g_timing && ((g_timing_mask >> act) & 1)) { e0 = next_event(act); e1 = next_event(act); }
    if (e0) (void)hipEventRecord(e0, st);
    count_path(sk ? GEMM_PATH_P8SK : GEMM_PATH_P8, act);
    const int rc = launch_gemm_p8(a, act, out, st, sk != 0, tm);
    if (e1) (void)hipEventRecord(e1, st);
    return rc;
  }
  if (batch == 1 && (g_force_tiles == 8 || w4_auto) && w4_supported(a, act, out)) {
    hipEvent_t e0 = nullptr, e1 = nullptr;
    if (g_timing && ((g_timing_mask >> act) & 1)) { e0 = next_event(act); e1 = next_event(act); }
    if (e0) (void)hipEventRecord(e0, st);
    count_path(GEMM_PATH_W4, act);
    const int rc = launch_gemm_w4(a, act, out, st, 0);
    if (e1) (void)hipEventRecord(e1, st);
    return rc;
  }
  if (batch == 1 && (g_force_tiles == 4 || (g_force_tiles == 0 && big_shape && a.K >= 4096))) {
    const long nb = (long)((a.M + BIG - 1) / BIG) * ((a.N + BIG - 1) / BIG);
    dim3 g4((unsigned)nb, 1, 1);
#define PTK_BIG2_CASE(ACT_, OUT_)                                                               \
    if (act == ACT_ && out == OUT_) {                                                           \
      hipEvent_t e0 = nullptr, e1 = nullptr;                                                    \
      if (g_timing && ((g_timing_mask >> act) & 1)) { e0 = next_event(act); e1 = next_event(act); }                             \
      if (e0) (void)hipEventRecord(e0, st);                                                     \
      count_path(GEMM_PATH_BIG2, act);                                                          \
      hipLaunchKernelGGL((gemm_big2_kernel<ACT_, OUT_>), g4, dim3(512), 0, st, a);              \
      if (e1) (void)hipEventRecord(e1, st);                                                     \
      return hipGetLastError() == hipSuccess ? 0 : set_error("gemm launch failed");            \
    }
    PTK_BIG2_CASE(ACT_NONE, OUT_BF16)
    PTK_BIG2_CASE(ACT_NONE, OUT_F32)
    PTK_BIG2_CASE(ACT_NONE, OUT_F32_BFR)
    PTK_BIG2_CASE(ACT_GELU_TANH, OUT_BF16)
    PTK_BIG2_CASE(ACT_GELU_ERF, OUT_BF16)
    PTK_BIG2_CASE(ACT_GEGLU, OUT_BF16)
    PTK_BIG2_CASE(ACT_GELU_ERF_BWD, OUT_BF16)
    PTK_BIG2_CASE(ACT_GEGLU_BWD, OUT_BF16)
#undef PTK_BIG2_CASE
    return set_error("gemm: unsupported (act=%d, out=%d)", act, out);
  }
  const bool big = batch == 1 && g_force_tiles != 1 && (g_force_tiles == 2 || big_shape);
  if (big) {
    const long nb = (long)((a.M + BIG - 1) / BIG) * ((a.N + BIG - 1) / BIG);
    dim3 g2((unsigned)nb, 1, 1);
#define PTK_BIG_CASE(ACT_, OUT_)                                                                \
    if (act == ACT_ && out == OUT_) {                                                           \
      hipEvent_t e0 = nullptr, e1 = nullptr;                                                    \
      if (g_timing && ((g_timing_mask >> act) & 1)) { e0 = next_event(act); e1 = next_event(act); }                             \
      if (e0) (void)hipEventRecord(e0, st);                                                     \
      count_path(GEMM_PATH_BIG, act);                                                           \
      hipLaunchKernelGGL((gemm_big_kernel<ACT_, OUT_>), g2, dim3(512), 0, st, a);               \
      if (e1) (void)hipEventRecord(e1, st);                                                     \
      return hipGetLastError() == hipSuccess ? 0 : set_error("gemm launch failed");            \
    }
    PTK_BIG_CASE(ACT_NONE, OUT_BF16)
    PTK_BIG_CASE(ACT_NONE, OUT_F32)
    PTK_BIG_CASE(ACT_NONE, OUT_F32_BFR)
    PTK_BIG_CASE(ACT_GELU_TANH, OUT_BF16)
    PTK_BIG_CASE(ACT_GELU_ERF, OUT_BF16)
    PTK_BIG_CASE(ACT_GEGLU, OUT_BF16)
    PTK_BIG_CASE(ACT_GELU_ERF_BWD, OUT_BF16)
    PTK_BIG_CASE(ACT_GEGLU_BWD, OUT_BF16)
#undef PTK_BIG_CASE
    return set_error("gemm: unsupported (act=%d, out=%d)", act, out);
  }
  dim3 grid((unsigned)ntile, 1, (unsigned)batch);
  PTK_GEMM_CASE(ACT_NONE, OUT_BF16)
  PTK_GEMM_CASE(ACT_NONE, OUT_F32)
  PTK_GEMM_CASE(ACT_NONE, OUT_F32_BFR)
  PTK_GEMM_CASE(ACT_GELU_TANH, OUT_BF16)
  PTK_GEMM_CASE(ACT_GELU_ERF, OUT_BF16)
  PTK_GEMM_CASE(ACT_GEGLU, OUT_BF16)
  PTK_GEMM_CASE(ACT_GELU_ERF_BWD, OUT_BF16)
  PTK_GEMM_CASE(ACT_GEGLU_BWD, OUT_BF16)
  return set_error("gemm: unsupported (act=%d, out=%d)", act, out);
}

// the K-sliced 8-wave GEMM (gemm_w4.hip launch_gemm_p8_kslices) with launch_gemm's census ("p8") and timers
int gemm_p8_kslices(const GemmArgs& a, int slices, hipStream_t st) {
  if (a.M <= 0 || a.N <= 0) return 0;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  if (g_timing && (g_timing_mask & 1)) { e0 = next_event(ACT_NONE); e1 = next_event(ACT_NONE); }
  if (e0) (void)hipEventRecord(e0, st);
  count_path(GEMM_PATH_P8, ACT_NONE);
  const int rc = launch_gemm_p8_kslices(a, slices, st);
  if (e1) (void)hipEventRecord(e1, st);
  return rc;
}

// the token-major weight-grad GEMM (gemm_tn.hip) with launch_gemm's census and live timers (class ACT_NONE)
int gemm_tn(const GemmArgs& a, int out, int slices, void* slab, hipStream_t st, long k_rows) {
  if (a.M <= 0 || a.N <= 0) return 0;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  if (g_timing && (g_timing_mask & 1)) { e0 = next_event(ACT_NONE); e1 = next_event(ACT_NONE); }
  if (e0) (void)hipEventRecord(e0, st);
  count_path(GEMM_PATH_TN, ACT_NONE);
  const int rc = launch_gemm_tn(a, out, slices, slab, st, k_rows);
  if (e1) (void)hipEventRecord(e1, st);
  return rc;
}

}  // namespace ptk

#ifdef PTK_STAMPS
extern "C" int ptk_debug_epi_mode(int m) {
  return hipMemcpyToSymbol(HIP_SYMBOL(ptk::g_epi_mode), &m, sizeof(int), 0, hipMemcpyHostToDevice) == hipSuccess ? 0 : -1;
}
extern "C" int ptk_debug_stamps_read(void* host, size_t bytes) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(ptk::g_stamps), bytes, 0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
#endif
