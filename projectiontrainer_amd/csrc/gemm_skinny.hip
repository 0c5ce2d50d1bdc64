// Skinny GEMM for the KV-cache decode: C[M, N] = A[M, K] . B[N, K]^T with M <= 64 rows (one token per decode row)
// and N up to the vocabulary.  At M <= 64 the product is a stream of the weight matrix B (N x K bf16, read once)
// against a few A rows that stay in L2: the 256x256-tile kernels would run a handful of mostly-empty tiles, each
// walking the whole K on one CU (measured 47 us per decode projection, ~70 % of a decode step).  Here every
// workgroup owns 128 columns of N and a slice of K, so the grid covers the CUs (K split until ~512 workgroups);
// each wave streams the B rows of its 16 columns straight into MFMA fragments (no LDS: nothing is shared between
// the waves but the A rows, which come from L1/L2; each wave covers 32 columns, so every A fragment feeds two
// MFMAs), 4 k-steps of loads in flight.
//   v_mfma_f32_16x16x32_bf16 with the B rows as the A operand: lane l holds C[16 mb + (l & 15)][n0 + 4 (l >> 4) + j]
//   (j < 4: four consecutive columns of one row -> 16-B partial stores).
// K-split partials [ksplit][M][N] fp32 are summed in split order by skinny_reduce_kernel, which also runs the
// epilogue (bf16 rounding; GEGLU on the interleaved gate|up columns, as the training path's gate|up epilogue:
// h = bf16(bf16(gelu_tanh(bf16 g)) * bf16 u)).  With one split the GEMM kernel rounds and stores C itself.
#include "common.h"
#include "ptk_internal.h"

namespace ptk {

constexpr int SK_COLS = 128;  // columns per workgroup (4 waves x 2 blocks of 16)
constexpr int SK_AHEAD = 4;   // k-steps of fragment loads in flight per wave

template <int MB, bool DIRECT>
__global__ void __launch_bounds__(256) gemm_skinny_kernel(const bf16_t* __restrict__ A, long lda,
                                                          const bf16_t* __restrict__ B, long ldb, int M, int N, int K,
                                                          int ks_len, float* __restrict__ part,
                                                          bf16_t* __restrict__ C, long ldc) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r = lane & 15, g = lane >> 4;
  const int n0 = blockIdx.x * SK_COLS + 32 * wave;   // the wave's two 16-column blocks: n0, n0 + 16
  const int z = blockIdx.y, nks = K / 32;
  const int ks0 = z * ks_len, ks1 = min(nks, ks0 + ks_len);
  const bf16_t* bp[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) bp[h] = B + (long)min(n0 + 16 * h + r, N - 1) * ldb + 8 * g;
  const bf16_t* ap[MB];
#pragma unroll
  for (int mb = 0; mb < MB; ++mb) ap[mb] = A + (long)min(16 * mb + r, M - 1) * lda + 8 * g;
  f32x4_t acc[MB][2];
#pragma unroll
  for (int mb = 0; mb < MB; ++mb) acc[mb][0] = acc[mb][1] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
  bf16x8_t bq[SK_AHEAD][2], aq[SK_AHEAD][MB];
#pragma unroll
  for (int i = 0; i < SK_AHEAD; ++i) {
    const int ks = min(ks0 + i, ks1 - 1);
#pragma unroll
    for (int h = 0; h < 2; ++h) bq[i][h] = *reinterpret_cast<const bf16x8_t*>(bp[h] + 32 * ks);
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) aq[i][mb] = *reinterpret_cast<const bf16x8_t*>(ap[mb] + 32 * ks);
  }
  for (int ks = ks0; ks < ks1; ks += SK_AHEAD) {
#pragma unroll
    for (int i = 0; i < SK_AHEAD; ++i) {
      if (ks + i < ks1) {
#pragma unroll
        for (int mb = 0; mb < MB; ++mb)
#pragma unroll
          for (int h = 0; h < 2; ++h)
            acc[mb][h] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bq[i][h], aq[i][mb], acc[mb][h], 0, 0, 0);
      }
      const int kn = min(ks + i + SK_AHEAD, ks1 - 1);   // (past the end: a re-load, unused)
#pragma unroll
      for (int h = 0; h < 2; ++h) bq[i][h] = *reinterpret_cast<const bf16x8_t*>(bp[h] + 32 * kn);
#pragma unroll
      for (int mb = 0; mb < MB; ++mb) aq[i][mb] = *reinterpret_cast<const bf16x8_t*>(ap[mb] + 32 * kn);
    }
  }
  // lane: row 16 mb + r, columns n0 + 16 h + 4 g .. + 3
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int nc = n0 + 16 * h + 4 * g;
    if (nc >= N) continue;
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) {
      const int m = 16 * mb + r;
      if (m >= M) continue;
      if constexpr (DIRECT) {
        u16x4_t u;
        u[0] = f2bf(acc[mb][h][0]); u[1] = f2bf(acc[mb][h][1]); u[2] = f2bf(acc[mb][h][2]); u[3] = f2bf(acc[mb][h][3]);
        *reinterpret_cast<u16x4_t*>(C + (long)m * ldc + nc) = u;
      } else {
        *reinterpret_cast<float4*>(part + ((long)z * M + m) * N + nc) =
            make_float4(acc[mb][h][0], acc[mb][h][1], acc[mb][h][2], acc[mb][h][3]);
      }
    }
  }
}

// partials [S][M][N] -> C (bf16): ACT_NONE C[m][n] = bf16(sum); ACT_GEGLU C[m][16 q + i] (N / 2 columns) from the
// gate column 32 q + i and the up column 32 q + 16 + i
template <int ACT>
__global__ void __launch_bounds__(256) skinny_reduce_kernel(const float* __restrict__ part, int S, int M, int N,
                                                            bf16_t* __restrict__ C, long ldc) {
  const int NO = ACT == ACT_GEGLU ? N / 2 : N;
  const long i = (long)blockIdx.x * 256 + threadIdx.x;   // 2 outputs per thread
  const long total = (long)M * NO / 2;
  if (i >= total) return;
  const int m = (int)(2 * i / NO), j = (int)(2 * i - (long)m * NO);
  if constexpr (ACT == ACT_GEGLU) {
    const int q = j / 16, ii = j % 16;   // j, j + 1 share q (16 | NO)
    const long cg = (long)m * N + 32 * q + ii, cu = cg + 16;
    float g0 = 0.f, g1 = 0.f, u0 = 0.f, u1 = 0.f;
    for (int s = 0; s < S; ++s) {
      const float* p = part + (long)s * M * N;
      g0 += p[cg]; g1 += p[cg + 1]; u0 += p[cu]; u1 += p[cu + 1];
    }
    uint32_t a, b, h;
    geglu_fwd2(bfround2(f32x2_t{g0, g1}), bfround2(f32x2_t{u0, u1}), a, b, h);
    *reinterpret_cast<uint32_t*>(C + (long)m * ldc + j) = h;
  } else {
    const long c = (long)m * N + j;
    float v0 = 0.f, v1 = 0.f;
    for (int s = 0; s < S; ++s) {
      const float* p = part + (long)s * M * N + c;
      v0 += p[0]; v1 += p[1];
    }
    *reinterpret_cast<uint32_t*>(C + (long)m * ldc + j) = pkbf2(f32x2_t{v0, v1});
  }
}

// K split: as many splits as bring the grid to ~512 workgroups, each split >= 2 k-steps
void skinny_plan(int M, int N, int K, int& splits, int& ks_len) {
  const int nblk = (N + SK_COLS - 1) / SK_COLS, nks = K / 32;
  int s = std::max(1, std::min((512 + nblk - 1) / nblk, nks / 2));
  ks_len = (nks + s - 1) / s;
  splits = (nks + ks_len - 1) / ks_len;
  (void)M;
}
size_t skinny_part_bytes(int M, int N, int K) {
  int s, l;
  skinny_plan(M, N, K, s, l);
  return s > 1 ? (size_t)s * M * N * 4 : 0;
}
bool skinny_supported(int M, int N, int K, long lda, long ldb, long ldc, int act) {
  return M >= 1 && M <= 64 && N % SK_COLS == 0 && K % 32 == 0 && K >= 64 && lda % 8 == 0 && ldb % 8 == 0 &&
         ldc % 2 == 0 && (act == ACT_NONE || (act == ACT_GEGLU && N % 32 == 0));
}

int launch_gemm_skinny(const bf16_t* A, long lda, const bf16_t* B, long ldb, bf16_t* C, long ldc, int M, int N,
                       int K, int act, float* part, size_t part_bytes, hipStream_t st) {
  if (!skinny_supported(M, N, K, lda, ldb, ldc, act))
    return set_error("gemm_skinny: M %d (<= 64), N %d (%% 128), K %d (%% 32), act %d unsupported", M, N, K, act);
  int S, ks_len;
  skinny_plan(M, N, K, S, ks_len);
  const bool direct = S == 1 && act == ACT_NONE;
  if (!direct && part_bytes < (size_t)S * M * N * 4) return set_error("gemm_skinny: partial buffer too small");
  const dim3 grid((unsigned)(N / SK_COLS), (unsigned)S);
  const int mb = (M + 15) / 16;
#define SKL(MB_, D_) hipLaunchKernelGGL((gemm_skinny_kernel<MB_, D_>), grid, dim3(256), 0, st, A, lda, B, ldb, M, N, K, \
                                        ks_len, part, C, ldc)
  if (direct) {
    if (mb == 1) SKL(1, true); else if (mb == 2) SKL(2, true); else if (mb == 3) SKL(3, true); else SKL(4, true);
  } else {
    if (mb == 1) SKL(1, false); else if (mb == 2) SKL(2, false); else if (mb == 3) SKL(3, false); else SKL(4, false);
  }
#undef SKL
  if (hipGetLastError() != hipSuccess) return set_error("gemm_skinny launch failed");
  if (direct) return 0;
  const int NO = act == ACT_GEGLU ? N / 2 : N;
  const long total = (long)M * NO / 2;
  if (act == ACT_GEGLU)
    hipLaunchKernelGGL(skinny_reduce_kernel<ACT_GEGLU>, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, part,
                       S, M, N, C, ldc);
  else
    hipLaunchKernelGGL(skinny_reduce_kernel<ACT_NONE>, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, part,
                       S, M, N, C, ldc);
  return hipGetLastError() == hipSuccess ? 0 : set_error("skinny_reduce launch failed");
}

}  // namespace ptk
