// Flash attention forward for gfx950 (bf16 in/out, fp32 softmax state).
//
// One workgroup = 8 waves = 128 query rows of one (batch, kv-head) z; each
// wave owns 16 rows.  Per 64-key tile (K and V staged global->LDS by
// LDS-DMA, double-buffered):
//   S^T[64 keys x 16 q] = K . Q^T        MFMA 16x16x32, A = K rows from LDS,
//                                        B = Q fragments kept in registers
//   online softmax per query column      (lane's column = its query row; the
//                                        column's 64 keys live in 4 lanes:
//                                        2 shuffles per reduction)
//   O^T[D x 16 q] += V^T . P^T           A = V^T via ds_read_b64_tr_b16 on
//                                        the row-major V tile, B = P^T taken
//                                        straight from the S^T accumulators
//                                        (k order permuted identically on
//                                        both operands: no LDS round trip)
// O^T's layout puts a query on the same lane as its softmax state, so the
// per-tile rescale needs no cross-lane traffic.  Masks: key padding / key
// length, causal (query position = row / qdiv), sliding window k > q - W.
// Writes O (bf16, row-remapped) and LSE = ln(sum exp(score)) per row (fp32)
// for the backward.  Semantics: softmax(scale * Q K^T + mask) V, as
// TF/models/siglip/modeling_siglip.py:289-300 and gemma3 :365-379 (sdpa).
#include <algorithm>
#include <cstdlib>
#include <functional>
#include <queue>
#include <type_traits>
#include <vector>
#include "common.h"
#include "ptk_internal.h"

namespace ptk {

typedef __attribute__((ext_vector_type(4))) short s16x4_t;
typedef const __attribute__((address_space(1))) void* fa_gptr_t;
typedef __attribute__((address_space(3))) void* fa_lptr_t;

// LDS-DMA of 16 B per lane (lds: wave-uniform base; lane i lands at lds + 16 i).  Inline asm on purpose:
// for the builtin, hipcc's wait-count pass assumes any later LDS read may alias an in-flight DMA and
// inserts s_waitcnt vmcnt(0) before the first one of every tile, draining the whole K/V ring (tiles t+1..t+3)
// each iteration.  The kernels publish landed tiles themselves (counted vm_wait + barrier), so the DMA is
// kept out of the compiler's view.
PTK_DEV void fa_glds16(const void* src, void* lds) {
  const uint32_t m0 = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(fa_lptr_t)lds);
  // M0 is passed through the {m0} constraint: hipcc writes it and knows the asm reads it (never an
  // undeclared M0 write inside the asm; the s_nop keeps the M0 -> LDS-DMA wait state)
  asm volatile("s_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(src), "{m0}"(m0) : "memory");
}

// 16-B chunk swizzles (chunk index within a row of D/8 chunks)
template <int D>
PTK_DEV int swz_k(int r) { return D == 256 ? (r & 15) : ((r >> 1) & 7); }     // ds_read_b128 row reads
template <int D>
PTK_DEV int swz_v(int r) { return D == 256 ? 2 * (r & 7) : 2 * ((r >> 1) & 3); }  // ds_read_b64_tr_b16
// d 256 tiles read both by rows (ds_read_b128, 16 rows x one chunk) and transposed (ds_read_b64_tr_b16,
// 8 rows x two adjacent chunks per 32-lane half).  With the b128 lane groups {0-3,12-15,20-27},
// {4-11,16-19,28-31}, ... (MI355X_MICROARCH.md, LDS table) a row swizzle f keeps the row reads
// conflict-free iff f(r) and f(r ^ 8) ^ 1 never collide, and the transposed reads iff f(r) >> 1 is
// distinct over each octet of rows: f(r) = 2 (r & 7) meets both.  (The former ((r & 7) << 1) | (r >> 3)
// met the second only: 2-way conflicts on every row read, 32-40 % of the backward kernels' LDS cycles.)
PTK_DEV int swz_rt(int r) { return (r & 7) << 1; }
template <int D>
PTK_DEV int swz_kt(int r) { return D == 256 ? swz_rt(r) : swz_k<D>(r); }


// s_waitcnt vmcnt(n) for a wave-uniform runtime n (the immediate must be a literal)
PTK_DEV void vm_wait(int n) {
  switch (n) {
#define PTK_VMW(k) case k: asm volatile("s_waitcnt vmcnt(" #k ")" ::: "memory"); break;
    PTK_VMW(0) PTK_VMW(1) PTK_VMW(2) PTK_VMW(3) PTK_VMW(4) PTK_VMW(5) PTK_VMW(6) PTK_VMW(7)
    PTK_VMW(8) PTK_VMW(9) PTK_VMW(10) PTK_VMW(11) PTK_VMW(12) PTK_VMW(13) PTK_VMW(14) PTK_VMW(15)
    PTK_VMW(16) PTK_VMW(17) PTK_VMW(18) PTK_VMW(19) PTK_VMW(20)
#undef PTK_VMW
    default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
  }
}

// wait for a register loaded from global memory before the K/V loop (an empty asm that reads and writes it):
// otherwise hipcc's wait-count pass places the wait at the first use INSIDE the loop, every iteration,
// where its s_waitcnt vmcnt also drains the LDS-DMA ring
template <typename T>
PTK_DEV void fa_pin(T& x) { asm volatile("" : "+v"(x)); }

// K/V tiles of 32 keys in a 4-deep LDS ring (tile t+3 staged while tile t computes); every wave
// issues the same number of LDS-DMA ops per tile (its share of K, V and, when present, 4 of the
// tile's key_valid flags), so one counted vmcnt serves all waves.
constexpr int FA_NBUF = 4;
template <int D, int KT>
struct FaRing {
  static constexpr int CPR = D / 8;                      // 16-B chunks per row
  static constexpr int TILE = KT * D * 2;                // one K or V tile
  static constexpr int INST = KT * CPR / 64;             // wave-instructions per tensor per tile
  static constexpr int PER_WAVE = INST >= 8 ? INST / 8 : 1;   // per tensor per wave (8 waves)
  static constexpr int KV_LANES = KT / 32;               // 16-B key_valid pieces per wave per tile
  static constexpr int KV_OFF = FA_NBUF * 2 * TILE;      // key_valid flags, KT*4 B per buffer
  static constexpr int BYTES = KV_OFF + FA_NBUF * KT * 4;
};
// key tile per head dim: d 256 keeps 32 keys (4 x 32 KiB ring); d 64 amortises the per-tile softmax,
// barrier and DMA issue over 64 keys
template <int D>
constexpr int fa_kt() { return D == 256 ? 32 : 64; }

// QG query groups of 16 rows per wave (block = 8 waves x 16 QG rows): with QG = 2 every K fragment
// (ds_read_b128) and V^T fragment (ds_read_b64_tr_b16) read from LDS feeds two MFMAs, halving the LDS
// traffic per FLOP — at head_dim 256 the 16-row form reads as many LDS bytes per tile as its MFMAs
// take cycles (8 waves x 32 KiB per 32-key tile)
template <int D, int QG>
__global__ void __launch_bounds__(512, 1) attn_fwd_kernel(FlashArgs a) {
  constexpr int KT = fa_kt<D>();
  using R = FaRing<D, KT>;
  constexpr int KS = D / 32;                 // MFMA k-steps over the head dim
  constexpr int DS = D / 16;                 // 16-wide d sub-tiles
  constexpr int MS = KT / 16, ST = KT / 32;  // 16-key score sub-tiles, 32-key P.V k-steps
  constexpr int BR = 128 * QG;               // query rows per block
  constexpr int WR = 16 * QG;                // query rows per wave
  __shared__ __attribute__((aligned(16))) char smem[R::BYTES];   // (K, V) x4, key_valid x4

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, c16 = lane & 15;
  // heaviest (latest, for causal) row blocks first; z fastest
  const int nqb = (a.rows + BR - 1) / BR, nz = gridDim.x / nqb;
  const int z = blockIdx.x % nz, z0 = z / a.zin, z1 = z - z0 * a.zin;
  const int r0 = (nqb - 1 - (int)(blockIdx.x / nz)) * BR;
  const bf16_t* Q = a.Q + z0 * a.sQ0 + z1 * a.sQ1;
  const bf16_t* K = a.K + z0 * a.sK0 + z1 * a.sK1;
  const bf16_t* V = a.V + z0 * a.sK0 + z1 * a.sK1;
  const long b = z / a.zdiv;
  const int* kvl = a.key_valid ? a.key_valid + b * a.nkeys : nullptr;

  // key range of the block (causal / window skip)
  const int pos_lo = r0 / a.qdiv, pos_hi = min(r0 + BR - 1, a.rows - 1) / a.qdiv;
  int k_hi = a.nkeys;
  int k_lo = 0;
  if (a.causal) {
    k_hi = min(k_hi, pos_hi + 1);
    if (a.window > 0) k_lo = max(0, pos_lo - a.window + 1);
  }
  const int t_lo = k_lo / KT, t_hi = (k_hi + KT - 1) / KT;

  // Q fragments: B operand of S^T = K Q^T, lane holds Q[row c16 of group qg][8g + 32ks .. +7]
  const int wrow0 = r0 + wave * WR;
  int qrow[QG], qpos[QG];
  bf16x8_t qf[QG][KS];
#pragma unroll
  for (int qg = 0; qg < QG; ++qg) {
    qrow[qg] = wrow0 + qg * 16 + c16;
    const int qrow_c = min(qrow[qg], a.rows - 1);
    qpos[qg] = qrow_c / a.qdiv;
    const long qa = map_row(a.qmap, qrow_c);
    const bf16_t* qp = Q + qa * a.ldq + 8 * g;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) qf[qg][ks] = *reinterpret_cast<const bf16x8_t*>(qp + 32 * ks);
  }
#pragma unroll
  for (int qg = 0; qg < QG; ++qg)
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) fa_pin(qf[qg][ks]);
  const int causal = a.causal != 0, nowin = a.window <= 0;
  const bool unmasked = !kvl && !causal && nowin;
  // query positions of this wave's rows (interior-tile test)
  const int wpos_lo = min(wrow0, a.rows - 1) / a.qdiv;
  const int wpos_hi = min(wrow0 + WR - 1, a.rows - 1) / a.qdiv;

  const int ops = (R::INST >= 8 ? 2 * R::PER_WAVE : 1) + (kvl ? 1 : 0);   // LDS-DMA ops per wave per tile
  auto stage = [&](int t, int buf) {
    char* kb = smem + buf * 2 * R::TILE;
    char* vb = kb + R::TILE;
    if constexpr (R::INST >= 8) {
#pragma unroll
      for (int j = 0; j < R::PER_WAVE; ++j) {
        const int inst = wave * R::PER_WAVE + j;
        const int row = inst * (64 / R::CPR) + lane / R::CPR;
        const int pch = lane % R::CPR;
        const int key = min(t * KT + row, a.nkeys - 1);
        fa_glds16(K + (long)key * a.ldk + 8 * (pch ^ swz_k<D>(row)), kb + inst * 1024);
        fa_glds16(V + (long)key * a.ldk + 8 * (pch ^ swz_v<D>(row)), vb + inst * 1024);
      }
    } else {   // fewer than 8 wave-instructions per tensor: waves split K / V
      const int inst = wave & (R::INST - 1);
      const int row = inst * (64 / R::CPR) + lane / R::CPR;
      const int pch = lane % R::CPR;
      const int key = min(t * KT + row, a.nkeys - 1);
      if (wave < R::INST)
        fa_glds16(K + (long)key * a.ldk + 8 * (pch ^ swz_k<D>(row)), kb + inst * 1024);
      else
        fa_glds16(V + (long)key * a.ldk + 8 * (pch ^ swz_v<D>(row)), vb + inst * 1024);
    }
    if (kvl && lane < R::KV_LANES)   // 4 flags per lane
      fa_glds16(kvl + min(t * KT + 4 * (wave * R::KV_LANES + lane), a.nkeys - 4),
                smem + R::KV_OFF + buf * (KT * 4) + wave * (R::KV_LANES * 16));
  };

  f32x4_t o[QG][DS];
#pragma unroll
  for (int qg = 0; qg < QG; ++qg)
#pragma unroll
    for (int i = 0; i < DS; ++i) o[qg][i] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
  float m_run[QG], l_run[QG];
#pragma unroll
  for (int qg = 0; qg < QG; ++qg) { m_run[qg] = -INFINITY; l_run[qg] = 0.f; }
  const float sl2 = a.scale * 1.4426950408889634f;   // scores in log2 units

#pragma unroll
  for (int i = 0; i < FA_NBUF - 1; ++i)
    if (t_lo + i < t_hi) stage(t_lo + i, i);
  // waves whose rows all lie past the last row (the half-empty last block when rows % 128 = 64, e.g.
  // SigLIP's 576 patches) only stage and keep the barriers; their SIMD time goes to the co-resident block
  const bool idle = wrow0 >= a.rows;
  for (int t = t_lo; t < t_hi; ++t) {
    const int buf = (t - t_lo) & (FA_NBUF - 1);
    vm_wait(ops * min(FA_NBUF - 2, t_hi - 1 - t));
    // raw barrier (the counted wait above publishes tile t; every LDS read of the buffer restaged below
    // was consumed by an MFMA or a compare in the previous iteration)
    __builtin_amdgcn_s_barrier();
    if (t + FA_NBUF - 1 < t_hi) stage(t + FA_NBUF - 1, (buf + FA_NBUF - 1) & (FA_NBUF - 1));
    if (idle) continue;
    const char* kb = smem + buf * 2 * R::TILE;
    const char* vb = kb + R::TILE;
    const int* kvs = reinterpret_cast<const int*>(smem + R::KV_OFF + buf * (KT * 4));

    // ---- S^T = K Q^T : s[qg][ms] holds keys 16ms + 4g + j, query column c16 of group qg
    f32x4_t s[QG][MS];
#pragma unroll
    for (int ms = 0; ms < MS; ++ms) {
#pragma unroll
      for (int qg = 0; qg < QG; ++qg) s[qg][ms] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
      const int row = ms * 16 + c16;
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        const int ch = (ks * 4 + g) ^ swz_k<D>(row);
        const bf16x8_t kf = *reinterpret_cast<const bf16x8_t*>(kb + row * (D * 2) + ch * 16);
#pragma unroll
        for (int qg = 0; qg < QG; ++qg)
          s[qg][ms] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf, qf[qg][ks], s[qg][ms], 0, 0, 0);
      }
    }
    // ---- mask + online softmax.  Running max in raw score units; p = exp2(s*c - m*c) is one FMA and
    // one v_exp (c = scale*log2 e > 0 keeps the argmax).  A tile every key of which is visible to every
    // row of this wave (all keys valid, below the causal diagonal, inside the window) skips the mask.
    bool interior = (t + 1) * KT <= a.nkeys && (unmasked || ((!causal || t * KT + KT - 1 <= wpos_lo) &&
                                                             (nowin || t * KT > wpos_hi - a.window)));
    if (interior && kvl) interior = __all(lane >= KT || kvs[lane] != 0);
    bf16x8_t pf[QG][ST];
    float alpha[QG];
    bool rescale = false;
#pragma unroll
    for (int qg = 0; qg < QG; ++qg) {
      float mt = -INFINITY;
      if (interior) {
#pragma unroll
        for (int ms = 0; ms < MS; ++ms)
#pragma unroll
          for (int j = 0; j < 4; ++j) mt = fmaxf(mt, s[qg][ms][j]);
      } else {
#pragma unroll
        for (int ms = 0; ms < MS; ++ms) {
          const int kbase = t * KT + ms * 16 + 4 * g;
          int kv[4] = {1, 1, 1, 1};
          if (kvl) {
            const int4 v4 = *reinterpret_cast<const int4*>(kvs + ms * 16 + 4 * g);
            kv[0] = v4.x; kv[1] = v4.y; kv[2] = v4.z; kv[3] = v4.w;
          }
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int key = kbase + j;
            const int ok = (int)(key < a.nkeys) & (int)(kv[j] != 0) & ((int)(key <= qpos[qg]) | !causal) &
                           ((int)(key > qpos[qg] - a.window) | nowin);
            const float v = ok ? s[qg][ms][j] : -INFINITY;
            s[qg][ms][j] = v;
            mt = fmaxf(mt, v);
          }
        }
      }
      mt = xor32_max(xor16_max(mt));
      const float m_new = fmaxf(m_run[qg], mt);
      alpha[qg] = (m_new == -INFINITY) ? 1.f : __builtin_amdgcn_exp2f((m_run[qg] - m_new) * sl2);
      const float mc = (m_new == -INFINITY) ? 0.f : m_new * sl2;
      float rs = 0.f;
#pragma unroll
      for (int ms = 0; ms < MS; ++ms)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float p = __builtin_amdgcn_exp2f(fmaf(s[qg][ms][j], sl2, -mc));   // exp2(-inf) = 0 for masked keys
          rs += p;   // fp32 row sum (P itself enters P.V in bf16)
          pf[qg][ms >> 1][(ms & 1) * 4 + j] = (short)f2bf(p);
        }
      rs = xor32_sum(xor16_sum(rs));
      l_run[qg] = l_run[qg] * alpha[qg] + rs;
      m_run[qg] = m_new;
      rescale = rescale || alpha[qg] != 1.f;
    }
    if (__any(rescale)) {   // no row's running max moved: nothing to rescale (common after a few tiles)
#pragma unroll
      for (int qg = 0; qg < QG; ++qg)
#pragma unroll
        for (int i = 0; i < DS; ++i) o[qg][i] *= alpha[qg];
    }

    // ---- O^T += V^T P^T : A = V^T (tr reads), k order of step st = {32st+4g+0..3, 32st+16+4g+0..3}
    const int q4 = c16 >> 2, p4 = c16 & 3;
#pragma unroll
    for (int ds = 0; ds < DS; ++ds) {
#pragma unroll
      for (int st = 0; st < ST; ++st) {
        bf16x8_t vf;
#pragma unroll
        for (int hh = 0; hh < 2; ++hh) {
          const int row = (2 * st + hh) * 16 + 4 * g + q4;
          const int ch = (2 * ds + (p4 >> 1)) ^ swz_v<D>(row);
          const char* addr = vb + row * (D * 2) + ch * 16 + 8 * (p4 & 1);
          const s16x4_t r = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4_t*)(addr));
          vf[4 * hh + 0] = r[0]; vf[4 * hh + 1] = r[1]; vf[4 * hh + 2] = r[2]; vf[4 * hh + 3] = r[3];
        }
#pragma unroll
        for (int qg = 0; qg < QG; ++qg)
          o[qg][ds] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf, pf[qg][st], o[qg][ds], 0, 0, 0);
      }
    }
  }

  // ---- epilogue: O[q][d] = O^T[d][q] / l ; lane holds d = 16ds + 4g + j for query c16
#pragma unroll
  for (int qg = 0; qg < QG; ++qg) {
    if (qrow[qg] >= a.rows) continue;
    const float inv = l_run[qg] > 0.f ? 1.f / l_run[qg] : 0.f;
    const long orow = map_row(a.omap, qrow[qg]);
    bf16_t* op = a.O + z0 * a.sO0 + z1 * a.sO1 + orow * a.ldo + 4 * g;
#pragma unroll
    for (int ds = 0; ds < DS; ++ds) {
      u16x4_t u;
      u[0] = f2bf(o[qg][ds][0] * inv); u[1] = f2bf(o[qg][ds][1] * inv);
      u[2] = f2bf(o[qg][ds][2] * inv); u[3] = f2bf(o[qg][ds][3] * inv);
      *reinterpret_cast<u16x4_t*>(op + 16 * ds) = u;
    }
    if (a.lse && g == 0)
      a.lse[(long)z * a.rows + qrow[qg]] = (m_run[qg] * sl2 + log2f(l_run[qg])) * 0.6931471805599453f;
  }
}

// ---------------------------------------------------------------- d-256 helpers
// online softmax with a deferred running max: it moves only when a tile's max exceeds it by more than
// FA_DEFER (log2 units; P <= 2^FA_DEFER is exact enough in fp32 sums and bf16 operands), so the O rescale
// runs a few times per row block instead of on most tiles
constexpr float FA_DEFER = 8.f;
constexpr int FA_MAXT = 128;   // key tiles (of 32) the mask table holds: nkeys <= 4096

// diagnostic build (make fastamps): s_memtime stamps of the 32-row d-256 kernels' phases per workgroup, kept in
// registers and written by lane 0 of wave 0 at the end (no extra memory op inside the counted-vmcnt pipeline)
#ifdef PTK_FA_STAMPS
__device__ unsigned long long g_fa_stamps[4][1 << 13][8];   // [kernel: fwd, dQ, dK/dV, fwd64][workgroup][stamp]
#define FA_STAMP(i) st_[i] = __builtin_amdgcn_s_memtime()
#define FA_STAMPS_DECL unsigned long long st_[8] = {}; st_[5] = __builtin_amdgcn_s_memrealtime(); FA_STAMP(0)
#define FA_STAMPS_WRITE(kid, ntiles)                                                               \
  if (threadIdx.x == 0) {                                                                          \
    FA_STAMP(4);                                                                                   \
    st_[6] = __builtin_amdgcn_s_memrealtime();                                                     \
    st_[7] = (unsigned long long)(ntiles);                                                         \
    for (int i_ = 0; i_ < 8; ++i_) g_fa_stamps[kid][blockIdx.x & ((1 << 13) - 1)][i_] = st_[i_];   \
  }
#else
#define FA_STAMP(i) (void)0
#define FA_STAMPS_DECL (void)0
#define FA_STAMPS_WRITE(kid, ntiles) (void)0
#endif

#define FA_DMA(VOFF, SOFF, RSRC, LDS)                                                                      \
  asm volatile("s_nop 0\n\tbuffer_load_dwordx4 %0, %2, %3 offen lds"                                     \
               :: "v"(VOFF), "{m0}"(LDS), "s"(RSRC), "s"(SOFF) : "memory")
typedef __attribute__((ext_vector_type(4))) unsigned int fa_u32x4_t;
PTK_DEV fa_u32x4_t fa_rsrc(const void* base, uint32_t bytes) {
  const uint64_t p = (uint64_t)base;
  fa_u32x4_t r;
  r[0] = __builtin_amdgcn_readfirstlane((uint32_t)p);
  r[1] = __builtin_amdgcn_readfirstlane((uint32_t)(p >> 32));   // stride 0: raw buffer
  r[2] = __builtin_amdgcn_readfirstlane(bytes);                  // num_records: reads past it return 0
  r[3] = 0x00020000u;
  return r;
}
PTK_DEV uint32_t fa_lds_addr(const void* p) { return (uint32_t)(uintptr_t)(fa_lptr_t)p; }
// the kernel's FlashArgs argument (offset 0 of the kernarg segment) behind a pointer the compiler cannot see
// through: the persistent kernels read the per-item fields by scalar loads at item boundaries instead of keeping
// some 50 SGPRs of arguments live across the K/V loop (which spilled)
typedef const FlashArgs __attribute__((address_space(4)))* fa_kargs_ptr_t;
PTK_DEV const FlashArgs& fa_kernarg() {
#if defined(__HIP_DEVICE_COMPILE__)
  fa_kargs_ptr_t pk = (fa_kargs_ptr_t)__builtin_amdgcn_kernarg_segment_ptr();
  asm volatile("" : "+s"(pk));
  return *(const FlashArgs*)pk;
#else
  __builtin_unreachable();
#endif
}
template <int N> using fa_ic = std::integral_constant<int, N>;

// per-tile 32-bit key masks (key valid and < nkeys) of tiles [t_lo, t_hi) into LDS, tile tt by wave tt % NW:
// every key_valid load of the wave issued before the first ballot waits (8 tiles at a time), so the table
// costs one memory latency, not one per tile
template <int NW>
PTK_DEV void fa_key_masks(const int* kvl, int nkeys, int t_lo, int t_hi, int wave, int lane, uint32_t* kmask_s) {
  constexpr int KT = 32;
  for (int base = t_lo + wave; base < t_hi; base += 8 * NW) {
    int v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int key = (base + NW * j) * KT + (lane & 31);
      v[j] = (kvl && base + NW * j < t_hi) ? kvl[min(key, nkeys - 1)] : 1;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int tt = base + NW * j;
      const uint64_t m = __ballot(tt * KT + (lane & 31) < nkeys && v[j] != 0);
      if (tt < t_hi && lane == 0) kmask_s[tt] = (uint32_t)m;
    }
  }
}

// ---------------------------------------------------------------- forward, head_dim 256, 32 rows per wave
// One workgroup = 4 waves (one per SIMD, the whole 512-entry register file each) = 128 query rows of one z;
// each wave owns 32 rows and runs v_mfma_f32_32x32x16_bf16 (32 cycles, 32x32 outputs), so every K / V^T
// fragment read from LDS feeds twice the FLOPs of the 16-row form (whose 8 waves read 256 KiB of LDS per
// 32-key tile, the LDS array's whole 256 B/clk at the MFMA rate).  Per 32-key tile and wave:
//   S^T[32 keys x 32 q] = K Q^T        16 MFMAs, one accumulator chain; A = K rows (ds_read_b128), B = Q
//                                      fragments held in registers for the whole block
//   online softmax                     lane = query column c32, 16 keys (8i + 4h + j) per lane: 15 max + one
//                                      permlane32 swap; the running sum stays per lane half (summed once at
//                                      the end), the running max moves only by more than FA_DEFER
//   O^T[256 d x 32 q] += V^T P^T       16 MFMAs (8 d blocks x 2 key steps); B = P straight from the S^T
//                                      accumulators (registers 8kk..8kk+7 = keys 16kk + 8(j>>2) + 4h + (j&3)),
//                                      A = V^T by ds_read_b64_tr_b16 in that same key order
// Software pipeline inside the wave: iteration t issues QK^T of tile t+1 beside the softmax of tile t, then
// P.V of tile t, so the MFMA pipe has independent work while the softmax VALU runs.  K / V tiles by LDS-DMA
// (8 x 1 KiB pieces per wave per tile) into 4-deep rings, one counted vmcnt + barrier per tile.
// LDS images (32 rows x 512 B, chunk c of row r at chunk c ^ swz(r)): K swz = r & 15 (the b128 row reads of
// 16 distinct keys per lane group hit 16 distinct bank quads), V swz = 4 (r & 3) (each 32-lane half of a
// transposed read takes 4 rows r..r+3 x 64 B: 4 distinct bank quads of 16).
__global__ void __launch_bounds__(256, 1) attn_fwd256w_kernel(FlashArgs a, int nz, int nitems) {
  constexpr int D = 256, KT = 32, NB = 4;
  constexpr int TILE = KT * D * 2;   // 16 KiB
  __shared__ __attribute__((aligned(16))) char smem[2 * NB * TILE + FA_MAXT * 4];
  char* const kring = smem;
  char* const vring = smem + NB * TILE;
  uint32_t* const kmask_s = reinterpret_cast<uint32_t*>(smem + 2 * NB * TILE);
  FA_STAMPS_DECL;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int h = lane >> 5, c32 = lane & 31;
  const int nqb = (a.rows + 127) / 128;
  const int causal = a.causal != 0, nowin = a.window <= 0;

  // ---- work items (row block of 128 query rows, z), heaviest (latest) row blocks first: item i is row block
  // nqb - 1 - i / nz of z = i % nz.  Workgroup b runs items b, 2G - 1 - b, 2G + b, .. (G = gridDim.x; a grid of
  // one workgroup per item runs one each).  Per-item state, set by begin_item:
  int z0 = 0, z1 = 0, t_lo = 0, t_hi = 0, wrow0 = 0, qrow = 0, qpos = 0, wpos_lo = 0, wpos_hi = 0;
  long zi = 0;
  fa_u32x4_t rsk, rsv;
  bf16x8_t qf[16];
  // begin_item part 1: the item's geometry and its key-mask table (kmask_s: every wave must have passed its last
  // read of the previous item's table); part 2: the Q fragments (B operand of S^T = K Q^T for k-step ks: lane holds
  // Q[row c32][16 ks + 8 h .. +7]), whose loads stay in flight until the K/V loop needs them
  auto begin_item = [&](int item) __attribute__((always_inline)) {
    const FlashArgs& a = fa_kernarg();
    const int z = item % nz;
    zi = z;
    z0 = z / a.zin;
    z1 = z - z0 * a.zin;
    const int r0 = (nqb - 1 - item / nz) * 128;
    const long b = z / a.zdiv;
    const int* kvl = a.key_valid ? a.key_valid + b * a.nkeys : nullptr;
    const int pos_lo = r0 / a.qdiv, pos_hi = min(r0 + 127, a.rows - 1) / a.qdiv;
    int k_hi = a.nkeys, k_lo = 0;
    if (a.causal) {
      k_hi = min(k_hi, pos_hi + 1);
      if (a.window > 0) k_lo = max(0, pos_lo - a.window + 1);
    }
    t_lo = k_lo / KT;
    t_hi = (k_hi + KT - 1) / KT;
    wrow0 = r0 + wave * 32;
    qrow = wrow0 + c32;
    wpos_lo = min(wrow0, a.rows - 1) / a.qdiv;
    wpos_hi = min(wrow0 + 31, a.rows - 1) / a.qdiv;
    fa_key_masks<4>(kvl, a.nkeys, t_lo, t_hi, wave, lane, kmask_s);
    const bf16_t* K = a.K + z0 * a.sK0 + z1 * a.sK1;
    const bf16_t* V = a.V + z0 * a.sK0 + z1 * a.sK1;
    rsk = fa_rsrc(K, (uint32_t)((long)a.nkeys * a.ldk * 2));
    rsv = fa_rsrc(V, (uint32_t)((long)a.nkeys * a.ldk * 2));
  };
  auto load_q = [&]() __attribute__((always_inline)) {
    const FlashArgs& a = fa_kernarg();
    const int qrow_c = min(qrow, a.rows - 1);
    qpos = qrow_c / a.qdiv;
    const bf16_t* qp = a.Q + z0 * a.sQ0 + z1 * a.sQ1 + map_row(a.qmap, qrow_c) * a.ldq + 8 * h;
#pragma unroll
    for (int ks = 0; ks < 16; ++ks) qf[ks] = *reinterpret_cast<const bf16x8_t*>(qp + 16 * ks);
  };

  // ---- DMA: wave w stages rows 8w..8w+7 of each tile (4 pieces of 2 rows x 512 B per tensor); lane i of a
  // piece writes LDS row 8w + 2j + (i >> 5), chunk i & 31, fetched from logical chunk (i & 31) ^ swz(row)
  uint32_t dk[4], dv[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int row = wave * 8 + 2 * j + h;
    dk[j] = (uint32_t)row * (uint32_t)a.ldk * 2u + 16u * (c32 ^ (row & 15));
    dv[j] = (uint32_t)row * (uint32_t)a.ldk * 2u + 16u * (c32 ^ (4 * (row & 3)));
  }
  const uint32_t lds_k = __builtin_amdgcn_readfirstlane(fa_lds_addr(kring) + wave * 4096);
  const uint32_t lds_v = __builtin_amdgcn_readfirstlane(fa_lds_addr(vring) + wave * 4096);
  const uint32_t tile_bytes = __builtin_amdgcn_readfirstlane((uint32_t)KT * (uint32_t)a.ldk * 2u);
  auto stage = [&](int bb, int t) __attribute__((always_inline)) {
    const uint32_t so = __builtin_amdgcn_readfirstlane((uint32_t)t * tile_bytes);
#pragma unroll
    for (int j = 0; j < 4; ++j) FA_DMA(dk[j], so, rsk, lds_k + bb * TILE + j * 1024);
#pragma unroll
    for (int j = 0; j < 4; ++j) FA_DMA(dv[j], so, rsv, lds_v + bb * TILE + j * 1024);
  };
  // the first three tiles of the item into ring slots 0..2 (past the last tile: re-loads of it, never read)
  auto stage_first = [&]() __attribute__((always_inline)) {
    if (t_lo < t_hi) {
#pragma unroll
      for (int i = 0; i < 3; ++i) stage(i, min(t_lo + i, t_hi - 1));
    }
  };

  // ---- LDS read addresses (lane part; the ring slot and the rest are immediates).
  // K: row c32, logical chunk 2ks + h -> (2ks + h) ^ (c32 & 15): 8 bases for ks & 7, ks >> 3 = +256 B.
  // V^T (tr read, key step kk, half r, d block db): lane 4q+p of group G = lane >> 4 reads row
  // 16kk + 8r + 4h + q, logical chunk 4db + 2(G & 1) + (p >> 1), byte 8 (p & 1); swz = 4q, so the chunk is
  // 4 ((db & 3) ^ q) + 2(G & 1) + (p >> 1) + 16 (db >> 2): 4 bases for db & 3, kk / r / db >> 2 immediates.
  uint32_t kaddr[8], vaddr[4];   // LDS byte addresses
  {
#pragma unroll
    for (int i = 0; i < 8; ++i)
      kaddr[i] = fa_lds_addr(kring) + c32 * (D * 2) + (((2 * i + h) ^ (c32 & 15)) * 16);
    const int G = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
    const int vrow = 4 * h + q;
#pragma unroll
    for (int i = 0; i < 4; ++i)
      vaddr[i] = fa_lds_addr(vring) + vrow * (D * 2) + (4 * (i ^ q) + 2 * (G & 1) + (p >> 1)) * 16 + 8 * (p & 1);
  }

  typedef __attribute__((ext_vector_type(16))) float f32x16_t;
  f32x16_t o[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) o[i] = (f32x16_t){};
  float m_run = -INFINITY, l_run = 0.f;   // l_run: this lane half's partial row sum
  const float sl2 = a.scale * 1.4426950408889634f;   // scores in log2 units
  const float defer = FA_DEFER / sl2;                 // the deferral in raw score units

  // ---- MFMA and LDS helpers.  The P.V MFMAs are inline asm with O tied to VGPRs (with the builtin, hipcc
  // keeps O in AGPRs and moves it through VGPRs around the rescale, 256 moves per pair of tiles); QK^T uses
  // the builtin, so hipcc sees its operands and results.  Volatile asm keeps its source order, and no LDS
  // read moves across it, so the loops below place every read, MFMA and softmax piece themselves (one slot
  // per MFMA, pinned by sched_barrier): reads run 3 (K) or 2 (V) MFMAs ahead of their use.  Hazards hipcc
  // does not see through the asm: each asm MFMA opens with s_nop 2, the wait states of a VALU write (P, the
  // rescaled O, or any copy the compiler places) right before it; O is read by VALU only in the next
  // iteration's rescale, after the barrier and 16 MFMAs, and in the epilogue, after its own s_nops
  // (tests/test_asm_hazards.py checks the emitted code for both).
  auto kload = [&](uint32_t so, int ks) __attribute__((always_inline)) {
    return *reinterpret_cast<const __attribute__((address_space(3))) bf16x8_t*>(
        (uintptr_t)(kaddr[ks & 7] + so + (ks >> 3) * 256));
  };
  // V^T fragment of key step kk, d block db: two transposed reads (keys 16kk + 8r + 4h + 0..3)
  auto vload = [&](uint32_t so, int kk, int db) __attribute__((always_inline)) {
    bf16x8_t vf;
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const uint32_t addr = vaddr[db & 3] + so + (16 * kk + 8 * r) * (D * 2) + (db >> 2) * 256;
      const s16x4_t x = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4_t*)(uintptr_t)addr);
      vf[4 * r + 0] = x[0]; vf[4 * r + 1] = x[1]; vf[4 * r + 2] = x[2]; vf[4 * r + 3] = x[3];
    }
    return vf;
  };
  auto vmax3 = [](float x, float y, float z) __attribute__((always_inline)) {
    float r;   // (plain fmaxf adds a canonicalising v_max per MFMA-produced operand)
    asm("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(x), "v"(y), "v"(z));
    return r;
  };

  // the mask of tile t on its scores (tiles every key of which every row of the wave sees skip it: all keys
  // valid, below the causal diagonal, inside the window).  Run at the top of the iteration, in a block of its
  // own, so the softmax pieces below have no branch.
  auto mask = [&](int t, f32x16_t& s) __attribute__((always_inline)) {
    const uint32_t km = kmask_s[t];
    const bool interior = km == 0xffffffffu && (!causal || t * KT + KT - 1 <= wpos_lo) &&
                          (nowin || t * KT > wpos_hi - a.window);
    if (interior) return;
    // this row's visible keys of the tile as a 32-bit mask: valid, kl <= qpos - t KT (causal),
    // kl > qpos - W - t KT (window); lane half h holds keys 8i + 4h + j
    uint32_t vis = km;
    if (causal) {
      const int d = qpos - t * KT;
      vis &= d >= 31 ? 0xffffffffu : (d < 0 ? 0u : (2u << d) - 1u);
      if (!nowin) {
        const int e = d - a.window;
        vis &= e < 0 ? 0xffffffffu : (e >= 31 ? 0u : ~((2u << e) - 1u));
      }
    }
    vis >>= 4 * h;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int kl = (r & 3) + 8 * (r >> 2);
      s[r] = ((vis >> kl) & 1u) ? s[r] : -INFINITY;
    }
  };

  // Phase A of an iteration: QK^T of the next tile (16 MFMAs, if QK) beside the online softmax of the
  // current tile's masked scores (if SM) in 16 slots: 0-3 the row max (v_max3), 4 the half-wave max swap and
  // the running max / rescale factor, 5-12 two exponentials each (P to bf16, fp32 row sum), 13 the running
  // sum.  The running max moves only by more than FA_DEFER; the row sum stays per lane half.
  float alpha = 1.f;
  auto phase_a = [&](auto QK, auto SM, uint32_t so, f32x16_t& s_next, const f32x16_t& s, bf16x8_t (&pf)[2])
      __attribute__((always_inline)) {
    constexpr bool qk = decltype(QK)::value, sm = decltype(SM)::value;
    bf16x8_t kf[4];
    if (qk) {
      kf[0] = kload(so, 0);
      kf[1] = kload(so, 1);
      kf[2] = kload(so, 2);
    }
    float mt = 0.f, m_new = 0.f, mc = 0.f, rs = 0.f;
#pragma unroll
    for (int ks = 0; ks < 16; ++ks) {
      if (qk) {
        if (ks + 3 < 16) kf[(ks + 3) & 3] = kload(so, ks + 3);
        s_next = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf[ks & 3], qf[ks], ks == 0 ? (f32x16_t){} : s_next, 0, 0, 0);
      }
      if (sm) {
        if (ks == 0) mt = vmax3(vmax3(s[0], s[1], s[2]), s[3], s[4]);
        else if (ks < 3) mt = vmax3(vmax3(mt, s[4 * ks + 1], s[4 * ks + 2]), s[4 * ks + 3], s[4 * ks + 4]);
        else if (ks == 3) mt = vmax3(mt, s[13], vmax3(s[14], s[15], s[15]));
        else if (ks == 4) {
          // the half-wave swap in asm: hipcc does not see that the v_max3 asm above is the VALU write the
          // permlane reads, so the 2 wait states of that hazard are written out here
          float mt2 = mt;
          asm volatile("s_nop 1\n\tv_permlane32_swap_b32 %0, %1" : "+v"(mt), "+v"(mt2));
          mt = fmaxf(mt, mt2);
          const bool up = mt > m_run + defer;   // m_run = -inf: any finite tile max moves it
          m_new = up ? mt : m_run;
          alpha = (up && m_run != -INFINITY) ? __builtin_amdgcn_exp2f((m_run - m_new) * sl2) : 1.f;
          mc = (m_new == -INFINITY) ? 0.f : m_new * sl2;
        } else if (ks <= 12) {
          const int r = 2 * (ks - 5);
          const float p0 = __builtin_amdgcn_exp2f(fmaf(s[r], sl2, -mc));   // exp2(-inf) = 0 for masked keys
          const float p1 = __builtin_amdgcn_exp2f(fmaf(s[r + 1], sl2, -mc));
          rs += p0 + p1;
          pf[r >> 3][r & 7] = (short)f2bf(p0);
          pf[r >> 3][(r & 7) + 1] = (short)f2bf(p1);
          // pin the pair here: otherwise hipcc sinks the exponentials past the rescale branch to their use
          asm volatile("" : "+v"(pf[r >> 3]));
        } else if (ks == 13) {
          l_run = l_run * alpha + rs;
          m_run = m_new;
        }
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  auto rescale = [&]() __attribute__((always_inline)) {
    if (__any(alpha != 1.f)) {
#pragma unroll
      for (int i = 0; i < 8; ++i) o[i] *= alpha;
    }
  };
  // Phase B: O^T += V^T P^T (16 MFMAs, key step outer so one accumulator's two MFMAs are 8 apart), V^T reads
  // two MFMAs ahead; the next tile's 8 LDS-DMA pieces (if ST) go out one per two MFMAs.
  auto phase_b = [&](auto ST, uint32_t so, const bf16x8_t (&pf)[2], int bb_st, int t_st)
      __attribute__((always_inline)) {
    constexpr bool st = decltype(ST)::value;
    bf16x8_t vf[3];
    vf[0] = vload(so, 0, 0);
    vf[1] = vload(so, 0, 1);
    uint32_t sso = 0;
    if (st) sso = __builtin_amdgcn_readfirstlane((uint32_t)t_st * tile_bytes);
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int kk = i >> 3, db = i & 7;
      if (i + 2 < 16) vf[(i + 2) % 3] = vload(so, (i + 2) >> 3, (i + 2) & 7);
      asm volatile("s_nop 2\n\tv_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+v"(o[db]) : "v"(vf[i % 3]), "v"(pf[kk]));
      if (st && (i & 1) == 0) {
        const int j = i >> 1;   // pieces K0..K3, V0..V3
        if (j < 4) FA_DMA(dk[j], sso, rsk, lds_k + bb_st * TILE + j * 1024);
        else FA_DMA(dv[j - 4], sso, rsv, lds_v + bb_st * TILE + (j - 4) * 1024);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  };

  // Tile t lives in ring slot (t - t_lo) % NB.  At iteration t the wave waits for tile t+1 (tile t+2 may
  // stay in flight), the barrier publishes it, and tile t+3 is staged into the slot of tile t-1, whose last
  // readers (QK^T of t-1 at iteration t-2, P.V of t-1 at iteration t-1) every wave has passed.  Past the last
  // tile the stage re-loads tile t_hi - 1 into that free slot (never read), so every iteration issues the
  // same 8 pieces and waits with the same count.  Fully masked tiles are computed like the others
  // (exp2(-inf) = 0).  The loop body is unrolled by two so the two score accumulators swap roles without a
  // copy.
  // Persistent items: after an item's last P.V, a barrier (every wave is done with the ring and the key-mask
  // table), then the next item's key masks, Q loads and first three K / V tiles are issued BEFORE this item's
  // epilogue, so their latency runs under the epilogue's normalisation and stores.
  int item = blockIdx.x, round_k = 0;
  begin_item(item);
  load_q();
#pragma unroll
  for (int ks = 0; ks < 16; ++ks) fa_pin(qf[ks]);
  __syncthreads();   // key masks published (no LDS-DMA in flight yet)
  FA_STAMP(1);
  stage_first();
  using T_ = std::true_type;
  using F_ = std::false_type;
  f32x16_t sa, sb;
  bf16x8_t pf[2];
  auto slot = [&](int t) { return (uint32_t)((t - t_lo) & (NB - 1)) * (uint32_t)TILE; };
  auto iter = [&](int t, f32x16_t& s_cur, f32x16_t& s_next) __attribute__((always_inline)) {
    mask(t, s_cur);
    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    phase_a(T_{}, T_{}, slot(t + 1), s_next, s_cur, pf);
    rescale();
    phase_b(T_{}, slot(t), pf, (t - t_lo + 3) & (NB - 1), min(t + 3, t_hi - 1));
  };
  for (;;) {
    if (t_lo < t_hi) {
      asm volatile("s_waitcnt vmcnt(16)" ::: "memory");   // tile t_lo landed (tiles t_lo + 1, + 2 in flight)
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) o[i] = (f32x16_t){};
    m_run = -INFINITY;
    l_run = 0.f;
    sb = (f32x16_t){};
    phase_a(T_{}, F_{}, 0, sa, sb, pf);   // QK^T of tile t_lo (t_lo == t_hi: slot 0 holds nothing, unused)
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");   // its MFMA results -> the first VALU reads
    FA_STAMP(2);
    int t = t_lo;
    for (; t + 2 < t_hi; t += 2) {
      iter(t, sa, sb);
      iter(t + 1, sb, sa);
    }
    if (t + 1 < t_hi) {
      iter(t, sa, sb);
      ++t;
      sa = sb;
    }
    if (t < t_hi) {   // the last tile: softmax and P.V only
      mask(t, sa);
      phase_a(F_{}, T_{}, 0, sb, sa, pf);
      rescale();
      phase_b(F_{}, slot(t), pf, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // (the item's stream is done; nothing else in flight)
    FA_STAMP(3);

    // ---- epilogue: O[q][d] = O^T[d][q] / l.  Lane half h holds d = 32db + 8i + 4h + (0..3) for query c32;
    // one permlane32 swap per register pair (i = 2m, 2m + 1) gives the lower half d 32db + 16m + 0..7 and the
    // upper half 32db + 16m + 8..15, stored 16 B per lane.  Its outputs' addresses are taken before the next
    // item's state replaces this one's.
    const float l_tot = l_run + xor32_get(l_run);
    const FlashArgs& ka = fa_kernarg();
    const bool row_ok = qrow < ka.rows;
    bf16_t* op = ka.O + z0 * ka.sO0 + z1 * ka.sO1 + map_row(ka.omap, row_ok ? qrow : 0) * ka.ldo + 8 * h;
    float* lsep = ka.lse ? ka.lse + zi * ka.rows + qrow : nullptr;
    const float lse_v = (m_run * sl2 + log2f(l_tot)) * 0.6931471805599453f;
    // snake order over rounds of G items (round k: workgroup b takes item kG + b for even k, kG + G - 1 - b for
    // odd k): a heavy row block pairs with a light one (the causal tiles per item fall with the item index);
    // round-robin measured slower than one workgroup per item, r05
    ++round_k;
    const int next = round_k * (int)gridDim.x +
                     ((round_k & 1) ? (int)gridDim.x - 1 - (int)blockIdx.x : (int)blockIdx.x);
    if (next < nitems) {
      __builtin_amdgcn_s_barrier();   // every wave is past its last read of the ring and of the mask table
      begin_item(next);
      load_q();
      stage_first();
    }
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");   // the last P.V MFMAs -> VALU reads of O
    if (row_ok) {
      const float inv = l_tot > 0.f ? 1.f / l_tot : 0.f;
#pragma unroll
      for (int db = 0; db < 8; ++db) {
#pragma unroll
        for (int m = 0; m < 2; ++m) {
          uint32_t w[4];   // packed bf16 pairs: registers (i = 2m: 0-1, i = 2m + 1: 2-3)
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const int r = 8 * m + 2 * k;
            w[k] = (uint32_t)f2bf(o[db][r] * inv) | ((uint32_t)f2bf(o[db][r + 1] * inv) << 16);
          }
          // lower half keeps registers of i = 2m and takes the upper half's i = 2m; the upper half keeps i = 2m+1
          const auto s0 = __builtin_amdgcn_permlane32_swap(w[0], w[2], false, false);
          const auto s1 = __builtin_amdgcn_permlane32_swap(w[1], w[3], false, false);
          *reinterpret_cast<uint4*>(op + 32 * db + 16 * m) = make_uint4(s0[0], s1[0], s0[1], s1[1]);
        }
      }
      if (lsep && h == 0) *lsep = lse_v;
    }
    if (next >= nitems) break;
    item = next;
#pragma unroll
    for (int ks = 0; ks < 16; ++ks) fa_pin(qf[ks]);
    // the next item's key masks published; raw barrier: its LDS-DMA stays in flight (a __syncthreads would drain it)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  }
  FA_STAMPS_WRITE(0, t_hi - t_lo);
}

// ============================================================================ backward
// FA2-style split without atomics:
//   delta[r] = sum_d dO[r][d] * O[r][d]
//   dQ kernel  (per 128 query rows, 8 waves x 16 rows, K/V tiles streamed):
//     S^T = K Q^T, dP^T = V dO^T, P^T = exp(S^T*scale - LSE), dS^T = P^T (dP^T - delta)
//     dQ^T += K^T dS^T            (A = K^T by ds_read_b64_tr_b16, B = dS^T from registers)
//   dKV kernel (per 64 keys; wave = 16 keys x half of each 64-row query chunk):
//     S = Q K^T, dP = dO V^T (keys on the lane), P, dS
//     dV^T += dO^T P, dK^T += Q^T dS   (A = dO^T / Q^T by tr reads, B = P / dS from registers)
//   then dQ *= scale, dK *= scale.  GQA: the query rows of all G heads of a kv head are one
//   z-batch, so dK/dV sum over the group for free.
template <int D>
__global__ void __launch_bounds__(256) attn_delta_kernel(FlashBwdArgs a, int nz) {
  // DELTA_RPW rows per wave, every row's loads issued before the first reduction (latency-bound otherwise:
  // one 512-B row pair per wave)
  constexpr int EPL = D / 64, RPW = 4;
  const int lane = threadIdx.x & 63;
  const long gr0 = ((long)blockIdx.x * 4 + (threadIdx.x >> 6)) * RPW;
  const long total = (long)nz * a.rows;
  if (gr0 >= total) return;
  bf16_t ov[RPW][EPL], dv[RPW][EPL];
#pragma unroll
  for (int i = 0; i < RPW; ++i) {
    const long gr = min(gr0 + i, total - 1);
    const long z = gr / a.rows;
    const int r = (int)(gr - z * a.rows);
    const int z0 = (int)(z / a.zin), z1 = (int)(z - (long)z0 * a.zin);
    const bf16_t* op = a.O + z0 * a.sO0 + z1 * a.sO1 + map_row(a.omap, r) * a.ldo + lane * EPL;
    const bf16_t* dp = a.dO + gr * D + lane * EPL;
#pragma unroll
    for (int e = 0; e < EPL; ++e) { ov[i][e] = op[e]; dv[i][e] = dp[e]; }
  }
#pragma unroll
  for (int i = 0; i < RPW; ++i) {
    float s = 0.f;
#pragma unroll
    for (int e = 0; e < EPL; ++e) s += bf2f(ov[i][e]) * bf2f(dv[i][e]);
    s = warp_sum(s);
    if (lane == 0 && gr0 + i < total) a.delta[gr0 + i] = s;
  }
}

template <int D>
__global__ void __launch_bounds__(512, 1) attn_bwd_dq_kernel(FlashBwdArgs a) {
  constexpr int FA_KT = 32;
  using R = FaRing<D, FA_KT>;
  constexpr int KS = D / 32;
  constexpr int DS = D / 16;
  __shared__ __attribute__((aligned(16))) char smem[R::BYTES];   // (K, V) x4, key_valid x4

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, c16 = lane & 15;
  // heaviest (latest, for causal) row blocks first; z fastest
  const int nqb = (a.rows + 127) / 128, nz = gridDim.x / nqb;
  const long z = blockIdx.x % nz;
  const int r0 = (nqb - 1 - (int)(blockIdx.x / nz)) * 128;
  const bf16_t* K = a.K + z * (long)a.nkeys * D;
  const bf16_t* V = a.V + z * (long)a.nkeys * D;
  const long b = z / a.zdiv;
  const int* kvl = a.key_valid ? a.key_valid + b * a.nkeys : nullptr;
  const int pos_lo = r0 / a.qdiv, pos_hi = min(r0 + 127, a.rows - 1) / a.qdiv;
  int k_hi = a.nkeys, k_lo = 0;
  if (a.causal) {
    k_hi = min(k_hi, pos_hi + 1);
    if (a.window > 0) k_lo = max(0, pos_lo - a.window + 1);
  }
  const int t_lo = k_lo / FA_KT, t_hi = (k_hi + FA_KT - 1) / FA_KT;

  const int qrow = r0 + wave * 16 + c16;
  const int qrow_c = min(qrow, a.rows - 1);
  const long qoff = (z * a.rows + qrow_c) * (long)D + 8 * g;
  bf16x8_t qf[KS], df[KS];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    qf[ks] = *reinterpret_cast<const bf16x8_t*>(a.Q + qoff + 32 * ks);
    df[ks] = *reinterpret_cast<const bf16x8_t*>(a.dO + qoff + 32 * ks);
  }
  const float L2E = 1.4426950408889634f;
  float lse2 = a.lse[z * a.rows + qrow_c] * L2E;
  float dlt = a.delta[z * a.rows + qrow_c];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    fa_pin(qf[ks]);
    fa_pin(df[ks]);
  }
  fa_pin(lse2);
  fa_pin(dlt);
  const int qpos = qrow_c / a.qdiv;
  const float sl2 = a.scale * L2E;
  const int causal = a.causal != 0, nowin = a.window <= 0;
  const int wpos_lo = min(r0 + wave * 16, a.rows - 1) / a.qdiv;
  const int wpos_hi = min(r0 + wave * 16 + 15, a.rows - 1) / a.qdiv;

  const int ops = (R::INST >= 8 ? 2 * R::PER_WAVE : 1) + (kvl ? 1 : 0);
  auto stage = [&](int t, int buf) {
    char* kb = smem + buf * 2 * R::TILE;
    char* vb = kb + R::TILE;
    if constexpr (R::INST >= 8) {
#pragma unroll
      for (int j = 0; j < R::PER_WAVE; ++j) {
        const int inst = wave * R::PER_WAVE + j;
        const int row = inst * (64 / R::CPR) + lane / R::CPR;
        const int lch = (lane % R::CPR) ^ swz_kt<D>(row);
        const int key = min(t * FA_KT + row, a.nkeys - 1);
        fa_glds16(K + (long)key * D + 8 * lch, kb + inst * 1024);
        fa_glds16(V + (long)key * D + 8 * lch, vb + inst * 1024);
      }
    } else {
      const int inst = wave & (R::INST - 1);
      const int row = inst * (64 / R::CPR) + lane / R::CPR;
      const int lch = (lane % R::CPR) ^ swz_kt<D>(row);
      const int key = min(t * FA_KT + row, a.nkeys - 1);
      if (wave < R::INST)
        fa_glds16(K + (long)key * D + 8 * lch, kb + inst * 1024);
      else
        fa_glds16(V + (long)key * D + 8 * lch, vb + inst * 1024);
    }
    if (kvl && lane == 0)
      fa_glds16(kvl + min(t * FA_KT + 4 * wave, a.nkeys - 4), smem + R::KV_OFF + buf * 128 + wave * 16);
  };

  f32x4_t acc[DS];
#pragma unroll
  for (int i = 0; i < DS; ++i) acc[i] = (f32x4_t){0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int i = 0; i < FA_NBUF - 1; ++i)
    if (t_lo + i < t_hi) stage(t_lo + i, i);
  for (int t = t_lo; t < t_hi; ++t) {
    const int buf = (t - t_lo) & (FA_NBUF - 1);
    vm_wait(ops * min(FA_NBUF - 2, t_hi - 1 - t));
    // raw barrier (the counted wait above publishes tile t; every LDS read of the buffer restaged below
    // was consumed by an MFMA or a compare in the previous iteration)
    __builtin_amdgcn_s_barrier();
    if (t + FA_NBUF - 1 < t_hi) stage(t + FA_NBUF - 1, (buf + FA_NBUF - 1) & (FA_NBUF - 1));
    const char* kb = smem + buf * 2 * R::TILE;
    const char* vb = kb + R::TILE;
    const int* kvs = reinterpret_cast<const int*>(smem + R::KV_OFF + buf * (FA_KT * 4));
    f32x4_t s[2], dp[2];
#pragma unroll
    for (int ms = 0; ms < 2; ++ms) {
      s[ms] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
      dp[ms] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
      const int row = ms * 16 + c16;
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        const int ch = (ks * 4 + g) ^ swz_kt<D>(row);
        const bf16x8_t kf = *reinterpret_cast<const bf16x8_t*>(kb + row * (D * 2) + ch * 16);
        const bf16x8_t vf = *reinterpret_cast<const bf16x8_t*>(vb + row * (D * 2) + ch * 16);
        s[ms] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf, qf[ks], s[ms], 0, 0, 0);
        dp[ms] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf, df[ks], dp[ms], 0, 0, 0);
      }
    }
    bf16x8_t dsf;
    // tile visible to every row of the wave (valid keys, below the diagonal, inside the window): no mask
    bool interior = (t + 1) * FA_KT <= a.nkeys && (!causal || t * FA_KT + FA_KT - 1 <= wpos_lo) &&
                    (nowin || t * FA_KT > wpos_hi - a.window);
    if (interior && kvl) interior = __all(lane >= FA_KT || kvs[lane] != 0);
    if (interior) {
#pragma unroll
      for (int ms = 0; ms < 2; ++ms)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float p = __builtin_amdgcn_exp2f(fmaf(s[ms][j], sl2, -lse2));
          dsf[ms * 4 + j] = (short)f2bf(bfround(p) * (dp[ms][j] - dlt));
        }
    } else {
#pragma unroll
      for (int ms = 0; ms < 2; ++ms) {
        const int kbase = t * FA_KT + ms * 16 + 4 * g;
        int kv[4] = {1, 1, 1, 1};
        if (kvl) {
          const int4 v4 = *reinterpret_cast<const int4*>(kvs + ms * 16 + 4 * g);
          kv[0] = v4.x; kv[1] = v4.y; kv[2] = v4.z; kv[3] = v4.w;
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int key = kbase + j;
          const int ok = (int)(key < a.nkeys) & (int)(kv[j] != 0) & ((int)(key <= qpos) | !causal) &
                         ((int)(key > qpos - a.window) | nowin);
          const float p = __builtin_amdgcn_exp2f(ok ? fmaf(s[ms][j], sl2, -lse2) : -INFINITY);
          dsf[ms * 4 + j] = (short)f2bf(bfround(p) * (dp[ms][j] - dlt));
        }
      }
    }
    const int q4 = c16 >> 2, p4 = c16 & 3;
#pragma unroll
    for (int ds = 0; ds < DS; ++ds) {
      bf16x8_t kt;
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {
        const int row = hh * 16 + 4 * g + q4;
        const int ch = (2 * ds + (p4 >> 1)) ^ swz_kt<D>(row);
        const char* addr = kb + row * (D * 2) + ch * 16 + 8 * (p4 & 1);
        const s16x4_t r = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4_t*)(addr));
        kt[4 * hh + 0] = r[0]; kt[4 * hh + 1] = r[1]; kt[4 * hh + 2] = r[2]; kt[4 * hh + 3] = r[3];
      }
      acc[ds] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kt, dsf, acc[ds], 0, 0, 0);
    }
  }
  if (qrow >= a.rows) return;
  bf16_t* op = a.dQ + (z * a.rows + qrow) * (long)D + 4 * g;
#pragma unroll
  for (int ds = 0; ds < DS; ++ds) {
    u16x4_t u;
    u[0] = f2bf(acc[ds][0] * a.scale); u[1] = f2bf(acc[ds][1] * a.scale);
    u[2] = f2bf(acc[ds][2] * a.scale); u[3] = f2bf(acc[ds][3] * a.scale);
    *reinterpret_cast<u16x4_t*>(op + 16 * ds) = u;
  }
}

// ---------------------------------------------------------------- forward, head_dim 64 (SigLIP)
// The 16-rows-per-wave, 8-wave structure at head_dim 64: 64-key tiles (8 KiB per tensor: one LDS-DMA piece per
// tensor per wave), K/V rings of 4 slots (64 KiB, so two blocks can share a CU), the loop unrolled by
// the ring depth, per-tile key masks, deferred running max, late waves one phase behind.  Per tile and
// wave: S^T = K Q^T (8 MFMAs), 16 scores per lane, O^T += V^T P^T (8 MFMAs).
__global__ void __launch_bounds__(512, 2) attn_fwd64_kernel(FlashArgs a) {
  constexpr int D = 64, KT = 64, KS = 2, DS = 4, MS = 4, ST = 2, NB = 4;
  constexpr int TILE = KT * D * 2;   // 8 KiB
  __shared__ __attribute__((aligned(16))) char smem[2 * NB * TILE + FA_MAXT * 4];
  char* const kring = smem;
  char* const vring = smem + NB * TILE;
  uint32_t* const kmask_s = reinterpret_cast<uint32_t*>(smem + 2 * NB * TILE);   // 2 words per 64-key tile
  FA_STAMPS_DECL;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, c16 = lane & 15;
  const int nqb = (a.rows + 127) / 128, nz = gridDim.x / nqb;
  // XCD-aware order: blocks b and b + 8 share an XCD (and its L2); the nqb row blocks of one z take consecutive
  // slots of one XCD, so its K / V are fetched from HBM once and re-read from that L2 (the z-major order re-read
  // them from HBM per row block: 415 MB per SigLIP layer against 151 MB of Q, K, V, O)
  int z, qb;
  const int G = gridDim.x;
  if (a.variant == 0 && (G & 7) == 0 && ((G >> 3) % nqb) == 0) {
    const int u = (int)(blockIdx.x & 7) * (G >> 3) + (int)(blockIdx.x >> 3);
    z = u / nqb;
    qb = u - z * nqb;
  } else {
    z = blockIdx.x % nz;
    qb = blockIdx.x / nz;
  }
  const int z0 = z / a.zin, z1 = z - z0 * a.zin;
  const int r0 = (nqb - 1 - qb) * 128;
  const bf16_t* Q = a.Q + z0 * a.sQ0 + z1 * a.sQ1;
  const bf16_t* K = a.K + z0 * a.sK0 + z1 * a.sK1;
  const bf16_t* V = a.V + z0 * a.sK0 + z1 * a.sK1;
  const long b = z / a.zdiv;
  const int* kvl = a.key_valid ? a.key_valid + b * a.nkeys : nullptr;

  const int pos_lo = r0 / a.qdiv, pos_hi = min(r0 + 127, a.rows - 1) / a.qdiv;
  int k_hi = a.nkeys, k_lo = 0;
  if (a.causal) {
    k_hi = min(k_hi, pos_hi + 1);
    if (a.window > 0) k_lo = max(0, pos_lo - a.window + 1);
  }
  const int t_lo = k_lo / KT, t_hi = (k_hi + KT - 1) / KT;

  // key masks: word 2t + h covers keys 64t + 32h .. +31
  for (int tt = wave; tt < 2 * t_hi; tt += 8) {
    const int key = tt * 32 + (lane & 31);
    const bool ok = key < a.nkeys && (!kvl || kvl[min(key, a.nkeys - 1)] != 0);
    const uint64_t m = __ballot(ok);
    if (lane == 0) kmask_s[tt] = (uint32_t)m;
  }

  const int wrow0 = r0 + wave * 16;
  const int qrow = wrow0 + c16;
  const int qrow_c = min(qrow, a.rows - 1);
  const int qpos = qrow_c / a.qdiv;
  bf16x8_t qf[KS];
  {
    const bf16_t* qp = Q + map_row(a.qmap, qrow_c) * a.ldq + 8 * g;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) qf[ks] = *reinterpret_cast<const bf16x8_t*>(qp + 32 * ks);
  }
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) fa_pin(qf[ks]);
  __syncthreads();
  FA_STAMP(1);

  const int causal = a.causal != 0, nowin = a.window <= 0;
  const int wpos_lo = min(wrow0, a.rows - 1) / a.qdiv;
  const int wpos_hi = min(wrow0 + 15, a.rows - 1) / a.qdiv;

  // DMA: wave w stages rows 8w..8w+7 of each tile (one 1-KiB piece per tensor)
  const fa_u32x4_t rsk = fa_rsrc(K, (uint32_t)((long)a.nkeys * a.ldk * 2));
  const fa_u32x4_t rsv = fa_rsrc(V, (uint32_t)((long)a.nkeys * a.ldk * 2));
  uint32_t dk, dv;
  {
    const int row = wave * 8 + (lane >> 3);
    dk = (uint32_t)row * (uint32_t)a.ldk * 2u + 16u * ((lane & 7) ^ swz_k<D>(row));
    dv = (uint32_t)row * (uint32_t)a.ldk * 2u + 16u * ((lane & 7) ^ swz_v<D>(row));
  }
  const uint32_t lds_k = __builtin_amdgcn_readfirstlane(fa_lds_addr(kring) + wave * 1024);
  const uint32_t lds_v = __builtin_amdgcn_readfirstlane(fa_lds_addr(vring) + wave * 1024);
  const uint32_t tile_bytes = __builtin_amdgcn_readfirstlane((uint32_t)KT * (uint32_t)a.ldk * 2u);
  auto stage = [&](int bb, int t) __attribute__((always_inline)) {
    const uint32_t so = __builtin_amdgcn_readfirstlane((uint32_t)t * tile_bytes);
    FA_DMA(dk, so, rsk, lds_k + bb * TILE);
    FA_DMA(dv, so, rsv, lds_v + bb * TILE);
  };
  // K rows 16ms + c16, chunk (4ks + g) ^ ((row >> 1) & 7): the swizzle does not depend on ms (immediate);
  // V^T rows 16(2st + hh) + 4g + q4, chunk (2ds + (p4 >> 1)) ^ 2((row >> 1) & 3): independent of st, hh
  int koff[KS];
  const char* vaddr[DS];
  {
    const int q4 = c16 >> 2, p4 = c16 & 3, vrow = 4 * g + q4;
#pragma unroll
    for (int i = 0; i < KS; ++i) koff[i] = c16 * (D * 2) + ((i * 4 + g) ^ swz_k<D>(c16)) * 16;
#pragma unroll
    for (int i = 0; i < DS; ++i) {
      const uint32_t va = fa_lds_addr(vring) + vrow * (D * 2) + ((2 * i + (p4 >> 1)) ^ swz_v<D>(vrow)) * 16 + 8 * (p4 & 1);
      vaddr[i] = (const char*)(fa_lptr_t)(uintptr_t)__builtin_amdgcn_readfirstlane(0) + va;
    }
  }

  f32x4_t o[DS];
#pragma unroll
  for (int i = 0; i < DS; ++i) o[i] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
  float m_run = -INFINITY, l_run = 0.f;
  const float sl2 = a.scale * 1.4426950408889634f;
  const float defer = FA_DEFER / sl2;
  const bool idle = wrow0 >= a.rows;   // rows past the end (SigLIP's half-empty last block)

  auto sync = [&](int bb, int t) __attribute__((always_inline)) {
    if (t + 1 < t_hi) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (t + 2 < t_hi) stage((bb + 2) % NB, t + 2);
  };
  auto qk = [&](auto BUF, f32x4_t (&s)[MS]) __attribute__((always_inline)) {
    constexpr int bb = decltype(BUF)::value;
    const char* kb = kring + bb * TILE;
#pragma unroll
    for (int ms = 0; ms < MS; ++ms) {
      s[ms] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        const bf16x8_t kf = *reinterpret_cast<const bf16x8_t*>(kb + koff[ks] + ms * 16 * (D * 2));
        s[ms] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf, qf[ks], s[ms], 0, 0, 0);
      }
    }
  };
  // P for the k order of the P.V step st: {32st + 4g + 0..3, 32st + 16 + 4g + 0..3}
  auto softmax = [&](int t, f32x4_t (&s)[MS], bf16x8_t (&pf)[ST]) __attribute__((always_inline)) {
    const uint32_t km0 = kmask_s[2 * t], km1 = kmask_s[2 * t + 1];
    const bool interior = (km0 & km1) == 0xffffffffu && (!causal || t * KT + KT - 1 <= wpos_lo) &&
                          (nowin || t * KT > wpos_hi - a.window);
    float mt = -INFINITY;
    if (interior) {
#pragma unroll
      for (int ms = 0; ms < MS; ++ms)
#pragma unroll
        for (int j = 0; j < 4; ++j) mt = fmaxf(mt, s[ms][j]);
    } else {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        uint32_t vis = h ? km1 : km0;
        if (causal) {
          const int d = qpos - (t * KT + 32 * h);
          vis &= d >= 31 ? 0xffffffffu : (d < 0 ? 0u : (2u << d) - 1u);
          if (!nowin) {
            const int e = d - a.window;
            vis &= e < 0 ? 0xffffffffu : (e >= 31 ? 0u : ~((2u << e) - 1u));
          }
        }
#pragma unroll
        for (int m2 = 0; m2 < 2; ++m2)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int ms = 2 * h + m2, kl = m2 * 16 + 4 * g + j;
            const float v = ((vis >> kl) & 1u) ? s[ms][j] : -INFINITY;
            s[ms][j] = v;
            mt = fmaxf(mt, v);
          }
      }
    }
    mt = xor32_max(xor16_max(mt));
    const bool up = mt > m_run + defer;
    const float m_new = up ? mt : m_run;
    const float alpha = (up && m_run != -INFINITY) ? __builtin_amdgcn_exp2f((m_run - m_new) * sl2) : 1.f;
    const float mc = (m_new == -INFINITY) ? 0.f : m_new * sl2;
    float rs = 0.f;
#pragma unroll
    for (int ms = 0; ms < MS; ++ms)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float p = __builtin_amdgcn_exp2f(fmaf(s[ms][j], sl2, -mc));
        rs += p;
        pf[ms >> 1][(ms & 1) * 4 + j] = (short)f2bf(p);
      }
    rs = xor32_sum(xor16_sum(rs));
    l_run = l_run * alpha + rs;
    m_run = m_new;
    if (__any(alpha != 1.f)) {
#pragma unroll
      for (int i = 0; i < DS; ++i) o[i] *= alpha;
    }
  };
  auto pv = [&](auto BUF, const bf16x8_t (&pf)[ST]) __attribute__((always_inline)) {
    constexpr int bb = decltype(BUF)::value;
#pragma unroll
    for (int ds = 0; ds < DS; ++ds)
#pragma unroll
      for (int st = 0; st < ST; ++st) {
        bf16x8_t vf;
#pragma unroll
        for (int hh = 0; hh < 2; ++hh) {
          const char* addr = vaddr[ds] + bb * TILE + (2 * st + hh) * 16 * (D * 2);
          const s16x4_t r = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4_t*)(addr));
          vf[4 * hh + 0] = r[0]; vf[4 * hh + 1] = r[1]; vf[4 * hh + 2] = r[2]; vf[4 * hh + 3] = r[3];
        }
        o[ds] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf, pf[st], o[ds], 0, 0, 0);
      }
  };
  auto early = [&](auto BUF, int t) __attribute__((always_inline)) {
    constexpr int bb = decltype(BUF)::value;
    sync(bb, t);
    if (idle) return;
    f32x4_t s[MS];
    bf16x8_t pf[ST];
    qk(BUF, s);
    softmax(t, s, pf);
    pv(BUF, pf);
  };
  bf16x8_t pprev[ST];
  auto late = [&](auto BUF, int t) __attribute__((always_inline)) {
    constexpr int bb = decltype(BUF)::value;
    if (t < t_hi) sync(bb, t);
    if (idle) return;
    if (t > t_lo) pv(fa_ic<(bb + NB - 1) % NB>{}, pprev);
    if (t == t_hi) return;
    f32x4_t s[MS];
    qk(BUF, s);
    softmax(t, s, pprev);
  };
  if (t_lo < t_hi) stage(0, t_lo);
  if (t_lo + 1 < t_hi) stage(1, t_lo + 1);
  FA_STAMP(2);
  if (wave < 4) {
    for (int t = t_lo; t < t_hi;) {
      early(fa_ic<0>{}, t);
      if (++t >= t_hi) break;
      early(fa_ic<1>{}, t);
      if (++t >= t_hi) break;
      early(fa_ic<2>{}, t);
      if (++t >= t_hi) break;
      early(fa_ic<3>{}, t);
      ++t;
    }
  } else {
    for (int t = t_lo; t <= t_hi;) {
      late(fa_ic<0>{}, t);
      if (++t > t_hi) break;
      late(fa_ic<1>{}, t);
      if (++t > t_hi) break;
      late(fa_ic<2>{}, t);
      if (++t > t_hi) break;
      late(fa_ic<3>{}, t);
      ++t;
    }
  }
  FA_STAMP(3);
  if (qrow >= a.rows) return;
  const float inv = l_run > 0.f ? 1.f / l_run : 0.f;
  bf16_t* op = a.O + z0 * a.sO0 + z1 * a.sO1 + map_row(a.omap, qrow) * a.ldo + 4 * g;
#pragma unroll
  for (int ds = 0; ds < DS; ++ds) {
    u16x4_t u;
    u[0] = f2bf(o[ds][0] * inv); u[1] = f2bf(o[ds][1] * inv);
    u[2] = f2bf(o[ds][2] * inv); u[3] = f2bf(o[ds][3] * inv);
    *reinterpret_cast<u16x4_t*>(op + 16 * ds) = u;
  }
  if (a.lse && g == 0)
    a.lse[(long)z * a.rows + qrow] = (m_run * sl2 + log2f(l_run)) * 0.6931471805599453f;
  FA_STAMPS_WRITE(3, t_hi - t_lo);
}

// ---------------------------------------------------------------- dQ, head_dim 256, 32 rows per wave
// attn_fwd256w_kernel's structure applied to the dQ pass: 4 waves (one per SIMD) x 32 query rows, 32x32x16
// MFMAs, K / V tiles of 32 keys by LDS-DMA into 4-deep rings, one counted vmcnt + barrier per tile.  Per tile
// and wave:
//   S^T = K Q^T, dP^T = V dO^T   32 MFMAs, A = K / V rows (ds_read_b128), B = the wave's Q / dO fragments,
//                                held in registers for the whole block
//   P = exp2(S scale log2e - LSE log2e) (bf16), dS = P (dP - delta) (bf16)   lane = query column: the row's
//                                LSE and delta are per lane, no cross-lane work at all
//   dQ^T[256 d x 32 q] += K^T dS^T   16 MFMAs, A = K^T by ds_read_b64_tr_b16 from the same K tile, B = dS^T
//                                straight from the accumulator layout (keys 16kk + 8(j>>2) + 4h + (j&3)),
//                                dQ^T accumulated in AGPRs
// Software pipeline: iteration t issues S / dP of tile t+1 (phase A) beside dS of tile t, then dQ of tile t
// (phase B) with the next DMA pieces.  The K image serves row reads and transposed reads: chunk c of row r at
// c ^ (4 (r & 3) | ((r >> 2) & 3)) (16 distinct chunk quads for the b128 lane groups, 4 distinct bank quads
// for the 4 rows of a transposed read); the V image uses it too (row reads only).  It also computes delta = rowsum(dO O) (attn_delta_kernel's job)
// from the dO fragments it holds, and runs before the dK/dV kernel, which reads it.  Same arithmetic as
// the generic attn_bwd_dq_kernel (P rounded to bf16 before the product, as the dK/dV kernel does).
PTK_DEV int swz_dual(int r) { return ((r & 3) << 2) | ((r >> 2) & 3); }

#ifndef DQ_RA
#define DQ_RA 2   // dQ kernel: LDS fragment reads issued this many MFMAs ahead of their use
#endif
typedef const FlashBwdArgs __attribute__((address_space(4)))* fb_kargs_ptr_t;
PTK_DEV const FlashBwdArgs& fb_kernarg() {   // fa_kernarg's laundered pointer for the backward arguments
#if defined(__HIP_DEVICE_COMPILE__)
  fb_kargs_ptr_t pk = (fb_kargs_ptr_t)__builtin_amdgcn_kernarg_segment_ptr();
  asm volatile("" : "+s"(pk));
  return *(const FlashBwdArgs*)pk;
#else
  __builtin_unreachable();
#endif
}

__global__ void __launch_bounds__(256, 1) attn_bwd_dq256w_kernel(FlashBwdArgs a, int nz, int nitems) {
  constexpr int D = 256, KT = 32, NB = 4;
  constexpr int TILE = KT * D * 2;
  typedef __attribute__((ext_vector_type(16))) float f32x16_t;
  // ring slot b: the K tile at 2b TILE, the V tile at (2b + 1) TILE, so one base register addresses both
  __shared__ __attribute__((aligned(16))) char smem[2 * NB * TILE + FA_MAXT * 4];
  char* const kring = smem;
  uint32_t* const kmask_s = reinterpret_cast<uint32_t*>(smem + 2 * NB * TILE);
  FA_STAMPS_DECL;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int h = lane >> 5, c32 = lane & 31;
  const int nqb = (a.rows + 127) / 128;
  const float L2E = 1.4426950408889634f;
  const float sl2 = a.scale * L2E;
  const int causal = a.causal != 0, nowin = a.window <= 0;

  // ---- work items (row block of 128 query rows, z), heaviest (latest) row blocks first, in
  // attn_fwd256w_kernel's snake order over rounds of the persistent grid.  Per-item state (begin_item, load_qdo):
  long z = 0;
  int t_lo = 0, t_hi = 0, wrow0 = 0, qrow = 0, qpos = 0, wpos_lo = 0, wpos_hi = 0;
  float lse2 = 0.f, dlt = 0.f;
  fa_u32x4_t rsk, rsv;
  bf16x8_t qf[16], df[16], of[16];   // Q, dO fragments (B operands, k-step ks: row c32, d 16 ks + 8 h .. +7); O
  auto begin_item = [&](int item) __attribute__((always_inline)) {
    const FlashBwdArgs& a = fb_kernarg();
    z = item % nz;
    const int r0 = (nqb - 1 - item / nz) * 128;
    const long b = z / a.zdiv;
    const int* kvl = a.key_valid ? a.key_valid + b * a.nkeys : nullptr;
    const int pos_lo = r0 / a.qdiv, pos_hi = min(r0 + 127, a.rows - 1) / a.qdiv;
    int k_hi = a.nkeys, k_lo = 0;
    if (a.causal) {
      k_hi = min(k_hi, pos_hi + 1);
      if (a.window > 0) k_lo = max(0, pos_lo - a.window + 1);
    }
    t_lo = k_lo / KT;
    t_hi = (k_hi + KT - 1) / KT;
    wrow0 = r0 + wave * 32;
    qrow = wrow0 + c32;
    wpos_lo = min(wrow0, a.rows - 1) / a.qdiv;
    wpos_hi = min(wrow0 + 31, a.rows - 1) / a.qdiv;
    fa_key_masks<4>(kvl, a.nkeys, t_lo, t_hi, wave, lane, kmask_s);
    rsk = fa_rsrc(a.K + z * (long)a.nkeys * D, (uint32_t)((long)a.nkeys * D * 2));
    rsv = fa_rsrc(a.V + z * (long)a.nkeys * D, (uint32_t)((long)a.nkeys * D * 2));
  };
  // the item's Q, dO, O fragments and LSE (loads left in flight); delta = rowsum(dO O) once they landed
  auto load_qdo = [&]() __attribute__((always_inline)) {
    const FlashBwdArgs& a = fb_kernarg();
    const int qrow_c = min(qrow, a.rows - 1);
    qpos = qrow_c / a.qdiv;
    const long qoff = (z * a.rows + qrow_c) * (long)D + 8 * h;
#pragma unroll
    for (int ks = 0; ks < 16; ++ks) {
      qf[ks] = *reinterpret_cast<const bf16x8_t*>(a.Q + qoff + 16 * ks);
      df[ks] = *reinterpret_cast<const bf16x8_t*>(a.dO + qoff + 16 * ks);
    }
    lse2 = a.lse[z * a.rows + qrow_c] * L2E;
    const long z0 = z / a.zin, z1 = z - z0 * a.zin;
    const bf16_t* orow = a.O + z0 * a.sO0 + z1 * a.sO1 + map_row(a.omap, qrow_c) * a.ldo + 8 * h;
#pragma unroll
    for (int ks = 0; ks < 16; ++ks) of[ks] = *reinterpret_cast<const bf16x8_t*>(orow + 16 * ks);
  };
  auto finish_qdo = [&]() __attribute__((always_inline)) {
    float acc0 = 0.f;
#pragma unroll
    for (int ks = 0; ks < 16; ++ks)
#pragma unroll
      for (int e = 0; e < 8; ++e) acc0 += bf2f((bf16_t)of[ks][e]) * bf2f((bf16_t)df[ks][e]);
    dlt = xor32_sum(acc0);
    const FlashBwdArgs& a = fb_kernarg();
    if (h == 0 && qrow < a.rows) a.delta[z * a.rows + qrow] = dlt;
#pragma unroll
    for (int ks = 0; ks < 16; ++ks) {
      fa_pin(qf[ks]);
      fa_pin(df[ks]);
    }
  };

  // ---- DMA: wave w stages rows 8w..8w+7 of each tile (4 pieces of 2 rows x 512 B per tensor)
  uint32_t dk[4], dv[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int row = wave * 8 + 2 * j + h;
    dk[j] = (uint32_t)row * (D * 2) + 16u * (c32 ^ swz_dual(row));
    dv[j] = dk[j];
  }
  const uint32_t lds_k = __builtin_amdgcn_readfirstlane(fa_lds_addr(kring) + wave * 4096);
  const uint32_t lds_v = lds_k + TILE;
  constexpr uint32_t tile_bytes = KT * D * 2;
  auto stage = [&](int bb, int t) __attribute__((always_inline)) {
    const uint32_t so = __builtin_amdgcn_readfirstlane((uint32_t)t * tile_bytes);
#pragma unroll
    for (int j = 0; j < 4; ++j) FA_DMA(dk[j], so, rsk, lds_k + bb * 2 * TILE + j * 1024);
#pragma unroll
    for (int j = 0; j < 4; ++j) FA_DMA(dv[j], so, rsv, lds_v + bb * 2 * TILE + j * 1024);
  };
  // the first three tiles of the item into ring slots 0..2 (past the last tile: re-loads of it, never read)
  auto stage_first = [&]() __attribute__((always_inline)) {
    if (t_lo < t_hi) {
#pragma unroll
      for (int i = 0; i < 3; ++i) stage(i, min(t_lo + i, t_hi - 1));
    }
  };

  // ---- LDS read addresses.  Row reads (K and V, k-step ks): row c32, logical chunk 2ks + h: 8 bases for
  // ks & 7 (both tiles use swz_dual), ks >> 3 = +256 B, the V tile +TILE.  Transposed K reads (key step kk, half r, d block db): lane 4q+p of group
  // G reads row 16kk + 8r + 4h + q, logical chunk 4db + 2(G & 1) + (p >> 1); with swz_dual the physical chunk
  // is 4((db & 3) ^ q) + ((2(G & 1) + (p >> 1)) ^ ((2r + h) & 3)) + 16 (db >> 2): 8 bases for (db & 3, r).
  uint32_t kaddr[8], taddr[8];
  {
#pragma unroll
    for (int i = 0; i < 8; ++i) kaddr[i] = fa_lds_addr(kring) + c32 * (D * 2) + (((2 * i + h) ^ swz_dual(c32)) * 16);
    const int G = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int dbl = i & 3, r = i >> 2;
      const int row = 8 * r + 4 * h + q;
      const int ch = (4 * dbl + 2 * (G & 1) + (p >> 1)) ^ swz_dual(row);
      taddr[i] = fa_lds_addr(kring) + row * (D * 2) + ch * 16 + 8 * (p & 1);
    }
  }
  auto rload = [&](int tensor, uint32_t so, int ks) __attribute__((always_inline)) {
    return *reinterpret_cast<const __attribute__((address_space(3))) bf16x8_t*>(
        (uintptr_t)(kaddr[ks & 7] + so + tensor * TILE + (ks >> 3) * 256));
  };
  auto tload = [&](uint32_t so, int kk, int db) __attribute__((always_inline)) {
    bf16x8_t vf;
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const uint32_t addr = taddr[(db & 3) + 4 * r] + so + 16 * kk * (D * 2) + (db >> 2) * 256;
      const s16x4_t x = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4_t*)(uintptr_t)addr);
      vf[4 * r + 0] = x[0]; vf[4 * r + 1] = x[1]; vf[4 * r + 2] = x[2]; vf[4 * r + 3] = x[3];
    }
    return vf;
  };

  f32x16_t acc[8];   // dQ^T: d block db, lane = query column

  // visibility of tile t for this row (all ones when the tile is interior for the wave)
  auto vis_of = [&](int t) __attribute__((always_inline)) {
    const uint32_t km = kmask_s[t];
    const bool interior = km == 0xffffffffu && (!causal || t * KT + KT - 1 <= wpos_lo) &&
                          (nowin || t * KT > wpos_hi - a.window);
    uint32_t vis = km;
    if (!interior && causal) {
      const int d = qpos - t * KT;
      vis &= d >= 31 ? 0xffffffffu : (d < 0 ? 0u : (2u << d) - 1u);
      if (!nowin) {
        const int e = d - a.window;
        vis &= e < 0 ? 0xffffffffu : (e >= 31 ? 0u : ~((2u << e) - 1u));
      }
    }
    return interior ? 0xffffffffu : (vis >> (4 * h));
  };

  // Phase A: S^T, dP^T of the next tile (32 MFMAs, if MM) beside dS of the current tile (if DS) in the
  // slots of the first 16 MFMAs: two keys per slot (P = exp2, bf16 round, dS = P (dP - delta), bf16).
  auto phase_a = [&](auto MM, auto DSC, uint32_t so, f32x16_t& s_n, f32x16_t& p_n, const f32x16_t& s,
                     const f32x16_t& dp, uint32_t vis, bf16x8_t (&dsf)[2]) __attribute__((always_inline)) {
    constexpr bool mm = decltype(MM)::value, dsc = decltype(DSC)::value;
    constexpr int RA = DQ_RA, RN = DQ_RA + 1;   // K / V row reads RA k-steps ahead of their MFMAs
    bf16x8_t kf[RN], vf[RN];
    if (mm) {
#pragma unroll
      for (int i = 0; i < RA; ++i) { kf[i] = rload(0, so, i); vf[i] = rload(1, so, i); }
    }
#pragma unroll
    for (int ks = 0; ks < 16; ++ks) {
      if (mm) {
        if (ks + RA < 16) {
          kf[(ks + RA) % RN] = rload(0, so, ks + RA);
          vf[(ks + RA) % RN] = rload(1, so, ks + RA);
        }
        s_n = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf[ks % RN], qf[ks], ks == 0 ? (f32x16_t){} : s_n, 0, 0, 0);
        p_n = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf[ks % RN], df[ks], ks == 0 ? (f32x16_t){} : p_n, 0, 0, 0);
      }
      if (dsc && ks < 8) {
        const int r = 2 * ks;
        float d2[2];
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          const int kl = ((r + e) & 3) + 8 * ((r + e) >> 2);
          const float pe = __builtin_amdgcn_exp2f(((vis >> kl) & 1u) ? fmaf(s[r + e], sl2, -lse2) : -INFINITY);
          d2[e] = bfround(pe) * (dp[r + e] - dlt);
        }
        dsf[r >> 3][r & 7] = (short)f2bf(d2[0]);
        dsf[r >> 3][(r & 7) + 1] = (short)f2bf(d2[1]);
        asm volatile("" : "+v"(dsf[r >> 3]));   // keep the pair here (not sunk to the dQ MFMAs)
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  // Phase B: dQ^T += K^T dS^T (16 MFMAs, key step outer), K^T reads two MFMAs ahead, the next DMA pieces
  // (if ST) one per two MFMAs.  (All MFMAs of this kernel are builtins: no VALU touches dQ^T before the
  // epilogue, so hipcc has no reason to move it between register files, and it inserts the hazard waits.)
  auto phase_b = [&](auto ST, uint32_t so, const bf16x8_t (&dsf)[2], int bb_st, int t_st)
      __attribute__((always_inline)) {
    constexpr bool st = decltype(ST)::value;
    constexpr int RA = DQ_RA, RN = DQ_RA + 1;
    bf16x8_t tf[RN];
#pragma unroll
    for (int i = 0; i < RA; ++i) tf[i] = tload(so, i >> 3, i & 7);
    uint32_t sso = 0;
    if (st) sso = __builtin_amdgcn_readfirstlane((uint32_t)t_st * tile_bytes);
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int kk = i >> 3, db = i & 7;
      if (i + RA < 16) tf[(i + RA) % RN] = tload(so, (i + RA) >> 3, (i + RA) & 7);
      acc[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(tf[i % RN], dsf[kk], acc[db], 0, 0, 0);
      if (st && (i & 1) == 0) {
        const int j = i >> 1;
        if (j < 4) FA_DMA(dk[j], sso, rsk, lds_k + bb_st * 2 * TILE + j * 1024);
        else FA_DMA(dv[j - 4], sso, rsv, lds_v + bb_st * 2 * TILE + (j - 4) * 1024);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  };

  // Persistent items (attn_fwd256w_kernel's scheme): after an item's last dQ MFMAs, a barrier (every wave is done
  // with the ring and the key-mask table), then the next item's key masks, Q / dO / O loads and first three K / V
  // tiles are issued BEFORE this item's dQ epilogue, so their latency runs under its scaling and stores; the next
  // item's delta follows the epilogue.
  int item = blockIdx.x, round_k = 0;
  begin_item(item);
  load_qdo();
  finish_qdo();
  __syncthreads();   // key masks published (no LDS-DMA in flight yet)
  FA_STAMP(1);
  stage_first();
  using T_ = std::true_type;
  using F_ = std::false_type;
  f32x16_t sa, pa, sb, pb;
  bf16x8_t dsf[2];
  auto slot = [&](int t) { return (uint32_t)((t - t_lo) & (NB - 1)) * (uint32_t)(2 * TILE); };
  auto iter = [&](int t, f32x16_t& s_c, f32x16_t& p_c, f32x16_t& s_n, f32x16_t& p_n) __attribute__((always_inline)) {
    const uint32_t vis = vis_of(t);
    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    phase_a(T_{}, T_{}, slot(t + 1), s_n, p_n, s_c, p_c, vis, dsf);
    phase_b(T_{}, slot(t), dsf, (t - t_lo + 3) & (NB - 1), min(t + 3, t_hi - 1));
  };
  for (;;) {
    if (t_lo < t_hi) {
      asm volatile("s_waitcnt vmcnt(16)" ::: "memory");   // tile t_lo landed (t_lo + 1, + 2 in flight)
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] = (f32x16_t){};
    sb = (f32x16_t){};
    pb = (f32x16_t){};
    phase_a(T_{}, F_{}, 0, sa, pa, sb, pb, 0u, dsf);
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");   // its MFMA results -> the first VALU reads
    FA_STAMP(2);
    int t = t_lo;
    for (; t + 2 < t_hi; t += 2) {
      iter(t, sa, pa, sb, pb);
      iter(t + 1, sb, pb, sa, pa);
    }
    if (t + 1 < t_hi) {
      iter(t, sa, pa, sb, pb);
      ++t;
      sa = sb;
      pa = pb;
    }
    if (t < t_hi) {
      phase_a(F_{}, T_{}, 0, sb, pb, sa, pa, vis_of(t), dsf);
      phase_b(F_{}, slot(t), dsf, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // (the item's stream is done; nothing else in flight)
    FA_STAMP(3);

    // ---- dQ[q][d] = scale dQ^T[d][q] (bf16), 16-B stores after one permlane32 swap per register pair; the
    // output address is taken before the next item's state replaces this one's
    const FlashBwdArgs& ka = fb_kernarg();
    const bool row_ok = qrow < ka.rows;
    bf16_t* op = ka.dQ + (z * ka.rows + (row_ok ? qrow : 0)) * (long)D + 8 * h;
    ++round_k;
    const int next = round_k * (int)gridDim.x +
                     ((round_k & 1) ? (int)gridDim.x - 1 - (int)blockIdx.x : (int)blockIdx.x);
    if (next < nitems) {
      __builtin_amdgcn_s_barrier();   // every wave is past its last read of the ring and of the mask table
      begin_item(next);
      load_qdo();
      stage_first();
    }
    if (row_ok) {
#pragma unroll
      for (int db = 0; db < 8; ++db) {
#pragma unroll
        for (int m = 0; m < 2; ++m) {
          uint32_t w[4];
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const int r = 8 * m + 2 * k;
            w[k] = (uint32_t)f2bf(acc[db][r] * ka.scale) | ((uint32_t)f2bf(acc[db][r + 1] * ka.scale) << 16);
          }
          const auto s0 = __builtin_amdgcn_permlane32_swap(w[0], w[2], false, false);
          const auto s1 = __builtin_amdgcn_permlane32_swap(w[1], w[3], false, false);
          *reinterpret_cast<uint4*>(op + 32 * db + 16 * m) = make_uint4(s0[0], s1[0], s0[1], s1[1]);
        }
      }
    }
    if (next >= nitems) break;
    item = next;
    finish_qdo();
    // the next item's key masks published; raw barrier: its LDS-DMA stays in flight (a __syncthreads would drain it)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  }
  FA_STAMPS_WRITE(1, t_hi - t_lo);
}


template <int D>
__global__ void __launch_bounds__(256, 1) attn_bwd_dkv_kernel(FlashBwdArgs a) {
  // 4 waves x 16 keys; one wave per SIMD so K/V fragments (B operands) and the dK^T/dV^T
  // accumulators (128 fp32 per lane at D = 256) stay in the 512-entry register file.
  constexpr int CPR = D / 8;
  constexpr int TILE_BYTES = 64 * D * 2;     // 64 query rows of Q or dO
  constexpr int KS = D / 32;
  constexpr int DS = D / 16;
  __shared__ __attribute__((aligned(16))) char smem[4 * TILE_BYTES + 2 * 512];   // Q0 dO0 Q1 dO1, (lse|delta) x2

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, c16 = lane & 15;
  const long z = blockIdx.y;
  const int k0 = blockIdx.x * 64;
  const int key = k0 + wave * 16 + c16;
  const int key_c = min(key, a.nkeys - 1);
  const long b = z / a.zdiv;
  const bf16_t* Qz = a.Q + z * (long)a.rows * D;
  const bf16_t* dOz = a.dO + z * (long)a.rows * D;
  bf16x8_t kf[KS], vf[KS];
  {
    const long ko = (z * a.nkeys + key_c) * (long)D + 8 * g;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      kf[ks] = *reinterpret_cast<const bf16x8_t*>(a.K + ko + 32 * ks);
      vf[ks] = *reinterpret_cast<const bf16x8_t*>(a.V + ko + 32 * ks);
    }
  }
  const bool key_ok = key < a.nkeys && (!a.key_valid || a.key_valid[b * a.nkeys + key_c] != 0);
  int r_lo = 0, r_hi = a.rows;
  if (a.causal) {
    r_lo = min(a.rows, k0 * a.qdiv);
    if (a.window > 0) r_hi = min(a.rows, (k0 + 64 + a.window - 1) * a.qdiv);
  }
  const int c_lo = r_lo / 64, c_hi = (r_hi + 63) / 64;
  const float L2E = 1.4426950408889634f;
  const float sl2 = a.scale * L2E;

  constexpr int ROWS_PER_INST = 64 / CPR;
  constexpr int INSTS = CPR / 4;              // per wave per tile (4 waves)
  auto stage = [&](int c, int buf) {
    char* qb = smem + buf * 2 * TILE_BYTES;
    char* ob = qb + TILE_BYTES;
#pragma unroll
    for (int j = 0; j < INSTS; ++j) {
      const int inst = wave * INSTS + j;
      const int row = inst * ROWS_PER_INST + lane / CPR;
      const int pch = lane % CPR;
      const int qr = min(c * 64 + row, a.rows - 1);
      const int lch = pch ^ swz_k<D>(row);
      fa_glds16(Qz + (long)qr * D + 8 * lch, qb + inst * 1024);
      fa_glds16(dOz + (long)qr * D + 8 * lch, ob + inst * 1024);
    }
    // the chunk's 64 LSE and 64 delta values ride in the same LDS-DMA batch (rows % 64 == 0)
    if (wave == 0 && lane < 32) {
      const float* srcv = (lane < 16 ? a.lse : a.delta) + z * a.rows + c * 64 + 4 * (lane & 15);
      fa_glds16(srcv, smem + 4 * TILE_BYTES + buf * 512);
    }
  };

  f32x4_t dv[DS], dk[DS];
#pragma unroll
  for (int i = 0; i < DS; ++i) {
    dv[i] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
    dk[i] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
  }
  const int q4 = c16 >> 2, p4 = c16 & 3;
  if (c_lo < c_hi) stage(c_lo, 0);
  for (int c = c_lo; c < c_hi; ++c) {
    const int buf = (c - c_lo) & 1;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (c + 1 < c_hi) stage(c + 1, buf ^ 1);
    const char* qb = smem + buf * 2 * TILE_BYTES;
    const char* ob = qb + TILE_BYTES;
#pragma unroll
    for (int kst = 0; kst < 2; ++kst) {          // two 32-query k-steps of the dV/dK products
      bf16x8_t pf, dsf;
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {
        const int qt = 2 * kst + hh;
        f32x4_t s = (f32x4_t){0.f, 0.f, 0.f, 0.f}, dp = (f32x4_t){0.f, 0.f, 0.f, 0.f};
        const int row = qt * 16 + c16;
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
          const int ch = (ks * 4 + g) ^ swz_k<D>(row);
          const bf16x8_t qa = *reinterpret_cast<const bf16x8_t*>(qb + row * (D * 2) + ch * 16);
          const bf16x8_t oa = *reinterpret_cast<const bf16x8_t*>(ob + row * (D * 2) + ch * 16);
          s = __builtin_amdgcn_mfma_f32_16x16x32_bf16(qa, kf[ks], s, 0, 0, 0);
          dp = __builtin_amdgcn_mfma_f32_16x16x32_bf16(oa, vf[ks], dp, 0, 0, 0);
        }
        const int qbase = c * 64 + qt * 16 + 4 * g;
        const float* ld = reinterpret_cast<const float*>(smem + 4 * TILE_BYTES + buf * 512);
        const float4 l4 = *reinterpret_cast<const float4*>(ld + qt * 16 + 4 * g);
        const float4 d4 = *reinterpret_cast<const float4*>(ld + 64 + qt * 16 + 4 * g);
        const float lv[4] = {l4.x, l4.y, l4.z, l4.w}, dl[4] = {d4.x, d4.y, d4.z, d4.w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int q = qbase + j;
          const int pos = q / a.qdiv;
          bool ok = key_ok && q < a.rows;
          if (a.causal) ok = ok && key <= pos;
          if (a.window > 0) ok = ok && key > pos - a.window;
          const float p = ok ? __builtin_amdgcn_exp2f(s[j] * sl2 - lv[j] * L2E) : 0.f;
          const bf16_t pb = f2bf(p);
          pf[4 * hh + j] = (short)pb;
          dsf[4 * hh + j] = (short)f2bf(bf2f(pb) * (dp[j] - dl[j]));
        }
      }
#pragma unroll
      for (int ds = 0; ds < DS; ++ds) {
        bf16x8_t ot, qt_;
#pragma unroll
        for (int hh = 0; hh < 2; ++hh) {
          const int row = (2 * kst + hh) * 16 + 4 * g + q4;
          const int ch = (2 * ds + (p4 >> 1)) ^ swz_k<D>(row);
          const int off = row * (D * 2) + ch * 16 + 8 * (p4 & 1);
          const s16x4_t ro = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4_t*)(ob + off));
          const s16x4_t rq = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4_t*)(qb + off));
          ot[4 * hh + 0] = ro[0]; ot[4 * hh + 1] = ro[1]; ot[4 * hh + 2] = ro[2]; ot[4 * hh + 3] = ro[3];
          qt_[4 * hh + 0] = rq[0]; qt_[4 * hh + 1] = rq[1]; qt_[4 * hh + 2] = rq[2]; qt_[4 * hh + 3] = rq[3];
        }
        dv[ds] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ot, pf, dv[ds], 0, 0, 0);
        dk[ds] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(qt_, dsf, dk[ds], 0, 0, 0);
      }
    }
  }
  if (key >= a.nkeys) return;
  bf16_t* dvp = a.dV + (z * a.nkeys + key) * (long)D + 4 * g;
  bf16_t* dkp = a.dK + (z * a.nkeys + key) * (long)D + 4 * g;
#pragma unroll
  for (int ds = 0; ds < DS; ++ds) {
    u16x4_t uv, uk;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      uv[j] = f2bf(dv[ds][j]);
      uk[j] = f2bf(dk[ds][j] * a.scale);
    }
    *reinterpret_cast<u16x4_t*>(dvp + 16 * ds) = uv;
    *reinterpret_cast<u16x4_t*>(dkp + 16 * ds) = uk;
  }
}


// ---------------------------------------------------------------- dK/dV, head_dim 256
// 4 waves x 32 keys = one 128-key slab per workgroup.  K/V fragments of the wave's 32 keys stay in
// registers (B operands), dK^T/dV^T (256 fp32 per lane) accumulate in the AGPR half of the 512-entry
// file (one wave per SIMD); 32-row Q/dO chunks (+ their LSE/delta) arrive by LDS-DMA, double-buffered.
// Per chunk and wave: 128 MFMAs against 64 KB of LDS reads (half the bytes/MFMA of 16 keys/wave).
// Causal slabs differ up to 11x in query rows, so a slab with more than `dkv_target` chunks is cut
// into query pieces (~equal chunks); pieces of a split slab write fp32 partials that
// attn_dkv_reduce_kernel sums in piece order (deterministic).  Blocks are ordered slab-major,
// heaviest slabs first.
// (DKV_KEYS, DKV_CH, dkv_slab_chunks, dkv_pieces, dkv_part_base: ptk_internal.h — qknorm_rope_bwd
// sums the partials itself when the reduce is deferred)

template <int KPW>   // keys per wave: 32 (4 waves, one per SIMD) or 16 (8 waves, two per SIMD)
__global__ void __launch_bounds__(DKV_KEYS / KPW * 64, 1) attn_bwd_dkv256_kernel(FlashBwdArgs a) {
  constexpr int D = 256, KS = D / 32, DS = D / 16;
  constexpr int KG = KPW / 16, NW = DKV_KEYS / KPW;   // 16-key groups per wave, waves
  constexpr int IPW = 16 / NW;                        // staging wave-instructions per tensor per wave
  constexpr int OPS = 2 * IPW + 1;                    // LDS-DMA ops per wave per chunk
  constexpr int TILE = DKV_CH * D * 2;   // 16 KiB: 32 rows of Q or dO
  constexpr int NBUF = 4;                 // ring depth: chunk c+3 is staged while chunk c computes
  __shared__ __attribute__((aligned(16))) char smem[NBUF * 2 * TILE + NBUF * 256];   // (Q, dO) x4, (lse|delta) x4

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, c16 = lane & 15;
  // ---- block -> (slab, piece, z)
  const int nz = a.nz;
  const int item = blockIdx.x / nz;
  const long z = blockIdx.x - (long)item * nz;
  const int s = a.dkv_item_slab[item], piece = a.dkv_item_piece[item];
  const int P = dkv_pieces(a, s);
  int base = 0;   // partial slots are numbered slab-major over the split slabs
  for (int s2 = 0; s2 < s; ++s2) {
    const int P2 = dkv_pieces(a, s2);
    if (P2 > 1) base += P2;
  }
  int c0, c1;
  {
    int lo, hi;
    dkv_slab_chunks(a, s, lo, hi);
    const int n = hi - lo;
    c0 = lo + (int)((long)piece * n / P);
    c1 = lo + (int)((long)(piece + 1) * n / P);
  }
  const long b = z / a.zdiv;
  const int kw = s * DKV_KEYS + wave * KPW;   // the wave's first key

  bf16x8_t kf[KG][KS], vf[KG][KS];
  int key[KG];
  bool kok[KG];
#pragma unroll
  for (int kg = 0; kg < KG; ++kg) {
    key[kg] = kw + 16 * kg + c16;
    const int kc = min(key[kg], a.nkeys - 1);
    const long ko = (z * a.nkeys + kc) * (long)D + 8 * g;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      kf[kg][ks] = *reinterpret_cast<const bf16x8_t*>(a.K + ko + 32 * ks);
      vf[kg][ks] = *reinterpret_cast<const bf16x8_t*>(a.V + ko + 32 * ks);
    }
    kok[kg] = key[kg] < a.nkeys && (!a.key_valid || a.key_valid[b * a.nkeys + kc] != 0);
  }
#pragma unroll
  for (int kg = 0; kg < KG; ++kg)
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      fa_pin(kf[kg][ks]);
      fa_pin(vf[kg][ks]);
    }
  const bf16_t* Qz = a.Q + z * (long)a.rows * D;
  const bf16_t* dOz = a.dO + z * (long)a.rows * D;
  const float L2E = 1.4426950408889634f;
  const float sl2 = a.scale * L2E;
  const int qshift = (a.qdiv & (a.qdiv - 1)) == 0 ? __builtin_ctz(a.qdiv) : -1;
  const int causal = a.causal != 0, nowin = a.window <= 0;
  bool kall = true;
#pragma unroll
  for (int kg = 0; kg < KG; ++kg) kall = kall && kok[kg];
  const bool wkall = __all(kall);   // every key of the wave valid

  // staging: 32 rows x 32 16-B chunks per tensor = 16 wave-instructions (IPW per wave), plus the
  // chunk's LSE|delta (256 B) spread over all waves: OPS LDS-DMA ops per wave per chunk, so one
  // counted vmcnt serves every wave
  const float* lse_base = a.lse;
  const float* delta_base = a.delta;
  auto stage = [&](int c, int buf) {
    char* qb = smem + buf * 2 * TILE;
    char* ob = qb + TILE;
#pragma unroll
    for (int j = 0; j < IPW; ++j) {
      const int inst = wave * IPW + j;
      const int row = inst * 2 + (lane >> 5);
      const int lch = (lane & 31) ^ swz_rt(row);
      const long src = (long)(c * DKV_CH + row) * D + 8 * lch;
      fa_glds16(Qz + src, qb + inst * 1024);
      fa_glds16(dOz + src, ob + inst * 1024);
    }
    if (lane < 16 / NW) {
      const int item = wave * (16 / NW) + lane;   // 0-7 LSE, 8-15 delta (4 floats each)
      // select between the two (uniform) base pointers arithmetically: a per-lane `? :` on the kernel
      // argument fields compiles to a load of the pointer from the kernarg segment, whose vmcnt(0) wait
      // drained the whole DMA ring every chunk
      const long off = z * a.rows + c * DKV_CH + 4 * (item & 7);
      const float* srcv = (item < 8 ? lse_base : delta_base) + off;
      fa_glds16(srcv, smem + NBUF * 2 * TILE + buf * 256 + wave * (256 / NW));
    }
  };

  f32x4_t dv[DS][KG], dk[DS][KG];
#pragma unroll
  for (int i = 0; i < DS; ++i)
#pragma unroll
    for (int kg = 0; kg < KG; ++kg) {
      dv[i][kg] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
      dk[i][kg] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
    }
  const int q4 = c16 >> 2, p4 = c16 & 3;
#pragma unroll
  for (int i = 0; i < NBUF - 1; ++i)
    if (c0 + i < c1) stage(c0 + i, i);
  for (int c = c0; c < c1; ++c) {
    const int buf = (c - c0) & (NBUF - 1);
    // chunk c landed; chunks c+1, c+2 may stay in flight (9 ops each)
    const int ahead = min(NBUF - 2, c1 - 1 - c);
    if (ahead >= 2) {
      if constexpr (OPS == 9) asm volatile("s_waitcnt vmcnt(18)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
    } else if (ahead == 1) {
      if constexpr (OPS == 9) asm volatile("s_waitcnt vmcnt(9)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    // raw barrier: __syncthreads() here compiles to vmcnt(0) + barrier and would drain the ring.
    // Every wave's share of chunk c landed (counted wait above); its reads of chunk c-1's buffer
    // were consumed by MFMAs before this point.
    __builtin_amdgcn_s_barrier();
    if (c + NBUF - 1 < c1) stage(c + NBUF - 1, (buf + NBUF - 1) & (NBUF - 1));
    const char* qb = smem + buf * 2 * TILE;
    const char* ob = qb + TILE;
    const float* ld = reinterpret_cast<const float*>(smem + NBUF * 2 * TILE + buf * 256);

    // ---- S = Q K^T, dP = dO V^T for 32 rows x 32 keys (key on the lane)
    f32x4_t sc[2][KG], dp[2][KG];
#pragma unroll
    for (int qt = 0; qt < 2; ++qt)
#pragma unroll
      for (int kg = 0; kg < KG; ++kg) {
        sc[qt][kg] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
        dp[qt][kg] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
      }
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) {
      const int row = qt * 16 + c16;
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        const int ch = (ks * 4 + g) ^ swz_rt(row);
        const bf16x8_t qa = *reinterpret_cast<const bf16x8_t*>(qb + row * (D * 2) + ch * 16);
        const bf16x8_t oa = *reinterpret_cast<const bf16x8_t*>(ob + row * (D * 2) + ch * 16);
#pragma unroll
        for (int kg = 0; kg < KG; ++kg) {
          sc[qt][kg] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(qa, kf[kg][ks], sc[qt][kg], 0, 0, 0);
          dp[qt][kg] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(oa, vf[kg][ks], dp[qt][kg], 0, 0, 0);
        }
      }
    }
    // ---- P = exp(S*scale - LSE) (bf16), dS = P (dP - delta) (bf16); k order of the next products:
    //      slot 4qt + j of lane group g <-> query row 16qt + 4g + j
    bf16x8_t pf[KG], dsf[KG];
    // chunk rows all see all of the wave's keys (valid, below the diagonal, inside the window): no mask
    const int cpos_lo = (c * DKV_CH) / a.qdiv, cpos_hi = (c * DKV_CH + DKV_CH - 1) / a.qdiv;
    const bool interior = wkall && (!causal || kw + KPW - 1 <= cpos_lo) && (nowin || kw > cpos_hi - a.window);
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) {
      const float4 l4 = *reinterpret_cast<const float4*>(ld + qt * 16 + 4 * g);
      const float4 d4 = *reinterpret_cast<const float4*>(ld + 32 + qt * 16 + 4 * g);
      const float lv[4] = {l4.x * L2E, l4.y * L2E, l4.z * L2E, l4.w * L2E}, dl[4] = {d4.x, d4.y, d4.z, d4.w};
      if (interior) {
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int kg = 0; kg < KG; ++kg) {
            const bf16_t pb = f2bf(__builtin_amdgcn_exp2f(fmaf(sc[qt][kg][j], sl2, -lv[j])));
            pf[kg][4 * qt + j] = (short)pb;
            dsf[kg][4 * qt + j] = (short)f2bf(bf2f(pb) * (dp[qt][kg][j] - dl[j]));
          }
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int qrow = c * DKV_CH + qt * 16 + 4 * g + j;
          const int pos = qshift >= 0 ? (qrow >> qshift) : qrow / a.qdiv;
#pragma unroll
          for (int kg = 0; kg < KG; ++kg) {
            // branch-free mask (short-circuit && turns into exec-mask control flow per element)
            const int ok = (int)kok[kg] & ((int)(key[kg] <= pos) | !causal) & ((int)(key[kg] > pos - a.window) | nowin);
            const float p = __builtin_amdgcn_exp2f(ok ? fmaf(sc[qt][kg][j], sl2, -lv[j]) : -INFINITY);
            const bf16_t pb = f2bf(p);
            pf[kg][4 * qt + j] = (short)pb;
            dsf[kg][4 * qt + j] = (short)f2bf(bf2f(pb) * (dp[qt][kg][j] - dl[j]));
          }
        }
      }
    }
    // ---- dV^T += dO^T P, dK^T += Q^T dS (A operands by transposed LDS reads)
#pragma unroll
    for (int ds = 0; ds < DS; ++ds) {
      bf16x8_t ot, qt_;
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {
        const int row = hh * 16 + 4 * g + q4;
        const int ch = (2 * ds + (p4 >> 1)) ^ swz_rt(row);
        const int off = row * (D * 2) + ch * 16 + 8 * (p4 & 1);
        const s16x4_t ro = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4_t*)(ob + off));
        const s16x4_t rq = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4_t*)(qb + off));
        ot[4 * hh + 0] = ro[0]; ot[4 * hh + 1] = ro[1]; ot[4 * hh + 2] = ro[2]; ot[4 * hh + 3] = ro[3];
        qt_[4 * hh + 0] = rq[0]; qt_[4 * hh + 1] = rq[1]; qt_[4 * hh + 2] = rq[2]; qt_[4 * hh + 3] = rq[3];
      }
#pragma unroll
      for (int kg = 0; kg < KG; ++kg) {
        dv[ds][kg] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ot, pf[kg], dv[ds][kg], 0, 0, 0);
        dk[ds][kg] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(qt_, dsf[kg], dk[ds][kg], 0, 0, 0);
      }
    }
  }
  // ---- outputs: lane holds dV^T[16ds + 4g + j][key]
  if (P == 1) {
#pragma unroll
    for (int kg = 0; kg < KG; ++kg) {
      if (key[kg] >= a.nkeys) continue;
      bf16_t* dvp = a.dV + (z * a.nkeys + key[kg]) * (long)D + 4 * g;
      bf16_t* dkp = a.dK + (z * a.nkeys + key[kg]) * (long)D + 4 * g;
#pragma unroll
      for (int ds = 0; ds < DS; ++ds) {
        u16x4_t uv, uk;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          uv[j] = f2bf(dv[ds][kg][j]);
          uk[j] = f2bf(dk[ds][kg][j] * a.scale);
        }
        *reinterpret_cast<u16x4_t*>(dvp + 16 * ds) = uv;
        *reinterpret_cast<u16x4_t*>(dkp + 16 * ds) = uk;
      }
    }
  } else {
    // partial slot [base + piece][z]: [dK | dV][128 keys][D] fp32
    float* part = a.dkv_part + ((long)(base + piece) * nz + z) * (2L * DKV_KEYS * D);
#pragma unroll
    for (int kg = 0; kg < KG; ++kg) {
      const int kl = wave * KPW + 16 * kg + c16;
      float* pk = part + (long)kl * D + 4 * g;
      float* pv = pk + (long)DKV_KEYS * D;
#pragma unroll
      for (int ds = 0; ds < DS; ++ds) {
        *reinterpret_cast<float4*>(pk + 16 * ds) = make_float4(dk[ds][kg][0], dk[ds][kg][1], dk[ds][kg][2], dk[ds][kg][3]);
        *reinterpret_cast<float4*>(pv + 16 * ds) = make_float4(dv[ds][kg][0], dv[ds][kg][1], dv[ds][kg][2], dv[ds][kg][3]);
      }
    }
  }
}

// dK/dV (head_dim 256), instruction-lean form of attn_bwd_dkv256_kernel<32> (same slab / piece plan, same
// arithmetic in the same order, so the same results): Q, dO and the chunk's LSE | delta arrive by
// buffer_load ... lds with per-lane offsets fixed for the kernel and the chunk's byte offset in an SGPR;
// separate Q and dO rings with the chunk loop unrolled by the ring depth (every LDS read = lane offset +
// immediate); the causal / window position test by shift (query heads per kv head a power of two); a wave
// whose 32 keys are all invisible to a chunk's rows (the causal diagonal and the window edge of the slab)
// skips that chunk's MFMAs.
#ifndef DKV_VACC
#define DKV_VACC 1   // dK/dV kernel: S / dP MFMAs from inline asm with VGPR accumulators (0 = builtins)
#endif
#ifndef DKV_PD
#define DKV_PD 2   // dK/dV kernel: LDS fragment groups read ahead of their MFMAs (0 = hipcc's own placement)
#endif
__global__ void __launch_bounds__(256, 1) attn_bwd_dkv256b_kernel(FlashBwdArgs a) {
  constexpr int D = 256, KS = D / 32, DS = D / 16, KPW = 32, KG = 2, NB = 4;
  constexpr int TILE = DKV_CH * D * 2;   // 16 KiB: 32 rows of Q or dO
  __shared__ __attribute__((aligned(16))) char smem[2 * NB * TILE + NB * 256];   // Q ring, dO ring, (lse|delta) ring
  char* const qring = smem;
  char* const oring = smem + NB * TILE;
  const float* const ldring = reinterpret_cast<const float*>(smem + 2 * NB * TILE);
  FA_STAMPS_DECL;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, c16 = lane & 15;
  const int nz = a.nz;
  const int item = blockIdx.x / nz;
  const long z = blockIdx.x - (long)item * nz;
  const int s = a.dkv_item_slab[item], piece = a.dkv_item_piece[item];
  const int P = dkv_pieces(a, s);
  int base = 0;
  for (int s2 = 0; s2 < s; ++s2) {
    const int P2 = dkv_pieces(a, s2);
    if (P2 > 1) base += P2;
  }
  int c0, c1;
  {
    int lo, hi;
    dkv_slab_chunks(a, s, lo, hi);
    const int n = hi - lo;
    c0 = lo + (int)((long)piece * n / P);
    c1 = lo + (int)((long)(piece + 1) * n / P);
  }
  const long b = z / a.zdiv;
  const int kw = s * DKV_KEYS + wave * KPW;   // the wave's first key

  bf16x8_t kf[KG][KS], vf[KG][KS];
  int key[KG];
  bool kok[KG];
#pragma unroll
  for (int kg = 0; kg < KG; ++kg) {
    key[kg] = kw + 16 * kg + c16;
    const int kc = min(key[kg], a.nkeys - 1);
    const long ko = (z * a.nkeys + kc) * (long)D + 8 * g;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      kf[kg][ks] = *reinterpret_cast<const bf16x8_t*>(a.K + ko + 32 * ks);
      vf[kg][ks] = *reinterpret_cast<const bf16x8_t*>(a.V + ko + 32 * ks);
    }
    kok[kg] = key[kg] < a.nkeys && (!a.key_valid || a.key_valid[b * a.nkeys + kc] != 0);
  }
#pragma unroll
  for (int kg = 0; kg < KG; ++kg)
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      fa_pin(kf[kg][ks]);
      fa_pin(vf[kg][ks]);
    }
  FA_STAMP(1);
  FA_STAMP(2);
  const float L2E = 1.4426950408889634f;
  const float sl2 = a.scale * L2E;
  const int qshift = __builtin_ctz(a.qdiv);   // host guarantees a power of two
  const int causal = a.causal != 0, nowin = a.window <= 0;
  bool kall = true;
#pragma unroll
  for (int kg = 0; kg < KG; ++kg) kall = kall && kok[kg];
  const bool wkall = __all(kall);   // every key of the wave valid

  // ---- DMA: wave w stages rows 8w..8w+7 of a chunk's Q and dO (4 pieces of 2 rows each), and one piece of
  // the chunk's LSE (waves 0, 1) or delta (waves 2, 3): 9 ops per wave per chunk
  const fa_u32x4_t rsq = fa_rsrc(a.Q + z * (long)a.rows * D, (uint32_t)((long)a.rows * D * 2));
  const fa_u32x4_t rso = fa_rsrc(a.dO + z * (long)a.rows * D, (uint32_t)((long)a.rows * D * 2));
  const fa_u32x4_t rsl = fa_rsrc(wave < 2 ? (const void*)(a.lse + z * a.rows) : (const void*)(a.delta + z * a.rows),
                                 (uint32_t)((long)a.rows * 4));
  uint32_t dof[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int row = (wave * 4 + j) * 2 + (lane >> 5);
    dof[j] = (uint32_t)row * (D * 2) + 16u * ((lane & 31) ^ swz_rt(row));
  }
  const uint32_t dol = (uint32_t)lane * 16u + (uint32_t)(wave & 1) * 64u;
  const uint32_t lds_q = __builtin_amdgcn_readfirstlane(fa_lds_addr(qring) + wave * 4096);
  const uint32_t lds_o = __builtin_amdgcn_readfirstlane(fa_lds_addr(oring) + wave * 4096);
  // (lse | delta) slot: [32 LSE | 32 delta] floats; wave w's 4 lanes land 64 B at slot + 64 w
  const uint32_t lds_l = __builtin_amdgcn_readfirstlane(fa_lds_addr(smem + 2 * NB * TILE) + wave * 64);
  auto stage = [&](int bb, int c) __attribute__((always_inline)) {
    const uint32_t so = __builtin_amdgcn_readfirstlane((uint32_t)c * (uint32_t)TILE);
#pragma unroll
    for (int j = 0; j < 4; ++j) FA_DMA(dof[j], so, rsq, lds_q + bb * TILE + j * 1024);
#pragma unroll
    for (int j = 0; j < 4; ++j) FA_DMA(dof[j], so, rso, lds_o + bb * TILE + j * 1024);
    const uint32_t sl = __builtin_amdgcn_readfirstlane((uint32_t)c * (uint32_t)(DKV_CH * 4));
    if (lane < 4) FA_DMA(dol, sl, rsl, lds_l + bb * 256);
  };

  // ---- LDS read offsets (lane part; slot, k-step and row-group parts are immediates)
  int roff[4], toff[8];
  {
    const int q4 = c16 >> 2, p4 = c16 & 3, trow = 4 * g + q4;
#pragma unroll
    for (int i = 0; i < 4; ++i) roff[i] = c16 * (D * 2) + ((i * 4 + g) ^ swz_rt(c16)) * 16;
#pragma unroll
    for (int i = 0; i < 8; ++i) toff[i] = trow * (D * 2) + ((2 * i + (p4 >> 1)) ^ swz_rt(trow)) * 16 + 8 * (p4 & 1);
  }
  const char* const obase = (const char*)(fa_lptr_t)(uintptr_t)__builtin_amdgcn_readfirstlane(0) + fa_lds_addr(oring);

  f32x4_t dv[DS][KG], dk[DS][KG];
#pragma unroll
  for (int i = 0; i < DS; ++i)
#pragma unroll
    for (int kg = 0; kg < KG; ++kg) {
      dv[i][kg] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
      dk[i][kg] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
    }

  auto step = [&](auto BUF, int c) __attribute__((always_inline)) {
    constexpr int bb = decltype(BUF)::value;
    // chunk c landed; chunks c+1, c+2 may stay in flight (9 ops each)
    const int ahead = c1 - 1 - c;
    if (ahead >= 2) asm volatile("s_waitcnt vmcnt(18)" ::: "memory");
    else if (ahead == 1) asm volatile("s_waitcnt vmcnt(9)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (c + NB - 1 < c1) stage((bb + NB - 1) % NB, c + NB - 1);
    // rows of this chunk: positions cpos_lo..cpos_hi; the wave's keys kw..kw+31
    const int cpos_lo = (c * DKV_CH) >> qshift, cpos_hi = (c * DKV_CH + DKV_CH - 1) >> qshift;
    if ((causal && kw > cpos_hi) || (!nowin && kw + KPW - 1 <= cpos_lo - a.window)) return;   // all invisible
    const char* qb = qring + bb * TILE;
    const char* ob = obase + bb * TILE;
    const float* ld = ldring + bb * 64;

    // ---- S = Q K^T, dP = dO V^T for 32 rows x 32 keys (key on the lane)
    f32x4_t sc[2][KG], dp[2][KG];
#pragma unroll
    for (int qt = 0; qt < 2; ++qt)
#pragma unroll
      for (int kg = 0; kg < KG; ++kg) {
        sc[qt][kg] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
        dp[qt][kg] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
      }
    // group i = (qt, ks): Q and dO fragments read DKV_PD groups ahead of their MFMAs (as in the dV/dK loop)
    bf16x8_t qar[DKV_PD + 1], oar[DKV_PD + 1];
    auto ldr = [&](int i) __attribute__((always_inline)) {
      const int qt = i / KS, ks = i % KS;
      const int off = roff[ks & 3] + (ks >> 2) * 256 + qt * 16 * (D * 2);
      qar[i % (DKV_PD + 1)] = *reinterpret_cast<const bf16x8_t*>(qb + off);
      oar[i % (DKV_PD + 1)] = *reinterpret_cast<const bf16x8_t*>(ob + off);
    };
#pragma unroll
    for (int i = 0; i < DKV_PD; ++i) ldr(i);
#pragma unroll
    for (int i = 0; i < 2 * KS; ++i) {
      const int qt = i / KS, ks = i % KS;
      if (DKV_PD > 0) {
        if (i + DKV_PD < 2 * KS) ldr(i + DKV_PD);
        __builtin_amdgcn_sched_barrier(0);
      } else {
        ldr(i);
      }
#pragma unroll
      for (int kg = 0; kg < KG; ++kg) {
        if (DKV_VACC) {
          // S and dP accumulate in VGPRs (asm): with the builtin, hipcc put them in AGPRs and moved 32 of
          // the dK/dV accumulators out to VGPRs and back around every chunk
          if (ks == 0) {
            asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, 0"
                         : "=&v"(sc[qt][kg]) : "v"(qar[i % (DKV_PD + 1)]), "v"(kf[kg][ks]));
            asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, 0"
                         : "=&v"(dp[qt][kg]) : "v"(oar[i % (DKV_PD + 1)]), "v"(vf[kg][ks]));
          } else {
            asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0"
                         : "+v"(sc[qt][kg]) : "v"(qar[i % (DKV_PD + 1)]), "v"(kf[kg][ks]));
            asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0"
                         : "+v"(dp[qt][kg]) : "v"(oar[i % (DKV_PD + 1)]), "v"(vf[kg][ks]));
          }
        } else {
          sc[qt][kg] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(qar[i % (DKV_PD + 1)], kf[kg][ks], sc[qt][kg], 0, 0, 0);
          dp[qt][kg] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(oar[i % (DKV_PD + 1)], vf[kg][ks], dp[qt][kg], 0, 0, 0);
        }
      }
      if (DKV_PD > 0) __builtin_amdgcn_sched_barrier(0);
    }
    if (DKV_VACC) {
      // the last asm MFMAs' results -> the softmax VALU reads (10 wait states for 16x16x32; 12 here)
      asm volatile("s_nop 7\n\ts_nop 3" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
    }
    // ---- P = exp(S*scale - LSE) (bf16), dS = P (dP - delta) (bf16); slot 4qt + j of lane group g <-> row 16qt + 4g + j
    bf16x8_t pf[KG], dsf[KG];
    const bool interior = wkall && (!causal || kw + KPW - 1 <= cpos_lo) && (nowin || kw > cpos_hi - a.window);
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) {
      const float4 l4 = *reinterpret_cast<const float4*>(ld + qt * 16 + 4 * g);
      const float4 d4 = *reinterpret_cast<const float4*>(ld + 32 + qt * 16 + 4 * g);
      const float lv[4] = {l4.x * L2E, l4.y * L2E, l4.z * L2E, l4.w * L2E}, dl[4] = {d4.x, d4.y, d4.z, d4.w};
      if (interior) {
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int kg = 0; kg < KG; ++kg) {
            const bf16_t pb = f2bf(__builtin_amdgcn_exp2f(fmaf(sc[qt][kg][j], sl2, -lv[j])));
            pf[kg][4 * qt + j] = (short)pb;
            dsf[kg][4 * qt + j] = (short)f2bf(bf2f(pb) * (dp[qt][kg][j] - dl[j]));
          }
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int pos = (c * DKV_CH + qt * 16 + 4 * g + j) >> qshift;
#pragma unroll
          for (int kg = 0; kg < KG; ++kg) {
            const int ok = (int)kok[kg] & ((int)(key[kg] <= pos) | !causal) & ((int)(key[kg] > pos - a.window) | nowin);
            const float p = __builtin_amdgcn_exp2f(ok ? fmaf(sc[qt][kg][j], sl2, -lv[j]) : -INFINITY);
            const bf16_t pb = f2bf(p);
            pf[kg][4 * qt + j] = (short)pb;
            dsf[kg][4 * qt + j] = (short)f2bf(bf2f(pb) * (dp[qt][kg][j] - dl[j]));
          }
        }
      }
    }
    // ---- dV^T += dO^T P, dK^T += Q^T dS (A operands by transposed LDS reads), the reads of group ds + DKV_PD
    // issued before the MFMAs of group ds (a ring of DKV_PD + 1 fragment pairs; sched_barrier keeps hipcc from
    // sinking the reads to just before their use, which left each group's LDS latency exposed)
    bf16x8_t otr[DKV_PD + 1], qtr[DKV_PD + 1];
    auto ldt = [&](int ds) __attribute__((always_inline)) {
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {
        const int off = toff[ds & 7] + (ds >> 3) * 256 + hh * 16 * (D * 2);
        const s16x4_t ro = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4_t*)(ob + off));
        const s16x4_t rq = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4_t*)(qb + off));
        bf16x8_t& ot = otr[ds % (DKV_PD + 1)];
        bf16x8_t& qt_ = qtr[ds % (DKV_PD + 1)];
        ot[4 * hh + 0] = ro[0]; ot[4 * hh + 1] = ro[1]; ot[4 * hh + 2] = ro[2]; ot[4 * hh + 3] = ro[3];
        qt_[4 * hh + 0] = rq[0]; qt_[4 * hh + 1] = rq[1]; qt_[4 * hh + 2] = rq[2]; qt_[4 * hh + 3] = rq[3];
      }
    };
#pragma unroll
    for (int ds = 0; ds < DKV_PD; ++ds) ldt(ds);
#pragma unroll
    for (int ds = 0; ds < DS; ++ds) {
      if (DKV_PD > 0) {
        if (ds + DKV_PD < DS) ldt(ds + DKV_PD);
        __builtin_amdgcn_sched_barrier(0);
      } else {
        ldt(ds);
      }
#pragma unroll
      for (int kg = 0; kg < KG; ++kg) {
        dv[ds][kg] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(otr[ds % (DKV_PD + 1)], pf[kg], dv[ds][kg], 0, 0, 0);
        dk[ds][kg] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(qtr[ds % (DKV_PD + 1)], dsf[kg], dk[ds][kg], 0, 0, 0);
      }
      if (DKV_PD > 0) __builtin_amdgcn_sched_barrier(0);
    }
  };

  // chunk c lives in ring slot (c - c0) % NB (compile-time in each unrolled copy)
  if (c0 < c1) stage(0, c0);
  if (c0 + 1 < c1) stage(1, c0 + 1);
  if (c0 + 2 < c1) stage(2, c0 + 2);
  for (int c = c0; c < c1;) {
    step(fa_ic<0>{}, c);
    if (++c >= c1) break;
    step(fa_ic<1>{}, c);
    if (++c >= c1) break;
    step(fa_ic<2>{}, c);
    if (++c >= c1) break;
    step(fa_ic<3>{}, c);
    ++c;
  }

  FA_STAMP(3);
  // ---- outputs: lane holds dV^T[16ds + 4g + j][key]
  if (P == 1) {
#pragma unroll
    for (int kg = 0; kg < KG; ++kg) {
      if (key[kg] >= a.nkeys) continue;
      bf16_t* dvp = a.dV + (z * a.nkeys + key[kg]) * (long)D + 4 * g;
      bf16_t* dkp = a.dK + (z * a.nkeys + key[kg]) * (long)D + 4 * g;
#pragma unroll
      for (int ds = 0; ds < DS; ++ds) {
        u16x4_t uv, uk;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          uv[j] = f2bf(dv[ds][kg][j]);
          uk[j] = f2bf(dk[ds][kg][j] * a.scale);
        }
        *reinterpret_cast<u16x4_t*>(dvp + 16 * ds) = uv;
        *reinterpret_cast<u16x4_t*>(dkp + 16 * ds) = uk;
      }
    }
  } else {
    float* part = a.dkv_part + ((long)(base + piece) * nz + z) * (2L * DKV_KEYS * D);
#pragma unroll
    for (int kg = 0; kg < KG; ++kg) {
      const int kl = wave * KPW + 16 * kg + c16;
      float* pk = part + (long)kl * D + 4 * g;
      float* pv = pk + (long)DKV_KEYS * D;
#pragma unroll
      for (int ds = 0; ds < DS; ++ds) {
        *reinterpret_cast<float4*>(pk + 16 * ds) = make_float4(dk[ds][kg][0], dk[ds][kg][1], dk[ds][kg][2], dk[ds][kg][3]);
        *reinterpret_cast<float4*>(pv + 16 * ds) = make_float4(dv[ds][kg][0], dv[ds][kg][1], dv[ds][kg][2], dv[ds][kg][3]);
      }
    }
  }
  FA_STAMPS_WRITE(2, c1 - c0);
}

// sums the partials of every split slab in piece order -> bf16 dK (x scale), dV
__global__ void __launch_bounds__(256) attn_dkv_reduce_kernel(FlashBwdArgs a) {
  constexpr int D = 256;
  const int s = blockIdx.y;
  const int P = dkv_pieces(a, s);
  if (P == 1) return;
  int base = 0;
  for (int t = 0; t < s; ++t) {
    const int pt = dkv_pieces(a, t);
    if (pt > 1) base += pt;
  }
  const long i = (long)blockIdx.x * 256 + threadIdx.x;   // float4 index in [nz][2][128][D/4]
  const long per_z = 2L * DKV_KEYS * D / 4;
  if (i >= (long)a.nz * per_z) return;
  const long z = i / per_z;
  const long r = i - z * per_z;
  const int which = (int)(r / (DKV_KEYS * D / 4));        // 0 = dK, 1 = dV
  const int kl = (int)((r / (D / 4)) % DKV_KEYS);
  const int d4 = (int)(r % (D / 4));
  const int key = s * DKV_KEYS + kl;
  if (key >= a.nkeys) return;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int pc = 0; pc < P; ++pc) {
    const float4 v = reinterpret_cast<const float4*>(a.dkv_part + ((long)(base + pc) * a.nz + z) * (2L * DKV_KEYS * D))[r];
    acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
  }
  const float m = which == 0 ? a.scale : 1.f;
  u16x4_t u;
  u[0] = f2bf(acc.x * m); u[1] = f2bf(acc.y * m); u[2] = f2bf(acc.z * m); u[3] = f2bf(acc.w * m);
  bf16_t* out = (which == 0 ? a.dK : a.dV) + (z * a.nkeys + key) * (long)D + 4 * d4;
  *reinterpret_cast<u16x4_t*>(out) = u;
}

static int num_cus() {
  static int n = 0;
  if (n == 0) {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) == hipSuccess &&
        hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && v > 0)
      n = v;
    else
      n = 256;
  }
  return n;
}

// Split plan.  Each block (one slab piece of one z) costs its query chunks plus a fixed overhead
// (K/V fragment loads, ring fill, dK/dV stores; ~1.5 chunks) and, for a piece of a split slab, the
// fp32 partial store (~1 chunk).  Blocks are dispatched heaviest first (LPT) onto num_cus() CUs
// (one block per CU: 129 KiB LDS); the target piece size is the candidate whose simulated makespan
// is smallest (causal slabs differ up to 11x, so one-piece-per-CU targets leave a third of the
// machine idle in the tail).
static double dkv_makespan(FlashBwdArgs& a, int nz, int nslab, int target, int ncu) {
  a.dkv_target = target;
  std::vector<double> cost;
  for (int s = 0; s < nslab; ++s) {
    int lo, hi;
    dkv_slab_chunks(a, s, lo, hi);
    const int n = hi - lo, P = dkv_pieces(a, s);
    for (int p = 0; p < P; ++p) {
      const int c = (int)((long)(p + 1) * n / P - (long)p * n / P);
      cost.push_back(c + 1.5 + (P > 1 ? 1.0 : 0.0));
    }
  }
  std::sort(cost.begin(), cost.end(), std::greater<double>());
  std::priority_queue<double, std::vector<double>, std::greater<double>> cu;
  for (int i = 0; i < ncu; ++i) cu.push(0.0);
  double span = 0.0;
  for (double c : cost)
    for (int z = 0; z < nz; ++z) {
      const double t = cu.top() + c;
      cu.pop();
      cu.push(t);
      span = std::max(span, t);
    }
  return span;
}

static void dkv_plan(FlashBwdArgs& a, int nz, int& nslab, long& npieces, long& nsplit) {
  a.nz = nz;
  nslab = (a.nkeys + DKV_KEYS - 1) / DKV_KEYS;
  long total = 0;
  for (int s = 0; s < nslab; ++s) {
    int lo, hi;
    a.dkv_target = 0;
    dkv_slab_chunks(a, s, lo, hi);
    total += hi - lo;
  }
  const int ncu = num_cus();
  // the work-item table holds 128 (slab, piece) entries: a target is admissible only if its pieces fit
  auto items_for = [&](int t) {
    long items = 0;
    a.dkv_target = t;
    for (int s = 0; s < nslab; ++s) items += dkv_pieces(a, s);
    return items;
  };
  int base = (int)std::max(4L, (total * nz + ncu - 1) / ncu);
  // few z (small batch, long sequence): the one-piece-per-CU target would cut slabs into more pieces than
  // the table holds; raise it until they fit (one piece per slab always does: nslab <= 128 is checked by
  // the caller)
  while (items_for(base) > 128 && base <= total) base += std::max(1, base / 8);
  int best = base;
  double best_span = dkv_makespan(a, nz, nslab, base, ncu);
  for (int k = 9; k >= 3; --k) {   // targets base * k / 12 (3/4 .. 1/4)
    const int t = std::max(4, base * k / 12);
    if (items_for(t) > 128) break;
    const double sp = dkv_makespan(a, nz, nslab, t, ncu);
    if (sp < best_span - 1e-9) { best_span = sp; best = t; }
  }
  a.dkv_target = best;
  // items (slab, piece) heaviest first; ties keep slab order
  std::vector<std::pair<int, int>> it;   // (-chunks, slab * 256 + piece)
  npieces = 0;
  nsplit = 0;
  for (int s = 0; s < nslab; ++s) {
    int lo, hi;
    dkv_slab_chunks(a, s, lo, hi);
    const int n = hi - lo, P = dkv_pieces(a, s);
    npieces += P;
    if (P > 1) nsplit += P;
    for (int p = 0; p < P; ++p)
      it.push_back({-(int)((long)(p + 1) * n / P - (long)p * n / P), s * 256 + p});
  }
  std::stable_sort(it.begin(), it.end(), [](const std::pair<int, int>& x, const std::pair<int, int>& y) {
    return x.first < y.first;
  });
  a.dkv_items = (int)it.size();
  for (size_t i = 0; i < it.size() && i < 128; ++i) {
    a.dkv_item_slab[i] = (unsigned char)(it[i].second >> 8);
    a.dkv_item_piece[i] = (unsigned char)(it[i].second & 255);
  }
}

size_t attn_bwd_workspace_bytes(const FlashBwdArgs& a0, int nz) {
  if (a0.D != 256 || a0.rows <= 0 || nz <= 0) return 0;
  FlashBwdArgs a = a0;
  int nslab;
  long np, ns;
  dkv_plan(a, nz, nslab, np, ns);
  return (size_t)ns * nz * 2 * DKV_KEYS * 256 * sizeof(float);
}

int launch_attn_bwd(const FlashBwdArgs& a, int nz, hipStream_t st, FlashBwdArgs* defer) {
  if (defer) {
    *defer = a;
    defer->dkv_deferred = 0;
  }
  if (a.rows <= 0 || nz <= 0) return 0;
  if (a.rows % 64 || a.nkeys % 64) return set_error("attn_bwd: rows (%d) and keys (%d) must be multiples of 64",
                                                   a.rows, a.nkeys);
  if (a.ldo & 7) return set_error("attn_bwd: O stride must be a multiple of 8");
  const dim3 gd((unsigned)(((long)nz * a.rows + 15) / 16)), gq((unsigned)((long)((a.rows + 127) / 128) * nz)),
      gk((unsigned)(a.nkeys / 64), (unsigned)nz);
  switch (a.D) {
    case 64:
      hipLaunchKernelGGL(attn_delta_kernel<64>, gd, dim3(256), 0, st, a, nz);
      hipLaunchKernelGGL(attn_bwd_dkv_kernel<64>, gk, dim3(256), 0, st, a);
      hipLaunchKernelGGL(attn_bwd_dq_kernel<64>, gq, dim3(512), 0, st, a);
      break;
    case 256: {
      FlashBwdArgs b = a;
      int nslab;
      long np, ns;
      dkv_plan(b, nz, nslab, np, ns);
      if (ns > 0 && (!b.dkv_part || b.dkv_part_bytes < (size_t)ns * nz * 2 * DKV_KEYS * 256 * sizeof(float))) {
        b.dkv_target = 0;   // no workspace: every slab in one piece, heaviest (lowest) slabs first
        np = nslab;
        ns = 0;
        b.dkv_items = nslab;
        for (int s = 0; s < nslab && s < 128; ++s) { b.dkv_item_slab[s] = (unsigned char)s; b.dkv_item_piece[s] = 0; }
      }
      if (b.dkv_items > 128 || nslab > 128) return set_error("attn_bwd: %d dK/dV work items over %d key slabs (max 128)", b.dkv_items, nslab);
      // the dQ kernel computes delta and runs first; past the 4096-key mask table the generic dQ kernel runs
      // after a separate delta pass and the dK/dV kernel
      const bool dq_new = (a.nkeys + 31) / 32 <= FA_MAXT;
      if (dq_new) {
        // persistent grid (attn_fwd256w_kernel's: one workgroup per CU over the row blocks heaviest first, the next
        // item's prologue beside this one's epilogue); PTK_ATTN_PERSIST=0 (A/B builds): one workgroup per item
        const bool persist = PTK_AB("PTK_ATTN_PERSIST", 1) != 0;
        const long nblk = (long)gq.x;
        const long g = persist ? std::min<long>(nblk, num_cus()) : nblk;
        hipLaunchKernelGGL(attn_bwd_dq256w_kernel, dim3((unsigned)g), dim3(256), 0, st, b, nz, (int)nblk);
      }
      else hipLaunchKernelGGL(attn_delta_kernel<256>, gd, dim3(256), 0, st, b, nz);
      // 32 keys per wave (one wave per SIMD) measured 209 us vs 252 us for 16 keys per wave (two per
      // SIMD, which spills the precomputed transposed-read addresses) at cfg2
      // the generic dK/dV kernel for GQA groups that are not a power of two and for very long query rows
      if ((b.qdiv & (b.qdiv - 1)) || (long)b.rows * 256 * 2 > 0x7fffffffL)
        hipLaunchKernelGGL(attn_bwd_dkv256_kernel<32>, dim3((unsigned)(np * nz)), dim3(256), 0, st, b);
      else
        hipLaunchKernelGGL(attn_bwd_dkv256b_kernel, dim3((unsigned)(np * nz)), dim3(256), 0, st, b);
      if (ns > 0 && defer) {
        *defer = b;
        defer->dkv_deferred = 1;
      } else if (ns > 0)
        hipLaunchKernelGGL(attn_dkv_reduce_kernel, dim3((unsigned)((nz * 2L * DKV_KEYS * 64 + 255) / 256), (unsigned)nslab),
                           dim3(256), 0, st, b);
      if (!dq_new) hipLaunchKernelGGL(attn_bwd_dq_kernel<256>, gq, dim3(512), 0, st, b);
      break;
    }
    default: return set_error("attn_bwd: head_dim %d unsupported (64, 256)", a.D);
  }
  return hipGetLastError() == hipSuccess ? 0 : set_error("attn_bwd launch failed");
}

int launch_attn_fwd(const FlashArgs& a, int nz, hipStream_t st) {
  if (a.rows <= 0 || nz <= 0) return 0;
  if (a.nkeys < 4) return set_error("attn_fwd: nkeys must be >= 4");
  if ((a.ldq | a.ldk | a.ldo) & 7) return set_error("attn_fwd: row strides must be multiples of 8");
  if (a.key_valid && (a.nkeys & 3)) return set_error("attn_fwd: key_valid rows must be a multiple of 4");
  const long nblk = (long)((a.rows + 127) / 128) * nz;
  if (nblk > 0x7fffffffL) return set_error("attn_fwd: too many blocks");
  dim3 grid((unsigned)nblk);
  switch (a.D) {
    case 64: {
      // the generic kernel past the 4096-key mask table
      if ((a.nkeys + 31) / 32 > FA_MAXT || (long)a.nkeys * a.ldk * 2 > 0x7fffffffL)
        hipLaunchKernelGGL((attn_fwd_kernel<64, 1>), grid, dim3(512), 0, st, a);
      else {
        FlashArgs b = a;
        b.variant = PTK_AB("PTK_FA64_XCD", 1) ? 0 : 1;   // 1: the z-major block order (A/B builds)
        hipLaunchKernelGGL(attn_fwd64_kernel, grid, dim3(512), 0, st, b);
      }
      break;
    }
    // QG = 2 (256-row blocks) measured slower on the Gemma3 step: 352 blocks of double work on 256 CUs
    // quantise worse than 704 (110 vs 78 us per layer), and it spills
    case 256: {
      // the generic kernel past the 4096-key mask table
      if ((a.nkeys + 31) / 32 > FA_MAXT || (long)a.nkeys * a.ldk * 2 > 0x7fffffffL)
        hipLaunchKernelGGL((attn_fwd_kernel<256, 1>), grid, dim3(512), 0, st, a);
      else {
        // persistent grid (one workgroup per CU walking the row blocks heaviest first, the next item's prologue
        // beside this one's epilogue); PTK_ATTN_PERSIST=0 (A/B builds): one workgroup per item (A/B, bit-identical)
        const bool persist = PTK_AB("PTK_ATTN_PERSIST", 1) != 0;
        const long g = persist ? std::min<long>(nblk, num_cus()) : nblk;
        hipLaunchKernelGGL(attn_fwd256w_kernel, dim3((unsigned)g), dim3(256), 0, st, a, nz, (int)nblk);
      }
      break;
    }
    default: return set_error("attn_fwd: head_dim %d unsupported (64, 256)", a.D);
  }
  return hipGetLastError() == hipSuccess ? 0 : set_error("attn_fwd launch failed");
}

}  // namespace ptk

#ifdef PTK_FA_STAMPS
extern "C" int ptk_debug_fa_stamps_read(void* host, size_t bytes) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(ptk::g_fa_stamps), bytes, 0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
#endif
