// Persistent 256x256-tile bf16 GEMM for gfx950: 4 waves, one per SIMD, 128x128 fp32 accumulator
// tile per wave (256 accumulator registers: the kernel runs at one wave per SIMD with the full
// 512-register file).
//
//   C[M,N] = epi( A[M,K] . B[N,K]^T )   (gemm_nt_kernel's contract at batch 1 and alpha = 1; other alphas go there)
//
// Why this shape: the Stage-1 step's projections are K = 1024..1536 deep, so a
// 256x256 tile runs only 16..24 K-tiles and the per-tile prologue (first DMA round trip) and
// epilogue (128 KiB of stores per CU, staged through LDS in gemm_big_kernel) cost as much as a
// third of the main loop.  Here
//   * one wave per SIMD software-pipelines its own LDS reads: the 16 ds_read_b128 fragments of
//     k-step s+1 are issued while the 64 MFMAs of k-step s run;
//   * LDS is a ring of five 32-deep k-step slots (160 KiB); the global->LDS stream (buffer_load ...
//     lds, 8 pieces per wave per k-step, one every 8 MFMAs, OOB rows read as zero) runs four
//     k-steps ahead and continues straight into the workgroup's NEXT tile, so the next tile's first
//     k-steps land while this tile's epilogue runs; one wait + barrier per pair of k-steps;
//   * the epilogue stores straight from the accumulators: the MFMA operands are swapped (C^T
//     orientation) so each lane holds 4 consecutive columns of one row, and one
//     v_permlane16_swap per dword pairs two 16-column MFMA tiles into 8 consecutive columns, i.e.
//     one 16-B store per lane (no LDS staging, no barrier); invalid rows store to a sink.
// Tiles are dealt round-robin over the persistent workgroups; the workgroups that share an XCD
// (b % 8) take consecutive tiles of the grouped (GROUP_M = 8) order, so a round's A row panels and
// B column panels are shared through that XCD's L2.
#include "common.h"
#include "ptk_internal.h"
#include "gemm_epi.h"
#include "gemm_persist.h"

#include <algorithm>
#include <cstdlib>
#include <type_traits>

#ifndef PTK_W4_RDS
#define PTK_W4_RDS 0      // diagnostic builds: fragment-read placement in the k-step (1 = two per group, groups 0..7)
#endif
#ifndef PTK_W4_DMS
#define PTK_W4_DMS 0      // diagnostic builds: DMA placement (1 = groups 8..15, 2 = groups 0..7, 3 = odd groups)
#endif
#ifndef PTK_P8_PRIO
#define PTK_P8_PRIO 1     // static s_setprio of the p8 kernel's younger half (waves 4-7): the two waves of a SIMD
                          // stop trading issue slots evenly and one runs ahead, so their LDS reads and MFMA
                          // bursts interleave (A/B r04: 298.5 vs 296.4 img/s, 3 rounds; 0 = diagnostic off)
#endif
#ifndef PTK_P8_MPRIO
#define PTK_P8_MPRIO 0    // diagnostic builds: s_setprio 1 around each p8 MFMA group (the issue arbitration
                          // between the two waves of a SIMD favours the one issuing MFMAs)
#endif

namespace ptk {

template <int ACT, int OUT, bool LEAN = false>
__global__ void __launch_bounds__(256, 1) gemm_w4_kernel(GemmArgs p, uint32_t a_bytes, uint32_t b_bytes,
                                                         uint32_t c_bytes) {
  __shared__ __attribute__((aligned(16))) char smem[W4_NSLOT * W4_SLOT];   // 160 KiB: the k-step ring
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wave >> 1, wc = wave & 1;
  const int nbm = (p.M + W4 - 1) / W4, nbn = (p.N + W4 - 1) / W4;
  const int ntile = nbm * nbn;
  const int G = gridDim.x;
  int loc;
  {
    const int b = blockIdx.x, q = G >> 3, rr = G & 7, x = b & 7;
    loc = (x < rr ? x * (q + 1) : rr * (q + 1) + (x - rr) * q) + (b >> 3);
  }
  if (loc >= ntile) return;
  const int nt = p.K / W4_KT;                              // 64-deep K-tiles per output tile
  const int nks = 2 * nt;                                  // 32-deep k-steps per output tile
  const int total_ks = ((ntile - loc + G - 1) / G) * nks;

  // A rows past M / B rows past N fall outside num_records and read as zero
  const u32x4_t rsa = w4_rsrc(p.A, a_bytes), rsb = w4_rsrc(p.B, b_bytes);

  // ---- global -> LDS stream, one ring slot (32 KiB: A and B, 256 rows x 64 B each) per k-step.
  // Wave w fills rows 64w..64w+63 of both operands: 4 + 4 pieces of 16 rows x 64 B.  Lane i of a
  // piece writes LDS row 16j + (i>>2), 16-B chunk i&3 (LDS image lane-linear) and fetches logical
  // chunk (i&3) ^ ((row>>1)&2): the XOR swizzle on the source address makes the fragment reads
  // bank-conflict free (every ds_read_b128 lane group covers the 64 banks once).
  uint32_t offa[4], offb[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int lr = wave * 64 + 16 * j + (lane >> 2);
    const int lc = (lane & 3) ^ ((lane >> 3) & 2);
    offa[j] = (uint32_t)lr * (uint32_t)p.lda * 2u + lc * 16;
    offb[j] = (uint32_t)lr * (uint32_t)p.ldb * 2u + lc * 16;
  }
  const uint32_t lds_base = __builtin_amdgcn_readfirstlane(lds_addr(smem));
  const uint32_t lds_dma = lds_base + wave * 64 * 64;      // this wave's rows in a slot
  // DMA cursor: tile dt, k-step dks, scalar offsets of its row panels.  Past the workgroup's last
  // k-step the cursor stays put and the stream re-loads that k-step into a free slot (never read),
  // so every k-step issues the same instructions.
  int dt = loc, dks = 0, dcount = 0;
  uint32_t dsa = 0, dsb = 0;
  auto dma_tile = [&](int t) {
    int bm, bn;
    w4_tile_coords(t, nbm, nbn, bm, bn);
    dsa = __builtin_amdgcn_readfirstlane((uint32_t)(bm * W4 + (int)p.amap.off) * (uint32_t)p.lda * 2u);
    dsb = __builtin_amdgcn_readfirstlane((uint32_t)(bn * W4) * (uint32_t)p.ldb * 2u);
  };
  auto dma_advance = [&]() {
    if (++dcount < total_ks) {
      if (++dks == nks) {
        dks = 0;
        dt += G;
        dma_tile(dt);
      }
    }
  };
  auto slot_next = [](uint32_t s) { s += W4_SLOT; return s == W4_NSLOT * W4_SLOT ? 0u : s; };

  // ---- fragments: A rows wr*128 + 16i + (lane&15), B rows wc*128 + 16j + (lane&15); logical 16-B
  // chunk lane>>4 of the slot's 64-B row
  const int frag_off = (lane & 15) * 64 + (((lane >> 4) ^ ((lane >> 1) & 2)) << 4);
  const uint32_t frag_a = lds_addr(smem) + wr * 128 * 64 + frag_off;
  const uint32_t frag_b = lds_addr(smem) + W4_SOPB + wc * 128 * 64 + frag_off;
  bf16x8_t fa0[8], fb0[8], fa1[8], fb1[8];
  f32x4_t acc[8][8];

// MFMA group q (0..15) of a k-step: 4 MFMAs of row block i = q/2, column blocks 4(q&1)..+3
#define W4_GROUP(FA, FB, Q, FIRST)                                                  \
  do {                                                                              \
    _Pragma("unroll") for (int jj = 0; jj < 4; ++jj) {                              \
      if (FIRST) W4_MFMA0(acc[(Q) >> 1][4 * ((Q) & 1) + jj], FB[4 * ((Q) & 1) + jj], FA[(Q) >> 1]); \
      else W4_MFMA(acc[(Q) >> 1][4 * ((Q) & 1) + jj], FB[4 * ((Q) & 1) + jj], FA[(Q) >> 1]);       \
    }                                                                               \
  } while (0)
// fragment read q (0..15) of the next k-step: q < 8 -> A row block q, else B column block q-8
#define W4_READ(FA, FB, BA, BB, Q)                                                  \
  do {                                                                              \
    if ((Q) < 8) W4_DSREAD(FA[(Q) & 7], BA, ((Q) & 7) * 1024);                      \
    else W4_DSREAD(FB[(Q) & 7], BB, ((Q) & 7) * 1024);                              \
  } while (0)
// every destination of the last 16 reads is pinned after the wait (no copy before the data lands)
#define W4_PIN(FA, FB)                                                                              \
  do {                                                                                              \
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");                                              \
    asm volatile("" : "+v"(FA[0]), "+v"(FA[1]), "+v"(FA[2]), "+v"(FA[3]), "+v"(FA[4]), "+v"(FA[5]),  \
                 "+v"(FA[6]), "+v"(FA[7]));                                                         \
    asm volatile("" : "+v"(FB[0]), "+v"(FB[1]), "+v"(FB[2]), "+v"(FB[3]), "+v"(FB[4]), "+v"(FB[5]),  \
                 "+v"(FB[6]), "+v"(FB[7]));                                                         \
  } while (0)

  // one k-step: 16 groups of 4 MFMAs on FA/FB; the 16 fragment reads of the next k-step (slot rs,
  // published by the last barrier) one per group in groups 0..7 and two per group in groups 8..11;
  // the 8 LDS-DMA pieces of k-step +4 (slot ws) in the even groups, i.e. one per 8 MFMAs: a
  // piece's issue cost (tens of cycles) is paid in MFMA time by a lone wave per SIMD and grows with
  // the density of memory instructions around it
  // (FIRST: the tile's first k-step, accumulators initialised by the MFMA; a compile-time constant
  // so that no branch sits between the MFMA groups)
  auto kstep = [&](auto first_c, const bf16x8_t (&FA)[8], const bf16x8_t (&FB)[8], bf16x8_t (&NA)[8],
                   bf16x8_t (&NB)[8], uint32_t rs, uint32_t ws) {
    constexpr bool first = decltype(first_c)::value;
    const uint32_t ba = frag_a + rs, bb = frag_b + rs;
    const uint32_t da = lds_dma + ws, db = da + W4_SOPB;
    const uint32_t sa = dsa + dks * (W4_KS * 2), sb = dsb + dks * (W4_KS * 2);
#pragma unroll
    for (int q = 0; q < 16; ++q) {
#if PTK_W4_RDS == 1
      if (q < 8) {
        W4_READ(NA, NB, ba, bb, 2 * q);
        W4_READ(NA, NB, ba, bb, 2 * q + 1);
      }
#else
      if (q < 8) {
        W4_READ(NA, NB, ba, bb, q);
      } else if (q < 12) {
        W4_READ(NA, NB, ba, bb, 8 + 2 * (q - 8));
        W4_READ(NA, NB, ba, bb, 9 + 2 * (q - 8));
      }
#endif
#if PTK_W4_DMS == 1
      if (q >= 8) {
        const int pc = q - 8;
#elif PTK_W4_DMS == 2
      if (q < 8) {
        const int pc = q;
#elif PTK_W4_DMS == 3
      if (q & 1) {
        const int pc = q >> 1;
#else
      if (!(q & 1)) {
        const int pc = q >> 1;   // pieces A0 B0 A1 B1 ... in groups 0, 2, .., 14
#endif
        if (pc & 1) W4_DMA(rsb, offb[pc >> 1], sb, db + (pc >> 1) * 1024);
        else W4_DMA(rsa, offa[pc >> 1], sa, da + (pc >> 1) * 1024);
      }
      W4_GROUP(FA, FB, q, first);
    }
  };

  // ---- prologue: k-steps 0..3 into slots 0..3; 0..2 landed and published, fragments of k-step 0
  // read, then a second barrier: k-step 1 overwrites slot 0 (ring invariant below)
  dma_tile(dt);
#pragma unroll
  for (int b = 0; b < 4; ++b) {
    const uint32_t da = lds_dma + b * W4_SLOT, db = da + W4_SOPB;
    const uint32_t sa = dsa + dks * (W4_KS * 2), sb = dsb + dks * (W4_KS * 2);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      W4_DMA(rsa, offa[j], sa, da + j * 1024);
      W4_DMA(rsb, offb[j], sb, db + j * 1024);
    }
    dma_advance();
  }
  asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  __builtin_amdgcn_s_barrier();
#pragma unroll
  for (int q = 0; q < 16; ++q) W4_READ(fa0, fb0, frag_a, frag_b, q);
  W4_PIN(fa0, fb0);
  __builtin_amdgcn_s_barrier();

  // ring invariant at k-step i (i counts over the workgroup's whole stream): fragments of i are in
  // registers; k-steps i+1 and (if i is even) i+2 have landed and are published; k-step i+3 is in
  // flight; k-step i+4 goes to slot (i+4) % 5, whose last reader (the fragment reads of k-step i-1,
  // done during k-step i-2) precedes the barrier that ends the last odd k-step <= i-1.  One wait +
  // barrier per pair of k-steps (after the odd one) publishes k-steps i+2 and i+3: vmcnt(8) leaves
  // only k-step i+4's 8 pieces in flight.  The epilogue's stores follow the barrier; the next wait
  // (two k-steps later) drains them too.
  uint32_t rs = W4_SLOT, ws = 4 * W4_SLOT;
  int t = loc, kt = 0;
#ifdef PTK_P8_STAMPS
  unsigned int stv_[4] = {0u, 0u, 0u, 0u};
  const int em_ = g_p8_epi_mode;
#endif
  for (int g = 0; g < total_ks; g += 2) {
    if (kt == 0) P8_STAMP(0, (t - loc) / G);
    if (kt == 0) kstep(std::true_type{}, fa0, fb0, fa1, fb1, rs, ws);
    else kstep(std::false_type{}, fa0, fb0, fa1, fb1, rs, ws);
    W4_PIN(fa1, fb1);
    dma_advance();
    rs = slot_next(rs);
    ws = slot_next(ws);
    kstep(std::false_type{}, fa1, fb1, fa0, fb0, rs, ws);
    W4_PIN(fa0, fb0);
    dma_advance();
    rs = slot_next(rs);
    ws = slot_next(ws);
    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (kt == 0) P8_STAMP(1, (t - loc) / G);
    if (kt == nt - 1) {
      P8_STAMP(2, (t - loc) / G);
      asm volatile("s_nop 7\n\ts_nop 7" ::: "memory");   // MFMA D -> accumulator read wait states
      int bm, bn;
      w4_tile_coords(t, nbm, nbn, bm, bn);
#ifdef PTK_P8_STAMPS
      if (em_ != 1)
#endif
      {
        const long row0 = (long)bm * W4 + wr * 128, col0 = (long)bn * W4 + wc * 128;
        if constexpr (LEAN && ACT == ACT_GEGLU_BWD)
          w4_epilogue_lean_glu<ACT, 8>(kernarg_args(), acc, row0, col0, lane, c_bytes);
        else if constexpr (LEAN) w4_epilogue_lean<ACT, 8>(kernarg_args(), acc, row0, col0, lane, c_bytes);
        else w4_epilogue<ACT, OUT>(kernarg_args(), acc, row0, col0, lane);
      }
      P8_STAMP(3, (t - loc) / G);
      t += G;
      kt = 0;
    } else {
      ++kt;
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // no LDS-DMA may land after the workgroup exits
#ifdef PTK_P8_STAMPS
  if (wave == 0 && blockIdx.x < 1024)
#pragma unroll
    for (int k = 0; k < 4; ++k) g_p8_stamps[blockIdx.x][k][lane] = stv_[k];
#endif
#undef W4_GROUP
#undef W4_READ
#undef W4_PIN
}

// the W4 path needs: batch 1, 16-B aligned rows of every operand it touches 8 columns at a time,
// N % 8 == 0, byte extents of A and B below 2^31 (32-bit buffer offsets)
bool w4_supported(const GemmArgs& a, int act, int out) {
  if (a.N % 8 || a.K % W4_KT) return false;
  if (a.alpha != 1.f) return false;   // the persistent epilogues take the accumulators as they are (no scale)
  if (a.row_stats) return false;   // the softmax-statistics epilogue lives in gemm.hip's epilogue only
  if (a.resid16 && (out != OUT_BF16 || a.ld_resid16 % 8)) return false;
  if ((a.ldc % 8) || (a.resid && a.ld_resid % 4) || (a.rowadd && a.ld_rowadd % 4)) return false;
  if ((a.aux || a.aux2) && a.ld_aux % 8) return false;
  if ((a.aux_in || a.aux_in2) && a.ld_aux_in % 8) return false;
  if (((uintptr_t)a.C | (uintptr_t)a.bias | (uintptr_t)a.resid | (uintptr_t)a.resid16 | (uintptr_t)a.rowadd | (uintptr_t)a.aux |
       (uintptr_t)a.aux2 | (uintptr_t)a.aux_in | (uintptr_t)a.aux_in2) & 15)
    return false;
  if (act == ACT_GEGLU && (a.N % 32)) return false;
  if (act == ACT_GEGLU_BWD && (!a.aux_in || !a.aux_in2 || (a.N % 16) || (a.ldc % 8))) return false;
  if (act == ACT_GELU_ERF_BWD && !a.aux_in) return false;
  if (out != OUT_BF16 && (act != ACT_NONE)) return false;
  if (a.amap.g != 0) return false;   // gathered A rows: not an affine row panel
  const double abytes = (double)(a.M + a.amap.off) * a.lda * 2, bbytes = (double)a.N * a.ldb * 2;
  return abytes < 2147483000.0 && bbytes < 2147483000.0;
}

static int g_num_cu = 0;

static int num_cu() {
  if (!g_num_cu) {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
      n = 256;
    g_num_cu = n;
  }
  return g_num_cu;
}

int device_cus() { return num_cu(); }

double w4_round_fill(long M, long N) {
  const long ntile = ((M + W4 - 1) / W4) * ((N + W4 - 1) / W4), cu = num_cu();
  return (double)ntile / (double)(((ntile + cu - 1) / cu) * cu);
}

// the lean bf16 epilogue (gemm_persist.h w4_epilogue_lean) applies: ACT_NONE / ACT_GELU_TANH into bf16 with at most
// a bias, the bf16-linear rounding and a bf16 residual (row-aligned with C, 16-B rows); a C row map that is an
// offset (cmap.g == 0, or a group map without skipped rows whose group stride equals its size: the identity
// plus cmap.off); whole 64-column wave ranges; C's extent (rows cmap.off .. M + cmap.off) below 2^31 bytes.
// c_bytes = that extent (num_records of the store resource: rows past M are dropped).  PTK_LEAN_EPI=0 (A/B builds,
// PTK_AB) keeps the general epilogue (bit-identical either way)
static bool lean_on() { return PTK_AB("PTK_LEAN_EPI", 1) != 0; }
// the lean GEGLU-backward epilogue (w4_epilogue_lean_glu): the saved g, u inputs with 16-B rows, no other epilogue
// input, an offset C row map, whole 128-column wave ranges, extents below 2^31 bytes
static bool lean_glu_ok(const GemmArgs& a, int act, int out, uint32_t& c_bytes) {
  if (!lean_on() || act != ACT_GEGLU_BWD || out != OUT_BF16) return false;
  if (a.bias || a.rowadd || a.resid || a.resid16 || a.bf16_linear || a.row_stats || a.alpha != 1.f) return false;
  const bool affine = a.cmap.g == 0 || (a.cmap.skip == 0 && a.cmap.gs == a.cmap.g);
  if (!affine || a.cmap.off < 0 || a.amap.g != 0 || a.N % 128 || a.ldc % 8 || ((uintptr_t)a.C & 15)) return false;
  if (!a.aux_in || !a.aux_in2 || a.ld_aux_in % 8 || a.ld_aux_in < a.N) return false;
  if (((uintptr_t)a.aux_in | (uintptr_t)a.aux_in2) & 15) return false;
  if (a.ldc < 2 * a.N) return false;
  const double side = (double)a.M * (double)a.ld_aux_in * 2.0;
  const double bytes = ((double)a.M + (double)a.cmap.off) * (double)a.ldc * 2.0;
  if (bytes >= 2147483000.0 || side >= 2147483000.0) return false;
  c_bytes = (uint32_t)bytes;
  return true;
}
bool lean_epilogue_ok(const GemmArgs& a, int act, int out, uint32_t& c_bytes) {
  if (act == ACT_GEGLU_BWD) return lean_glu_ok(a, act, out, c_bytes);
  if (!lean_on() || (act != ACT_NONE && act != ACT_GELU_TANH) || out != OUT_BF16) return false;
  if (a.rowadd || a.resid || a.aux || a.aux2 || a.aux_in || a.aux_in2 || a.row_stats || a.alpha != 1.f) return false;
  const bool affine = a.cmap.g == 0 || (a.cmap.skip == 0 && a.cmap.gs == a.cmap.g);
  if (!affine || a.cmap.off < 0 || a.N % 64 || a.ldc % 8 || a.ldc < a.N || ((uintptr_t)a.C & 15)) return false;
  if (a.bias && ((uintptr_t)a.bias & 15)) return false;
  if (a.resid16 && (a.ld_resid16 % 8 || ((uintptr_t)a.resid16 & 15))) return false;
  const double rows = (double)a.M + (double)a.cmap.off;
  const double bytes = rows * (double)a.ldc * 2.0, rbytes = a.resid16 ? rows * (double)a.ld_resid16 * 2.0 : 0.0;
  if (bytes >= 2147483000.0 || rbytes >= 2147483000.0) return false;
  c_bytes = (uint32_t)bytes;
  return true;
}

bool lean_epilogue_candidate(const GemmArgs& a) {
  uint32_t cb = 0;
  return lean_epilogue_ok(a, ACT_NONE, OUT_BF16, cb);
}

int launch_gemm_w4(const GemmArgs& a, int act, int out, hipStream_t st, int max_grid) {
  num_cu();
  const long ntile = (long)((a.M + W4 - 1) / W4) * ((a.N + W4 - 1) / W4);
  long grid = std::min<long>(ntile, max_grid > 0 ? max_grid : g_num_cu);
#ifdef PTK_P8_STAMPS
  if (const char* e = getenv("PTK_GEMM_GRID")) grid = std::min<long>(grid, atol(e));   // diagnostic: fewer CUs
#endif
  const long arows = a.M + a.amap.off;
  const uint32_t ab = (uint32_t)std::min<double>((double)arows * a.lda * 2, 2147483000.0);
  const uint32_t bb = (uint32_t)std::min<double>((double)a.N * a.ldb * 2, 2147483000.0);
  uint32_t cb = 0;
  if (lean_epilogue_ok(a, act, out, cb)) {
#define PTK_W4L_CASE(ACT_)                                                                                   \
    if (act == ACT_)                                                                                         \
      hipLaunchKernelGGL((gemm_w4_kernel<ACT_, OUT_BF16, true>), dim3((unsigned)grid), dim3(256), 0, st, a, ab, bb, cb);
    PTK_W4L_CASE(ACT_NONE)
    PTK_W4L_CASE(ACT_GELU_TANH)
    PTK_W4L_CASE(ACT_GEGLU_BWD)
#undef PTK_W4L_CASE
    return hipGetLastError() == hipSuccess ? 0 : set_error("gemm_w4 launch failed");
  }
#define PTK_W4_CASE(ACT_, OUT_)                                                                   \
  if (act == ACT_ && out == OUT_) {                                                               \
    hipLaunchKernelGGL((gemm_w4_kernel<ACT_, OUT_>), dim3((unsigned)grid), dim3(256), 0, st, a, ab, bb, 0u); \
    return hipGetLastError() == hipSuccess ? 0 : set_error("gemm_w4 launch failed");              \
  }
  PTK_W4_CASE(ACT_NONE, OUT_BF16)
  PTK_W4_CASE(ACT_NONE, OUT_F32)
  PTK_W4_CASE(ACT_NONE, OUT_F32_BFR)
  PTK_W4_CASE(ACT_GELU_TANH, OUT_BF16)
  PTK_W4_CASE(ACT_GELU_ERF, OUT_BF16)
  PTK_W4_CASE(ACT_GEGLU, OUT_BF16)
  PTK_W4_CASE(ACT_GELU_ERF_BWD, OUT_BF16)
  PTK_W4_CASE(ACT_GEGLU_BWD, OUT_BF16)
#undef PTK_W4_CASE
  return set_error("gemm_w4: unsupported (act=%d, out=%d)", act, out);
}


// ============================================================================ persistent 8-wave variant
// gemm_p8_kernel: the w4 kernel's persistent 256x256 tiles, k-step ring and register epilogue with 8 waves,
// two per SIMD.  Waves w and w + 4 share a SIMD; wave w computes rows wr*128 .. +128 and columns
// wc*128 + 64*(w >> 2) .. +64 of the tile (wr, wc from w & 3): a 128x64 fp32 accumulator (128 AGPRs), so
// each wave fits the 256-register budget of two waves per SIMD.  The LDS-DMA stream is split over all 8
// waves (4 pieces per wave per k-step instead of w4's 8), and each wave's pieces issue while its SIMD
// partner's MFMAs keep the matrix pipe busy: the per-piece issue cost that holds the 4-wave kernel's K loop
// at ~64 % of the MFMA floor is paid beside the partner's MFMAs, not instead of them.
// Fragments: B double-buffered (4 per k-step), A single-buffered and re-read in place one MFMA group after
// its last reader (the ping-pong kernel's consumer stream).  The tile's last k-step reads no fragments, so
// only the accumulators are live through the epilogue; the next tile's first fragments are read after it.
// The ring, the DMA cursor and the one wait + barrier per pair of k-steps are w4's; the waits are vmcnt(4).
namespace {
constexpr int P8_PIECES = 4;   // LDS-DMA pieces per wave per k-step

}

// ---- stream-K tail (P8Tail; SK kernels only).  A tile grid whose last round fills the persistent grid badly
// (Gemma3's N = 1152 projections: 440 tiles = 1.72 rounds of 256 CUs; SigLIP's N = 1024 ones: 288 = 1.13) runs
// its first R whole rounds data-parallel (tiles loc, loc + G, ..: the lock-step L2 sharing of the plain kernel)
// and spreads the K-tiles of the remaining tail tiles evenly over the first Gs workgroups (Gs <= G, chosen on
// the host: more workgroups shorten the tail round but cut each tile into more pieces, and every extra piece
// costs the fixup one more 256-KiB partial read): workgroup g < Gs takes the K-tile units
// [g U / Gs, (g + 1) U / Gs) of the tail's U = tail tiles x K-tiles, i.e. the end of one tail tile and / or the
// start of the next.  A tile covered by one workgroup runs the normal epilogue.  A tile split over workgroups
// g0 .. g1 (its pieces, in K order): every wave of a piece writes its 128x64 fp32 partial (32 KiB) to its
// workgroup's slot (slot 0 for the workgroup's first piece, 1 for its last), and p8_fixup_kernel, launched
// after the GEMM, sums each cut tile's pieces in K order (deterministic) and runs the tile's epilogue.  r04 let
// the wave arriving last at a per-(tile, wave) counter do that sum inside the GEMM: one wave loading a piece's
// row block at a time was latency-bound (~150 us on the Stage-2 d(gate|up) dX, profiles/r04_sk_ab.txt), where
// the fixup spreads the same loads over 8 waves x 8 row blocks per tile.  No wave waits for another workgroup.


// PTK_P8_CREAD (A/B builds only): the fragment reads as compiler-visible LDS loads (hipcc places them and counts
// their waits) instead of the asm reads with the counted lgkmcnt ladder -- gemm_tn.hip's form
#ifdef PTK_P8_CREAD
#define P8_DSREAD(DST, ADDR, OFF) \
  (DST) = *reinterpret_cast<const __attribute__((address_space(3))) bf16x8_t*>((uintptr_t)((ADDR) + (OFF)))
#define P8_LGKM(N) do { } while (0)
#define P8_BARRIER() do { __builtin_amdgcn_s_barrier(); asm volatile("" ::: "memory"); } while (0)
#else
#define P8_BARRIER() __builtin_amdgcn_s_barrier()
#define P8_DSREAD(DST, ADDR, OFF) W4_DSREAD(DST, ADDR, OFF)
#define P8_LGKM(N) asm volatile("s_waitcnt lgkmcnt(" #N ")" ::: "memory")
#endif
// TM: output tile height, 256, 224, 192 or 160.  Shorter tiles (TM / 32 row blocks of 16 per wave, the A image's
// last rows unused, waves 0 .. TM / 32 - 1 staging A, the others only B) fill the rounds of the persistent grid
// better where 256-row tiles leave a thin last round: Gemma3's N 1152 / 1024 projections at M 22 528 (440 -> 505
// tiles of 7/8 the work on 2 rounds), N 1536 (3 rounds either way, 7/8 the work), SigLIP's q|k|v at M 18 432,
// its fc1 on 192-row tiles (5 rounds of 256 -> 6 of 192) -- launch_gemm: p8_tile_height
template <int ACT, int OUT, bool SK, bool LEAN = false, int TM = 256>
__global__ void __launch_bounds__(512, 1) gemm_p8_kernel(GemmArgs p, uint32_t a_bytes, uint32_t b_bytes, P8Tail tl,
                                                         uint32_t c_bytes) {
  static_assert(TM == 256 || ((TM == 224 || TM == 192 || TM == 160) && !SK), "shorter tiles: whole tiles only");
  constexpr int RB = TM / 32;   // 16-row blocks per wave
  __shared__ __attribute__((aligned(16))) char smem[W4_NSLOT * W4_SLOT];   // 160 KiB: the k-step ring
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int hf = wave >> 2, wq = wave & 3, wr = wq >> 1, wc = wq & 1;
  const bool a_dma = TM == 256 || wave < RB;   // (shorter tiles: waves RB .. 7 stage no A rows)
  const int nbm = (p.M + TM - 1) / TM, nbn = (p.N + W4 - 1) / W4;
  const int ntile = nbm * nbn;
  const int G = gridDim.x;
  int loc;
  {
    const int b = blockIdx.x, q = G >> 3, rr = G & 7, x = b & 7;
    loc = (x < rr ? x * (q + 1) : rr * (q + 1) + (x - rr) * q) + (b >> 3);
  }
  const int nt = p.K / W4_KT;                              // 64-deep K-tiles per output tile
  // this workgroup's segments: whole tiles loc, loc + G, .. below dp_tiles, then (SK) its tail pieces
  const int dp_tiles = SK ? tl.dp_tiles : ntile;
  const int n_dp = loc < dp_tiles ? (dp_tiles - loc + G - 1) / G : 0;
  // tail units are pairs of K-tiles (nt is even for an SK launch), so every piece spans >= 2 K-tiles
  const int U = SK ? tl.units : 0, Gs = SK ? tl.gsplit : 1, nu = nt >> 1;
  const int u0 = SK && loc < Gs ? p8_start(loc, Gs, U) : 0, u1 = SK && loc < Gs ? p8_start(loc + 1, Gs, U) : 0;
  const int n_tail = u1 > u0 ? (u1 - 1) / nu - u0 / nu + 1 : 0;
  const int nseg = n_dp + n_tail;
  if (nseg == 0) return;
  const int total_ks = 2 * n_dp * nt + 4 * (u1 - u0);     // 32-deep k-steps of the workgroup's whole stream
  // segment table (SK): lane i holds segment i (the host keeps nseg <= 64) -- tile t, tail tile tt (-1 for a
  // whole data-parallel tile), K-tiles [k0, k1) and for a cut tail tile its pieces' first workgroup g0, their
  // count np, piece 0's slot s0 and this workgroup's slot -- read back by v_readlane at segment boundaries, so
  // the bookkeeping costs 3 VGPRs instead of a dozen SGPRs live across the K loop
  uint32_t segA = 0, segB = 0, segC = 0;
  if constexpr (SK) {
    const int i = lane;
    int t, k0, k1, tt;
    if (i < n_dp) {
      t = loc + i * G; k0 = 0; k1 = nt; tt = -1;
    } else {
      tt = u0 / nu + (i - n_dp);
      k0 = 2 * (max(u0, tt * nu) - tt * nu);
      k1 = 2 * (min(u1, (tt + 1) * nu) - tt * nu);
      t = dp_tiles + tt;
    }
    int g0 = 0, np = 1, s0 = 0, myslot = 0;
    if (tt >= 0 && i < nseg) {
      g0 = p8_owner((long)tt * nu, Gs, U);
      np = p8_owner((long)(tt + 1) * nu - 1, Gs, U) - g0 + 1;
      s0 = p8_start(g0, Gs, U) < tt * nu ? 1 : 0;
      myslot = u0 < tt * nu ? 1 : 0;
      if (np == 1) tt = -1;   // the whole tile in one piece: plain epilogue
    }
    segA = (uint32_t)t | ((uint32_t)(tt + 1) << 16);
    segB = (uint32_t)k0 | ((uint32_t)k1 << 16);
    segC = (uint32_t)g0 | ((uint32_t)np << 10) | ((uint32_t)s0 << 20) | ((uint32_t)myslot << 21);
  }
  // segment s -> output tile t, K-tiles [k0, k1) (tt: tail tile index, -1 for a whole tile)
  auto segment = [&](int s, int& t, int& k0, int& k1, int& tt) __attribute__((always_inline)) {
    if constexpr (!SK) {
      t = loc + s * G; k0 = 0; k1 = nt; tt = -1;
    } else {
      const uint32_t a = __builtin_amdgcn_readlane(segA, s), b = __builtin_amdgcn_readlane(segB, s);
      t = (int)(a & 0xffffu); tt = (int)(a >> 16) - 1;
      k0 = (int)(b & 0xffffu); k1 = (int)(b >> 16);
    }
  };
  const u32x4_t rsa = w4_rsrc(p.A, a_bytes), rsb = w4_rsrc(p.B, b_bytes);

  // global -> LDS: wave w fills rows 32w..32w+31 of both operands (2 + 2 pieces of 16 rows x 64 B), lane i of
  // a piece writes LDS row 16j + (i>>2), chunk i&3 and fetches logical chunk (i&3) ^ ((row>>1)&2) (w4's swizzle)
  uint32_t offa[2], offb[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int lr = wave * 32 + 16 * j + (lane >> 2);
    const int lc = (lane & 3) ^ ((lane >> 3) & 2);
    offa[j] = (uint32_t)lr * (uint32_t)p.lda * 2u + lc * 16;
    offb[j] = (uint32_t)lr * (uint32_t)p.ldb * 2u + lc * 16;
  }
  const uint32_t lds_base = __builtin_amdgcn_readfirstlane(lds_addr(smem));
  const uint32_t lds_dma = lds_base + wave * 32 * 64;
  // DMA cursor: segment dseg, k-step dks of its dlen (past the last k-step it stays put and re-loads that k-step
  // into a free slot, never read, so every k-step issues the same instructions)
  int dseg = 0, dks = 0, dlen = 0, dcount = 0;
  uint32_t dsa = 0, dsb = 0;
  auto dma_seg = [&](int s) {
    int t, k0, k1, tt;
    segment(s, t, k0, k1, tt);
    int bm, bn;
    w4_tile_coords(t, nbm, nbn, bm, bn);
    uint32_t kz = 0;   // K slices as row tiles (P8Tail::zslices): byte offset of slice z's K range
    if (!SK && tl.zslices > 1) {
      const int nbz = nbm / tl.zslices, z = bm / nbz;
      bm -= z * nbz;
      kz = (uint32_t)z * (uint32_t)p.K * 2u;
    }
    dsa = __builtin_amdgcn_readfirstlane((uint32_t)(bm * TM + (int)p.amap.off) * (uint32_t)p.lda * 2u + kz +
                                         (uint32_t)k0 * (W4_KT * 2));
    dsb = __builtin_amdgcn_readfirstlane((uint32_t)(bn * W4) * (uint32_t)p.ldb * 2u + kz + (uint32_t)k0 * (W4_KT * 2));
    dlen = 2 * (k1 - k0);
  };
  auto dma_advance = [&]() {
    if (++dcount < total_ks) {
      if (++dks == dlen) {
        dks = 0;
        dma_seg(++dseg);
      }
    }
  };
  auto slot_next = [](uint32_t s) { s += W4_SLOT; return s == W4_NSLOT * W4_SLOT ? 0u : s; };

  const int frag_off = (lane & 15) * 64 + (((lane >> 4) ^ ((lane >> 1) & 2)) << 4);
  const uint32_t frag_a = lds_addr(smem) + wr * (TM / 2) * 64 + frag_off;
  const uint32_t frag_b = lds_addr(smem) + W4_SOPB + (wc * 128 + hf * 64) * 64 + frag_off;
  bf16x8_t fa[8], fb0[4], fb1[4];
  f32x4_t acc[8][4];

  // all 12 fragments of the k-step in slot rs (after a barrier published it)
  auto read_frags = [&](uint32_t rs) __attribute__((always_inline)) {
    const uint32_t ba = frag_a + rs, bb = frag_b + rs;
#pragma unroll
    for (int r = 0; r < RB; ++r) P8_DSREAD(fa[r], ba, r * 1024);
#pragma unroll
    for (int r = 0; r < 4; ++r) P8_DSREAD(fb0[r], bb, r * 1024);
    P8_LGKM(0);
    asm volatile("" : "+v"(fa[0]), "+v"(fa[1]), "+v"(fa[2]), "+v"(fa[3]), "+v"(fa[4]), "+v"(fa[5]),
                 "+v"(fa[6]), "+v"(fa[7]));
    asm volatile("" : "+v"(fb0[0]), "+v"(fb0[1]), "+v"(fb0[2]), "+v"(fb0[3]));
  };

  // one k-step: 8 groups of 4 MFMAs (row block q x column blocks 0..3) on fa / FB.  RD: the next k-step's
  // fragments (slot rs) are read, B block q (q < 4) into NB before group q and A block q into fa[q] one group
  // after group q (A7 after the last group); issue order B0 B1 A0 B2 A1 B3 A2 .. A7, so before group q of the
  // next k-step lgkmcnt(n_q) leaves exactly the younger reads in flight (n = 6, 8, 8, 9, 10, 10, 10, 10).
  // The 4 LDS-DMA pieces of k-step +4 (slot ws) go out in the even groups (waves 0-3) or the odd groups
  // (waves 4-7), so the two waves of a SIMD do not issue theirs side by side.
  auto kstep = [&](auto first_c, auto read_c, auto half_c, bf16x8_t (&FB)[4], bf16x8_t (&NB)[4], uint32_t rs,
                   uint32_t ws) __attribute__((always_inline)) {
    constexpr bool first = decltype(first_c)::value, rd = decltype(read_c)::value;
    constexpr int half = decltype(half_c)::value;
    const uint32_t ba = frag_a + rs, bb = frag_b + rs;
    const uint32_t da = lds_dma + ws, db = da + W4_SOPB;
    const uint32_t sa = dsa + dks * (W4_KS * 2), sb = dsb + dks * (W4_KS * 2);
#pragma unroll
    for (int q = 0; q < RB; ++q) {
      // n_q = RB - 2, RB, RB, RB + 1, RB + 2, .. (8 groups: 6, 8, 8, 9, 10, 10, 10, 10; each A read fewer, one less)
      if constexpr (RB == 8) {
        if (q == 0) P8_LGKM(6);
        else if (q < 3) P8_LGKM(8);
        else if (q == 3) P8_LGKM(9);
        else P8_LGKM(10);
      } else if constexpr (RB == 7) {
        if (q == 0) P8_LGKM(5);
        else if (q < 3) P8_LGKM(7);
        else if (q == 3) P8_LGKM(8);
        else P8_LGKM(9);
      } else if constexpr (RB == 6) {
        if (q == 0) P8_LGKM(4);
        else if (q < 3) P8_LGKM(6);
        else if (q == 3) P8_LGKM(7);
        else P8_LGKM(8);
      } else {
        static_assert(RB == 5, "tile heights 256, 224, 192, 160");
        if (q == 0) P8_LGKM(3);
        else if (q < 3) P8_LGKM(5);
        else if (q == 3) P8_LGKM(6);
        else P8_LGKM(7);
      }
      asm volatile("" : "+v"(fa[q]));
      if (q == 0) asm volatile("" : "+v"(FB[0]), "+v"(FB[1]), "+v"(FB[2]), "+v"(FB[3]));
      if (rd && q < 4) P8_DSREAD(NB[q], bb, q * 1024);
      // pieces A0 B0 A1 B1: piece pc in group min(2 pc + half, RB - 1) -- the even (waves 0-3) or odd (waves 4-7)
      // groups, the pieces past the last group in it
#pragma unroll
      for (int pc = 0; pc < 4; ++pc) {
        if (q == (2 * pc + half < RB - 1 ? 2 * pc + half : RB - 1)) {
          if (pc & 1) W4_DMA(rsb, offb[pc >> 1], sb, db + (pc >> 1) * 1024);
          else if (a_dma) W4_DMA(rsa, offa[pc >> 1], sa, da + (pc >> 1) * 1024);
        }
      }
      if (PTK_P8_MPRIO) asm volatile("s_setprio 1" ::: "memory");
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) {
        if (first) W4_MFMA0(acc[q][jj], FB[jj], fa[q]);
        else W4_MFMA(acc[q][jj], FB[jj], fa[q]);
      }
      if (PTK_P8_MPRIO) asm volatile("s_setprio 0" ::: "memory");
      if (rd && q >= 1) P8_DSREAD(fa[q - 1], ba, (q - 1) * 1024);   // one group after its last reader
    }
    if (rd) P8_DSREAD(fa[RB - 1], ba, (RB - 1) * 1024);
  };

  // stream-K piece of a cut tail tile: the wave's 128x64 fp32 partial to its workgroup's slot (slot 0 for the
  // workgroup's first piece, 1 for its last); p8_fixup_kernel sums the pieces after the launch
  auto tail_store = [&](int slot) __attribute__((always_inline)) {
    float* mine = tl.slab + (((size_t)loc * 2 + slot) * 8 + wave) * P8_WAVE_FLOATS + lane * 4;
#pragma unroll
    for (int q = 0; q < 8; ++q)
#pragma unroll
      for (int jj = 0; jj < 4; ++jj)
        asm volatile("global_store_dwordx4 %0, %1, off" :: "v"(mine + (4 * q + jj) * 256), "a"(acc[q][jj])
                     : "memory");   // straight from the AGPRs (a VGPR copy invites hipcc to re-home acc)
  };

#ifdef PTK_P8_STAMPS
  unsigned int stv_[4] = {0u, 0u, 0u, 0u};
  const int em_ = g_p8_epi_mode;
#endif
  // the wait that leaves only the youngest k-step's pieces in flight: 4 per wave, 2 for the B-only waves
  auto vm_wait = [&]() __attribute__((always_inline)) {
    if (TM != 256 && !a_dma) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  };
  auto run = [&](auto half_c) __attribute__((always_inline)) {
    if (PTK_P8_PRIO && decltype(half_c)::value) __builtin_amdgcn_s_setprio(PTK_P8_PRIO);
    // prologue: k-steps 0..3 into slots 0..3; 0..2 landed and published; fragments of k-step 0 read
    dma_seg(0);
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const uint32_t da = lds_dma + b * W4_SLOT, db = da + W4_SOPB;
      const uint32_t sa = dsa + dks * (W4_KS * 2), sb = dsb + dks * (W4_KS * 2);
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        if (a_dma) W4_DMA(rsa, offa[j], sa, da + j * 1024);
        W4_DMA(rsb, offb[j], sb, db + j * 1024);
      }
      dma_advance();
    }
    vm_wait();
    P8_BARRIER();
    read_frags(0);
    P8_BARRIER();
    // ring invariant as gemm_w4_kernel's (k-step i's fragments in registers, i+1 / i+2 published, i+3 in
    // flight, i+4 issued into the slot of i-1); vmcnt(4) before each pair's barrier leaves only the youngest
    // k-step's 4 pieces in flight
    uint32_t rs = W4_SLOT, ws = 4 * W4_SLOT;
    // one pair of k-steps (one 64-deep K-tile), then the wait + barrier; the segment's first K-tile
    // initialises the accumulators (MFMA with C = 0) and its last reads no fragments.  Peeled per segment (no
    // branch between MFMA forms), so the 128 accumulators keep their registers across the K loop.
    auto pair = [&](auto first_c, auto last_c) __attribute__((always_inline)) {
      constexpr bool lst = decltype(last_c)::value;
      kstep(first_c, std::true_type{}, half_c, fb0, fb1, rs, ws);
      dma_advance();
      rs = slot_next(rs);
      ws = slot_next(ws);
      kstep(std::false_type{}, std::integral_constant<bool, !lst>{}, half_c, fb1, fb0, rs, ws);
      dma_advance();
      if (!lst) rs = slot_next(rs);   // last pair: rs stays on the next segment's first k-step
      ws = slot_next(ws);
      vm_wait();
      P8_BARRIER();
    };
    for (int s = 0; s < nseg; ++s) {
      int t, k0, k1, tt;
      segment(s, t, k0, k1, tt);
      P8_STAMP(0, s);
      pair(std::true_type{}, std::false_type{});   // (every segment spans >= 2 K-tiles: tail units are pairs)
      P8_STAMP(1, s);
      for (int kt = k0 + 1; kt < k1 - 1; ++kt) pair(std::false_type{}, std::false_type{});
      pair(std::false_type{}, std::true_type{});
      P8_STAMP(2, s);
      asm volatile("s_nop 7\n\ts_nop 7" ::: "memory");   // MFMA D -> accumulator read wait states
      int bm, bn;
      w4_tile_coords(t, nbm, nbn, bm, bn);
      const long row0 = (long)bm * TM + wr * (TM / 2), col0 = (long)bn * W4 + wc * 128 + hf * 64;
      if (!SK || tt < 0) {
#ifdef PTK_P8_STAMPS
        if (em_ != 1)
#endif
        {
          if constexpr (LEAN && ACT == ACT_GEGLU_BWD)
            w4_epilogue_lean_glu<ACT, 4>(kernarg_args(), acc, row0, col0, lane, c_bytes);
          else if constexpr (LEAN) w4_epilogue_lean<ACT, 4, RB>(kernarg_args(), acc, row0, col0, lane, c_bytes);
          else w4_epilogue<ACT, OUT, 4, RB>(kernarg_args(), acc, row0, col0, lane);
        }
      } else if constexpr (SK) {
        tail_store((int)((__builtin_amdgcn_readlane(segC, s) >> 21) & 1u));
      }
      P8_STAMP(3, s);
      // the next segment's first k-step (published by the barrier; harmless after the last).  Its slot is the
      // one the NEXT pair's second k-step restages (k-step i+6 lands in the slot of i+1), so a barrier keeps
      // a wave that finished its epilogue early from overwriting it before every wave has read it
      read_frags(rs);
      P8_BARRIER();
      rs = slot_next(rs);
    }
  };
  if (hf) run(std::integral_constant<int, 1>{});
  else run(std::integral_constant<int, 0>{});
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // no LDS-DMA may land after the workgroup exits
#ifdef PTK_P8_STAMPS
  if (wave == 0 && blockIdx.x < 1024)
#pragma unroll
    for (int k = 0; k < 4; ++k) g_p8_stamps[blockIdx.x][k][lane] = stv_[k];
#endif
}

#ifdef PTK_P8_STAMPS
}  // namespace ptk
extern "C" int ptk_debug_p8_stamps_read(void* host, size_t bytes) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(ptk::g_p8_stamps), bytes, 0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
extern "C" int ptk_debug_p8_epi_mode(int m) {
  return hipMemcpyToSymbol(HIP_SYMBOL(ptk::g_p8_epi_mode), &m, sizeof(int), 0, hipMemcpyHostToDevice) == hipSuccess ? 0 : -1;
}
namespace ptk {
#endif
// stream-K fixup (P8Tail): workgroup (tail tile tt, row block I); wave w sums row block I of its 128x64 partial
// over the tile's pieces in K order (4 x 16 B per lane per piece, up to 4 pieces' loads in flight) and runs the
// general epilogue of those 16 rows (w4_rows: bit-identical to the lean one).  Tiles that ran whole are skipped.
template <int ACT, int OUT, int I>
PTK_DEV void p8_fixup_rows(const GemmArgs& p, const float* slab, int g0, int np, int s0, int wave, long row0,
                           long col0, int lane) {
  f32x4_t sum[4];
  auto piece = [&](int jj) __attribute__((always_inline)) {
    return slab + ((((size_t)(g0 + jj) * 2 + (jj == 0 ? s0 : 0)) * 8 + wave) * P8_WAVE_FLOATS + lane * 4 + 4 * I * 256);
  };
  int jj = 0;
  for (; jj + 4 <= np; jj += 4) {
    f32x4_t v[4][4];
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int j = 0; j < 4; ++j) v[u][j] = *reinterpret_cast<const f32x4_t*>(piece(jj + u) + j * 256);
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int j = 0; j < 4; ++j) sum[j] = jj + u == 0 ? v[u][j] : sum[j] + v[u][j];
  }
  for (; jj < np; ++jj) {
    f32x4_t v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = *reinterpret_cast<const f32x4_t*>(piece(jj) + j * 256);
#pragma unroll
    for (int j = 0; j < 4; ++j) sum[j] = jj == 0 ? v[j] : sum[j] + v[j];
  }
  w4_rows<ACT, OUT, I, 4, false>(p, sum, row0, col0, lane, g_w4_sink + lane * 64);
}

template <int ACT, int OUT>
__global__ void __launch_bounds__(512) p8_fixup_kernel(GemmArgs p, P8Tail tl, int nu) {
  const int tt = blockIdx.x, I = blockIdx.y;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int hf = wave >> 2, wq = wave & 3, wr = wq >> 1, wc = wq & 1;
  const int U = tl.units, Gs = tl.gsplit;
  const int g0 = p8_owner((long)tt * nu, Gs, U);
  const int np = p8_owner((long)(tt + 1) * nu - 1, Gs, U) - g0 + 1;
  if (np == 1) return;   // the tile ran whole in one workgroup (epilogue done there)
  const int s0 = p8_start(g0, Gs, U) < tt * nu ? 1 : 0;
  const int nbm = (p.M + W4 - 1) / W4, nbn = (p.N + W4 - 1) / W4;
  int bm, bn;
  w4_tile_coords(tl.dp_tiles + tt, nbm, nbn, bm, bn);
  const long row0 = (long)bm * W4 + wr * 128, col0 = (long)bn * W4 + wc * 128 + hf * 64;
  switch (I) {
    case 0: p8_fixup_rows<ACT, OUT, 0>(p, tl.slab, g0, np, s0, wave, row0, col0, lane); break;
    case 1: p8_fixup_rows<ACT, OUT, 1>(p, tl.slab, g0, np, s0, wave, row0, col0, lane); break;
    case 2: p8_fixup_rows<ACT, OUT, 2>(p, tl.slab, g0, np, s0, wave, row0, col0, lane); break;
    case 3: p8_fixup_rows<ACT, OUT, 3>(p, tl.slab, g0, np, s0, wave, row0, col0, lane); break;
    case 4: p8_fixup_rows<ACT, OUT, 4>(p, tl.slab, g0, np, s0, wave, row0, col0, lane); break;
    case 5: p8_fixup_rows<ACT, OUT, 5>(p, tl.slab, g0, np, s0, wave, row0, col0, lane); break;
    case 6: p8_fixup_rows<ACT, OUT, 6>(p, tl.slab, g0, np, s0, wave, row0, col0, lane); break;
    default: p8_fixup_rows<ACT, OUT, 7>(p, tl.slab, g0, np, s0, wave, row0, col0, lane); break;
  }
}

int launch_p8_fixup(const GemmArgs& a, int act, int out, const P8Tail& tl, hipStream_t st) {
  const long ntile = (long)((a.M + W4 - 1) / W4) * ((a.N + W4 - 1) / W4);
  const dim3 grid((unsigned)(ntile - tl.dp_tiles), 8);
  const int nu = a.K / W4_KT / 2;
  if (act != ACT_NONE) return set_error("p8 fixup: ACT_NONE only");
  if (out == OUT_BF16) hipLaunchKernelGGL((p8_fixup_kernel<ACT_NONE, OUT_BF16>), grid, dim3(512), 0, st, a, tl, nu);
  else if (out == OUT_F32) hipLaunchKernelGGL((p8_fixup_kernel<ACT_NONE, OUT_F32>), grid, dim3(512), 0, st, a, tl, nu);
  else hipLaunchKernelGGL((p8_fixup_kernel<ACT_NONE, OUT_F32_BFR>), grid, dim3(512), 0, st, a, tl, nu);
  return hipGetLastError() == hipSuccess ? 0 : set_error("p8 fixup launch failed");
}

// the p8 path takes what the w4 path takes, at K >= 128 (a tile's first and last k-step pairs are peeled)
bool p8_supported(const GemmArgs& a, int act, int out) { return a.K >= 128 && w4_supported(a, act, out); }

// stream-K tail scratch (P8Tail): the arrival counters first (zeroed by p8_tail_scratch_zero at the start of
// every model-level call that uses it; each launch leaves them zero), then the partial slabs
constexpr size_t P8_CNT_BYTES = 16384;
size_t p8_tail_scratch_bytes() {
  num_cu();
  return P8_CNT_BYTES + (size_t)g_num_cu * 2 * 8 * P8_WAVE_FLOATS * sizeof(float);
}

// the stream-K plan of a launch.  Cost model of the tail round, in K-tiles of one workgroup (a 256x256x64 step,
// ~1.3 us): unsplit, nt; split over Gs workgroups, ceil(U / Gs) plus the partial writes of a workgroup's (at most
// two) cut pieces (a 256-KiB slab each, ~1 K-tile) and the fixup launch (~5 K-tiles).  The cheapest Gs is taken
// when it saves >= 10 % of the round.
size_t p8_slab_bytes(long G) { return (size_t)G * 2 * 8 * P8_WAVE_FLOATS * sizeof(float); }
P8Tail p8_tail_plan_ws(const GemmArgs& a, long ntile, long G, void* slab, long max_t0, long max_t1) {
  P8Tail tl;
  const long R = ntile / G, T = ntile - R * G, nt = a.K / W4_KT;
  if (!slab || T == 0 || (nt & 1)) return tl;
  if (!((R == 0 && T <= max_t0) || (R == 1 && T <= max_t1))) return tl;
  const long U = T * (nt / 2);                                // tail units: pairs of K-tiles
  double best = (double)nt * 0.9;
  long bestG = 0;
  for (long gs = T + 1; gs <= G; ++gs) {
    const long per = (U + gs - 1) / gs;                       // units of the busiest workgroup
    if (U / gs < 1) break;                                    // (every workgroup >= 1 unit)
    const double cost = 2.0 * (double)per + 2.0 + 5.0;
    if (cost < best - 1e-9) { best = cost; bestG = gs; }
  }
  if (!bestG || R + 3 > 64 || G > 1023 || ntile > 65535) return tl;   // the kernel's per-lane segment table
  tl.dp_tiles = (int)(R * G);
  tl.units = (int)U;
  tl.gsplit = (int)bestG;
  tl.slab = (float*)slab;
  return tl;
}

// the 8-wave kernel's plan: the scratch of the descriptor or the model-level scope (slabs after the counters).
// Long K only (K >= 4096: the fixup launch and the partial writes cost a few K-tiles), and a tail the split
// shortens without losing the lock-step L2 sharing of a round: a grid of at most 64 tiles, or one full round plus
// at most 128.  Measured (tools/sk_ab.py, r05, same box): SigLIP fc2 0.90x, projector fc2 0.91x, Stage 2's
// down / d(gate|up) dX 0.72 / 0.63x, projector dW1 (160 tiles, no full round) 0.90x; slower where many tiles
// share no full round (projector dW2 200 tiles 1.31x, the Stage-2 SigLIP fc2 144 tiles 1.11x, Gemma's 440-tile
// projections with 184 tail tiles 1.06-1.08x)
static P8Tail p8_tail_plan(const GemmArgs& a, long ntile, long G, int act, int out) {
  void* ws = a.tail_ws ? a.tail_ws : tail_scope();
  if (!ws || act != ACT_NONE || (out != OUT_BF16 && out != OUT_F32 && out != OUT_F32_BFR)) return P8Tail{};
  if (a.K < 4096) return P8Tail{};
#ifndef PTK_SK_MAXT1
#define PTK_SK_MAXT1 128   // A/B builds (make ablib AB_DEFS=-DPTK_SK_MAXT1=..) vary the one-round-plus-tail limit
#endif
  return p8_tail_plan_ws(a, ntile, G, (char*)ws + P8_CNT_BYTES, 64, PTK_SK_MAXT1);
}

// The model-level calls lend their tail scratch to every GEMM they launch (PTK_STREAMK=0 in an A/B build, PTK_AB:
// never, the default dispatch without the tail; r04's opt-in predates the parallel fixup)
static bool streamk_models() { return PTK_AB("PTK_STREAMK", 1) != 0; }
bool streamk_enabled() { return streamk_models(); }
static thread_local void* g_tail_scope = nullptr;
void* tail_scope() { return g_tail_scope; }
TailScratchScope::TailScratchScope(void* ws, hipStream_t st) : prev(g_tail_scope) {
  if (!streamk_models()) ws = nullptr;
  g_tail_scope = ws;   // (the counters ahead of the slabs are unused since the fixup kernel: no zero-fill)
  (void)st;
}
TailScratchScope::~TailScratchScope() { g_tail_scope = prev; }

// the model-level workspaces reserve tail scratch when it will be lent
size_t p8_tail_scratch_bytes_models() { return streamk_models() ? p8_tail_scratch_bytes() : 0; }

int p8_tail_split(const GemmArgs& a, int act, int out) {
  num_cu();
  const long ntile = (long)((a.M + W4 - 1) / W4) * ((a.N + W4 - 1) / W4);
  return p8_tail_plan(a, ntile, g_num_cu, act, out).gsplit;
}

// K-sliced plain fp32 GEMM on the 8-wave kernel (P8Tail::zslices): C[z][M][N] = A[:, zK:(z+1)K] B[:, zK:(z+1)K]^T
// for z < slices, a.K the slice depth; the slices run as S x M rows of persistent tiles in lock-step rounds
// (every slice's tiles share their operand panels through L2), the caller sums the partials.  Plain fp32 out,
// M % 256 == 0 (no tile straddles two slices), byte offsets within 4 GiB.
int launch_gemm_p8_kslices(const GemmArgs& a, int slices, hipStream_t st) {
  num_cu();
  if (slices < 1 || a.M % W4 || a.K < 128 || a.K % W4_KT || a.cmap.g || a.cmap.off || a.amap.g || a.amap.off ||
      a.bias || a.rowadd || a.resid || a.resid16 || a.aux || a.row_stats)
    return set_error("gemm_p8_kslices: unsupported operands");
  if ((double)a.M * a.lda * 2 + (double)slices * a.K * 2 >= 4293918720.0 ||
      (double)a.N * a.ldb * 2 + (double)slices * a.K * 2 >= 4293918720.0)
    return set_error("gemm_p8_kslices: operands past 4 GiB");
  GemmArgs g = a;
  g.M = a.M * slices;
  P8Tail tl;
  tl.zslices = slices;
  const long ntile = (long)(g.M / W4) * ((g.N + W4 - 1) / W4);
  const long grid = std::min<long>(ntile, g_num_cu);
  const uint32_t ab = (uint32_t)std::min<double>((double)a.M * a.lda * 2, 4294967040.0);
  const uint32_t bb = (uint32_t)std::min<double>((double)a.N * a.ldb * 2, 4294967040.0);
  hipLaunchKernelGGL((gemm_p8_kernel<ACT_NONE, OUT_F32, false>), dim3((unsigned)grid), dim3(512), 0, st, g, ab, bb, tl,
                     0u);
  return hipGetLastError() == hipSuccess ? 0 : set_error("gemm_p8_kslices launch failed");
}

// the tile height of a plain / GELU-tanh 8-wave GEMM without a stream-K tail: the TM of {256, 224, 192, 160} with the
// lowest tile rounds x (TM + 128), a tie with 256 rows going to the shorter tile (SigLIP fc1: 6 rounds of 192 = 5 of
// 256; +0.15 % on the cfg2 step over three same-box alternations, profiles/r05_tm160_ab.txt; with a 5 % margin it
// stayed at 256).  The 128 rows' worth per round is what shorter tiles do not shed (prologue, epilogue, the DMA / LDS work per MFMA): fitted to tools/p8_probe.py
// (r05, same box): Gemma o 59.6 / 54.1 / 68.5 us at 256 / 224 / 192 rows, dO 65.8 / 59.5 / 54.4, q|k|v 90.7 / 88.0
// / 81.4, down 340 / 312 / 407, SigLIP fc1 149 / 157 / 153 (on another box 154.7 at 256, 148.1 at 192); 160 rows:
// SigLIP o 52.1 -> 46.4 us (2 rounds of 160 vs 2 of 192), Gemma dO stays at 192 (57.6 vs 70.9), profiles/r05_tm160_ab.txt
int p8_tile_height(const GemmArgs& a, int act, int out) {
  num_cu();
  if (!(act == ACT_NONE || (act == ACT_GELU_TANH && out == OUT_BF16))) return 256;
  const long nbn = (a.N + W4 - 1) / W4, cu = g_num_cu;
  auto cost = [&](long tm) { return (double)((((a.M + tm - 1) / tm) * nbn + cu - 1) / cu) * (double)(tm + 128); };
  const double c256 = cost(256);
  int best = 256;
  double bc = c256;
  for (int tm : {224, 192, 160}) {
    const double c = cost(tm);
    if (c < bc || (c == bc && best == 256)) { bc = c; best = tm; }   // a tie with 256 rows goes to the shorter tile
  }
  return best;
}

template <int TM>
static int launch_p8_short(const GemmArgs& a, int act, int out, hipStream_t st, long grid) {
  const uint32_t ab = (uint32_t)std::min<double>((double)(a.M + a.amap.off) * a.lda * 2, 2147483000.0);
  const uint32_t bb = (uint32_t)std::min<double>((double)a.N * a.ldb * 2, 2147483000.0);
  const P8Tail tl{};
  uint32_t cb = 0;
  if (lean_epilogue_ok(a, act, out, cb)) {
    if (act == ACT_NONE)
      hipLaunchKernelGGL((gemm_p8_kernel<ACT_NONE, OUT_BF16, false, true, TM>), dim3((unsigned)grid), dim3(512), 0,
                         st, a, ab, bb, tl, cb);
    else
      hipLaunchKernelGGL((gemm_p8_kernel<ACT_GELU_TANH, OUT_BF16, false, true, TM>), dim3((unsigned)grid),
                         dim3(512), 0, st, a, ab, bb, tl, cb);
  } else if (act == ACT_GELU_TANH) {
    hipLaunchKernelGGL((gemm_p8_kernel<ACT_GELU_TANH, OUT_BF16, false, false, TM>), dim3((unsigned)grid), dim3(512),
                       0, st, a, ab, bb, tl, 0u);
  } else if (out == OUT_BF16) {
    hipLaunchKernelGGL((gemm_p8_kernel<ACT_NONE, OUT_BF16, false, false, TM>), dim3((unsigned)grid), dim3(512), 0,
                       st, a, ab, bb, tl, 0u);
  } else if (out == OUT_F32) {
    hipLaunchKernelGGL((gemm_p8_kernel<ACT_NONE, OUT_F32, false, false, TM>), dim3((unsigned)grid), dim3(512), 0,
                       st, a, ab, bb, tl, 0u);
  } else {
    hipLaunchKernelGGL((gemm_p8_kernel<ACT_NONE, OUT_F32_BFR, false, false, TM>), dim3((unsigned)grid), dim3(512),
                       0, st, a, ab, bb, tl, 0u);
  }
  return hipGetLastError() == hipSuccess ? 0 : set_error("gemm_p8 launch failed");
}

int launch_gemm_p8(const GemmArgs& a, int act, int out, hipStream_t st, bool sk, int tm) {
  num_cu();
  if (tm != 256 && !sk) {
    if (!(act == ACT_NONE || (act == ACT_GELU_TANH && out == OUT_BF16)))
      return set_error("gemm_p8: %d-row tiles take the plain / GELU-tanh epilogues only", tm);
    if (tm != 224 && tm != 192 && tm != 160) return set_error("gemm_p8: tile height %d (256, 224, 192, 160)", tm);
    const long ntm = (long)((a.M + tm - 1) / tm) * ((a.N + W4 - 1) / W4);
    const long grid = std::min<long>(ntm, g_num_cu);
    if (tm == 224) return launch_p8_short<224>(a, act, out, st, grid);
    if (tm == 192) return launch_p8_short<192>(a, act, out, st, grid);
    return launch_p8_short<160>(a, act, out, st, grid);
  }
  const long ntile = (long)((a.M + W4 - 1) / W4) * ((a.N + W4 - 1) / W4);
  // the stream-K plan only where launch_gemm's gates chose the tail split (its census counts it as p8sk)
  const P8Tail tl = sk ? p8_tail_plan(a, ntile, g_num_cu, act, out) : P8Tail{};
  long grid = tl.units ? g_num_cu : std::min<long>(ntile, g_num_cu);
#ifdef PTK_P8_STAMPS
  if (const char* e = getenv("PTK_GEMM_GRID")) grid = std::min<long>(grid, atol(e));   // diagnostic: fewer CUs
#endif
  const long arows = a.M + a.amap.off;
  const uint32_t ab = (uint32_t)std::min<double>((double)arows * a.lda * 2, 2147483000.0);
  const uint32_t bb = (uint32_t)std::min<double>((double)a.N * a.ldb * 2, 2147483000.0);
  uint32_t cb = 0;
  if (!tl.units && lean_epilogue_ok(a, act, out, cb)) {
#define PTK_P8L_CASE(ACT_)                                                                                   \
    if (act == ACT_)                                                                                         \
      hipLaunchKernelGGL((gemm_p8_kernel<ACT_, OUT_BF16, false, true>), dim3((unsigned)grid), dim3(512), 0, st, a, ab, \
                         bb, tl, cb);
    PTK_P8L_CASE(ACT_NONE)
    PTK_P8L_CASE(ACT_GELU_TANH)
    PTK_P8L_CASE(ACT_GEGLU_BWD)
#undef PTK_P8L_CASE
    return hipGetLastError() == hipSuccess ? 0 : set_error("gemm_p8 launch failed");
  }
#define PTK_P8_CASE(ACT_, OUT_)                                                                       \
  if (act == ACT_ && out == OUT_) {                                                                   \
    hipLaunchKernelGGL((gemm_p8_kernel<ACT_, OUT_, false>), dim3((unsigned)grid), dim3(512), 0, st, a, ab, bb, tl, 0u); \
    return hipGetLastError() == hipSuccess ? 0 : set_error("gemm_p8 launch failed");                  \
  }
#define PTK_P8SK_CASE(ACT_, OUT_)                                                                     \
  if (act == ACT_ && out == OUT_) {                                                                   \
    hipLaunchKernelGGL((gemm_p8_kernel<ACT_, OUT_, true>), dim3((unsigned)grid), dim3(512), 0, st, a, ab, bb, tl, 0u); \
    if (hipGetLastError() != hipSuccess) return set_error("gemm_p8 launch failed");                  \
    return launch_p8_fixup(a, act, out, tl, st);                                                      \
  }
  if (tl.units) {
    if (act == ACT_NONE && lean_epilogue_ok(a, act, out, cb)) {   // whole tiles take the lean epilogue
      hipLaunchKernelGGL((gemm_p8_kernel<ACT_NONE, OUT_BF16, true, true>), dim3((unsigned)grid), dim3(512), 0, st, a,
                         ab, bb, tl, cb);
      if (hipGetLastError() != hipSuccess) return set_error("gemm_p8 launch failed");
      return launch_p8_fixup(a, act, out, tl, st);
    }
    PTK_P8SK_CASE(ACT_NONE, OUT_BF16)
    PTK_P8SK_CASE(ACT_NONE, OUT_F32)
    PTK_P8SK_CASE(ACT_NONE, OUT_F32_BFR)
  }
  PTK_P8_CASE(ACT_NONE, OUT_BF16)
  PTK_P8_CASE(ACT_NONE, OUT_F32)
  PTK_P8_CASE(ACT_NONE, OUT_F32_BFR)
  PTK_P8_CASE(ACT_GELU_TANH, OUT_BF16)
  PTK_P8_CASE(ACT_GELU_ERF, OUT_BF16)
  PTK_P8_CASE(ACT_GEGLU, OUT_BF16)
  PTK_P8_CASE(ACT_GELU_ERF_BWD, OUT_BF16)
  PTK_P8_CASE(ACT_GEGLU_BWD, OUT_BF16)
#undef PTK_P8_CASE
#undef PTK_P8SK_CASE
  return set_error("gemm_p8: unsupported (act=%d, out=%d)", act, out);
}

}  // namespace ptk
