// Persistent 8-wave NT GEMM with whole-cache-line operand pieces (gfx950): gemm_p8_kernel's tiles, waves,
// MFMA / ds_read stream and epilogues over 64-deep LDS images.
//
// Why: gemm_p8_kernel stages 32-deep k-steps, so one LDS-DMA piece (64 lanes x 16 B) is 16 operand rows x 64 B --
// half a 128-B cache line per row, and every k-step asks the L2 for half-lines.  PMC on 8192^3 (tools/probes/
// tn_vs_nt.py, r05): the 8-wave NT kernel issues 133.5 M TCP->TCC read requests where the token-major TN kernel
// (gemm_tn.hip, whole 512-B k-rows per piece) issues 68.2 M for the same operand bytes, and the TN kernel runs
// 7-15 % faster per K-tile round on long K.  Here a piece is 8 rows x 128 B (whole lines):
//   * an LDS slot is one 64-deep K-tile: A [256 rows][128 B] + B [256 rows][128 B] = 64 KiB; two slots (the CU
//     has 160 KiB), so the DMA of K-tile i + 2 goes into K-tile i's slot as soon as its last fragments are read;
//   * K-tile i = k-steps a (k 0-31) and b (k 32-63).  During a: MFMAs of a, fragment reads of b (same slot).  Then
//     lgkmcnt(0) + vmcnt(0) + one barrier: every wave is done with slot i % 2 and K-tile i + 1 (DMA'd during the
//     previous b) has landed.  During b: MFMAs of b, fragment reads of K-tile i + 1's a (other slot), and the 8
//     DMA pieces per wave of K-tile i + 2 into slot i % 2.  One barrier per K-tile, a DMA latency window of about
//     one K-tile -- gemm_p8_kernel's (k-step j + 4 issued in j, waited at the end of the pair j, j + 1);
//   * 128-B rows need no swizzle: the ds_read_b128 lane groups {0-3,12-15,20-27}, .. of a fragment read (row
//     lane & 15, chunk 4h + lane >> 4) fall on 16 distinct 16-B bank groups (2 row + chunk mod 16).
// Fragments, MFMA order, counted lgkmcnt ladder, the stream-K tail (P8Tail) and every epilogue are
// gemm_p8_kernel's.
#include "common.h"
#include "ptk_internal.h"
#include "gemm_epi.h"
#include "gemm_persist.h"

#include <algorithm>
#include <type_traits>

namespace ptk {

namespace {
constexpr int PW_ROW = 128;                   // bytes per LDS row (64 bf16 of K)
constexpr int PW_OPB = W4 * PW_ROW;           // one operand's K-tile image: 32 KiB
constexpr int PW_SLOT = 2 * PW_OPB;           // A + B
}  // namespace

template <int ACT, int OUT, bool SK, bool LEAN = false>
__global__ void __launch_bounds__(512, 1) gemm_p8w_kernel(GemmArgs p, uint32_t a_bytes, uint32_t b_bytes, P8Tail tl,
                                                          uint32_t c_bytes) {
  __shared__ __attribute__((aligned(16))) char smem[2 * PW_SLOT];   // 128 KiB: two K-tile slots
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int hf = wave >> 2, wq = wave & 3, wr = wq >> 1, wc = wq & 1;
  const int nbm = (p.M + W4 - 1) / W4, nbn = (p.N + W4 - 1) / W4;
  const int ntile = nbm * nbn;
  const int G = gridDim.x;
  int loc;
  {
    const int b = blockIdx.x, q = G >> 3, rr = G & 7, x = b & 7;
    loc = (x < rr ? x * (q + 1) : rr * (q + 1) + (x - rr) * q) + (b >> 3);
  }
  const int nt = p.K / W4_KT;
  const int dp_tiles = SK ? tl.dp_tiles : ntile;
  const int n_dp = loc < dp_tiles ? (dp_tiles - loc + G - 1) / G : 0;
  const int U = SK ? tl.units : 0, Gs = SK ? tl.gsplit : 1, nu = nt >> 1;
  const int u0 = SK && loc < Gs ? p8_start(loc, Gs, U) : 0, u1 = SK && loc < Gs ? p8_start(loc + 1, Gs, U) : 0;
  const int n_tail = u1 > u0 ? (u1 - 1) / nu - u0 / nu + 1 : 0;
  const int nseg = n_dp + n_tail;
  if (nseg == 0) return;
  const int total_kt = n_dp * nt + 2 * (u1 - u0);          // K-tiles of the workgroup's whole stream
  // segment table (SK): gemm_p8_kernel's (tile, tail tile + 1, K-tiles [k0, k1), the cut piece's slot)
  uint32_t segA = 0, segB = 0;
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
    int myslot = 0;
    if (tt >= 0 && i < nseg) {
      const int np = p8_owner((long)(tt + 1) * nu - 1, Gs, U) - p8_owner((long)tt * nu, Gs, U) + 1;
      myslot = u0 < tt * nu ? 1 : 0;
      if (np == 1) tt = -1;
    }
    segA = (uint32_t)t | ((uint32_t)(tt + 1) << 16) | ((uint32_t)myslot << 31);
    segB = (uint32_t)k0 | ((uint32_t)k1 << 16);
  }
  auto segment = [&](int s, int& t, int& k0, int& k1, int& tt) __attribute__((always_inline)) {
    if constexpr (!SK) {
      t = loc + s * G; k0 = 0; k1 = nt; tt = -1;
    } else {
      const uint32_t a = (uint32_t)__builtin_amdgcn_readlane(segA, s), b = (uint32_t)__builtin_amdgcn_readlane(segB, s);
      t = (int)(a & 0xffffu); tt = (int)((a >> 16) & 0x7fffu) - 1;
      k0 = (int)(b & 0xffffu); k1 = (int)(b >> 16);
    }
  };
  const u32x4_t rsa = w4_rsrc(p.A, a_bytes), rsb = w4_rsrc(p.B, b_bytes);

  // global -> LDS: wave w fills rows 32w .. 32w + 31 of both images, 4 + 4 pieces of 8 rows x 128 B; lane i of
  // piece j writes row 32w + 8j + (i >> 3), chunk i & 7 (lane-linear: one whole line per 8 lanes)
  uint32_t offa[4], offb[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const uint32_t r = (uint32_t)(wave * 32 + 8 * j + (lane >> 3));
    offa[j] = r * (uint32_t)p.lda * 2u + (uint32_t)(lane & 7) * 16u;
    offb[j] = r * (uint32_t)p.ldb * 2u + (uint32_t)(lane & 7) * 16u;
  }
  const uint32_t lds_base = __builtin_amdgcn_readfirstlane(lds_addr(smem));
  const uint32_t lds_dma = lds_base + wave * 32 * PW_ROW;
  // DMA cursor (one K-tile at a time): segment dseg, K-tile dkt of its dlen; past the stream's last K-tile it
  // stays put and re-loads that K-tile into the slot nobody reads any more
  int dseg = 0, dkt = 0, dlen = 0, dcount = 0;
  uint32_t dsa = 0, dsb = 0;
  auto dma_seg = [&](int s) {
    int t, k0, k1, tt;
    segment(s, t, k0, k1, tt);
    int bm, bn;
    w4_tile_coords(t, nbm, nbn, bm, bn);
    dsa = __builtin_amdgcn_readfirstlane((uint32_t)(bm * W4 + (int)p.amap.off) * (uint32_t)p.lda * 2u +
                                         (uint32_t)k0 * (W4_KT * 2));
    dsb = __builtin_amdgcn_readfirstlane((uint32_t)(bn * W4) * (uint32_t)p.ldb * 2u + (uint32_t)k0 * (W4_KT * 2));
    dlen = k1 - k0;
  };
  auto dma_advance = [&]() {
    if (++dcount < total_kt) {
      if (++dkt == dlen) {
        dkt = 0;
        dma_seg(++dseg);
      }
    }
  };

  // fragment addresses (slot 0, k-step half 0): lane l reads row (l & 15) of its 16-row block, chunk l >> 4
  const uint32_t frag_off = (uint32_t)(lane & 15) * PW_ROW + (uint32_t)(lane >> 4) * 16u;
  const uint32_t frag_a = lds_base + (uint32_t)(wr * 128) * PW_ROW + frag_off;
  const uint32_t frag_b = lds_base + PW_OPB + (uint32_t)(wc * 128 + hf * 64) * PW_ROW + frag_off;
  bf16x8_t fa[8], fb0[4], fb1[4];
  f32x4_t acc[8][4];

  // all 12 fragments of k-step half h of the K-tile in slot rs
  auto read_frags = [&](uint32_t rs) __attribute__((always_inline)) {
    const uint32_t ba = frag_a + rs, bb = frag_b + rs;
#pragma unroll
    for (int r = 0; r < 8; ++r) W4_DSREAD(fa[r], ba, r * 16 * PW_ROW);
#pragma unroll
    for (int r = 0; r < 4; ++r) W4_DSREAD(fb0[r], bb, r * 16 * PW_ROW);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    asm volatile("" : "+v"(fa[0]), "+v"(fa[1]), "+v"(fa[2]), "+v"(fa[3]), "+v"(fa[4]), "+v"(fa[5]),
                 "+v"(fa[6]), "+v"(fa[7]));
    asm volatile("" : "+v"(fb0[0]), "+v"(fb0[1]), "+v"(fb0[2]), "+v"(fb0[3]));
  };

  // one k-step: gemm_p8_kernel's 8 groups of 4 MFMAs with the next k-step's fragments read from rs (half and
  // slot folded into the address), the same counted lgkmcnt ladder (6, 8, 8, 9, 10, ..).  DMA (the b half only):
  // the wave's 8 pieces of the K-tile two ahead into slot ws, one per group
  auto kstep = [&](auto first_c, auto read_c, auto dma_c, bf16x8_t (&FB)[4], bf16x8_t (&NB)[4], uint32_t rs,
                   uint32_t ws) __attribute__((always_inline)) {
    constexpr bool first = decltype(first_c)::value, rd = decltype(read_c)::value, dm = decltype(dma_c)::value;
    const uint32_t ba = frag_a + rs, bb = frag_b + rs;
    const uint32_t da = lds_dma + ws, db = da + PW_OPB;
    const uint32_t sa = dsa + dkt * (W4_KT * 2), sb = dsb + dkt * (W4_KT * 2);
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      if (q == 0) asm volatile("s_waitcnt lgkmcnt(6)" ::: "memory");
      else if (q < 3) asm volatile("s_waitcnt lgkmcnt(8)" ::: "memory");
      else if (q == 3) asm volatile("s_waitcnt lgkmcnt(9)" ::: "memory");
      else asm volatile("s_waitcnt lgkmcnt(10)" ::: "memory");
      asm volatile("" : "+v"(fa[q]));
      if (q == 0) asm volatile("" : "+v"(FB[0]), "+v"(FB[1]), "+v"(FB[2]), "+v"(FB[3]));
      if (rd && q < 4) W4_DSREAD(NB[q], bb, q * 16 * PW_ROW);
      if constexpr (dm) {   // pieces A0 B0 A1 B1 A2 B2 A3 B3
        const int j = q >> 1;
        if (q & 1) W4_DMA(rsb, offb[j], sb, db + j * 1024);
        else W4_DMA(rsa, offa[j], sa, da + j * 1024);
      }
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) {
        if (first) W4_MFMA0(acc[q][jj], FB[jj], fa[q]);
        else W4_MFMA(acc[q][jj], FB[jj], fa[q]);
      }
      if (rd && q >= 1) W4_DSREAD(fa[q - 1], ba, (q - 1) * 16 * PW_ROW);
    }
    if (rd) W4_DSREAD(fa[7], ba, 7 * 16 * PW_ROW);
  };

  auto tail_store = [&](int slot) __attribute__((always_inline)) {
    float* mine = tl.slab + (((size_t)loc * 2 + slot) * 8 + wave) * P8_WAVE_FLOATS + lane * 4;
#pragma unroll
    for (int q = 0; q < 8; ++q)
#pragma unroll
      for (int jj = 0; jj < 4; ++jj)
        asm volatile("global_store_dwordx4 %0, %1, off" :: "v"(mine + (4 * q + jj) * 256), "a"(acc[q][jj])
                     : "memory");
  };

  auto run = [&](auto half_c) __attribute__((always_inline)) {
    if (decltype(half_c)::value) __builtin_amdgcn_s_setprio(1);   // gemm_p8_kernel's static priority
    // prologue: K-tiles 0 and 1 into slots 0 and 1; K-tile 0 landed and published; its a fragments read
    dma_seg(0);
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      const uint32_t da = lds_dma + b * PW_SLOT, db = da + PW_OPB;
      const uint32_t sa = dsa + dkt * (W4_KT * 2), sb = dsb + dkt * (W4_KT * 2);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        W4_DMA(rsa, offa[j], sa, da + j * 1024);
        W4_DMA(rsb, offb[j], sb, db + j * 1024);
      }
      dma_advance();
    }
    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    read_frags(0);
    uint32_t cur = 0;   // slot of the K-tile being computed
    // one K-tile: k-step a (reads b), wait + barrier, k-step b (reads the next K-tile's a unless last, DMA of the
    // K-tile two ahead into this slot).  Peeled per segment: its first K-tile initialises the accumulators.
    auto ktile = [&](auto first_c, auto last_c) __attribute__((always_inline)) {
      constexpr bool lst = decltype(last_c)::value;
      const uint32_t nxt = cur ^ PW_SLOT;
      kstep(first_c, std::true_type{}, std::false_type{}, fb0, fb1, cur + 64, 0u);
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      kstep(std::false_type{}, std::integral_constant<bool, !lst>{}, std::true_type{}, fb1, fb0, nxt, cur);
      dma_advance();
      cur = nxt;
    };
    for (int s = 0; s < nseg; ++s) {
      int t, k0, k1, tt;
      segment(s, t, k0, k1, tt);
      ktile(std::true_type{}, std::false_type{});   // (every segment spans >= 2 K-tiles: K >= 128, tail units
      for (int kt = k0 + 1; kt < k1 - 1; ++kt) ktile(std::false_type{}, std::false_type{});   // are pairs)
      ktile(std::false_type{}, std::true_type{});
      asm volatile("s_nop 7\n\ts_nop 7" ::: "memory");   // MFMA D -> accumulator read wait states
      int bm, bn;
      w4_tile_coords(t, nbm, nbn, bm, bn);
      const long row0 = (long)bm * W4 + wr * 128, col0 = (long)bn * W4 + wc * 128 + hf * 64;
      if (!SK || tt < 0) {
        if constexpr (LEAN && ACT == ACT_GEGLU_BWD)
          w4_epilogue_lean_glu<ACT, 4>(kernarg_args(), acc, row0, col0, lane, c_bytes);
        else if constexpr (LEAN) w4_epilogue_lean<ACT, 4>(kernarg_args(), acc, row0, col0, lane, c_bytes);
        else w4_epilogue<ACT, OUT, 4>(kernarg_args(), acc, row0, col0, lane);
      } else if constexpr (SK) {
        tail_store((int)((uint32_t)__builtin_amdgcn_readlane(segA, s) >> 31));
      }
      // the next segment's first a fragments (slot cur: landed and published by the last K-tile's barrier); every
      // wave's reads complete (lgkmcnt(0)) before the barrier after which that slot is overwritten
      read_frags(cur);
    }
  };
  if (hf) run(std::integral_constant<int, 1>{});
  else run(std::integral_constant<int, 0>{});
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // no LDS-DMA may land after the workgroup exits
}

bool p8w_supported(const GemmArgs& a, int act, int out) { return p8_supported(a, act, out); }

int launch_gemm_p8w(const GemmArgs& a, int act, int out, hipStream_t st, const P8Tail& tl) {
  const long ntile = (long)((a.M + W4 - 1) / W4) * ((a.N + W4 - 1) / W4);
  const long cu = device_cus();
  const long grid = tl.units ? cu : std::min<long>(ntile, cu);
  const long arows = a.M + a.amap.off;
  const uint32_t ab = (uint32_t)std::min<double>((double)arows * a.lda * 2, 2147483000.0);
  const uint32_t bb = (uint32_t)std::min<double>((double)a.N * a.ldb * 2, 2147483000.0);
  uint32_t cb = 0;
  if (!tl.units && lean_epilogue_ok(a, act, out, cb)) {
#define PW_L(ACT_)                                                                                                 \
    if (act == ACT_)                                                                                               \
      hipLaunchKernelGGL((gemm_p8w_kernel<ACT_, OUT_BF16, false, true>), dim3((unsigned)grid), dim3(512), 0, st, a, \
                         ab, bb, tl, cb);
    PW_L(ACT_NONE)
    PW_L(ACT_GELU_TANH)
    PW_L(ACT_GEGLU_BWD)
#undef PW_L
    return hipGetLastError() == hipSuccess ? 0 : set_error("gemm_p8w launch failed");
  }
  if (tl.units) {
    if (act == ACT_NONE && lean_epilogue_ok(a, act, out, cb)) {
      hipLaunchKernelGGL((gemm_p8w_kernel<ACT_NONE, OUT_BF16, true, true>), dim3((unsigned)grid), dim3(512), 0, st, a,
                         ab, bb, tl, cb);
    } else if (act == ACT_NONE && out == OUT_BF16) {
      hipLaunchKernelGGL((gemm_p8w_kernel<ACT_NONE, OUT_BF16, true>), dim3((unsigned)grid), dim3(512), 0, st, a, ab,
                         bb, tl, 0u);
    } else if (act == ACT_NONE && out == OUT_F32) {
      hipLaunchKernelGGL((gemm_p8w_kernel<ACT_NONE, OUT_F32, true>), dim3((unsigned)grid), dim3(512), 0, st, a, ab,
                         bb, tl, 0u);
    } else if (act == ACT_NONE && out == OUT_F32_BFR) {
      hipLaunchKernelGGL((gemm_p8w_kernel<ACT_NONE, OUT_F32_BFR, true>), dim3((unsigned)grid), dim3(512), 0, st, a,
                         ab, bb, tl, 0u);
    } else {
      return set_error("gemm_p8w: stream-K tail for ACT_NONE only");
    }
    if (hipGetLastError() != hipSuccess) return set_error("gemm_p8w launch failed");
    return launch_p8_fixup(a, act, out, tl, st);
  }
#define PW_CASE(ACT_, OUT_)                                                                                      \
  if (act == ACT_ && out == OUT_) {                                                                              \
    hipLaunchKernelGGL((gemm_p8w_kernel<ACT_, OUT_, false>), dim3((unsigned)grid), dim3(512), 0, st, a, ab, bb, tl, \
                       0u);                                                                                      \
    return hipGetLastError() == hipSuccess ? 0 : set_error("gemm_p8w launch failed");                            \
  }
  PW_CASE(ACT_NONE, OUT_BF16)
  PW_CASE(ACT_NONE, OUT_F32)
  PW_CASE(ACT_NONE, OUT_F32_BFR)
  PW_CASE(ACT_GELU_TANH, OUT_BF16)
  PW_CASE(ACT_GELU_ERF, OUT_BF16)
  PW_CASE(ACT_GEGLU, OUT_BF16)
  PW_CASE(ACT_GELU_ERF_BWD, OUT_BF16)
  PW_CASE(ACT_GEGLU_BWD, OUT_BF16)
#undef PW_CASE
  return set_error("gemm_p8w: unsupported (act=%d, out=%d)", act, out);
}

}  // namespace ptk
