// Persistent bf16 GEMM whose epilogues run beside another wave's MFMAs (gfx950): two independent 4-wave groups
// per workgroup, each streaming its own 256x128 output tiles, the second group LAG phases behind the first.
//
//   C[M,N] = epi( A[M,K] . B[N,K]^T )   (the persistent kernels' contract: batch 1, alpha = 1, gemm_w4.hip)
//
// Why (DESIGN.md §5, round 4 stamps): the persistent 256x256 kernels lose 18-45 % of every launch to an epilogue
// during which no MFMA issues -- all waves of the CU reach their tile's end together.  Here the waves w and w + 4
// that share a SIMD belong to different groups (group = wave >> 2), and the groups' tile streams are offset, so
// while one group stores a tile (VALU + stores) its SIMD partners keep the matrix pipe busy with their own K loop.
//
//   * group tile 256 x 128; wave (wr, wc) of a group computes rows wr*128 .. +128, columns wc*64 .. +64: a 128x64
//     fp32 accumulator in 128 AGPRs (two waves per SIMD, 256 registers each), the p8 kernel's per-wave tile and
//     register epilogue (gemm_persist.h: whole-line bf16 stores, GELU / GEGLU / GEGLU-backward epilogues);
//   * each group has its own LDS ring of three 32-deep k-step slots (A 256 rows + B 128 rows x 64 B = 24 KiB;
//     2 x 72 KiB in all).  The stream runs two k-steps ahead: k-step i + 2 goes into the slot k-step i - 1 was
//     read from (its reads retired before the barrier that ended k-step i - 1);
//   * every workgroup barrier ends a PHASE, and both groups pass the same barriers: a k-step is two phases (P0:
//     its 12 fragment reads and MFMA groups 0-3; P1: MFMA groups 4-7; 3 LDS-DMA pieces of k-step i + 2 in each),
//     a tile's epilogue is DU_EPI phases (one 16-row block of the wave's accumulators each), so a tile is
//     2 * K/32 + DU_EPI phases.  Group 1 starts DU_LAG phases late (odd: its P0 -- the fragment reads -- always
//     meets group 0's P1 and vice versa; >= DU_EPI: the two groups' epilogues never coincide);
//   * publication: vmcnt(6) at the end of each P1 (the youngest 6 pieces -- k-step i + 3 -- stay in flight)
//     followed by the barrier; a group with nothing to do passes its barriers idle.
// Tiles are dealt over the 2G groups of the grid (group g of workgroup b takes tiles 2b + g, 2b + g + 2G, ..),
// with the XCD-aware workgroup remap and the grouped (GROUP_M = 8) tile order of the other persistent kernels.
#include "common.h"
#include "ptk_internal.h"
#include "gemm_epi.h"
#include "gemm_persist.h"

#include <algorithm>
#include <type_traits>

namespace ptk {

namespace {
constexpr int DU_BN = 128;                          // group tile columns (rows: W4 = 256)
constexpr int DU_SOPA = W4 * W4_KS * 2;             // A k-step image: 256 rows x 64 B = 16 KiB
constexpr int DU_SOPB = DU_BN * W4_KS * 2;          // B k-step image: 128 rows x 64 B = 8 KiB
constexpr int DU_SLOT = DU_SOPA + DU_SOPB;          // 24 KiB
constexpr int DU_NSLOT = 3;
constexpr int DU_RING = DU_NSLOT * DU_SLOT;         // 72 KiB per group
constexpr int DU_EPI = 8;                           // epilogue phases per tile (one 16-row block each)
constexpr int DU_LAG = 9;                           // group 1's start offset in phases (odd, >= DU_EPI)
constexpr int DU_PIECES = 6;                        // LDS-DMA pieces per wave per k-step (4 of A, 2 of B)
#ifndef DU_DMA_EARLY
#define DU_DMA_EARLY 0   // A/B: 1 = all six pieces of k-step i + 2 issued right after the fragment reads of k-step i
#endif
static_assert(DU_LAG % 2 == 1 && DU_LAG >= DU_EPI && DU_EPI % 2 == 0, "phase offsets");
}  // namespace

// SOLO: one group per workgroup (256 threads, 72 KiB of LDS, two workgroups per CU): the same tiles, ring and
// phases, the two groups of a CU independent (their own barriers) instead of LAG phases apart in one workgroup
template <int ACT, int OUT, bool SOLO>
__global__ void __launch_bounds__(SOLO ? 256 : 512, SOLO ? 2 : 1) gemm_dual_kernel(GemmArgs p, uint32_t a_bytes,
                                                                                   uint32_t b_bytes) {
  __shared__ __attribute__((aligned(16))) char smem[(SOLO ? 1 : 2) * DU_RING];   // the groups' rings
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int grp = SOLO ? 0 : wave >> 2, q = wave & 3, wr = q >> 1, wc = q & 1;
  const int nbm = (p.M + W4 - 1) / W4, nbn = (p.N + DU_BN - 1) / DU_BN;
  const int ntile = nbm * nbn;
  const int G = gridDim.x, G2 = SOLO ? G : 2 * G;
  int loc;
  {
    const int b = blockIdx.x, qq = G >> 3, rr = G & 7, x = b & 7;
    loc = (x < rr ? x * (qq + 1) : rr * (qq + 1) + (x - rr) * qq) + (b >> 3);
  }
  const int gid0 = SOLO ? loc : 2 * loc, gid = gid0 + grp;
  const int n0 = gid0 < ntile ? (ntile - gid0 + G2 - 1) / G2 : 0;
  const int n1 = (!SOLO && gid0 + 1 < ntile) ? (ntile - gid0 - 1 + G2 - 1) / G2 : 0;
  const int nmine = grp ? n1 : n0;
  const int nks = p.K / W4_KS;                      // 32-deep k-steps per tile
  const int per_tile = 2 * nks + DU_EPI;            // phases per tile
  const int total = max(n0 * per_tile, n1 ? DU_LAG + n1 * per_tile : 0);
  if (total == 0) return;                           // (n0 == 0 implies n1 == 0: uniform over the workgroup)
  const int lead = (grp && nmine) ? DU_LAG : 0;
  const int trail = total - lead - nmine * per_tile;
  const int total_ks = nmine * nks;

  const u32x4_t rsa = w4_rsrc(p.A, a_bytes), rsb = w4_rsrc(p.B, b_bytes);
  // global -> LDS: wave q of a group fills A rows 64q .. 64q + 63 (4 pieces) and B rows 32q .. 32q + 31 (2 pieces)
  // of each k-step image; lane i of a piece writes LDS row 16j + (i >> 2), 16-B chunk i & 3 and fetches logical
  // chunk (i & 3) ^ ((row >> 1) & 2) (gemm_w4's swizzle: conflict-free fragment reads)
  uint32_t offa[4], offb[2];
  {
    const int lc = (lane & 3) ^ ((lane >> 3) & 2);
#pragma unroll
    for (int j = 0; j < 4; ++j) offa[j] = (uint32_t)(q * 64 + 16 * j + (lane >> 2)) * (uint32_t)p.lda * 2u + lc * 16;
#pragma unroll
    for (int j = 0; j < 2; ++j) offb[j] = (uint32_t)(q * 32 + 16 * j + (lane >> 2)) * (uint32_t)p.ldb * 2u + lc * 16;
  }
  const uint32_t ring = __builtin_amdgcn_readfirstlane(lds_addr(smem)) + grp * DU_RING;
  const uint32_t dma_a = ring + q * 64 * 64, dma_b = ring + DU_SOPA + q * 32 * 64;
  // DMA cursor: tile dt of the group's stream, k-step dks; past the group's last k-step it stays put and the
  // stream re-loads that k-step into a free slot (never read), so every k-step issues the same instructions
  int dt = gid, dks = 0, dcount = 0;
  uint32_t dsa = 0, dsb = 0;
  auto dma_tile = [&](int t) {
    int bm, bn;
    w4_tile_coords(t, nbm, nbn, bm, bn);
    dsa = __builtin_amdgcn_readfirstlane((uint32_t)(bm * W4 + (int)p.amap.off) * (uint32_t)p.lda * 2u);
    dsb = __builtin_amdgcn_readfirstlane((uint32_t)(bn * DU_BN) * (uint32_t)p.ldb * 2u);
  };
  auto dma_advance = [&]() {
    if (++dcount < total_ks) {
      if (++dks == nks) {
        dks = 0;
        dt += G2;
        dma_tile(dt);
      }
    }
  };
  // piece pc of the cursor's k-step into slot ws: 0..3 = A rows 64q + 16pc, 4..5 = B rows 32q + 16(pc - 4)
  auto dma_piece = [&](int pc, uint32_t ws) __attribute__((always_inline)) {
    if (pc < 4) W4_DMA(rsa, offa[pc], dsa + dks * (W4_KS * 2), dma_a + ws + pc * 1024);
    else W4_DMA(rsb, offb[pc - 4], dsb + dks * (W4_KS * 2), dma_b + ws + (pc - 4) * 1024);
  };
  auto slot_next = [](uint32_t s) { s += DU_SLOT; return s == DU_RING ? 0u : s; };

  // fragments: A rows wr*128 + 16i + (lane & 15), B rows wc*64 + 16j + (lane & 15), logical chunk lane >> 4
  const int frag_off = (lane & 15) * 64 + (((lane >> 4) ^ ((lane >> 1) & 2)) << 4);
  const uint32_t frag_a = ring + wr * 128 * 64 + frag_off;
  const uint32_t frag_b = ring + DU_SOPA + wc * 64 * 64 + frag_off;
  bf16x8_t fa[8], fb[4];
  f32x4_t acc[8][4];
  constexpr int order[DU_PIECES] = {0, 4, 1, 2, 5, 3};   // A0 B0 A1 | A2 B1 A3

  // MFMA group g (row block g x column blocks 0..3) once its fragments have landed: the 12 reads are issued in the
  // order B0..B3, A0..A7, so group g waits with lgkmcnt(7 - g) (its A block and every younger read in flight)
#define DU_MGROUP(FIRST, G)                                                                       \
  do {                                                                                            \
    asm volatile("s_waitcnt lgkmcnt(%0)" :: "i"(7 - (G)) : "memory");                             \
    asm volatile("" : "+v"(fa[G]));                                                               \
    if ((G) == 0) asm volatile("" : "+v"(fb[0]), "+v"(fb[1]), "+v"(fb[2]), "+v"(fb[3]));          \
    _Pragma("unroll") for (int jj = 0; jj < 4; ++jj) {                                            \
      if (FIRST) W4_MFMA0(acc[G][jj], fb[jj], fa[G]);                                             \
      else W4_MFMA(acc[G][jj], fb[jj], fa[G]);                                                    \
    }                                                                                             \
  } while (0)
  uint32_t rs = 0;   // slot of the k-step being computed
  // one k-step: P0 (reads + MFMA groups 0-3 + DMA pieces 0-2), barrier, P1 (groups 4-7 + pieces 3-5), the wait that
  // publishes k-step i + 1 (only k-step i + 2's pieces stay in flight), barrier
  auto kstep = [&](auto first_c) __attribute__((always_inline)) {
    const uint32_t ws = slot_next(slot_next(rs));
    const uint32_t ba = frag_a + rs, bb = frag_b + rs;
#pragma unroll
    for (int j = 0; j < 4; ++j) W4_DSREAD(fb[j], bb, j * 1024);
#pragma unroll
    for (int i = 0; i < 8; ++i) W4_DSREAD(fa[i], ba, i * 1024);
    constexpr bool first = decltype(first_c)::value;
    if (DU_DMA_EARLY) {
#pragma unroll
      for (int pc = 0; pc < DU_PIECES; ++pc) dma_piece(order[pc], ws);
    }
    DU_MGROUP(first, 0);
    if (!DU_DMA_EARLY) dma_piece(order[0], ws);
    DU_MGROUP(first, 1);
    if (!DU_DMA_EARLY) dma_piece(order[1], ws);
    DU_MGROUP(first, 2);
    if (!DU_DMA_EARLY) dma_piece(order[2], ws);
    DU_MGROUP(first, 3);
    __builtin_amdgcn_s_barrier();
    DU_MGROUP(first, 4);
    if (!DU_DMA_EARLY) dma_piece(order[3], ws);
    DU_MGROUP(first, 5);
    if (!DU_DMA_EARLY) dma_piece(order[4], ws);
    DU_MGROUP(first, 6);
    if (!DU_DMA_EARLY) dma_piece(order[5], ws);
    DU_MGROUP(first, 7);
    dma_advance();
    asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    rs = slot_next(rs);
  };

  // prologue: k-steps 0 and 1 of the group's stream into slots 0 and 1; k-step 0 landed before the first barrier
  if (nmine) {
    dma_tile(dt);
#pragma unroll
    for (int b = 0; b < 2; ++b) {
#pragma unroll
      for (int pc = 0; pc < DU_PIECES; ++pc) dma_piece(pc, b * DU_SLOT);
      dma_advance();
    }
    asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  }
  __builtin_amdgcn_s_barrier();
  for (int i = 0; i < lead; ++i) __builtin_amdgcn_s_barrier();

  char* sink = g_w4_sink + lane * 64;
  for (int s = 0; s < nmine; ++s) {
    kstep(std::true_type{});
    for (int k = 1; k < nks; ++k) kstep(std::false_type{});
    asm volatile("s_nop 7\n\ts_nop 7" ::: "memory");   // MFMA D -> accumulator read wait states
    int bm, bn;
    w4_tile_coords(gid + s * G2, nbm, nbn, bm, bn);
    const long row0 = (long)bm * W4 + wr * 128, col0 = (long)bn * DU_BN + wc * 64;
    if constexpr (ACT == ACT_GEGLU_BWD) {
      // the saved g, u of row block I + 2 are loaded in phase I, used in phase I + 2 (three blocks in flight)
      u16x8_t G0[2], U0[2], G1[2], U1[2], G2_[2], U2[2];
      const GemmArgs& pa = kernarg_args();
      w4_gbwd_load<0, 2>(pa, row0, col0, lane, G0, U0);
      w4_gbwd_load<1, 2>(pa, row0, col0, lane, G1, U1);
#define DU_GB(I, GA, UA, GN, UN)                                                                  \
  do {                                                                                            \
    const GemmArgs& pk = kernarg_args();                                                          \
    if ((I) + 2 < 8) w4_gbwd_load<((I) + 2) & 7, 2>(pk, row0, col0, lane, GN, UN);                \
    w4_gbwd_rows<I, 2>(pk, acc[I], row0, col0, lane, sink, GA, UA);                               \
    __builtin_amdgcn_s_barrier();                                                                 \
  } while (0)
      DU_GB(0, G0, U0, G2_, U2);
      DU_GB(1, G1, U1, G0, U0);
      DU_GB(2, G2_, U2, G1, U1);
      DU_GB(3, G0, U0, G2_, U2);
      DU_GB(4, G1, U1, G0, U0);
      DU_GB(5, G2_, U2, G1, U1);
      DU_GB(6, G0, U0, G2_, U2);
      DU_GB(7, G1, U1, G0, U0);
#undef DU_GB
    } else {
#define DU_EP(I)                                                                                  \
  do {                                                                                            \
    w4_rows<ACT, OUT, I, 4>(kernarg_args(), acc[I], row0, col0, lane, sink);                      \
    __builtin_amdgcn_s_barrier();                                                                 \
  } while (0)
      DU_EP(0);
      DU_EP(1);
      DU_EP(2);
      DU_EP(3);
      DU_EP(4);
      DU_EP(5);
      DU_EP(6);
      DU_EP(7);
#undef DU_EP
    }
  }
  for (int i = 0; i < trail; ++i) __builtin_amdgcn_s_barrier();
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // no LDS-DMA may land after the workgroup exits
#undef DU_MGROUP
}

// the dual path takes what the persistent kernels take (gemm_w4.hip w4_supported)
bool dual_supported(const GemmArgs& a, int act, int out) { return w4_supported(a, act, out); }

int launch_gemm_dual(const GemmArgs& a, int act, int out, hipStream_t st, bool solo) {
  const long ntile = (long)((a.M + W4 - 1) / W4) * ((a.N + DU_BN - 1) / DU_BN);
  const long grid = solo ? std::min<long>(ntile, 2L * device_cus()) : std::min<long>((ntile + 1) / 2, device_cus());
  if (grid <= 0) return 0;
  const long arows = a.M + a.amap.off;
  const uint32_t ab = (uint32_t)std::min<double>((double)arows * a.lda * 2, 2147483000.0);
  const uint32_t bb = (uint32_t)std::min<double>((double)a.N * a.ldb * 2, 2147483000.0);
#define PTK_DU_CASE(ACT_, OUT_)                                                                       \
  if (act == ACT_ && out == OUT_) {                                                                   \
    if (solo)                                                                                         \
      hipLaunchKernelGGL((gemm_dual_kernel<ACT_, OUT_, true>), dim3((unsigned)grid), dim3(256), 0, st, a, ab, bb); \
    else                                                                                              \
      hipLaunchKernelGGL((gemm_dual_kernel<ACT_, OUT_, false>), dim3((unsigned)grid), dim3(512), 0, st, a, ab, bb); \
    return hipGetLastError() == hipSuccess ? 0 : set_error("gemm_dual launch failed");                \
  }
  PTK_DU_CASE(ACT_NONE, OUT_BF16)
  PTK_DU_CASE(ACT_NONE, OUT_F32)
  PTK_DU_CASE(ACT_NONE, OUT_F32_BFR)
  PTK_DU_CASE(ACT_GELU_TANH, OUT_BF16)
  PTK_DU_CASE(ACT_GELU_ERF, OUT_BF16)
  PTK_DU_CASE(ACT_GEGLU, OUT_BF16)
  PTK_DU_CASE(ACT_GELU_ERF_BWD, OUT_BF16)
  PTK_DU_CASE(ACT_GEGLU_BWD, OUT_BF16)
#undef PTK_DU_CASE
  return set_error("gemm_dual: unsupported (act=%d, out=%d)", act, out);
}

}  // namespace ptk
