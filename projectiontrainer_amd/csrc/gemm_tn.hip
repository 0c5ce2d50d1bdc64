// Persistent TN GEMM for gfx950: both operands K-major, as the unfrozen LLM's weight grads read them.
//
//   C[M,N] = A[K,M]^T . B[K,N]      (dW = dY^T X: A = dY [tokens][N_out], B = X [tokens][N_in], row-major)
//
// The weight grads of Stage 2 (Stage2/trainer.py:420-423, the backward through the unfrozen Gemma3) contract over
// the token dimension, which is the ROW dimension of both token-major operands.  The NT kernels need K-contiguous
// rows, so round 3-4 transposed every dY and X first (transpose_rows: 8.6 ms of a 118 ms micro-batch) and ran
// split-K 128x128 GEMMs on the copies.  Here the operands are read where they lie:
//   * gemm_p8_kernel's structure (8 waves, two per SIMD, 256x256 tiles, 128x64 fp32 accumulator per wave, the
//     five-slot k-step ring of 32-deep k-steps, the LDS-DMA stream four k-steps ahead into the next tile, one wait +
//     barrier per pair of k-steps);
//   * a k-step image of an operand is 32 k-rows x 256 columns (512 B per row, 16 KiB): one LDS-DMA piece (64 lanes
//     x 16 B) is two whole k-rows of the token-major matrix, wave w fills k-rows 4w .. 4w + 3 of A and of B;
//   * an MFMA fragment (lane 16G + i: column i of the 16-column block, k = 8G .. 8G + 7) is two ds_read_b64_tr_b16
//     transposed reads of rows 8G + 4r + q (lane 4q + p supplies row q's 8-B piece p of the block's 32-B span);
//     the 16-B chunk of row r sits at chunk ^ tn_swz(r), so the 8 rows one 32-lane half reads land on the 8
//     distinct 32-B slots of the 256-B bank row (the DMA fetches the source chunks in that permuted order, the
//     image stays lane-linear);
//   * K slices: a grid of `slices` copies of the tile set, slice z covering K rows [z kc, (z + 1) kc), each tile
//     of slice z writing fp32 partials to C + z M ldc (summed by splitk_reduce_kernel in slice order:
//     deterministic); one slice writes the bf16 weight-grad accumulate grad = bf16(grad + bf16(acc)) through the
//     lean epilogue (gemm_persist.h).
#include "common.h"
#include "ptk_internal.h"
#include "gemm_epi.h"
#include "gemm_persist.h"

#include <algorithm>
#include <type_traits>

namespace ptk {

namespace {
typedef __attribute__((ext_vector_type(4))) short s16x4_t;
// 16-B chunk swizzle of a k-row: rows differing in bits 0, 1 and 3 (the 8 rows a 32-lane half of a transposed read
// takes) get 8 distinct even XOR values, i.e. 8 distinct 32-B bank slots; row bit 2 (the second read) is free
constexpr int TN_ROW = 512;   // bytes per k-row of an image (256 bf16)
// the ring's barrier, also a compiler fence for the (compiler-visible) fragment reads of the slot it publishes
PTK_DEV void tn_barrier() {
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}
PTK_DEV uint32_t tn_swz(int row) { return 2u * (uint32_t)((row & 3) | (((row >> 3) & 1) << 2)); }

// fp32 partial epilogue of a K slice: the wave's 128 x 64 accumulators (register layout: row lane & 15, 8 columns
// per lane and column pair) stored as they are, rows past M dropped (an out-of-range buffer offset)
PTK_DEV void tn_epilogue_f32(const GemmArgs& p, f32x4_t (&acc)[8][4], long row0, long col0, int lane, uint32_t c_bytes,
                             uint32_t slice_off) {
  if (col0 >= p.N) return;
  const __amdgpu_buffer_rsrc_t rc = __builtin_amdgcn_make_buffer_rsrc(p.C, 0, (int)c_bytes, 0x00020000);
  const int q = lane >> 4;
  const int cb = 16 * (q & 1) + 8 * (q >> 1);
  const uint32_t ldc_bytes = __builtin_amdgcn_readfirstlane((uint32_t)p.ldc * 4u);
  const uint32_t vbase = (uint32_t)(row0 + (lane & 15)) * ldc_bytes + (uint32_t)(col0 + cb) * 4u + slice_off;
#define TN_EP(I)                                                                                                \
  do {                                                                                                          \
    _Pragma("unroll") for (int j = 0; j < 4; ++j) asm volatile("" : "+a"(acc[I][j]) :: "memory");               \
    const bool rv = row0 + 16 * (I) + (lane & 15) < p.M;                                                         \
    const uint32_t vr = rv ? vbase + (uint32_t)(16 * (I)) * ldc_bytes : 0x80000000u;                            \
    _Pragma("unroll") for (int pp = 0; pp < 2; ++pp) {                                                          \
      f32x4_t x = acc[I][2 * pp], y = acc[I][2 * pp + 1];                                                       \
      swap16(x, y);                                                                                              \
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4v_t, x), rc, vr + 128u * pp, 0, 0);        \
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4v_t, y), rc, vr + 128u * pp + 16u, 0, 0);  \
    }                                                                                                            \
  } while (0)
  TN_EP(0); TN_EP(1); TN_EP(2); TN_EP(3); TN_EP(4); TN_EP(5); TN_EP(6); TN_EP(7);
#undef TN_EP
}
}  // namespace

template <int OUT, bool SK>
__global__ void __launch_bounds__(512, 1) gemm_tn_kernel(GemmArgs p, uint32_t a_bytes, uint32_t b_bytes,
                                                          uint32_t c_bytes, int slices, P8Tail tl) {
  __shared__ __attribute__((aligned(16))) char smem[W4_NSLOT * W4_SLOT];   // 160 KiB: the k-step ring
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int hf = wave >> 2, wq = wave & 3, wr = wq >> 1, wc = wq & 1;
  const int nbm = (p.M + W4 - 1) / W4, nbn = (p.N + W4 - 1) / W4;
  const int ntz = nbm * nbn, ntile = ntz * slices;
  const int G = gridDim.x;
  int loc;
  {
    const int b = blockIdx.x, q = G >> 3, rr = G & 7, x = b & 7;
    loc = (x < rr ? x * (q + 1) : rr * (q + 1) + (x - rr) * q) + (b >> 3);
  }
  const int kc = p.K / slices;                             // K rows per slice (a multiple of 64)
  const int nt = kc / W4_KT;                               // 64-deep K-tiles per tile
  // this workgroup's segments: whole tiles loc, loc + G, .. below dp_tiles, then (SK, one slice) its tail pieces:
  // gemm_p8_kernel's stream-K tail (gemm_w4.hip), pieces summed by p8_fixup_kernel
  const int dp_tiles = SK ? tl.dp_tiles : ntile;
  const int n_dp = loc < dp_tiles ? (dp_tiles - loc + G - 1) / G : 0;
  const int U = SK ? tl.units : 0, Gs = SK ? tl.gsplit : 1, nu = nt >> 1;
  const int u0 = SK && loc < Gs ? p8_start(loc, Gs, U) : 0, u1 = SK && loc < Gs ? p8_start(loc + 1, Gs, U) : 0;
  const int n_tail = u1 > u0 ? (u1 - 1) / nu - u0 / nu + 1 : 0;
  const int nseg = n_dp + n_tail;
  if (nseg == 0) return;
  const int total_ks = 2 * n_dp * nt + 4 * (u1 - u0);     // 32-deep k-steps of the workgroup's whole stream
  // segment table (SK): lane i holds segment i -- tile t, tail tile tt + 1 (0: a whole tile), K-tiles [k0, k1) and
  // the slot of a cut piece -- read back by v_readlane at segment boundaries (gemm_p8_kernel's table)
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
      if (np == 1) tt = -1;   // the whole tile in one piece: plain epilogue
    }
    segA = (uint32_t)t | ((uint32_t)(tt + 1) << 16) | ((uint32_t)myslot << 31);
    segB = (uint32_t)k0 | ((uint32_t)k1 << 16);
  }
  // segment s -> tile t (slice z = t / ntz of the tile grid), K-tiles [k0, k1) of its slice, tail tile tt
  auto segment = [&](int s, int& t, int& k0, int& k1, int& tt) __attribute__((always_inline)) {
    if constexpr (!SK) {
      t = loc + s * G; k0 = 0; k1 = nt; tt = -1;
    } else {
      const uint32_t a = __builtin_amdgcn_readlane(segA, s), b = __builtin_amdgcn_readlane(segB, s);
      t = (int)(a & 0xffffu); tt = (int)((a >> 16) & 0x7fffu) - 1;
      k0 = (int)(b & 0xffffu); k1 = (int)(b >> 16);
    }
  };

  const u32x4_t rsa = w4_rsrc(p.A, a_bytes), rsb = w4_rsrc(p.B, b_bytes);
  // global -> LDS: wave w fills k-rows 4w + 2j + (lane >> 5) (j = 0, 1) of both images; lane i of a piece lands at
  // chunk i & 31 of its row and fetches logical chunk (i & 31) ^ tn_swz(row).  The whole source offset goes in the
  // VGPR offset (the buffer range check leaves soffset out): the last tile of an M (N) that is not a multiple of
  // 256 reads past the end of its k-row -- the next row's columns, harmless garbage for output rows past M -- and
  // on the last k-row past the end of the operand, where the range check returns zeros
  uint32_t offa[2], offb[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int row = wave * 4 + 2 * j + (lane >> 5);
    const uint32_t lc = (uint32_t)(lane & 31) ^ tn_swz(row);
    offa[j] = (uint32_t)row * (uint32_t)p.lda * 2u + lc * 16u;
    offb[j] = (uint32_t)row * (uint32_t)p.ldb * 2u + lc * 16u;
  }
  const uint32_t lds_base = __builtin_amdgcn_readfirstlane(lds_addr(smem));
  const uint32_t lds_dma = lds_base + wave * 4 * TN_ROW;
  const uint32_t kstep_a = __builtin_amdgcn_readfirstlane((uint32_t)W4_KS * (uint32_t)p.lda * 2u);
  const uint32_t kstep_b = __builtin_amdgcn_readfirstlane((uint32_t)W4_KS * (uint32_t)p.ldb * 2u);
  // DMA cursor: segment dseg (tile loc + dseg G), k-step dks; past the last k-step it stays put and re-loads that
  // k-step into a free slot (never read), so every k-step issues the same instructions
  int dseg = 0, dks = 0, dlen = 0, dcount = 0;
  uint32_t dsa = 0, dsb = 0;
  auto tile_coords = [&](int t, int& bm, int& bn, int& z) __attribute__((always_inline)) {
    z = t / ntz;
    w4_tile_coords(t - z * ntz, nbm, nbn, bm, bn);
  };
  auto dma_seg = [&](int s) {
    int t, k0, k1, tt, bm, bn, z;
    segment(s, t, k0, k1, tt);
    tile_coords(t, bm, bn, z);
    const uint32_t krow = (uint32_t)z * (uint32_t)kc + (uint32_t)k0 * W4_KT;   // first k-row of the segment
    dsa = __builtin_amdgcn_readfirstlane(krow * (uint32_t)p.lda * 2u + (uint32_t)(bm * W4) * 2u);
    dsb = __builtin_amdgcn_readfirstlane(krow * (uint32_t)p.ldb * 2u + (uint32_t)(bn * W4) * 2u);
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

  // fragment read addresses (slot 0, the first of the two transposed reads; the second is +4 rows = +2048 B):
  // lane 4q + p of group G reads row 8G + q, 8-B piece p of the 16-column block's 32-B span
  uint32_t ra[8], rb[4];
  {
    const int G4 = lane >> 4, q = (lane >> 2) & 3, pp = lane & 3;
    const int row = 8 * G4 + q;
    const uint32_t f = tn_swz(row), rowb = lds_base + (uint32_t)row * TN_ROW + 8u * (pp & 1);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const uint32_t c = (uint32_t)(wr * 16 + 2 * i) + (uint32_t)(pp >> 1);   // 16-B chunk of column wr*128 + 16i
      ra[i] = rowb + ((c ^ f) << 4);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t c = (uint32_t)(wc * 16 + hf * 8 + 2 * j) + (uint32_t)(pp >> 1);
      rb[j] = rowb + W4_SOPB + ((c ^ f) << 4);
    }
  }
  // (compiler-visible loads: hipcc counts them and waits before the MFMA that takes the fragment -- an asm pair
  // would have to be merged into one 128-bit register, a copy hipcc might place before an asm wait)
  auto trread = [](uint32_t addr) __attribute__((always_inline)) {
    typedef __attribute__((address_space(3))) s16x4_t* tr_ptr_t;
    const s16x4_t x0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((tr_ptr_t)(uintptr_t)addr);
    const s16x4_t x1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((tr_ptr_t)(uintptr_t)(addr + 4 * TN_ROW));
    return (bf16x8_t)__builtin_shufflevector(x0, x1, 0, 1, 2, 3, 4, 5, 6, 7);
  };
  bf16x8_t fa[8], fb0[4], fb1[4];
  f32x4_t acc[8][4];

  // all 12 fragments of the k-step in slot rs (after a barrier published it)
  auto read_frags = [&](uint32_t rs) __attribute__((always_inline)) {
#pragma unroll
    for (int r = 0; r < 8; ++r) fa[r] = trread(ra[r] + rs);
#pragma unroll
    for (int r = 0; r < 4; ++r) fb0[r] = trread(rb[r] + rs);
    asm volatile("" : "+v"(fa[0]), "+v"(fa[1]), "+v"(fa[2]), "+v"(fa[3]), "+v"(fa[4]), "+v"(fa[5]),
                 "+v"(fa[6]), "+v"(fa[7]));
    asm volatile("" : "+v"(fb0[0]), "+v"(fb0[1]), "+v"(fb0[2]), "+v"(fb0[3]));
  };

  // one k-step, gemm_p8_kernel's stream: 8 groups of 4 MFMAs (row block q x column blocks 0..3) on fa / FB; the
  // next k-step's B block q read into NB before group q (q < 4) and A block q into fa[q] one group after group q
  // (A7 after the last group).  Two transposed reads per fragment, waited for by hipcc before the fragment's
  // first MFMA (p8's counted waits would double to 12 .. 20, past lgkmcnt's 4-bit field).  The 4 LDS-DMA pieces
  // of k-step + 4 (slot ws) go out in the even (waves 0-3) or odd (waves 4-7) groups.
  auto kstep = [&](auto first_c, auto read_c, auto half_c, bf16x8_t (&FB)[4], bf16x8_t (&NB)[4], uint32_t rs,
                   uint32_t ws) __attribute__((always_inline)) {
    constexpr bool first = decltype(first_c)::value, rd = decltype(read_c)::value;
    constexpr int half = decltype(half_c)::value;
    const uint32_t da = lds_dma + ws, db = da + W4_SOPB;
    const uint32_t sa = dsa + dks * kstep_a, sb = dsb + dks * kstep_b;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      asm volatile("" : "+v"(fa[q]));
      if (q == 0) asm volatile("" : "+v"(FB[0]), "+v"(FB[1]), "+v"(FB[2]), "+v"(FB[3]));
      if (rd && q < 4) NB[q] = trread(rb[q] + rs);
      if ((q & 1) == half) {
        const int pc = q >> 1;   // pieces A0 B0 A1 B1
        if (pc & 1) W4_DMA(rsb, offb[pc >> 1] + sb, 0u, db + (pc >> 1) * 1024);
        else W4_DMA(rsa, offa[pc >> 1] + sa, 0u, da + (pc >> 1) * 1024);
      }
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) {
        if (first) W4_MFMA0(acc[q][jj], FB[jj], fa[q]);
        else W4_MFMA(acc[q][jj], FB[jj], fa[q]);
      }
      if (rd && q >= 1) fa[q - 1] = trread(ra[q - 1] + rs);   // one group after its last reader
    }
    if (rd) fa[7] = trread(ra[7] + rs);
  };

  // stream-K piece of a cut tail tile: the wave's 128x64 fp32 partial to its workgroup's slot (gemm_p8_kernel's)
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
    if (decltype(half_c)::value) __builtin_amdgcn_s_setprio(1);   // p8's static priority of the younger half
    // prologue: k-steps 0..3 into slots 0..3; 0..2 landed and published; fragments of k-step 0 read
    dma_seg(0);
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const uint32_t da = lds_dma + b * W4_SLOT, db = da + W4_SOPB;
      const uint32_t sa = dsa + dks * kstep_a, sb = dsb + dks * kstep_b;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        W4_DMA(rsa, offa[j] + sa, 0u, da + j * 1024);
        W4_DMA(rsb, offb[j] + sb, 0u, db + j * 1024);
      }
      dma_advance();
    }
    asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    tn_barrier();
    read_frags(0);
    tn_barrier();
    uint32_t rs = W4_SLOT, ws = 4 * W4_SLOT;
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
      asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      tn_barrier();
    };
    for (int s = 0; s < nseg; ++s) {
      int t, k0, k1, tt;
      segment(s, t, k0, k1, tt);
      pair(std::true_type{}, std::false_type{});   // (every segment spans >= 2 K-tiles: slices >= 128 deep, tail
      for (int kt = k0 + 1; kt < k1 - 1; ++kt) pair(std::false_type{}, std::false_type{});   // units are pairs)
      pair(std::false_type{}, std::true_type{});
      asm volatile("s_nop 7\n\ts_nop 7" ::: "memory");   // MFMA D -> accumulator read wait states
      int bm, bn, z;
      tile_coords(t, bm, bn, z);
      const long row0 = (long)bm * W4 + wr * 128, col0 = (long)bn * W4 + wc * 128 + hf * 64;
      if (!SK || tt < 0) {
        if constexpr (OUT == OUT_BF16) {
          w4_epilogue_lean<ACT_NONE, 4>(kernarg_args(), acc, row0, col0, lane, c_bytes);
        } else {
          const GemmArgs& pk = kernarg_args();
          tn_epilogue_f32(pk, acc, row0, col0, lane, c_bytes, (uint32_t)z * (uint32_t)pk.M * (uint32_t)pk.ldc * 4u);
        }
      } else if constexpr (SK) {
        tail_store((int)((uint32_t)__builtin_amdgcn_readlane(segA, s) >> 31));   // (readlane is signed)
      }
      // the next segment's first k-step (published by the barrier; harmless after the last); a barrier keeps a
      // wave that finished its epilogue early from overwriting it before every wave has read it
      read_frags(rs);
      tn_barrier();
      rs = slot_next(rs);
    }
  };
  if (hf) run(std::integral_constant<int, 1>{});
  else run(std::integral_constant<int, 0>{});
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // no LDS-DMA may land after the workgroup exits
}

// the TN path takes: 16-B aligned operands with 16-B k-rows, K split into `slices` equal slices of >= 128 rows (a
// multiple of 64), N % 64 == 0, operand extents below 4 GiB and C's below 2^31; OUT_BF16 only with the lean epilogue's form (the weight-grad
// accumulate: bf16_linear + resid16), OUT_F32 the partials of a K split ([slices][M][ldc])
bool tn_supported(const GemmArgs& a, int out, int slices) {
  if (slices < 1 || a.K % (W4_KT * slices) || a.K / slices < 2 * W4_KT) return false;
  if (a.N % 64 || a.lda % 8 || a.ldb % 8 || a.lda < a.M || a.ldb < a.N) return false;
  if (((uintptr_t)a.A | (uintptr_t)a.B | (uintptr_t)a.C) & 15) return false;
  if (a.amap.g || a.amap.off || a.bias || a.rowadd || a.resid || a.aux || a.aux_in || a.row_stats || a.alpha != 1.f)
    return false;
  // operand extents below 4 GiB less 1 MiB: 32-bit buffer offsets and num_records (the tied lm_head's dW reads the
  // 2 GiB d(logits) [4 096][262 144]); the last tile's read past its k-row never wraps
  const double ab = (double)a.K * a.lda * 2, bb = (double)a.K * a.ldb * 2;
  if (ab >= 4293918720.0 || bb >= 4293918720.0) return false;
  if (out == OUT_BF16) {
    uint32_t cb = 0;
    return slices == 1 && lean_epilogue_candidate(a) && lean_epilogue_ok(a, ACT_NONE, OUT_BF16, cb);
  }
  if (out != OUT_F32 || a.ldc % 4 || a.ldc < a.N || a.cmap.g || a.cmap.off || a.resid16 || a.bf16_linear) return false;
  return (double)slices * a.M * a.ldc * 4 < 2147483000.0;
}

// Slice count of a weight grad (a: the OUT_BF16 accumulate form).  Cost in us: the tile rounds of the persistent
// grid, each K / S / 64 K-tiles of ~1.15 us (a 256x256x64 step at ~75 % of one CU's MFMA rate) plus ~4 us of
// epilogue, and for S > 1 the fp32 partials written, read back and reduced with the bf16 accumulate
// ((8 S + 4) M N bytes at ~5 TB/s).  cfg4: dW_gate|up (54 x 5 tiles, K 14 336) 2 slices (partials capped by the
// workspace), dW_down (5 x 27) 1, dW_qkv (6 x 5) and dW_o (5 x 4) 8
int tn_slices(const GemmArgs& a, long part_floats) {
  const long tiles = (long)((a.M + W4 - 1) / W4) * ((a.N + W4 - 1) / W4), cu = device_cus();
  int best = 0;
  double best_us = 0;
  for (int S = 1; S <= 16; S *= 2) {
    GemmArgs f = a;
    int out = OUT_BF16;
    if (S > 1) {
      if ((double)S * a.M * a.N > (double)part_floats) break;
      f.C = reinterpret_cast<void*>((uintptr_t)256);   // (the partials' alignment is the workspace's, checked at launch)
      f.ldc = a.N;
      f.bf16_linear = 0;
      f.resid16 = nullptr;
      f.ld_resid16 = 0;
      out = OUT_F32;
    }
    if (!tn_supported(f, out, S)) continue;
    const long rounds = (tiles * S + cu - 1) / cu;
    const double us = (double)rounds * ((double)a.K / S / W4_KT * 1.15 + 4.0) +
                      (S > 1 ? (8.0 * S + 4.0) * (double)a.M * a.N / 5e6 : 0.0);
    if (!best || us < best_us) { best = S; best_us = us; }
  }
  return best;
}

size_t tn_slab_bytes() { return p8_slab_bytes(device_cus()); }

// the stream-K plan of a one-slice TN GEMM over `slab` (p8_slab_bytes(CUs) bytes): any tail of at most 256 tiles
// without a full round before it (the few-tile weight grads: dW_down 135 tiles, dW_qkv 30, dW_o 20), at most 64
// after one (dW_gate|up: 270 = 256 + 14)
P8Tail tn_tail_plan(const GemmArgs& a, void* slab) {
  const long ntile = (long)((a.M + W4 - 1) / W4) * ((a.N + W4 - 1) / W4);
  return p8_tail_plan_ws(a, ntile, device_cus(), slab, 256, 64);
}

int launch_gemm_tn(const GemmArgs& a, int out, int slices, void* slab, hipStream_t st, long k_rows) {
  if (!tn_supported(a, out, slices)) return set_error("gemm_tn: unsupported operands (M %d N %d K %d slices %d)", a.M, a.N, a.K, slices);
  if (k_rows < 0) k_rows = a.K;
  if (k_rows > a.K || k_rows <= a.K - W4_KT) return set_error("gemm_tn: k_rows %ld outside (K - 64, K] (K %d)", k_rows, a.K);
  const long ntile = (long)((a.M + W4 - 1) / W4) * ((a.N + W4 - 1) / W4) * slices;
  const P8Tail tl = slices == 1 && slab ? tn_tail_plan(a, slab) : P8Tail{};
  const long grid = tl.units ? device_cus() : std::min<long>(ntile, device_cus());
  // num_records end at row k_rows: a K padded to a multiple of 64 reads its last rows as zero
  const uint32_t ab = (uint32_t)((double)k_rows * a.lda * 2), bb = (uint32_t)((double)k_rows * a.ldb * 2);
  uint32_t cb = 0;
  if (out == OUT_BF16) {
    lean_epilogue_ok(a, ACT_NONE, OUT_BF16, cb);
    if (tl.units) {
      hipLaunchKernelGGL((gemm_tn_kernel<OUT_BF16, true>), dim3((unsigned)grid), dim3(512), 0, st, a, ab, bb, cb, 1, tl);
      if (hipGetLastError() != hipSuccess) return set_error("gemm_tn launch failed");
      return launch_p8_fixup(a, ACT_NONE, OUT_BF16, tl, st);
    }
    hipLaunchKernelGGL((gemm_tn_kernel<OUT_BF16, false>), dim3((unsigned)grid), dim3(512), 0, st, a, ab, bb, cb, 1, tl);
  } else {
    cb = (uint32_t)((double)slices * a.M * a.ldc * 4);
    hipLaunchKernelGGL((gemm_tn_kernel<OUT_F32, false>), dim3((unsigned)grid), dim3(512), 0, st, a, ab, bb, cb, slices,
                       tl);
  }
  return hipGetLastError() == hipSuccess ? 0 : set_error("gemm_tn launch failed");
}

}  // namespace ptk
