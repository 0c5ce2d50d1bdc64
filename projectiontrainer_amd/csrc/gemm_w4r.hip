// Register-staged operand stream for the persistent 4-wave GEMM (VERDICT r04 item 2's A/B: register-staged
// operands against LDS-DMA pieces).  Everything but the global -> LDS stream is gemm_w4_kernel's: 256x256 tiles
// dealt round-robin over the persistent workgroups, the five-slot ring of 32-deep k-steps, the 16 fragment reads
// of k-step i+1 under the 64 MFMAs of k-step i, one barrier per pair of k-steps, the register epilogues.  The
// stream: each wave's 8 KiB of a k-step (rows 64w..64w+63 of A and B, 16 rows x 64 B per 1-KiB piece, the
// same source swizzle and lane-linear LDS image as w4's DMA pieces) comes in by 8 buffer_load_dwordx4 into
// VGPRs and goes to LDS by 8 ds_write_b128.  Per pair of k-steps (e, e+1): groups 0..7 of k-step e load
// k-steps e+3 and e+4 into two staging sets of 32 VGPRs, groups 8..15 of k-step e+1 store them to slots
// (e+3) % 5 and (e+4) % 5, so a load has ~1.5 k-steps before its store and no staging value crosses the loop's
// back edge (compiler-counted vmcnt stays exact there).
//
// Ring check (e even): slot (e+3) % 5 was last read during k-step e-3 and slot (e+4) % 5 during e-2 (the
// fragments of k-steps e-2 and e-1), both before the pair barrier that ends k-step e-1; the stores (during
// e+1) are published by the barrier that ends e+1, before the fragment reads of k-steps e+3 and e+4 (during
// e+2 and e+3).  Every ds_write is waited (lgkmcnt(0)) at the end of
// its k-step, before any barrier.  The loads are compiler-visible builtins, so hipcc counts vmcnt for them (and
// for the epilogue's stores); there is no asm memory operation besides the stores and fragment reads.
#include "common.h"
#include "ptk_internal.h"
#include "gemm_epi.h"
#include "gemm_persist.h"

#include <algorithm>
#include <cstdlib>
#include <type_traits>

namespace ptk {

#define W4R_DSWRITE(ADDR, DATA, OFF) \
  asm volatile("ds_write_b128 %0, %1 offset:%2" :: "v"(ADDR), "v"(DATA), "i"(OFF) : "memory")

template <int ACT, int OUT, bool LEAN = false>
__global__ void __launch_bounds__(256, 1) gemm_w4r_kernel(GemmArgs p, uint32_t a_bytes, uint32_t b_bytes,
                                                          uint32_t c_bytes) {
  __shared__ __attribute__((aligned(16))) char smem[W4_NSLOT * W4_SLOT];
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
  const int nt = p.K / W4_KT;
  const int nks = 2 * nt;
  const int total_ks = ((ntile - loc + G - 1) / G) * nks;

  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc((void*)p.A, 0, (int)a_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc((void*)p.B, 0, (int)b_bytes, 0x00020000);
  uint32_t offa[4], offb[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int lr = wave * 64 + 16 * j + (lane >> 2);
    const int lc = (lane & 3) ^ ((lane >> 3) & 2);
    offa[j] = (uint32_t)lr * (uint32_t)p.lda * 2u + lc * 16;
    offb[j] = (uint32_t)lr * (uint32_t)p.ldb * 2u + lc * 16;
  }
  // this lane's 16 B of piece j of a slot: lane-linear, as the DMA image
  const uint32_t lds_st = lds_addr(smem) + wave * 64 * 64 + lane * 16;
  // load cursor: tile lt, k-step lks; past the stream's last k-step it stays put (re-loads, never stored
  // where it is read)
  int lt = loc, lks = 0, lcount = 0;
  uint32_t lsa = 0, lsb = 0;
  auto load_tile = [&](int t) {
    int bm, bn;
    w4_tile_coords(t, nbm, nbn, bm, bn);
    lsa = __builtin_amdgcn_readfirstlane((uint32_t)(bm * W4 + (int)p.amap.off) * (uint32_t)p.lda * 2u);
    lsb = __builtin_amdgcn_readfirstlane((uint32_t)(bn * W4) * (uint32_t)p.ldb * 2u);
  };
  auto load_advance = [&]() {
    if (++lcount < total_ks) {
      if (++lks == nks) {
        lks = 0;
        lt += G;
        load_tile(lt);
      }
    }
  };
  // the cursor's k-step as the scalar offsets of its two row panels; the cursor moves on
  struct Cur { uint32_t sa, sb; };
  auto cur_take = [&]() {
    const Cur c{lsa + (uint32_t)lks * (W4_KS * 2), lsb + (uint32_t)lks * (W4_KS * 2)};
    load_advance();
    return c;
  };
  // piece pc = 0..7 of a k-step: A pieces 0, 2, 4, 6, B pieces 1, 3, 5, 7 (w4's DMA order)
  auto load_piece = [&](u32x4v_t (&S)[8], int pc, const Cur& c) {
    if (pc & 1) S[pc] = __builtin_amdgcn_raw_buffer_load_b128(rb, offb[pc >> 1], c.sb, 0);
    else S[pc] = __builtin_amdgcn_raw_buffer_load_b128(ra, offa[pc >> 1], c.sa, 0);
  };
  auto store_piece = [&](const u32x4v_t (&S)[8], int pc, uint32_t ws) {
    const uint32_t a = lds_st + ws + ((pc & 1) ? (uint32_t)W4_SOPB : 0u);
    switch (pc >> 1) {   // the piece offset as the instruction's immediate
      case 0: W4R_DSWRITE(a, S[pc], 0); break;
      case 1: W4R_DSWRITE(a, S[pc], 1024); break;
      case 2: W4R_DSWRITE(a, S[pc], 2048); break;
      default: W4R_DSWRITE(a, S[pc], 3072); break;
    }
  };
  auto slot_next = [](uint32_t s) { s += W4_SLOT; return s == W4_NSLOT * W4_SLOT ? 0u : s; };

  const int frag_off = (lane & 15) * 64 + (((lane >> 4) ^ ((lane >> 1) & 2)) << 4);
  const uint32_t frag_a = lds_addr(smem) + wr * 128 * 64 + frag_off;
  const uint32_t frag_b = lds_addr(smem) + W4_SOPB + wc * 128 * 64 + frag_off;
  bf16x8_t fa0[8], fb0[8], fa1[8], fb1[8];
  f32x4_t acc[8][8];
  u32x4v_t s0[8], s1[8];

#define W4R_GROUP(FA, FB, Q, FIRST)                                                                  \
  do {                                                                                               \
    _Pragma("unroll") for (int jj = 0; jj < 4; ++jj) {                                               \
      if (FIRST) W4_MFMA0(acc[(Q) >> 1][4 * ((Q) & 1) + jj], FB[4 * ((Q) & 1) + jj], FA[(Q) >> 1]); \
      else W4_MFMA(acc[(Q) >> 1][4 * ((Q) & 1) + jj], FB[4 * ((Q) & 1) + jj], FA[(Q) >> 1]);       \
    }                                                                                                \
  } while (0)
#define W4R_READ(FA, FB, BA, BB, Q)                               \
  do {                                                            \
    if ((Q) < 8) W4_DSREAD(FA[(Q) & 7], BA, ((Q) & 7) * 1024);    \
    else W4_DSREAD(FB[(Q) & 7], BB, ((Q) & 7) * 1024);            \
  } while (0)
#define W4R_PIN(FA, FB)                                                                             \
  do {                                                                                              \
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");                                              \
    asm volatile("" : "+v"(FA[0]), "+v"(FA[1]), "+v"(FA[2]), "+v"(FA[3]), "+v"(FA[4]), "+v"(FA[5]),  \
                 "+v"(FA[6]), "+v"(FA[7]));                                                         \
    asm volatile("" : "+v"(FB[0]), "+v"(FB[1]), "+v"(FB[2]), "+v"(FB[3]), "+v"(FB[4]), "+v"(FB[5]),  \
                 "+v"(FB[6]), "+v"(FB[7]));                                                         \
  } while (0)

  // one k-step: w4's 16 MFMA groups and fragment reads of the next k-step (slot rs).  Even k-step e of a pair:
  // the loads of k-steps e+3 (c0 -> s0) and e+4 (c1 -> s1), two per group in groups 0..7; odd k-step e+1: their
  // stores to slots ws0, ws1, two per group in groups 8..15.  The staging registers never cross the loop's
  // back edge (loaded and stored within one pair)
  auto kstep = [&](auto first_c, auto odd_c, const bf16x8_t (&FA)[8], const bf16x8_t (&FB)[8], bf16x8_t (&NA)[8],
                   bf16x8_t (&NB)[8], uint32_t rs, const Cur& c0, const Cur& c1, uint32_t ws0, uint32_t ws1) {
    constexpr bool first = decltype(first_c)::value, odd = decltype(odd_c)::value;
    const uint32_t ba = frag_a + rs, bb = frag_b + rs;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      if (q < 8) {
        W4R_READ(NA, NB, ba, bb, q);
        if constexpr (!odd) {
          load_piece(s0, q, c0);
          load_piece(s1, q, c1);
        }
      } else {
        if (q < 12) {
          W4R_READ(NA, NB, ba, bb, 8 + 2 * (q - 8));
          W4R_READ(NA, NB, ba, bb, 9 + 2 * (q - 8));
        }
        if constexpr (odd) {
          store_piece(s0, q - 8, ws0);
          store_piece(s1, q - 8, ws1);
        }
      }
      W4R_GROUP(FA, FB, q, first);
    }
  };

  // ---- prologue: k-steps 0..2 loaded and stored to slots 0..2
  load_tile(lt);
#pragma unroll
  for (int b = 0; b < 3; ++b) {
    const Cur c = cur_take();
#pragma unroll
    for (int pc = 0; pc < 8; ++pc) load_piece(s0, pc, c);
#pragma unroll
    for (int pc = 0; pc < 8; ++pc) store_piece(s0, pc, (uint32_t)b * W4_SLOT);
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
#pragma unroll
  for (int q = 0; q < 16; ++q) W4R_READ(fa0, fb0, frag_a, frag_b, q);
  W4R_PIN(fa0, fb0);
  __builtin_amdgcn_s_barrier();

  uint32_t rs = W4_SLOT, ws = 3 * W4_SLOT;   // ws: slot of k-step e+3 (e: the pair's even k-step)
  int t = loc, kt = 0;
  for (int g = 0; g < total_ks; g += 2) {
    const Cur c0 = cur_take(), c1 = cur_take();
    const uint32_t ws1 = slot_next(ws);
    if (kt == 0) kstep(std::true_type{}, std::false_type{}, fa0, fb0, fa1, fb1, rs, c0, c1, ws, ws1);
    else kstep(std::false_type{}, std::false_type{}, fa0, fb0, fa1, fb1, rs, c0, c1, ws, ws1);
    W4R_PIN(fa1, fb1);
    rs = slot_next(rs);
    kstep(std::false_type{}, std::true_type{}, fa1, fb1, fa0, fb0, rs, c0, c1, ws, ws1);
    W4R_PIN(fa0, fb0);
    rs = slot_next(rs);
    ws = slot_next(ws1);
    __builtin_amdgcn_s_barrier();
    if (kt == nt - 1) {
      asm volatile("s_nop 7\n\ts_nop 7" ::: "memory");   // MFMA D -> accumulator read wait states
      int bm, bn;
      w4_tile_coords(t, nbm, nbn, bm, bn);
      const long row0 = (long)bm * W4 + wr * 128, col0 = (long)bn * W4 + wc * 128;
      if constexpr (LEAN && ACT == ACT_GEGLU_BWD)
        w4_epilogue_lean_glu<ACT, 8>(kernarg_args(), acc, row0, col0, lane, c_bytes);
      else if constexpr (LEAN) w4_epilogue_lean<ACT, 8>(kernarg_args(), acc, row0, col0, lane, c_bytes);
      else w4_epilogue<ACT, OUT>(kernarg_args(), acc, row0, col0, lane);
      t += G;
      kt = 0;
    } else {
      ++kt;
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#undef W4R_GROUP
#undef W4R_READ
#undef W4R_PIN
}

int launch_gemm_w4r(const GemmArgs& a, int act, int out, hipStream_t st) {
  const long ntile = (long)((a.M + W4 - 1) / W4) * ((a.N + W4 - 1) / W4);
  const long grid = std::min<long>(ntile, device_cus());
  const long arows = a.M + a.amap.off;
  const uint32_t ab = (uint32_t)std::min<double>((double)arows * a.lda * 2, 2147483000.0);
  const uint32_t bb = (uint32_t)std::min<double>((double)a.N * a.ldb * 2, 2147483000.0);
  uint32_t cb = 0;
  if (lean_epilogue_ok(a, act, out, cb)) {
#define PTK_W4RL_CASE(ACT_)                                                                                   \
    if (act == ACT_)                                                                                          \
      hipLaunchKernelGGL((gemm_w4r_kernel<ACT_, OUT_BF16, true>), dim3((unsigned)grid), dim3(256), 0, st, a, ab, bb, cb);
    PTK_W4RL_CASE(ACT_NONE)
    PTK_W4RL_CASE(ACT_GELU_TANH)
    PTK_W4RL_CASE(ACT_GEGLU_BWD)
#undef PTK_W4RL_CASE
    return hipGetLastError() == hipSuccess ? 0 : set_error("gemm_w4r launch failed");
  }
#define PTK_W4R_CASE(ACT_, OUT_)                                                                    \
  if (act == ACT_ && out == OUT_) {                                                                 \
    hipLaunchKernelGGL((gemm_w4r_kernel<ACT_, OUT_>), dim3((unsigned)grid), dim3(256), 0, st, a, ab, bb, 0u); \
    return hipGetLastError() == hipSuccess ? 0 : set_error("gemm_w4r launch failed");              \
  }
  PTK_W4R_CASE(ACT_NONE, OUT_BF16)
  PTK_W4R_CASE(ACT_NONE, OUT_F32)
  PTK_W4R_CASE(ACT_NONE, OUT_F32_BFR)
  PTK_W4R_CASE(ACT_GELU_TANH, OUT_BF16)
  PTK_W4R_CASE(ACT_GELU_ERF, OUT_BF16)
  PTK_W4R_CASE(ACT_GEGLU, OUT_BF16)
  PTK_W4R_CASE(ACT_GELU_ERF_BWD, OUT_BF16)
  PTK_W4R_CASE(ACT_GEGLU_BWD, OUT_BF16)
#undef PTK_W4R_CASE
  return set_error("gemm_w4r: unsupported (act=%d, out=%d)", act, out);
}

}  // namespace ptk
