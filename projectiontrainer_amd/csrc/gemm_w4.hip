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

#include <algorithm>
#include <cstdlib>
#include <type_traits>

#ifndef PTK_W4_RDS
#define PTK_W4_RDS 0      // diagnostic builds: fragment-read placement in the k-step (1 = two per group, groups 0..7)
#endif
#ifndef PTK_W4_DMS
#define PTK_W4_DMS 0      // diagnostic builds: DMA placement (1 = groups 8..15, 2 = groups 0..7, 3 = odd groups)
#endif
#ifndef PTK_W4_LINES
#define PTK_W4_LINES 1    // whole 128-B lines in the epilogues (row pairs exchanged by DPP), bit flags: 1 the bf16
                          // stores of the plain / GELU and GEGLU-backward epilogues, 4 the gate|up stores (measured
                          // slower, off); 0 the register layout everywhere (A/B).  (The GEGLU-backward g, u loads as
                          // whole lines measured equal, 500.8 vs 494.1 us, and were removed.)
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

namespace {
constexpr int W4 = 256;                  // output tile edge
constexpr int W4_KT = 64;                // K granularity of the path (a pair of k-steps per barrier)
constexpr int W4_KS = 32;                // k-step depth: one MFMA 16x16x32 deep, one ring slot
constexpr int W4_SOPB = W4 * W4_KS * 2;  // one operand's k-step image: 256 rows x 64 B = 16 KiB
constexpr int W4_SLOT = 2 * W4_SOPB;     // A + B per ring slot
constexpr int W4_NSLOT = 5;              // ring depth: 5 x 32 KiB = the CU's 160 KiB of LDS
constexpr uint32_t W4_OOB = 0x80000000u; // voffset beyond every buffer's num_records -> zeros
typedef __attribute__((address_space(3))) void* lds_ptr_t;

__device__ char g_w4_sink[64 * 64];      // store target of rows/columns outside C (64 B per lane)

// RowMap in 32-bit arithmetic (every row index of the step fits an int; 64-bit division is a
// software routine on gfx950)
PTK_DEV int map_row32(const RowMap& m, int r) {
  if (m.g == 0) return r + (int)m.off;
  const int q = (int)((unsigned)r / (unsigned)m.g), s = r - q * m.g;
  if (s < m.skip) return -1;
  return q * (int)m.gs + s + (int)m.off;
}

PTK_DEV void add8(float* v, const float* s) {
  const float4 a = *reinterpret_cast<const float4*>(s), b = *reinterpret_cast<const float4*>(s + 4);
  v[0] += a.x; v[1] += a.y; v[2] += a.z; v[3] += a.w; v[4] += b.x; v[5] += b.y; v[6] += b.z; v[7] += b.w;
}

// diagnostic build (make ablib AB_NAME=p8stamps AB_SRC=gemm_w4.hip AB_DEFS=-DPTK_P8_STAMPS; tools/p8_stamps.py):
// s_memtime stamps of wave 0 of the persistent GEMMs (w4 and p8) per segment -- 0 segment start, 1 first K-tile done (its end wait passed), 2 K loop
// done, 3 epilogue issued -- kept in VGPR lanes (lane = segment) so no memory op enters the counted vmcnt
// pipeline, written at the end; g_p8_epi_mode 1 skips the epilogue (wrong results: K-loop-only timing)
#ifdef PTK_P8_STAMPS
__device__ unsigned int g_p8_stamps[1024][4][64];
__device__ int g_p8_epi_mode;
#define P8_STAMP(K, S)                                                                   \
  do {                                                                                   \
    unsigned long long t_;                                                               \
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)); \
    stv_[K] = lane == ((S) & 63) ? (unsigned int)t_ : stv_[K];                           \
  } while (0)
#else
#define P8_STAMP(K, S) (void)0
#endif

// per-lane row state of one row block, computed once for its four 8-column groups: the row's
// validity, its clamped index and the element offsets of its rows in C (after the row map), the
// residual and the side inputs / outputs (the 64-bit products and the row-map division stay out of
// the per-store path)
struct W4Row {
  bool rv;          // r < M
  bool cv;          // r < M and mapped (C row exists)
  long ro_aux;      // rl * ld_aux
  long ro_auxin;    // rl * ld_aux_in
  long ro_rowadd;   // (rl % rowadd_period) * ld_rowadd
  long ro_c;        // cr * ldc
  long ro_resid;    // cr * ld_resid
  long ro_resid16;  // cr * ld_resid16
};
PTK_DEV W4Row w4_row(const GemmArgs& p, long r) {
  W4Row w;
  w.rv = r < p.M;
  const long rl = w.rv ? r : 0;
  const long cr = w.rv ? map_row32(p.cmap, (int)r) : -1;
  w.cv = cr >= 0;
  const long crl = w.cv ? cr : 0;
  w.ro_aux = rl * p.ld_aux;
  w.ro_auxin = rl * p.ld_aux_in;
  w.ro_rowadd = p.rowadd ? (long)((unsigned)rl % (unsigned)p.rowadd_period) * p.ld_rowadd : 0;
  w.ro_c = crl * p.ldc;
  w.ro_resid = crl * p.ld_resid;
  w.ro_resid16 = crl * p.ld_resid16;
  return w;
}

// 8 consecutive columns [c, c+8) of one row (c % 8 == 0); rows r >= M, unmapped rows and columns
// c >= N store into the sink
template <int ACT, int OUT, bool STORE = true>
PTK_DEV void w4_epi8(const GemmArgs& p, const W4Row& w, long c_, float* v, char* sink) {
  const bool cin = c_ < p.N;                // N % 8 == 0: c < N covers all 8 columns
  const bool rv = w.rv && cin, sv = w.cv && cin;
  const long c = cin ? c_ : 0;
  if (p.bias) add8(v, p.bias + c);
  if (p.bf16_linear) {   // bf16(acc + bias) before the row-add / bf16 residual (a bf16 nn.Linear)
#pragma unroll
    for (int e = 0; e < 8; e += 2) {
      const f32x2_t y = bfround2(f32x2_t{v[e], v[e + 1]});
      v[e] = y.x;
      v[e + 1] = y.y;
    }
  }
  if (p.rowadd) add8(v, p.rowadd + w.ro_rowadd + c);
  if constexpr (ACT == ACT_GELU_TANH) {
#pragma unroll
    for (int e = 0; e < 8; e += 2) {
      const f32x2_t y = gelu_tanh2(bfround2(f32x2_t{v[e], v[e + 1]}));
      v[e] = y.x;
      v[e + 1] = y.y;
    }
  } else if constexpr (ACT == ACT_GELU_ERF) {
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = bfround(v[e]);
    if (p.aux) stbf8(rv ? p.aux + w.ro_aux + c : reinterpret_cast<bf16_t*>(sink), v);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = gelu_erf(v[e]);
  } else if constexpr (ACT == ACT_GELU_ERF_BWD) {
    float a[8];
    ldbf8(p.aux_in + w.ro_auxin + c, a);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = bfround(v[e]) * gelu_erf_grad(a[e]);
  }
  if (p.resid) add8(v, p.resid + w.ro_resid + c);
  if (p.resid16) {   // bf16 residual (may alias C: each lane reads its own 8 columns before storing them)
    float r[8];
    ldbf8(sv ? p.resid16 + w.ro_resid16 + c : reinterpret_cast<const bf16_t*>(sink), r);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] += r[e];
  }
  if constexpr (!STORE) {
    return;   // the caller stores v (the whole-line bf16 stores)
  } else if constexpr (OUT == OUT_BF16) {
    stbf8(sv ? reinterpret_cast<bf16_t*>(p.C) + w.ro_c + c : reinterpret_cast<bf16_t*>(sink), v);
  } else {
    if constexpr (OUT == OUT_F32_BFR) {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = bfround(v[e]);
    }
    float* d = sv ? reinterpret_cast<float*>(p.C) + w.ro_c + c : reinterpret_cast<float*>(sink);
    *reinterpret_cast<float4*>(d) = make_float4(v[0], v[1], v[2], v[3]);
    *reinterpret_cast<float4*>(d + 4) = make_float4(v[4], v[5], v[6], v[7]);
  }
}

// Whole-line stores.  In the register layout lane (r = lane & 15, q = lane >> 4) holds 8 consecutive columns of row
// r, so a store instruction writes 16 rows x 64 B: half of each 128-B line, the other half by the next instruction.
// The persistent GEMMs' epilogues took 11-56 k cycles per tile (tools/p8_stamps.py,
// profiles/r04_gemm_epilogue_stamps.jsonl) and the same stores written as whole lines measured ~40 % shorter.  For
// two chunks X (row r, line chunk cx(q)) and Y (row r, line chunk cy(q)) that together cover a line of every row,
// one DPP exchange with lane r ^ 8 (row_ror:8) lets store 1 write rows 0-7 and store 2 rows 8-15 whole: lanes
// r < 8 store X at row r and the partner's X at row r + 8, lanes r >= 8 the partner's Y at row r - 8 and Y at row
// r, both at chunk (r < 8 ? cx : cy).  The row offsets travel the same way.
// keep `old` in lanes r < 8 (HI = false) or r >= 8 (HI = true) of each 16-lane row, take lane r ^ 8's `src` in
// the others: one DPP move (row_ror:8, bank mask = the 4-lane banks written), no select
template <bool HI>
PTK_DEV uint32_t w4_x8(uint32_t old, uint32_t src) {
  return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)src, 0x128, 0xf, HI ? 0x3 : 0xc, false);
}
template <bool HI>
PTK_DEV uint4 w4_x8(const uint4& old, const uint4& src) {
  return uint4{w4_x8<HI>(old.x, src.x), w4_x8<HI>(old.y, src.y), w4_x8<HI>(old.z, src.z), w4_x8<HI>(old.w, src.w)};
}
// store 1 (rows 0-7): X in lanes r < 8, the partner's Y in lanes r >= 8; store 2 (rows 8-15): the partner's X in
// lanes r < 8, Y in lanes r >= 8
PTK_DEV void w4_line_pair(const uint4& X, const uint4& Y, bool, uint4& d1, uint4& d2) {
  d1 = w4_x8<false>(X, Y);
  d2 = w4_x8<true>(Y, X);
}
PTK_DEV uint4 w4_pack8(const float* v) {
  u16x8_t u;
#pragma unroll
  for (int e = 0; e < 8; ++e) u[e] = f2bf(v[e]);
  return __builtin_bit_cast(uint4, u);
}
// row offsets (elements) of the two stores of a row pair, -1 = sink: own is this lane's row (valid flag ok)
PTK_DEV void w4_pair_rows(long own, bool ok, bool, long& o1, long& o2) {
  const uint64_t m = (uint64_t)(ok ? own : -1);
  const uint32_t lo32 = (uint32_t)m, hi32 = (uint32_t)(m >> 32);
  o1 = (long)(((uint64_t)w4_x8<false>(hi32, hi32) << 32) | w4_x8<false>(lo32, lo32));
  o2 = (long)(((uint64_t)w4_x8<true>(hi32, hi32) << 32) | w4_x8<true>(lo32, lo32));
}

// row block I of the wave's tile: lane holds C[row0 + 16I + (lane&15)][col0 + 16j + 4(lane>>4) + e]
// (one function per row block so every accumulator index is a compile-time constant)
template <int ACT, int OUT, int I, int NJ = 8, bool AGPR = true>
PTK_DEV void w4_rows(const GemmArgs& p, f32x4_t (&a)[NJ], long row0, long col0, int lane, char* sink) {
  // pin the accumulator reads to this row block (otherwise hipcc reads all 256 up front and spills); values
  // summed in VGPRs (the stream-K reducer) are pinned there instead
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    if constexpr (AGPR) asm volatile("" : "+a"(a[j]) :: "memory");
    else asm volatile("" : "+v"(a[j]) :: "memory");
  }
  const int q = lane >> 4;
  const int cb = 16 * (q & 1) + 8 * (q >> 1);
  const long r = row0 + 16 * I + (lane & 15);
  if constexpr (ACT == ACT_GEGLU) {
    const W4Row w = w4_row(p, r);
    if constexpr ((PTK_W4_LINES & 4) && NJ == 8) {
      // (bit 4 only: measured slower on gate|up, 710 vs 696 us -- its three outputs' exchanges add VALU
      // to an epilogue that is VALU-heavy already, profiles/r04_gemm_lines_ab.txt)
      // the wave's 64 h columns are one line of every row: X = column pair 0 (line chunk cb / 8), Y = pair 1
      const bool lo = (lane & 8) == 0;
      long a1, a2, c1, c2;
      w4_pair_rows(w.ro_aux, w.rv, lo, a1, a2);
      w4_pair_rows(w.ro_c, w.cv, lo, c1, c2);
      uint4 G[2], U[2], H[2];
#pragma unroll
      for (int pp = 0; pp < 2; ++pp) {
        f32x4_t g0 = a[4 * pp], g1 = a[4 * pp + 2];
        f32x4_t u0 = a[4 * pp + 1], u1 = a[4 * pp + 3];
        swap16(g0, g1);
        swap16(u0, u1);
        const float g[8] = {g0[0], g0[1], g0[2], g0[3], g1[0], g1[1], g1[2], g1[3]};
        const float u[8] = {u0[0], u0[1], u0[2], u0[3], u1[0], u1[1], u1[2], u1[3]};
        uint32_t gp[4], up[4], hp[4];
#pragma unroll
        for (int e = 0; e < 8; e += 2) {
          gp[e / 2] = __builtin_bit_cast(uint32_t, __builtin_convertvector(f32x2_t{g[e], g[e + 1]}, bf16x2_t));
          up[e / 2] = __builtin_bit_cast(uint32_t, __builtin_convertvector(f32x2_t{u[e], u[e + 1]}, bf16x2_t));
          const f32x2_t hh = bfround2(gelu_tanh2(bf2x2(gp[e / 2]))) * bf2x2(up[e / 2]);
          hp[e / 2] = __builtin_bit_cast(uint32_t, __builtin_convertvector(hh, bf16x2_t));
        }
        G[pp] = uint4{gp[0], gp[1], gp[2], gp[3]};
        U[pp] = uint4{up[0], up[1], up[2], up[3]};
        H[pp] = uint4{hp[0], hp[1], hp[2], hp[3]};
      }
      const long hc = col0 / 2 + (lo ? cb : 32 + cb);
      const bool cin = 2 * hc < p.N;
      uint4 d1, d2;
      if (p.aux) {
        w4_line_pair(G[0], G[1], lo, d1, d2);
        *reinterpret_cast<uint4*>(a1 >= 0 && cin ? reinterpret_cast<char*>(p.aux + a1 + hc) : sink) = d1;
        *reinterpret_cast<uint4*>(a2 >= 0 && cin ? reinterpret_cast<char*>(p.aux + a2 + hc) : sink) = d2;
      }
      if (p.aux2) {
        w4_line_pair(U[0], U[1], lo, d1, d2);
        *reinterpret_cast<uint4*>(a1 >= 0 && cin ? reinterpret_cast<char*>(p.aux2 + a1 + hc) : sink) = d1;
        *reinterpret_cast<uint4*>(a2 >= 0 && cin ? reinterpret_cast<char*>(p.aux2 + a2 + hc) : sink) = d2;
      }
      w4_line_pair(H[0], H[1], lo, d1, d2);
      bf16_t* C = reinterpret_cast<bf16_t*>(p.C);
      *reinterpret_cast<uint4*>(c1 >= 0 && cin ? reinterpret_cast<char*>(C + c1 + hc) : sink) = d1;
      *reinterpret_cast<uint4*>(c2 >= 0 && cin ? reinterpret_cast<char*>(C + c2 + hc) : sink) = d2;
      return;
    }
    // GEMM columns: 16-wide gate / up groups alternate (interleaved weights); tiles 4pp, 4pp+2 are
    // gate and 4pp+1, 4pp+3 up for h columns [col0/2 + 32pp, +32)
#pragma unroll
    for (int pp = 0; pp < NJ / 4; ++pp) {
      f32x4_t g0 = a[4 * pp], g1 = a[4 * pp + 2];
      f32x4_t u0 = a[4 * pp + 1], u1 = a[4 * pp + 3];
      swap16(g0, g1);
      swap16(u0, u1);
      const float g[8] = {g0[0], g0[1], g0[2], g0[3], g1[0], g1[1], g1[2], g1[3]};
      const float u[8] = {u0[0], u0[1], u0[2], u0[3], u1[0], u1[1], u1[2], u1[3]};
      // g, u rounded to bf16 once: the packed dwords are stored as they are and unpacked for the math
      uint32_t gp[4], up[4], hp[4];
#pragma unroll
      for (int e = 0; e < 8; e += 2) {
        gp[e / 2] = __builtin_bit_cast(uint32_t, __builtin_convertvector(f32x2_t{g[e], g[e + 1]}, bf16x2_t));
        up[e / 2] = __builtin_bit_cast(uint32_t, __builtin_convertvector(f32x2_t{u[e], u[e + 1]}, bf16x2_t));
        const f32x2_t hh = bfround2(gelu_tanh2(bf2x2(gp[e / 2]))) * bf2x2(up[e / 2]);
        hp[e / 2] = __builtin_bit_cast(uint32_t, __builtin_convertvector(hh, bf16x2_t));
      }
      const long hc = col0 / 2 + 32 * pp + cb;
      const bool cin = 2 * hc < p.N;
      const bool rv = w.rv && cin, sv = w.cv && cin;
      bf16_t* sk = reinterpret_cast<bf16_t*>(sink);
      if (p.aux) *reinterpret_cast<uint4*>(rv ? p.aux + w.ro_aux + hc : sk) = uint4{gp[0], gp[1], gp[2], gp[3]};
      if (p.aux2) *reinterpret_cast<uint4*>(rv ? p.aux2 + w.ro_aux + hc : sk) = uint4{up[0], up[1], up[2], up[3]};
      *reinterpret_cast<uint4*>(sv ? reinterpret_cast<bf16_t*>(p.C) + w.ro_c + hc : sk) = uint4{hp[0], hp[1], hp[2], hp[3]};
    }
  } else {
    const W4Row w = w4_row(p, r);
    if constexpr (OUT == OUT_BF16 && (PTK_W4_LINES & 1)) {
      // column pairs (2m, 2m + 1) = the 64-column line m of every row: X = pair 2m (line chunk cb / 8), Y = 2m + 1
      const bool lo = (lane & 8) == 0;
      long o1, o2;
      w4_pair_rows(w.ro_c, w.cv, lo, o1, o2);
#pragma unroll
      for (int m = 0; m < NJ / 4; ++m) {
        uint4 X, Y;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int pp = 2 * m + h;
          f32x4_t x = a[2 * pp], y = a[2 * pp + 1];
          swap16(x, y);
          float v[8] = {x[0], x[1], x[2], x[3], y[0], y[1], y[2], y[3]};
          w4_epi8<ACT, OUT, false>(p, w, col0 + 32 * pp + cb, v, sink);
          (h ? Y : X) = w4_pack8(v);
        }
        uint4 d1, d2;
        w4_line_pair(X, Y, lo, d1, d2);
        const long c = col0 + 64 * m + (lo ? cb : 32 + cb);
        bf16_t* C = reinterpret_cast<bf16_t*>(p.C);
        *reinterpret_cast<uint4*>(o1 >= 0 && c < p.N ? reinterpret_cast<char*>(C + o1 + c) : sink) = d1;
        *reinterpret_cast<uint4*>(o2 >= 0 && c < p.N ? reinterpret_cast<char*>(C + o2 + c) : sink) = d2;
      }
      return;
    }
#pragma unroll
    for (int pp = 0; pp < NJ / 2; ++pp) {
      f32x4_t x = a[2 * pp], y = a[2 * pp + 1];
      swap16(x, y);
      float v[8] = {x[0], x[1], x[2], x[3], y[0], y[1], y[2], y[3]};
      w4_epi8<ACT, OUT>(p, w, col0 + 32 * pp + cb, v, sink);
    }
  }
}

// GEGLU backward (GEMM output = dh [M, I]; writes dg, du into the interleaved [M, 2I] layout, as
// geglu_bwd_kernel does): the saved g and u of row block I, 8 columns per lane and column pair pp,
// loaded one row block ahead of their use so their latency runs under the previous block's math
template <int I, int NP = 4>
PTK_DEV void w4_gbwd_load(const GemmArgs& p, long row0, long col0, int lane, u16x8_t (&G)[NP], u16x8_t (&U)[NP]) {
  const int q = lane >> 4;
  const int cb = 16 * (q & 1) + 8 * (q >> 1);
  const long r = row0 + 16 * I + (lane & 15);
  const long rl = r < p.M ? r : 0;
#pragma unroll
  for (int pp = 0; pp < NP; ++pp) {
    const long c = col0 + 32 * pp + cb;
    const long cl = c < p.N ? c : 0;
    G[pp] = *reinterpret_cast<const u16x8_t*>(p.aux_in + rl * p.ld_aux_in + cl);
    U[pp] = *reinterpret_cast<const u16x8_t*>(p.aux_in2 + rl * p.ld_aux_in + cl);
  }
}
template <int I, int NP = 4>
PTK_DEV void w4_gbwd_rows(const GemmArgs& p, f32x4_t (&a)[2 * NP], long row0, long col0, int lane, char* sink,
                          const u16x8_t (&G)[NP], const u16x8_t (&U)[NP]) {
#pragma unroll
  for (int j = 0; j < 2 * NP; ++j) asm volatile("" : "+a"(a[j]) :: "memory");
  const int q = lane >> 4;
  const int cb = 16 * (q & 1) + 8 * (q >> 1);
  const long r = row0 + 16 * I + (lane & 15);
  const W4Row w = w4_row(p, r);
#pragma unroll
  for (int pp = 0; pp < NP; ++pp) {
    f32x4_t x = a[2 * pp], y = a[2 * pp + 1];
    swap16(x, y);
    const float v[8] = {x[0], x[1], x[2], x[3], y[0], y[1], y[2], y[3]};
    const uint4 gw = __builtin_bit_cast(uint4, G[pp]), uw = __builtin_bit_cast(uint4, U[pp]);
    const uint32_t gv[4] = {gw.x, gw.y, gw.z, gw.w}, uv[4] = {uw.x, uw.y, uw.z, uw.w};
    float dg[8], du[8];
#pragma unroll
    for (int e = 0; e < 8; e += 2) {   // packed pairs: the same per-element math as gelu_tanh_fg
      const f32x2_t d = bfround2(f32x2_t{v[e], v[e + 1]}), g = bf2x2(gv[e / 2]), u = bf2x2(uv[e / 2]);
      f32x2_t f, df;
      gelu_tanh_fg2(g, f, df);
      const f32x2_t a = bfround2(d * u) * df, b = d * bfround2(f);
      dg[e] = a.x;
      dg[e + 1] = a.y;
      du[e] = b.x;
      du[e + 1] = b.y;
    }
    const long c = col0 + 32 * pp + cb;
    if constexpr (PTK_W4_LINES & 1) {
      // column pair pp = output line pp of every row (64 dg | du columns): X = dg (line chunk 4 (cb >> 4) +
      // ((cb >> 3) & 1)), Y = du (two chunks on)
      const bool lo = (lane & 8) == 0;
      long o1, o2;
      w4_pair_rows(w.ro_c, w.cv, lo, o1, o2);
      uint4 d1, d2;
      w4_line_pair(w4_pack8(dg), w4_pack8(du), lo, d1, d2);
      const long oc = 2 * col0 + 64 * pp + 8 * (4 * (cb >> 4) + ((cb >> 3) & 1) + (lo ? 0 : 2));
      bf16_t* C = reinterpret_cast<bf16_t*>(p.C);
      *reinterpret_cast<uint4*>(o1 >= 0 && c < p.N ? reinterpret_cast<char*>(C + o1 + oc) : sink) = d1;
      *reinterpret_cast<uint4*>(o2 >= 0 && c < p.N ? reinterpret_cast<char*>(C + o2 + oc) : sink) = d2;
      continue;
    }
    bf16_t* o = w.cv && c < p.N ? reinterpret_cast<bf16_t*>(p.C) + w.ro_c + (c >> 4) * 32 + (c & 15)
                                : reinterpret_cast<bf16_t*>(sink);
    stbf8(o, dg);
    stbf8(o + 16, du);
  }
}

// the wave's 128 x 16NJ accumulator tile (8 row blocks of NJ 16x16 MFMA tiles)
template <int ACT, int OUT, int NJ = 8>
PTK_DEV void w4_epilogue(const GemmArgs& p, f32x4_t (&acc)[8][NJ], long row0, long col0, int lane) {
  char* sink = g_w4_sink + lane * 64;
  if constexpr (ACT == ACT_GEGLU_BWD) {
    constexpr int NP = NJ / 2;
    u16x8_t G0[NP], U0[NP], G1[NP], U1[NP];
    w4_gbwd_load<0, NP>(p, row0, col0, lane, G0, U0);
    w4_gbwd_load<1, NP>(p, row0, col0, lane, G1, U1);
    w4_gbwd_rows<0, NP>(p, acc[0], row0, col0, lane, sink, G0, U0);
    w4_gbwd_load<2, NP>(p, row0, col0, lane, G0, U0);
    w4_gbwd_rows<1, NP>(p, acc[1], row0, col0, lane, sink, G1, U1);
    w4_gbwd_load<3, NP>(p, row0, col0, lane, G1, U1);
    w4_gbwd_rows<2, NP>(p, acc[2], row0, col0, lane, sink, G0, U0);
    w4_gbwd_load<4, NP>(p, row0, col0, lane, G0, U0);
    w4_gbwd_rows<3, NP>(p, acc[3], row0, col0, lane, sink, G1, U1);
    w4_gbwd_load<5, NP>(p, row0, col0, lane, G1, U1);
    w4_gbwd_rows<4, NP>(p, acc[4], row0, col0, lane, sink, G0, U0);
    w4_gbwd_load<6, NP>(p, row0, col0, lane, G0, U0);
    w4_gbwd_rows<5, NP>(p, acc[5], row0, col0, lane, sink, G1, U1);
    w4_gbwd_load<7, NP>(p, row0, col0, lane, G1, U1);
    w4_gbwd_rows<6, NP>(p, acc[6], row0, col0, lane, sink, G0, U0);
    w4_gbwd_rows<7, NP>(p, acc[7], row0, col0, lane, sink, G1, U1);
    return;
  }
  w4_rows<ACT, OUT, 0, NJ>(p, acc[0], row0, col0, lane, sink);
  w4_rows<ACT, OUT, 1, NJ>(p, acc[1], row0, col0, lane, sink);
  w4_rows<ACT, OUT, 2, NJ>(p, acc[2], row0, col0, lane, sink);
  w4_rows<ACT, OUT, 3, NJ>(p, acc[3], row0, col0, lane, sink);
  w4_rows<ACT, OUT, 4, NJ>(p, acc[4], row0, col0, lane, sink);
  w4_rows<ACT, OUT, 5, NJ>(p, acc[5], row0, col0, lane, sink);
  w4_rows<ACT, OUT, 6, NJ>(p, acc[6], row0, col0, lane, sink);
  w4_rows<ACT, OUT, 7, NJ>(p, acc[7], row0, col0, lane, sink);
}

// the kernel's own GemmArgs argument (offset 0 of the kernarg segment) behind a pointer the compiler cannot
// see through: the epilogue reloads its fields (s_load) instead of keeping some 30 SGPRs of arguments live
// across the K loop (which spilled SGPRs)
typedef const GemmArgs __attribute__((address_space(4)))* kargs_ptr_t;
PTK_DEV const GemmArgs& kernarg_args() {
#if defined(__HIP_DEVICE_COMPILE__)
  // laundered in the constant address space, so the fields come in by scalar loads (lgkmcnt): a vector load of
  // an argument would make hipcc wait vmcnt(0) before its use, i.e. for every LDS-DMA piece of the next tile
  // the stream already has in flight (r04: -15 % on the gate|up GEMM)
  kargs_ptr_t pk = (kargs_ptr_t)__builtin_amdgcn_kernarg_segment_ptr();
  asm volatile("" : "+s"(pk));
  return *(const GemmArgs*)pk;
#else
  __builtin_unreachable();   // host pass: device code only
#endif
}

PTK_DEV void w4_tile_coords(int t, int nbm, int nbn, int& bm, int& bn) {
  const int per_group = 8 * nbn;
  const int first_m = (t / per_group) * 8;
  const int gsz = min(nbm - first_m, 8);
  bm = first_m + (t % per_group) % gsz;
  bn = (t % per_group) / gsz;
}
}  // namespace

// ---- main-loop primitives as inline asm: hipcc neither reorders volatile asm statements nor splits
// the AGPR accumulators, so the instruction stream below is exactly the source order.  Waits are
// explicit (hipcc does not count asm memory operations): lgkmcnt(0) before a fragment's first MFMA,
// vmcnt before the barrier that publishes an LDS-DMA K-tile.
typedef __attribute__((ext_vector_type(4))) unsigned int u32x4_t;

#define W4_MFMA(ACC, FB, FA) asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(ACC) : "v"(FB), "v"(FA))
#define W4_MFMA0(ACC, FB, FA) asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, 0" : "=a"(ACC) : "v"(FB), "v"(FA))
#define W4_DSREAD(DST, ADDR, OFF) asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(DST) : "v"(ADDR), "i"(OFF))
// one 1-KiB LDS-DMA piece: M0 = wave-uniform LDS destination, passed through the {m0} constraint so that
// hipcc writes M0 itself and knows the asm reads it (an M0 write hidden inside the asm would break any
// M0 value hipcc keeps live, e.g. for an indexed register move or a spill sequence).
// PTK_W4_DMA_POL (diagnostic builds, make w4pol): cache-policy bits on the pieces (1 sc1, 2 sc0, 3 nt);
// measured (tools/gemm_ab.sh, r03): sc1 / sc0 within +-1 % of none on every step shape, nt 2x slower
#if PTK_W4_DMA_POL == 1
#define W4_POL " sc1"
#elif PTK_W4_DMA_POL == 2
#define W4_POL " sc0"
#elif PTK_W4_DMA_POL == 3
#define W4_POL " nt"
#else
#define W4_POL ""
#endif
#define W4_DMA(RSRC, VOFF, SOFF, LDS)                                                                      \
  asm volatile("s_nop 0\n\tbuffer_load_dwordx4 %0, %2, %3 offen" W4_POL " lds"                            \
               :: "v"(VOFF), "{m0}"(LDS), "s"(RSRC), "s"(SOFF) : "memory")

PTK_DEV u32x4_t w4_rsrc(const void* base, uint32_t bytes) {
  const uint64_t a = (uint64_t)base;
  u32x4_t r;
  r[0] = __builtin_amdgcn_readfirstlane((uint32_t)a);
  r[1] = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));   // stride 0: raw buffer
  r[2] = __builtin_amdgcn_readfirstlane(bytes);                  // num_records (bytes)
  r[3] = 0x00020000u;
  return r;
}
PTK_DEV uint32_t lds_addr(const void* p) { return (uint32_t)(uintptr_t)(lds_ptr_t)p; }


template <int ACT, int OUT>
__global__ void __launch_bounds__(256, 1) gemm_w4_kernel(GemmArgs p, uint32_t a_bytes, uint32_t b_bytes) {
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
      w4_epilogue<ACT, OUT>(kernarg_args(), acc, (long)bm * W4 + wr * 128, (long)bn * W4 + wc * 128, lane);
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
#define PTK_W4_CASE(ACT_, OUT_)                                                                   \
  if (act == ACT_ && out == OUT_) {                                                               \
    hipLaunchKernelGGL((gemm_w4_kernel<ACT_, OUT_>), dim3((unsigned)grid), dim3(256), 0, st, a, ab, bb); \
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
// costs its reducer one more 256-KiB partial read): workgroup g < Gs takes the K-tile units
// [g U / Gs, (g + 1) U / Gs) of the tail's U = tail tiles x K-tiles, i.e. the end of one tail tile and / or the
// start of the next.  A tile covered by one workgroup runs the normal epilogue.  A tile split
// over workgroups g0 .. g1 (its pieces, in K order) is finished by the wave that arrives last: every wave of a
// piece writes its 128x64 fp32 partial (32 KiB, write-through `sc1` stores) to its workgroup's slot (slot 0
// for the workgroup's first piece, 1 for its last), drains it (vmcnt(0)) and adds 1 to the (tile, wave)
// arrival counter (agent scope); the wave whose add returns pieces - 1 loads the other pieces' partials
// (`sc1` loads: MI355X_MICROARCH.md's hand-off row "one lane per storing wave, agent atomic add, sc1 stores
// and loads"), sums all pieces in K order (deterministic: the same sum whichever piece arrives last), resets
// the counter (every launch leaves the counters zero) and runs the fused epilogue.  No wave ever waits for
// another workgroup, so the grid needs no co-residency.
struct P8Tail {
  int dp_tiles = 0;           // tiles [0, dp_tiles) run whole (R rounds of G)
  int units = 0;              // U = tail tiles x K-tile pairs (0: no tail split)
  int gsplit = 0;             // Gs: workgroups sharing the tail
  float* slab = nullptr;      // [G][2 slots][8 waves][128 x 64] fp32 partials
  uint32_t* cnt = nullptr;    // [tail tiles][8 waves] arrival counters
};
constexpr size_t P8_WAVE_FLOATS = 128 * 64;

// the tail tile's pieces are summed in K order: piece jj of tile tt belongs to workgroup g0 + jj, whose partial
// sits in its slot 0 if the piece is that workgroup's first (its unit range starts inside the tile), else slot 1
PTK_DEV int p8_owner(long x, int G, int U) { return (int)(((x + 1) * G - 1) / U); }   // workgroup of unit x
PTK_DEV int p8_start(int g, int G, int U) { return (int)(((long)g * U) / G); }

// row block I of the reducer: the tile's partials summed in K order (the reducer's own piece too, read back
// from its slab: the accumulators are dead by then), then the fused epilogue of the row block.  Piece jj of the
// tile belongs to workgroup g0 + jj; its partial sits in that workgroup's slot 0, except piece 0's when the
// workgroup's range started in an earlier tile (s0 = 1: its slot 1)
template <int ACT, int OUT, int I>
PTK_DEV void p8_tail_rows(const GemmArgs& p, const float* slab, int g0, int np, int s0, int wave, long row0,
                          long col0, int lane, char* sink) {
  // sc1 buffer loads through the builtin (hipcc sees them and waits for their data itself: an asm load whose
  // result register hipcc copies before an asm wait reads garbage -- the first version of this reducer did)
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)slab, 0, 0x7fffffff, 0x00020000);
  f32x4_t sum[4];
  for (int jj = 0; jj < np; ++jj) {
    const uint32_t off = (uint32_t)(((((g0 + jj) * 2 + (jj == 0 ? s0 : 0)) * 8 + wave) * (int)P8_WAVE_FLOATS +
                                     lane * 4 + 4 * I * 256) * 4);
#pragma unroll
    for (int j = 0; j < 4; ++j) {   // K order: piece 0, 1, ..
      const f32x4_t v = __builtin_bit_cast(f32x4_t, __builtin_amdgcn_raw_buffer_load_b128(rs, off + j * 1024, 0, 16));
      sum[j] = jj == 0 ? v : sum[j] + v;
    }
  }
  w4_rows<ACT, OUT, I, 4, false>(p, sum, row0, col0, lane, sink);
}

template <int ACT, int OUT>
PTK_DEV void p8_tail_epilogue(const GemmArgs& p, const float* slab, int g0, int np, int s0, int wave, long row0,
                              long col0, int lane) {
  char* sink = g_w4_sink + lane * 64;
  p8_tail_rows<ACT, OUT, 0>(p, slab, g0, np, s0, wave, row0, col0, lane, sink);
  p8_tail_rows<ACT, OUT, 1>(p, slab, g0, np, s0, wave, row0, col0, lane, sink);
  p8_tail_rows<ACT, OUT, 2>(p, slab, g0, np, s0, wave, row0, col0, lane, sink);
  p8_tail_rows<ACT, OUT, 3>(p, slab, g0, np, s0, wave, row0, col0, lane, sink);
  p8_tail_rows<ACT, OUT, 4>(p, slab, g0, np, s0, wave, row0, col0, lane, sink);
  p8_tail_rows<ACT, OUT, 5>(p, slab, g0, np, s0, wave, row0, col0, lane, sink);
  p8_tail_rows<ACT, OUT, 6>(p, slab, g0, np, s0, wave, row0, col0, lane, sink);
  p8_tail_rows<ACT, OUT, 7>(p, slab, g0, np, s0, wave, row0, col0, lane, sink);
}

template <int ACT, int OUT, bool SK>
__global__ void __launch_bounds__(512, 1) gemm_p8_kernel(GemmArgs p, uint32_t a_bytes, uint32_t b_bytes, P8Tail tl) {
  __shared__ __attribute__((aligned(16))) char smem[W4_NSLOT * W4_SLOT];   // 160 KiB: the k-step ring
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
    dsa = __builtin_amdgcn_readfirstlane((uint32_t)(bm * W4 + (int)p.amap.off) * (uint32_t)p.lda * 2u +
                                         (uint32_t)k0 * (W4_KT * 2));
    dsb = __builtin_amdgcn_readfirstlane((uint32_t)(bn * W4) * (uint32_t)p.ldb * 2u + (uint32_t)k0 * (W4_KT * 2));
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
  const uint32_t frag_a = lds_addr(smem) + wr * 128 * 64 + frag_off;
  const uint32_t frag_b = lds_addr(smem) + W4_SOPB + (wc * 128 + hf * 64) * 64 + frag_off;
  bf16x8_t fa[8], fb0[4], fb1[4];
  f32x4_t acc[8][4];

  // all 12 fragments of the k-step in slot rs (after a barrier published it)
  auto read_frags = [&](uint32_t rs) __attribute__((always_inline)) {
    const uint32_t ba = frag_a + rs, bb = frag_b + rs;
#pragma unroll
    for (int r = 0; r < 8; ++r) W4_DSREAD(fa[r], ba, r * 1024);
#pragma unroll
    for (int r = 0; r < 4; ++r) W4_DSREAD(fb0[r], bb, r * 1024);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
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
    for (int q = 0; q < 8; ++q) {
      if (q == 0) asm volatile("s_waitcnt lgkmcnt(6)" ::: "memory");
      else if (q < 3) asm volatile("s_waitcnt lgkmcnt(8)" ::: "memory");
      else if (q == 3) asm volatile("s_waitcnt lgkmcnt(9)" ::: "memory");
      else asm volatile("s_waitcnt lgkmcnt(10)" ::: "memory");
      asm volatile("" : "+v"(fa[q]));
      if (q == 0) asm volatile("" : "+v"(FB[0]), "+v"(FB[1]), "+v"(FB[2]), "+v"(FB[3]));
      if (rd && q < 4) W4_DSREAD(NB[q], bb, q * 1024);
      if ((q & 1) == half) {
        const int pc = q >> 1;   // pieces A0 B0 A1 B1
        if (pc & 1) W4_DMA(rsb, offb[pc >> 1], sb, db + (pc >> 1) * 1024);
        else W4_DMA(rsa, offa[pc >> 1], sa, da + (pc >> 1) * 1024);
      }
      if (PTK_P8_MPRIO) asm volatile("s_setprio 1" ::: "memory");
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) {
        if (first) W4_MFMA0(acc[q][jj], FB[jj], fa[q]);
        else W4_MFMA(acc[q][jj], FB[jj], fa[q]);
      }
      if (PTK_P8_MPRIO) asm volatile("s_setprio 0" ::: "memory");
      if (rd && q >= 1) W4_DSREAD(fa[q - 1], ba, (q - 1) * 1024);   // one group after its last reader
    }
    if (rd) W4_DSREAD(fa[7], ba, 7 * 1024);
  };

  // stream-K hand-off of one wave's 128x64 partial (P8Tail): returns true when this wave arrived last and must
  // sum the pieces and run the epilogue
  auto tail_arrive = [&](int tt, int np, int slot) __attribute__((always_inline)) -> bool {
    float* mine = tl.slab + (((size_t)loc * 2 + slot) * 8 + wave) * P8_WAVE_FLOATS + lane * 4;
#pragma unroll
    for (int q = 0; q < 8; ++q)
#pragma unroll
      for (int jj = 0; jj < 4; ++jj)
        asm volatile("global_store_dwordx4 %0, %1, off sc1" :: "v"(mine + (4 * q + jj) * 256), "a"(acc[q][jj])
                     : "memory");   // straight from the AGPRs (a VGPR copy invites hipcc to re-home acc)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    uint32_t old = 0;
    if (lane == 0)
      old = __hip_atomic_fetch_add(tl.cnt + tt * 8 + wave, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    old = __builtin_amdgcn_readfirstlane(old);
    return (int)old == np - 1;
  };

#ifdef PTK_P8_STAMPS
  unsigned int stv_[4] = {0u, 0u, 0u, 0u};
  const int em_ = g_p8_epi_mode;
#endif
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
        W4_DMA(rsa, offa[j], sa, da + j * 1024);
        W4_DMA(rsb, offb[j], sb, db + j * 1024);
      }
      dma_advance();
    }
    asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    read_frags(0);
    __builtin_amdgcn_s_barrier();
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
      asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      __builtin_amdgcn_s_barrier();
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
      const long row0 = (long)bm * W4 + wr * 128, col0 = (long)bn * W4 + wc * 128 + hf * 64;
      if (!SK || tt < 0) {
#ifdef PTK_P8_STAMPS
        if (em_ != 1)
#endif
        w4_epilogue<ACT, OUT, 4>(kernarg_args(), acc, row0, col0, lane);
      } else if constexpr (SK) {
        const uint32_t c = __builtin_amdgcn_readlane(segC, s);
        const int g0 = (int)(c & 1023u), np = (int)((c >> 10) & 1023u), s0 = (int)((c >> 20) & 1u);
        if (tail_arrive(tt, np, (int)((c >> 21) & 1u))) {
          // agent-scope acquire before reading the other pieces (the hand-off is per wave with the counter's
          // returned value as the signal, not one of MI355X_MICROARCH.md's measured sc1-only rows; the
          // invalidate also drops any line of the slab an earlier launch left in this XCD's caches)
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          p8_tail_epilogue<ACT, OUT>(kernarg_args(), tl.slab, g0, np, s0, wave, row0, col0, lane);
          if (lane == 0) __hip_atomic_store(tl.cnt + tt * 8 + wave, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
      }
      P8_STAMP(3, s);
      // the next segment's first k-step (published by the barrier; harmless after the last).  Its slot is the
      // one the NEXT pair's second k-step restages (k-step i+6 lands in the slot of i+1), so a barrier keeps
      // a wave that finished its epilogue early from overwriting it before every wave has read it
      read_frags(rs);
      __builtin_amdgcn_s_barrier();
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
// ~1.7 us): unsplit, nt; split over Gs workgroups, ceil(U / Gs) plus, where a tile is cut, one partial write
// and (pieces - 1) partial reads by its reducer, each ~HANDOFF K-tiles (a 256-KiB slab at the ~70 GB/s one
// workgroup moves across XCDs: ~3.7 us).  The cheapest Gs is taken when it saves >= 10 % of the round.
constexpr double P8_HANDOFF_KTILES = 2.4;
static P8Tail p8_tail_plan(const GemmArgs& a, long ntile, long G, int act, int out) {
  P8Tail tl;
  void* ws = a.tail_ws ? a.tail_ws : tail_scope();   // (the scope is lent only under PTK_STREAMK=1)
  if (!ws || act != ACT_NONE || (out != OUT_BF16 && out != OUT_F32 && out != OUT_F32_BFR)) return tl;
  const long R = ntile / G, T = ntile - R * G, nt = a.K / W4_KT;
  if (T == 0 || T * 8 * 4 > (long)P8_CNT_BYTES || (nt & 1)) return tl;
  // only few tail tiles -- a grid of at most 64 tiles, or one full round plus at most 24: where the tail split
  // measured faster than the same launch unsplit (tools/sk_ab.py, profiles/r04_sk_ab.txt: Stage 2's weight grads
  // and M = 14 336 projections at 0.43-0.80 of the time).  With more tail tiles the pieces of a tile stream
  // different K ranges at the same time, the L2 sharing of a lock-step round is lost, and every Stage-1 shape
  // measured slower (1.1-1.4x)
  if (!((R == 0 && T <= 64) || (R == 1 && T <= 24))) return tl;
  const long U = T * (nt / 2);                                // tail units: pairs of K-tiles
  double best = (double)nt * 0.9;
  long bestG = 0;
  for (long gs = T + 1; gs <= G; ++gs) {
    const long per = (U + gs - 1) / gs;                       // units of the busiest workgroup
    const long lo = U / gs;                                   // units of the least busy (>= 1 needed)
    if (lo < 1) break;
    const long pieces = (nt / 2 + lo - 1) / lo + 1;           // most pieces one tile can be cut into
    const double cost = 2.0 * (double)per + P8_HANDOFF_KTILES * (double)pieces;
    if (cost < best - 1e-9) { best = cost; bestG = gs; }
  }
  if (!bestG || R + 3 > 64 || G > 1023 || ntile > 65535) return tl;   // the kernel's per-lane segment table
  tl.dp_tiles = (int)(R * G);
  tl.units = (int)U;
  tl.gsplit = (int)bestG;
  tl.cnt = (uint32_t*)ws;
  tl.slab = (float*)((char*)ws + P8_CNT_BYTES);
  return tl;
}

// The model-level calls lend their tail scratch only under PTK_STREAMK=1: on the whole step the stream-K tail
// measured slower than the dispatch without it (r04, same box: Stage-2 cfg4 130.7 vs 137.0 img/s against its
// split-K 128x128 weight grads; no Stage-1 shape qualifies), so it stays an opt-in of the model path and a
// per-call option of ptk_gemm (ptk_gemm_desc.tail_ws)
static bool streamk_models() {
  static const bool v = [] { const char* e = getenv("PTK_STREAMK"); return e && e[0] == '1'; }();
  return v;
}
static thread_local void* g_tail_scope = nullptr;
void* tail_scope() { return g_tail_scope; }
TailScratchScope::TailScratchScope(void* ws, hipStream_t st) : prev(g_tail_scope) {
  if (!streamk_models()) ws = nullptr;
  g_tail_scope = ws;
  if (ws) status = launch_zero(ws, P8_CNT_BYTES, st);
}
TailScratchScope::~TailScratchScope() { g_tail_scope = prev; }

// the model-level workspaces reserve tail scratch only when it will be lent (PTK_STREAMK=1)
size_t p8_tail_scratch_bytes_models() { return streamk_models() ? p8_tail_scratch_bytes() : 0; }

int p8_tail_split(const GemmArgs& a, int act, int out) {
  num_cu();
  const long ntile = (long)((a.M + W4 - 1) / W4) * ((a.N + W4 - 1) / W4);
  return p8_tail_plan(a, ntile, g_num_cu, act, out).gsplit;
}

int launch_gemm_p8(const GemmArgs& a, int act, int out, hipStream_t st, bool sk) {
  num_cu();
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
#define PTK_P8_CASE(ACT_, OUT_)                                                                       \
  if (act == ACT_ && out == OUT_) {                                                                   \
    hipLaunchKernelGGL((gemm_p8_kernel<ACT_, OUT_, false>), dim3((unsigned)grid), dim3(512), 0, st, a, ab, bb, tl); \
    return hipGetLastError() == hipSuccess ? 0 : set_error("gemm_p8 launch failed");                  \
  }
#define PTK_P8SK_CASE(ACT_, OUT_)                                                                     \
  if (act == ACT_ && out == OUT_) {                                                                   \
    hipLaunchKernelGGL((gemm_p8_kernel<ACT_, OUT_, true>), dim3((unsigned)grid), dim3(512), 0, st, a, ab, bb, tl); \
    return hipGetLastError() == hipSuccess ? 0 : set_error("gemm_p8 launch failed");                  \
  }
  if (tl.units) {
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
