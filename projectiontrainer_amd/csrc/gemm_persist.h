// Shared pieces of the persistent GEMM kernels (gemm_w4.hip: 4-wave and 8-wave 256x256; gemm_tn.hip: the token-major
// weight-grad kernel): tile constants, the register epilogues (plain / GELU / GEGLU / GEGLU backward,
// whole-line bf16 stores), the grouped tile order, the laundered kernarg pointer and the inline-asm MFMA /
// ds_read / LDS-DMA primitives.  Included by the .hip files only (device code, anonymous namespace).
#pragma once
#include "common.h"
#include "ptk_internal.h"
#include "gemm_epi.h"

#ifndef PTK_W4_LINES
#define PTK_W4_LINES 1    // whole 128-B lines in the epilogues (row pairs exchanged by DPP), bit flags: 1 the bf16
                          // stores of the plain / GELU and GEGLU-backward epilogues, 4 the gate|up stores (measured
                          // slower, off); 0 the register layout everywhere (A/B).  (The GEGLU-backward g, u loads as
                          // whole lines measured equal, 500.8 vs 494.1 us, and were removed.)
#endif
#ifndef PTK_W4_DMA_POL
#define PTK_W4_DMA_POL 0
#endif

namespace ptk {

typedef __attribute__((ext_vector_type(4))) unsigned int u32x4v_t;

// stream-K tail of the persistent 8-wave kernels (gemm_w4.hip gemm_p8_kernel, gemm_tn.hip gemm_tn_kernel): the
// plan (p8_tail_plan) and the fixup that sums the cut tiles' pieces (launch_p8_fixup), described in gemm_w4.hip
struct P8Tail {
  int dp_tiles = 0;           // tiles [0, dp_tiles) run whole (R rounds of G)
  int units = 0;              // U = tail tiles x K-tile pairs (0: no tail split)
  int gsplit = 0;             // Gs: workgroups sharing the tail
  float* slab = nullptr;      // [G][2 slots][8 waves][128 x 64] fp32 partials
  // K slices as extra row tiles (no tail split): the grid's M = zslices x the real M; virtual row tile bm covers
  // real rows (bm % (nbm / zslices)) x 256 and K rows [z K, (z + 1) K) of the operands (z = bm / (nbm / zslices)),
  // so slice z's fp32 partial lands at output rows z M_real .. (gemm_p8_kslices)
  int zslices = 1;
};
constexpr size_t P8_WAVE_FLOATS = 128 * 64;
// the plan of a GEMM with ntile tiles on a grid of G over scratch ws (nullptr: no split); the tail is split only
// for R == 0 with at most max_t0 tail tiles or R == 1 with at most max_t1
P8Tail p8_tail_plan_ws(const GemmArgs& a, long ntile, long G, void* ws, long max_t0, long max_t1);
size_t p8_slab_bytes(long G);
// the cut tail tiles' pieces summed in K order + the tile epilogue (ACT_NONE; the general epilogue's forms)
int launch_p8_fixup(const GemmArgs& a, int act, int out, const P8Tail& tl, hipStream_t st);

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
        uint32_t gp[4], up[4], hp[4];   // gp / up: the backward's factors a = gelu(g), b = gelu'(g) u
#pragma unroll
        for (int e = 0; e < 8; e += 2)
          geglu_fwd2(bfround2(f32x2_t{g[e], g[e + 1]}), bfround2(f32x2_t{u[e], u[e + 1]}), gp[e / 2], up[e / 2],
                     hp[e / 2]);
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
      // g, u rounded to bf16 once; stored: h and the backward's factors a = gelu(g) (aux), b = gelu'(g) u (aux2)
      uint32_t gp[4], up[4], hp[4];
#pragma unroll
      for (int e = 0; e < 8; e += 2)
        geglu_fwd2(bfround2(f32x2_t{g[e], g[e + 1]}), bfround2(f32x2_t{u[e], u[e + 1]}), gp[e / 2], up[e / 2],
                   hp[e / 2]);
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
// geglu_bwd_kernel does): the forward's saved factors a = gelu(g) (aux_in), b = gelu'(g) u (aux_in2) of row block
// I, 8 columns per lane and column pair pp, loaded one row block ahead of their use so their latency runs under
// the previous block's math (G holds a, U holds b)
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
    for (int e = 0; e < 8; e += 2) {   // the forward's factors (G: a = gelu(g), U: b = gelu'(g) u): two multiplies
      f32x2_t a, b;
      geglu_bwd2(bfround2(f32x2_t{v[e], v[e + 1]}), gv[e / 2], uv[e / 2], a, b);
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

// Lean bf16 epilogue (chosen on the host by lean_epilogue_ok: ACT_NONE or ACT_GELU_TANH, OUT_BF16, an optional
// bias / bf16-linear rounding / bf16 residual (SigLIP's linears), no row-add or fp32 residual, a C row map that
// is an offset (cmap.g == 0, or a group map that is the identity), N % 64 == 0).  The values are w4_epi8's, in
// its order (bias, bf16(linear), GELU-tanh, + bf16 residual), and the whole-line row-pair exchange is
// w4_rows' (bit-identical); what goes is the per-store address work -- row validity, row-map offsets, sink
// selects and 64-bit addresses per row block.  Stores (and residual loads) go through buffer resources whose
// num_records end at row M (rows past M fall outside them: stores dropped, loads zero), with one per-lane
// 32-bit offset computed once per tile plus a uniform row-block offset (kept in the VGPR offset: the range check
// does not include soffset).  The bias of the wave's columns is loaded once per tile.  A wave whose 16NJ columns
// start at or past N stores nothing (N % 64 == 0: a wave's columns are all inside N or all outside).
struct LeanEpi {
  __amdgpu_buffer_rsrc_t rc, rr;   // C, resid16
  uint32_t voff, ldc_bytes;        // store 1 of row block 0 / line 0 (row lane & 7, chunk lo ? cb : 32 + cb)
  uint32_t roff, ldr_bytes;        // resid16 of row block 0 (row lane & 15, columns col0 + cb)
  bool hb, lin, hr;
};
template <int ACT, int I, int NJ>
PTK_DEV void w4_rows_lean(f32x4_t (&a)[NJ], const LeanEpi& e, const float (&bias)[NJ / 2][8]) {
#pragma unroll
  for (int j = 0; j < NJ; ++j) asm volatile("" : "+a"(a[j]) :: "memory");
  u16x8_t res[NJ / 2];
  if (e.hr) {
#pragma unroll
    for (int pp = 0; pp < NJ / 2; ++pp)
      res[pp] = __builtin_bit_cast(u16x8_t, __builtin_amdgcn_raw_buffer_load_b128(
                                                e.rr, e.roff + (uint32_t)(16 * I) * e.ldr_bytes + 64u * pp, 0, 0));
  }
#pragma unroll
  for (int m = 0; m < NJ / 4; ++m) {
    uint4 X, Y;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int pp = 2 * m + h;
      f32x4_t x = a[2 * pp], y = a[2 * pp + 1];
      swap16(x, y);
      float v[8] = {x[0], x[1], x[2], x[3], y[0], y[1], y[2], y[3]};
      if (e.hb) {
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] += bias[pp][k];
      }
      if (e.lin) {
#pragma unroll
        for (int k = 0; k < 8; k += 2) {
          const f32x2_t r = bfround2(f32x2_t{v[k], v[k + 1]});
          v[k] = r.x;
          v[k + 1] = r.y;
        }
      }
      if constexpr (ACT == ACT_GELU_TANH) {
#pragma unroll
        for (int k = 0; k < 8; k += 2) {
          const f32x2_t r = gelu_tanh2(bfround2(f32x2_t{v[k], v[k + 1]}));
          v[k] = r.x;
          v[k + 1] = r.y;
        }
      }
      if (e.hr) {
        const uint4 rw = __builtin_bit_cast(uint4, res[pp]);
        const uint32_t rv[4] = {rw.x, rw.y, rw.z, rw.w};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const f32x2_t r = bf2x2(rv[k]);
          v[2 * k] += r.x;
          v[2 * k + 1] += r.y;
        }
      }
      (h ? Y : X) = w4_pack8(v);
    }
    uint4 d1, d2;
    w4_line_pair(X, Y, false, d1, d2);
    const uint32_t v1 = e.voff + (uint32_t)(16 * I) * e.ldc_bytes + 128u * m;   // rows 16I + (lane & 7), line m
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4v_t, d1), e.rc, v1, 0, 0);
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4v_t, d2), e.rc, v1 + 8u * e.ldc_bytes, 0, 0);
  }
}
template <int ACT, int NJ, int RB = 8>   // RB: 16-row blocks per wave (7, 6, 5: the 224- / 192- / 160-row tiles)
PTK_DEV void w4_epilogue_lean(const GemmArgs& p, f32x4_t (&acc)[8][NJ], long row0, long col0, int lane,
                              uint32_t c_bytes) {
  if (col0 >= p.N) return;
  LeanEpi e;
  const int q = lane >> 4;
  const int cb = 16 * (q & 1) + 8 * (q >> 1);
  const bool lo = (lane & 8) == 0;
  const uint32_t crow0 = (uint32_t)(row0 + p.cmap.off);
  e.rc = __builtin_amdgcn_make_buffer_rsrc(p.C, 0, (int)c_bytes, 0x00020000);
  e.ldc_bytes = __builtin_amdgcn_readfirstlane((uint32_t)p.ldc * 2u);
  // store 1 of a row pair writes row (lane & 7) of the row block, store 2 row 8 + (lane & 7), both at line chunk
  // lo ? cb : 32 + cb (w4_line_pair)
  e.voff = (crow0 + (lane & 7)) * e.ldc_bytes + (uint32_t)(col0 + (lo ? cb : 32 + cb)) * 2u;
  e.hb = p.bias != nullptr;
  e.lin = p.bf16_linear != 0;
  e.hr = p.resid16 != nullptr;
  e.ldr_bytes = __builtin_amdgcn_readfirstlane((uint32_t)p.ld_resid16 * 2u);
  e.rr = __builtin_amdgcn_make_buffer_rsrc((void*)p.resid16, 0, (int)(c_bytes / e.ldc_bytes * e.ldr_bytes), 0x00020000);
  e.roff = (crow0 + (lane & 15)) * e.ldr_bytes + (uint32_t)(col0 + cb) * 2u;
  float bias[NJ / 2][8];
  if (e.hb) {
#pragma unroll
    for (int pp = 0; pp < NJ / 2; ++pp) {
      const float4 b0 = *reinterpret_cast<const float4*>(p.bias + col0 + 32 * pp + cb);
      const float4 b1 = *reinterpret_cast<const float4*>(p.bias + col0 + 32 * pp + cb + 4);
      bias[pp][0] = b0.x; bias[pp][1] = b0.y; bias[pp][2] = b0.z; bias[pp][3] = b0.w;
      bias[pp][4] = b1.x; bias[pp][5] = b1.y; bias[pp][6] = b1.z; bias[pp][7] = b1.w;
    }
  }
  w4_rows_lean<ACT, 0, NJ>(acc[0], e, bias);
  w4_rows_lean<ACT, 1, NJ>(acc[1], e, bias);
  w4_rows_lean<ACT, 2, NJ>(acc[2], e, bias);
  w4_rows_lean<ACT, 3, NJ>(acc[3], e, bias);
  w4_rows_lean<ACT, 4, NJ>(acc[4], e, bias);
  if constexpr (RB > 5) w4_rows_lean<ACT, 5, NJ>(acc[5], e, bias);
  if constexpr (RB > 6) w4_rows_lean<ACT, 6, NJ>(acc[6], e, bias);
  if constexpr (RB > 7) w4_rows_lean<ACT, 7, NJ>(acc[7], e, bias);
}

// Lean GEGLU-backward epilogue (lean_glu_ok): w4_gbwd_rows' values and whole-line dg | du stores, the saved factors
// a, b loaded by buffer loads one row block ahead (rows past M read as zero and their stores are dropped)
#ifndef PTK_GBWD_AHEAD
#define PTK_GBWD_AHEAD 2   // row blocks of saved g, u in flight in the lean GEGLU-backward epilogue (A/B builds)
#endif
struct LeanGbwd {
  __amdgpu_buffer_rsrc_t rgi, rui, rc;
  uint32_t vin, ldin_bytes, vout, ldc_bytes;
};
template <int NP>
PTK_DEV void w4_gbwd_load_lean(const LeanGbwd& e, int I, u16x8_t (&G)[NP], u16x8_t (&U)[NP]) {
#pragma unroll
  for (int pp = 0; pp < NP; ++pp) {
    const uint32_t o = e.vin + (uint32_t)(16 * I) * e.ldin_bytes + 64u * pp;
    G[pp] = __builtin_bit_cast(u16x8_t, __builtin_amdgcn_raw_buffer_load_b128(e.rgi, o, 0, 0));
    U[pp] = __builtin_bit_cast(u16x8_t, __builtin_amdgcn_raw_buffer_load_b128(e.rui, o, 0, 0));
  }
}
template <int NP>
PTK_DEV void w4_gbwd_rows_lean(f32x4_t (&a)[2 * NP], const LeanGbwd& e, int I, const u16x8_t (&G)[NP],
                               const u16x8_t (&U)[NP]) {
#pragma unroll
  for (int j = 0; j < 2 * NP; ++j) asm volatile("" : "+a"(a[j]) :: "memory");
#pragma unroll
  for (int pp = 0; pp < NP; ++pp) {
    f32x4_t x = a[2 * pp], y = a[2 * pp + 1];
    swap16(x, y);
    const float v[8] = {x[0], x[1], x[2], x[3], y[0], y[1], y[2], y[3]};
    const uint4 gw = __builtin_bit_cast(uint4, G[pp]), uw = __builtin_bit_cast(uint4, U[pp]);
    const uint32_t gv[4] = {gw.x, gw.y, gw.z, gw.w}, uv[4] = {uw.x, uw.y, uw.z, uw.w};
    float dg[8], du[8];
#pragma unroll
    for (int k = 0; k < 8; k += 2) {   // w4_gbwd_rows' math
      f32x2_t aa, bb;
      geglu_bwd2(bfround2(f32x2_t{v[k], v[k + 1]}), gv[k / 2], uv[k / 2], aa, bb);
      dg[k] = aa.x;
      dg[k + 1] = aa.y;
      du[k] = bb.x;
      du[k + 1] = bb.y;
    }
    uint4 d1, d2;
    w4_line_pair(w4_pack8(dg), w4_pack8(du), false, d1, d2);
    const uint32_t o1 = e.vout + (uint32_t)(16 * I) * e.ldc_bytes + 128u * pp;
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4v_t, d1), e.rc, o1, 0, 0);
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4v_t, d2), e.rc, o1 + 8u * e.ldc_bytes, 0, 0);
  }
}
// (a lean gate|up GEGLU epilogue -- the same buffer-resource addressing for its g, u, h register-layout stores --
// measured 1 % slower than w4_rows' on the 4-wave kernel, 762.7 vs 755.7 us, profiles/r05_lean_epilogue_ab.txt, and
// is not kept)
template <int ACT, int NJ>
PTK_DEV void w4_epilogue_lean_glu(const GemmArgs& p, f32x4_t (&acc)[8][NJ], long row0, long col0, int lane,
                                  uint32_t c_bytes) {
  static_assert(ACT == ACT_GEGLU_BWD, "lean GEGLU backward only");
  if (col0 >= p.N) return;
  const int q = lane >> 4;
  const int cb = 16 * (q & 1) + 8 * (q >> 1);
  const uint32_t rows = (uint32_t)p.M;
  const uint32_t ldc_bytes = __builtin_amdgcn_readfirstlane((uint32_t)p.ldc * 2u);
  const uint32_t crow0 = (uint32_t)(row0 + p.cmap.off);
  {
    constexpr int NP = NJ / 2;
    LeanGbwd e;
    e.ldin_bytes = __builtin_amdgcn_readfirstlane((uint32_t)p.ld_aux_in * 2u);
    e.ldc_bytes = ldc_bytes;
    e.rgi = __builtin_amdgcn_make_buffer_rsrc((void*)p.aux_in, 0, (int)(rows * e.ldin_bytes), 0x00020000);
    e.rui = __builtin_amdgcn_make_buffer_rsrc((void*)p.aux_in2, 0, (int)(rows * e.ldin_bytes), 0x00020000);
    e.rc = __builtin_amdgcn_make_buffer_rsrc(p.C, 0, (int)c_bytes, 0x00020000);
    e.vin = ((uint32_t)row0 + (lane & 15)) * e.ldin_bytes + (uint32_t)(col0 + cb) * 2u;
    // dg | du line pp of rows (lane & 7) / 8 + (lane & 7): w4_gbwd_rows' output column map
    const bool lo = (lane & 8) == 0;
    e.vout = (crow0 + (lane & 7)) * ldc_bytes +
             (uint32_t)(2 * col0 + 8 * (4 * (cb >> 4) + ((cb >> 3) & 1) + (lo ? 0 : 2))) * 2u;
    // the saved g, u of row block i + D load while row block i computes (D row blocks in flight)
    constexpr int D = PTK_GBWD_AHEAD;
    u16x8_t G[D][NP], U[D][NP];
#pragma unroll
    for (int i = 0; i < D; ++i) w4_gbwd_load_lean<NP>(e, i, G[i], U[i]);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      w4_gbwd_rows_lean<NP>(acc[i], e, i, G[i % D], U[i % D]);
      if (i + D < 8) w4_gbwd_load_lean<NP>(e, i + D, G[i % D], U[i % D]);
    }
  }
}

// the wave's 128 x 16NJ accumulator tile (8 row blocks of NJ 16x16 MFMA tiles)
template <int ACT, int OUT, int NJ = 8, int RB = 8>
PTK_DEV void w4_epilogue(const GemmArgs& p, f32x4_t (&acc)[8][NJ], long row0, long col0, int lane) {
  char* sink = g_w4_sink + lane * 64;
  static_assert(RB == 8 || ACT != ACT_GEGLU_BWD, "the GEGLU backward epilogue runs 8 row blocks");
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
  if constexpr (RB > 5) w4_rows<ACT, OUT, 5, NJ>(p, acc[5], row0, col0, lane, sink);
  if constexpr (RB > 6) w4_rows<ACT, OUT, 6, NJ>(p, acc[6], row0, col0, lane, sink);
  if constexpr (RB > 7) w4_rows<ACT, OUT, 7, NJ>(p, acc[7], row0, col0, lane, sink);
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

// stream-K tail units: the tail tile's pieces are summed in K order: piece jj of tile tt belongs to workgroup
// g0 + jj, whose partial sits in its slot 0 if the piece is that workgroup's first (its unit range starts inside
// the tile), else slot 1
PTK_DEV int p8_owner(long x, int G, int U) { return (int)(((x + 1) * G - 1) / U); }   // workgroup of unit x
PTK_DEV int p8_start(int g, int G, int U) { return (int)(((long)g * U) / G); }

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


}  // namespace ptk
