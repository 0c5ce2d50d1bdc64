// Model-level orchestration of the Stage-1 hot path (host side of libptk).
//
// ptk_siglip_fwd        SigLIP vision tower forward (modeling_siglip.py:576-619)
// ptk_gemma3_loss_fwd_bwd  Gemma3 forward + causal-LM loss + dX backward
//                       (modeling_gemma3.py:511-659, loss_utils.py:49-67)
//
// Each call is a fixed sequence of kernel launches on the caller's stream using
// a caller-provided workspace (sized by the *_workspace_bytes query), so it can
// be captured into a hipGraph.  Layouts (row-major, token rows b*S + s):
//   LLM hidden x: f32 [B*Spad, H] (fp32 residual stream, as the reference's
//   autocast keeps it); GEMM operands bf16.  Attention per (b, kv-head) z:
//   Q [B,Hkv,S,G,D] (rows (s,j) contiguous), K/V [B,Hkv,S,D], scores/P
//   [B*Hkv, S*G, S].  QK^T and P.V run on the MFMA GEMM; masks/softmax are
//   row kernels.
#include <cstdlib>
#include <algorithm>
#include <math.h>
#include <string.h>

#include <vector>

#include "../../include/ptk.h"
#include "ptk_internal.h"

using namespace ptk;

namespace {

struct Bump {
  char* base;
  size_t off = 0;
  explicit Bump(void* b) : base((char*)b) {}
  template <class T>
  T* take(size_t n) {
    off = (off + 255) & ~(size_t)255;
    T* p = base ? reinterpret_cast<T*>(base + off) : nullptr;
    off += n * sizeof(T);
    return p;
  }
};

float bfround_host(float f) {
  uint32_t u;
  memcpy(&u, &f, 4);
  u += 0x7fffu + ((u >> 16) & 1u);
  u &= 0xffff0000u;
  memcpy(&f, &u, 4);
  return f;
}

constexpr int LM_SPLITK = 8;   // split-K for the vocab-long lm_head dX GEMM (R x H output, K = V)
constexpr int LM_KSLICES = 16; // its K slices on the 8-wave kernel (R % 256 == 0, V % 1024 == 0)

#define CK(x) \
  do {        \
    if ((x)) return -1; \
  } while (0)
// HIP runtime call: a failure records its own message (ptk_last_error) instead of leaving a stale one
#define CKH(x)                                                                       \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) return set_error("%s: %s", #x, hipGetErrorString(e_));    \
  } while (0)

static bool geglu_split() {
  const int v = PTK_AB("PTK_GEGLU_SPLIT", 0) == 1;   // A/B builds only
  return v != 0;
}
// Stage 2: the residual norm backward writes both norms' weight-grad partials itself (PTK_NORM_WG=0: the two
// separate rms_wgrad passes, A/B builds)
static bool norm_wg_fused() { return PTK_AB("PTK_NORM_WG", 1) != 0; }

// dR += rms_bwd(x2, w_pre, rstd_pre, dn); dt = bf16(rms_bwd(t, w_post, rstd_t, bf16(dR))); with g_pre / g_post
// (Stage 2) also accumulates both norms' weight grads.  wpart: the fused kernel's two partial sets back to back
static int residual_norm_bwd_grads(const float* x2, const float* w_pre, const float* rstd_pre, const bf16_t* dn,
                                   float* dR, const bf16_t* t, const float* w_post, const float* rstd_t, bf16_t* dt,
                                   int M, int H, bf16_t* g_pre, bf16_t* g_post, float* wpart, hipStream_t st) {
  const RowMap ident{0, 0, 0, 0};
  if (g_pre && norm_wg_fused()) {
    const int nb = residual_norm_bwd_wg_blocks(M);
    float* pq = wpart + rms_wgrad_finish_floats(nb, H);
    CK(launch_residual_norm_bwd_wg(x2, w_pre, rstd_pre, dn, dR, t, w_post, rstd_t, dt, M, H, wpart, pq, st));
    CK(launch_rms_wgrad_finish(wpart, nb, H, g_pre, st));
    return launch_rms_wgrad_finish(pq, nb, H, g_post, st);
  }
  if (g_pre) CK(launch_rms_wgrad_bdy(x2, H, ident, rstd_pre, dn, H, M, H, g_pre, wpart, st));
  CK(launch_residual_norm_bwd_bdn(x2, w_pre, rstd_pre, dn, dR, t, w_post, rstd_t, dt, M, H, st));
  if (g_pre) CK(launch_rms_wgrad_bx(t, H, ident, rstd_t, dR, H, 1, M, H, g_post, wpart, st));
  return 0;
}
// PTK_DKV_REDUCE_SPLIT=1: separate attn_dkv_reduce_kernel pass (A/B) instead of summing the split-slab
// dK/dV partials inside qknorm_rope_bwd
static bool dkv_reduce_split() {
  static const int v = [] { const char* e = getenv("PTK_DKV_REDUCE_SPLIT"); return e && e[0] == '1' ? 1 : 0; }();
  return v != 0;
}

// PTK_CE_TWO_PASS=1: the cross-entropy pass computes its own row statistics (two reads of the logits) instead
// of taking them from the lm_head GEMM's epilogue (A/B; tests/test_stage1_gpu.py checks both agree)
// PTK_LM_STATS_ONLY=1 (diagnostic builds only, -DPTK_DIAG: wrong results by construction): the lm_head GEMM
// computes its softmax statistics but skips the logits store -- the forward half of a fused lm_head + online-LSE
// CE, timed against the shipped chain.  The product library has no such switch.
static bool lm_stats_only() {
#ifdef PTK_DIAG
  static const int v = [] { const char* e = getenv("PTK_LM_STATS_ONLY"); return e && e[0] == '1' ? 1 : 0; }();
  return v != 0;
#else
  return false;
#endif
}

static bool ce_two_pass() {
  static const int v = [] { const char* e = getenv("PTK_CE_TWO_PASS"); return e && e[0] == '1' ? 1 : 0; }();
  return v != 0;
}

GemmArgs gemm(const void* A, long lda, const void* B, long ldb, void* C, long ldc, int M, int N, int K) {
  GemmArgs g;
  g.A = (const bf16_t*)A; g.B = (const bf16_t*)B; g.C = C;
  g.lda = lda; g.ldb = ldb; g.ldc = ldc;
  g.M = M; g.N = N; g.K = K;
  return g;
}

// ------------------------------------------------------------------ SigLIP
struct SiglipWs {
  bf16_t *patches, *h, *a, *qkv, *o, *mlp;
  void* tail;   // stream-K tail scratch of the tower's GEMMs
};

SiglipWs siglip_layout(Bump& bp, const ptk_siglip_config* c, int B) {
  const long D = c->hidden, I = c->intermediate, P = c->patch_size, Nn = (c->image_size / P) * (c->image_size / P);
  const long Np = (Nn + 63) / 64 * 64, M = B * Nn, H = c->heads, hd = D / H, Kp = (long)c->channels * P * P;
  SiglipWs w;
  w.patches = bp.take<bf16_t>(M * Kp);
  w.h = bp.take<bf16_t>(M * D);   // bf16 residual stream: the reference tower runs in pure bf16
  w.a = bp.take<bf16_t>(M * D);
  w.qkv = bp.take<bf16_t>(M * 3 * D);
  w.o = bp.take<bf16_t>(M * D);
  w.mlp = bp.take<bf16_t>(M * I);
  w.tail = bp.take<char>(p8_tail_scratch_bytes_models());
  return w;
}

// ------------------------------------------------------------------ Gemma3
struct GemmaLayerSave {
  float *x2, *rstd_in, *rstd_ao, *rstd_pre, *rstd_dn, *rstd_q, *rstd_k;
  // glu_a, glu_b: the GEGLU backward's factors the gate|up epilogue saves, bf16 gelu(gate) and gelu'(gate) * up
  // (common.h geglu_fwd2)
  bf16_t *qkv, *Q, *K, *V, *O, *ao, *glu_a, *glu_b, *dn;
  float* lse;
  // unfrozen LLM only: the GEMM inputs the weight grads contract with (input-norm / pre-ff-norm outputs,
  // GEGLU output); the frozen path keeps them in one scratch buffer
  bf16_t *xn_in = nullptr, *xn_ff = nullptr, *h = nullptr;
};
struct GemmaWs {
  std::vector<float*> x;          // L+1 residual-stream snapshots
  std::vector<GemmaLayerSave> L;
  bf16_t *P, *xn, *O, *h, *Vt, *Kt, *Qt, *dqkv, *dgu, *dao, *dO, *dS, *dST, *PT, *dOT, *dQ, *dK, *dV, *xf, *logits;
  bf16_t* dtmp;             // bf16 dX of the q|k|v / gate|up projections (see the workspace layout)
  float *S, *rstd_f, *row_loss, *dxf, *dxf_part, *count, *gscale, *delta;
  float* ce_stats = nullptr;   // the lm_head epilogue's softmax statistics [R][V / 64] (float2)
  float* dkv_part;          // split-query dK/dV partials of the attention backward
  size_t dkv_part_bytes;
  int32_t* key_valid;
  // unfrozen LLM only: feature-major GEMM operands of dW = dY^T X (K = tokens) and norm-grad partials
  bf16_t *TA = nullptr, *TB = nullptr, *TL = nullptr, *TX = nullptr;
  float* wpart = nullptr;
  void* eg_keys = nullptr;   // the embedding grad's sorted (id, position) keys
  float* skpart = nullptr;     // split-K partials (gemm_split)
  long sk_floats = 0;
  void* tail = nullptr;        // stream-K tail scratch of the model's GEMMs
};

GemmaWs gemma_layout(Bump& bp, const ptk_gemma3_config* c, int B, int T, int Sp, bool train = false) {
  const long H = c->hidden, I = c->inter, D = c->head_dim, Hq = c->heads, Hkv = c->kv_heads, G = Hq / Hkv;
  const long M = (long)B * Sp, Dq = Hq * D, Dqkv = (Hq + 2 * Hkv) * D, R = (long)B * T, V = c->vocab;
  const long Z = (long)B * Hkv, SG = (long)Sp * G;
  GemmaWs w;
  w.key_valid = bp.take<int32_t>(M);
  w.x.push_back(nullptr);   // x[0] is the caller's input buffer
  for (int l = 1; l <= c->layers; ++l) w.x.push_back(bp.take<float>(M * H));
  for (int l = 0; l < c->layers; ++l) {
    GemmaLayerSave s;
    s.x2 = bp.take<float>(M * H);
    s.rstd_in = bp.take<float>(M);
    s.rstd_ao = bp.take<float>(M);
    s.rstd_pre = bp.take<float>(M);
    s.rstd_dn = bp.take<float>(M);
    s.rstd_q = bp.take<float>(M * Hq);
    s.rstd_k = bp.take<float>(M * Hkv);
    s.qkv = bp.take<bf16_t>(M * Dqkv);
    s.Q = bp.take<bf16_t>(Z * SG * D);
    s.K = bp.take<bf16_t>(Z * Sp * D);
    s.V = bp.take<bf16_t>(Z * Sp * D);
    s.lse = bp.take<float>(Z * SG);
    s.O = bp.take<bf16_t>(M * Dq);
    s.ao = bp.take<bf16_t>(M * H);
    s.glu_a = bp.take<bf16_t>(M * I);
    s.glu_b = bp.take<bf16_t>(M * I);
    s.dn = bp.take<bf16_t>(M * H);
    if (train) {
      s.xn_in = bp.take<bf16_t>(M * H);
      s.xn_ff = bp.take<bf16_t>(M * H);
      s.h = bp.take<bf16_t>(M * I);
    }
    w.L.push_back(s);
  }
  w.P = nullptr;
  w.xn = bp.take<bf16_t>(M * H);
  w.O = nullptr;
  w.h = bp.take<bf16_t>(M * I);
  w.Vt = nullptr;
  w.Kt = nullptr;
  w.Qt = nullptr;
  w.S = nullptr;
  w.delta = bp.take<float>(Z * SG);
  {
    FlashBwdArgs fa;
    fa.rows = (int)SG; fa.nkeys = Sp; fa.D = (int)D; fa.qdiv = (int)G; fa.causal = 1;
    size_t nb = attn_bwd_workspace_bytes(fa, (int)Z);
    fa.window = c->sliding_window;
    if (c->sliding_window > 0) nb = std::max(nb, attn_bwd_workspace_bytes(fa, (int)Z));
    w.dkv_part_bytes = nb;
    w.dkv_part = nb ? bp.take<float>((long)(nb / sizeof(float))) : nullptr;
  }
  w.dqkv = bp.take<bf16_t>(M * Dqkv);
  w.dgu = bp.take<bf16_t>(M * 2 * I);
  // dX of the q|k|v and gate|up projections, bf16: the reference's autocast linear backward returns a bf16
  // input grad (upcast to fp32 only where it meets the fp32 norm / residual stream), so the norm backward
  // passes read bf16 values either way; stored as bf16 it moves half the bytes
  w.dtmp = bp.take<bf16_t>(M * H);
  w.dao = bp.take<bf16_t>(M * H);
  w.dO = bp.take<bf16_t>(Z * SG * D);
  w.dS = nullptr;
  w.dST = nullptr;
  w.PT = nullptr;
  w.dOT = nullptr;
  w.dQ = bp.take<bf16_t>(Z * SG * D);
  w.dK = bp.take<bf16_t>(Z * Sp * D);
  w.dV = bp.take<bf16_t>(Z * Sp * D);
  w.xf = bp.take<bf16_t>(R * H);
  w.rstd_f = bp.take<float>(R);
  w.logits = bp.take<bf16_t>(R * V);
  if (V % 64 == 0) w.ce_stats = bp.take<float>(R * (V / 64) * 2);
  w.row_loss = bp.take<float>(R);
  w.dxf = bp.take<float>(R * H);
  w.dxf_part = bp.take<float>((long)std::max(LM_SPLITK + 1, LM_KSLICES) * R * H);   // (+ a vocab remainder slot)
  w.count = bp.take<float>(4);
  w.gscale = bp.take<float>(4);
  if (train) {
    const long Rp = (R + 63) / 64 * 64;
    w.TA = bp.take<bf16_t>(std::max(std::max(2 * I, Dqkv), H) * M);
    w.TB = bp.take<bf16_t>(std::max(std::max(H, Dq), I) * M);
    w.TL = bp.take<bf16_t>(V * Rp);
    w.TX = bp.take<bf16_t>(H * Rp);
    // two norms' partials (the fused residual norm backward), or one norm's / the q,k norms'
    w.eg_keys = bp.take<char>((long)embed_grad_ws_bytes(B, T));
    w.wpart = bp.take<float>(std::max(std::max((long)rms_wgrad_partial_floats((int)M, (int)H),
                                               2L * rms_wgrad_finish_floats(residual_norm_bwd_wg_blocks((int)M), (int)H)),
                                      (long)qknorm_wgrad_partial_floats(M, (int)D)));
  }
  // split-K partials (gemm_split): 2 slices of the largest [M, H] / [2I, H] output, 4 of the small dW ones
  w.sk_floats = std::max(std::max(2 * M * H, 2 * 2 * I * H), 4 * std::max(Dqkv, H) * H);
  if (train) w.sk_floats = std::max(w.sk_floats, V * H);   // the tied embedding's fp32 dW before its accumulate
  // the stream-K slabs: the TN weight grads' and the long-K projections' (gemm_split)
  w.sk_floats = std::max(w.sk_floats, (long)(p8_tail_scratch_bytes() / sizeof(float)) + 64);
  if (train) w.sk_floats = std::max(w.sk_floats, (long)(tn_slab_bytes() / sizeof(float)));
  w.skpart = bp.take<float>(w.sk_floats);
  w.tail = bp.take<char>(p8_tail_scratch_bytes_models());
  return w;
}

// Split-K for long-K GEMMs whose 256x256 tile grid fills few of the CUs' rounds (measured, tools/splitk_probe.py
// r02: the cfg4 shapes dW_qkv 313 -> 73 us and dW_o 313 -> 68 us at 4 slices; dW_down, dW_gate|up, the
// d(gate|up) dX and the down projection at 280 tiles -8..-16 % at 2 slices; the cfg2 d(gate|up) dX at 440
// tiles is slower split, the vocab-wide lm_head dW too).  ACT_NONE only; OUT_F32, or OUT_BF16 with the
// optional bf16 accumulate (bf16_linear + resid16, the weight-grad epilogue).  The slices go to the batched
// 128x128 kernel as fp32 partials [S][M][N]; one pass sums them in slice order (deterministic).
int gemm_split(const GemmArgs& a, int out, float* part, long part_floats, hipStream_t st) {
  // the persistent kernel's stream-K tail takes the shapes it measured faster on (gemm_w4.hip p8_tail_plan:
  // Stage 2's weight grads and M = 14 336 projections) before any host-side split
  if (a.M >= 1024 && a.N >= 256 && a.N <= 16384 && p8_supported(a, ACT_NONE, out) && p8_tail_split(a, ACT_NONE, out))
    return launch_gemm(a, ACT_NONE, out, 1, st);
  // long-K GEMMs whose 256x256 tiles leave a thin last round (Stage 2's d(gate|up) dX and down projection at M =
  // 14 336: 280 tiles = 256 + 24): the 8-wave kernel's stream-K tail over the split-K scratch, its pieces summed by
  // p8_fixup_kernel (r05, tools/sk_ab.py same box: 419 / 216 us vs 662 / 298 unsplit; the 2-slice 128x128 split
  // below ran them at ~390 + 26 us on average)
  if (streamk_enabled() && a.K >= 4096 && part && (size_t)part_floats * sizeof(float) >= p8_tail_scratch_bytes() &&
      a.M >= 1024 && a.N >= 256 && a.N <= 16384) {
    GemmArgs b = a;
    b.tail_ws = part;
    if (p8_supported(b, ACT_NONE, out) && p8_tail_split(b, ACT_NONE, out)) return launch_gemm(b, ACT_NONE, out, 1, st);
  }
  // one partial round of 256x256 tiles: the 8-wave kernel unsplit (launch_gemm's single-round rule) beats the
  // split-K 128x128 slices (Stage 2 at bs 8: the down projection 133.6 vs 177.8 us); K <= 8192 as launch_gemm's own
  // single-round rule, so a longer K (Gemma3-4B's down projection, K 10 240) keeps the split
  if (a.M >= 4096 && a.K <= 8192 && (long)((a.M + 255) / 256) * ((a.N + 255) / 256) <= device_cus() && out == OUT_BF16 &&
      p8_supported(a, ACT_NONE, out) && lean_epilogue_candidate(a))
    return launch_gemm(a, ACT_NONE, out, 1, st);
  const long nbig = (long)((a.M + 255) / 256) * ((a.N + 255) / 256);
  int S = 1, kmin = 1024;
  if (a.K >= 4096 && nbig <= 64) S = 4;
  else if (a.K >= 4096 && nbig <= 300) S = 2;
  // small M (cfg1, bs 2: M = 520): the 128x128 tile grid alone leaves most CUs idle, so split K until
  // the slices fill about two blocks per CU (slices >= 256 deep)
  const long n128 = (long)((a.M + 127) / 128) * ((a.N + 127) / 128), cus = device_cus();
  if (n128 * 2 <= cus) {
    kmin = 256;
    while (n128 * S * 2 <= 2 * cus && a.K / (S * 2) >= kmin) S *= 2;
  }
  while (S > 1 && ((long)S * a.M * a.N > part_floats || a.K / S < kmin || a.N % 4 || a.ldc % 4)) S /= 2;
  const bool plain = !a.rowadd && !a.resid && !a.aux && !a.aux_in && a.amap.g == 0 && a.amap.off == 0 &&
                     a.cmap.g == 0 && a.cmap.off == 0 && a.bias == nullptr && a.alpha == 1.f;
  if (S == 1 || !plain || !part) return launch_gemm(a, ACT_NONE, out, 1, st);
  const int kc = (a.K / S + 63) / 64 * 64;
  const int nfull = a.K / kc, rem = a.K - nfull * kc;
  GemmArgs b = a;
  b.C = part; b.ldc = a.N; b.K = kc;
  b.sA0 = kc; b.sB0 = kc; b.sC0 = (long)a.M * a.N;
  b.bf16_linear = 0; b.resid16 = nullptr; b.ld_resid16 = 0;
  CK(launch_gemm(b, ACT_NONE, OUT_F32, nfull, st));
  if (rem) {
    GemmArgs r = b;
    r.A = a.A + (long)nfull * kc; r.B = a.B + (long)nfull * kc; r.K = rem;
    r.C = part + (long)nfull * a.M * a.N;
    CK(launch_gemm(r, ACT_NONE, OUT_F32, 1, st));
  }
  const bool bf = out == OUT_BF16;
  return launch_splitk_reduce(part, nfull + (rem ? 1 : 0), a.M, a.N, a.C, a.ldc, bf ? 1 : 0,
                              bf ? a.resid16 : nullptr, a.ld_resid16, st);
}

// dW (+)= dY^T X over K token rows into the bf16 .grad (bf16(grad + bf16(acc)), autograd's accumulation).  Both
// operands are token-major.  Ungathered rows (identity maps): the persistent TN GEMM reads them where they lie
// (a ragged row count padded to 64 with zero rows), K slices as fp32 partials summed in slice order (gemm_tn.hip).  Otherwise (the loss rows of the
// last layer, ragged row counts, PTK_WGRAD_TN=0) each is transposed to a K-contiguous feature-major copy (rows
// gathered through the map, zero-padded to a multiple of 64) for the NT GEMMs.
static int wgrad_tn_mode() { return PTK_AB("PTK_WGRAD_TN", 1); }   // A/B builds: PTK_WGRAD_TN=0 / 2
}  // namespace
namespace ptk {
int wgrad_tn_enabled() { return wgrad_tn_mode() != 0; }
}  // namespace ptk
namespace {
int weight_grad(const bf16_t* dy, long lddy, RowMap ymap, int Ny, const bf16_t* x, long ldx, RowMap xmap, int Nx,
                int rows, bf16_t* TA, bf16_t* TB, void* grad, float* skpart, long sk_floats, hipStream_t st,
                int tn = -1) {
  if (!grad) return 0;
  if (tn < 0) tn = wgrad_tn_mode();
  if (tn && ymap.g == 0 && ymap.off == 0 && xmap.g == 0 && xmap.off == 0 && rows > 0) {
    // A = dY [rows][Ny], B = X [rows][Nx]; K = rows padded to a multiple of 64, the pad rows past the operands'
    // buffer ranges read as zero
    const int Kp = (rows + 63) / 64 * 64;
    GemmArgs g = gemm(dy, lddy, x, ldx, grad, Nx, Ny, Nx, Kp);
    g.bf16_linear = 1;
    g.resid16 = (const bf16_t*)grad;
    g.ld_resid16 = Nx;
    // with a slab for the stream-K tail (the fp32 scratch): one slice, the tail round's K-tiles spread over the
    // CUs; otherwise equal K slices summed by splitk_reduce
    if (skpart && (size_t)sk_floats * sizeof(float) >= tn_slab_bytes() && tn_supported(g, OUT_BF16, 1))
      return gemm_tn(g, OUT_BF16, 1, skpart, st, rows);
    const int S = skpart ? tn_slices(g, sk_floats) : (tn_supported(g, OUT_BF16, 1) ? 1 : 0);
    if (S == 1) return gemm_tn(g, OUT_BF16, 1, nullptr, st, rows);
    if (S > 1) {
      GemmArgs b = g;
      b.C = skpart;
      b.ldc = Nx;
      b.bf16_linear = 0;
      b.resid16 = nullptr;
      b.ld_resid16 = 0;
      CK(gemm_tn(b, OUT_F32, S, nullptr, st, rows));
      return launch_splitk_reduce(skpart, S, Ny, Nx, grad, Nx, 1, (const bf16_t*)grad, Nx, st);
    }
  }
  if (tn == 2) return set_error("weight_grad: the TN path does not take Ny %d Nx %d rows %d", Ny, Nx, rows);
  // the transpose path: decided here on the host, so scratch that was left out because the caller expected the
  // TN path (identity maps) is caught before any launch (tn_supported rejects e.g. Ny / Nx % 64, 64 rows, unaligned
  // pointers or operands past 4 GiB)
  if (!TA || !TB)
    return set_error("weight_grad: Ny %d Nx %d rows %d take the transpose path, which needs ta / tb scratch", Ny, Nx,
                     rows);
  const int Kp = (rows + 63) / 64 * 64;
  CK(launch_transpose_rows(dy, lddy, ymap, rows, Ny, TA, Kp, Kp, st));
  CK(launch_transpose_rows(x, ldx, xmap, rows, Nx, TB, Kp, Kp, st));
  GemmArgs g = gemm(TA, Kp, TB, Kp, grad, Nx, Ny, Nx, Kp);
  g.bf16_linear = 1;
  g.resid16 = (const bf16_t*)grad;
  g.ld_resid16 = Nx;
  return gemm_split(g, OUT_BF16, skpart, sk_floats, st);
}

}  // namespace

extern "C" {

int ptk_weight_grad_bf16(const void* dy, int64_t lddy, int y_map_g, int64_t y_map_gs, int64_t y_map_off, int Ny,
                         const void* x, int64_t ldx, int x_map_g, int64_t x_map_gs, int64_t x_map_off, int Nx, int rows,
                         void* grad, void* ta, void* tb, float* part, int64_t part_floats, int mode, void* stream) {
  if (mode < 0 || mode > 2) return set_error("weight_grad: mode %d (0 auto, 1 transposes, 2 TN)", mode);
  if (Ny <= 0 || Nx <= 0 || rows <= 0) return 0;
  const RowMap ym{y_map_g, 0, y_map_gs, y_map_off}, xm{x_map_g, 0, x_map_gs, x_map_off};
  const bool tn_ok = mode != 1 && ym.g == 0 && ym.off == 0 && xm.g == 0 && xm.off == 0;
  if (!tn_ok && (!ta || !tb)) return set_error("weight_grad: the transpose path needs ta / tb scratch");
  return weight_grad((const bf16_t*)dy, lddy, ym, Ny, (const bf16_t*)x, ldx, xm, Nx, rows, (bf16_t*)ta, (bf16_t*)tb,
                     grad, part, part_floats, (hipStream_t)stream, mode == 0 ? -1 : (mode == 1 ? 0 : 2));
}

size_t ptk_siglip_workspace_bytes(const ptk_siglip_config* c, int batch) {
  Bump bp(nullptr);
  siglip_layout(bp, c, batch);
  return bp.off + 256;
}

int ptk_siglip_fwd(const ptk_siglip_config* c, const ptk_siglip_weights* wt, int B, const void* pixels, void* out,
                   void* ws, size_t ws_bytes, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (ws_bytes < ptk_siglip_workspace_bytes(c, B)) return set_error("siglip_fwd: workspace too small");
  if (c->hidden % c->heads) return set_error("siglip_fwd: hidden %% heads");
  const int D = c->hidden, I = c->intermediate, P = c->patch_size, Hh = c->heads, hd = D / Hh;
  const int Nn = (c->image_size / P) * (c->image_size / P), Np = (Nn + 63) / 64 * 64, M = B * Nn;
  const int Kp = c->channels * P * P;
  if (Kp % 64 || hd % 64) return set_error("siglip_fwd: patch dim %d and head dim %d must be multiples of 64", Kp, hd);
  Bump bp(ws);
  SiglipWs w = siglip_layout(bp, c, B);
  TailScratchScope tail(w.tail, st);
  CK(tail.status);
  StageScope stage_all("siglip.fwd", st);
  StageSeq sq(st);
  sq.next("siglip.embed");

  // K1 patch embed: im2col + GEMM; bf16(conv + bias) + pos -> bf16 residual stream (modeling_siglip.py:175-186)
  CK(launch_im2col((const bf16_t*)pixels, w.patches, B, c->channels, c->image_size, c->image_size, P, st));
  {
    GemmArgs g = gemm(w.patches, Kp, wt->patch_w, Kp, w.h, D, M, D, Kp);
    g.bias = wt->patch_b;
    g.bf16_linear = 1;
    g.rowadd = wt->pos; g.rowadd_period = Nn; g.ld_rowadd = D;
    CK(launch_gemm(g, ACT_NONE, OUT_BF16, 1, st));
  }
  for (int l = 0; l < c->layers; ++l) {
    const ptk_siglip_layer& L = wt->layers[l];
    sq.next("siglip.attn");
    CK(launch_layernorm_bf16(w.h, L.ln1_w, L.ln1_b, w.a, M, D, c->eps, st));
    {  // fused q|k|v projection
      GemmArgs g = gemm(w.a, D, L.wqkv, D, w.qkv, 3 * D, M, 3 * D, D);
      g.bias = L.bqkv;
      CK(launch_gemm(g, ACT_NONE, OUT_BF16, 1, st));
    }
    {  // softmax(Q K^T / sqrt(hd)) V per (b, head), flash (no score matrix in HBM)
      FlashArgs fa;
      fa.Q = w.qkv; fa.K = w.qkv + D; fa.V = w.qkv + 2 * D; fa.O = w.o;
      fa.rows = Nn; fa.nkeys = Nn; fa.D = hd;
      fa.ldq = fa.ldk = 3 * D; fa.ldo = D;
      fa.zin = Hh; fa.zdiv = Hh;
      fa.sQ0 = fa.sK0 = (long)Nn * 3 * D; fa.sQ1 = fa.sK1 = hd;
      fa.sO0 = (long)Nn * D; fa.sO1 = hd;
      fa.scale = 1.0f / sqrtf((float)hd);
      StageScope sf("siglip.flash", st);
      CK(launch_attn_fwd(fa, B * Hh, st));
    }
    {  // h = bf16(h + bf16(out_proj + bias))   (modeling_siglip.py:343-346, bf16 module)
      GemmArgs g = gemm(w.o, D, L.wo, D, w.h, D, M, D, D);
      g.bias = L.bo; g.bf16_linear = 1; g.resid16 = w.h; g.ld_resid16 = D;
      CK(launch_gemm(g, ACT_NONE, OUT_BF16, 1, st));
    }
    sq.next("siglip.mlp");
    CK(launch_layernorm_bf16(w.h, L.ln2_w, L.ln2_b, w.a, M, D, c->eps, st));
    {
      GemmArgs g = gemm(w.a, D, L.w1, D, w.mlp, I, M, I, D);
      g.bias = L.b1;
      CK(launch_gemm(g, ACT_GELU_TANH, OUT_BF16, 1, st));
    }
    {  // h = bf16(h + bf16(fc2 + bias))
      GemmArgs g = gemm(w.mlp, I, L.w2, I, w.h, D, M, D, I);
      g.bias = L.b2; g.bf16_linear = 1; g.resid16 = w.h; g.ld_resid16 = D;
      CK(launch_gemm(g, ACT_NONE, OUT_BF16, 1, st));
    }
  }
  sq.next("siglip.post_norm");
  CK(launch_layernorm_bf16(w.h, wt->post_w, wt->post_b, (bf16_t*)out, M, D, c->eps, st));
  return 0;
}

size_t ptk_gemma3_workspace_bytes(const ptk_gemma3_config* c, int batch, int text_len, int seq_pad) {
  Bump bp(nullptr);
  gemma_layout(bp, c, batch, text_len, seq_pad);
  return bp.off + 256;
}

size_t ptk_gemma3_train_workspace_bytes(const ptk_gemma3_config* c, int batch, int text_len, int seq_pad) {
  Bump bp(nullptr);
  gemma_layout(bp, c, batch, text_len, seq_pad, true);
  return bp.off + 256;
}

}  // extern "C"

namespace {

// Gemma3 forward + causal-LM loss + backward.  gr == nullptr: the frozen LLM of Stage 1 (dX only);
// otherwise every parameter's grad is accumulated into *gr as well (unfrozen LLM, Stage 2).
int gemma_run(const ptk_gemma3_config* c, const ptk_gemma3_weights* wt, const ptk_gemma3_batch* bt,
              const ptk_gemma3_grads* gr, void* ws, size_t ws_bytes, hipStream_t st, bool fwd_only = false) {
  const bool train = gr != nullptr;
  const int B = bt->batch, T = bt->text_len, Nv = bt->num_vision, Sp = bt->seq_pad, S = Nv + T;
  const int lo = bt->label_offset;
  if (Sp % 64 || S > Sp) return set_error("gemma3: seq_pad %d must be a multiple of 64 and >= %d", Sp, S);
  if (Sp > wt->rope_max_pos) return set_error("gemma3: seq_pad %d exceeds rope table (%d)", Sp, wt->rope_max_pos);
  if (c->heads % c->kv_heads) return set_error("gemma3: heads %% kv_heads");
  if (Nv < 1) return set_error("gemma3: num_vision must be >= 1");
  if (lo < 0 || lo >= T) return set_error("gemma3: label_offset %d outside [0, text_len %d)", lo, T);
  const size_t need = train ? ptk_gemma3_train_workspace_bytes(c, B, T, Sp) : ptk_gemma3_workspace_bytes(c, B, T, Sp);
  if (ws_bytes < need) return set_error("gemma3: workspace too small");
  if (c->vocab % 64 || c->vocab < 64 * LM_SPLITK) return set_error("gemma3: vocab must be a multiple of 64 and >= %d", 64 * LM_SPLITK);
  if (train && (!gr->layers || !gr->embed || !gr->final_norm)) return set_error("gemma3 train: grads missing");
  const int H = c->hidden, I = c->inter, D = c->head_dim, Hq = c->heads, Hkv = c->kv_heads, G = Hq / Hkv;
  const int M = B * Sp, Dq = Hq * D, Dqkv = (Hq + 2 * Hkv) * D, Tl = T - lo, R = B * Tl, V = c->vocab;
  const int Z = B * Hkv, SG = Sp * G, nl = c->layers;
  const float eps = c->eps, scale = 1.0f / sqrtf(c->query_pre_attn_scalar);
  Bump bp(ws);
  GemmaWs w = gemma_layout(bp, c, B, T, Sp, train);
  TailScratchScope tail(w.tail, st);
  CK(tail.status);
  AttnShape ash{B, Sp, Hq, Hkv, D};
  const RowMap ident{0, 0, 0, 0};
  const int Rp = (R + 63) / 64 * 64;
  StageSeq sq(st);
  sq.next("gemma.embed");

  // K11/K12: text embeddings (x bf16(sqrt H)), padded rows, key-valid mask; vision rows already in x
  const float escale = bfround_host(sqrtf((float)H));
  CK(launch_build_llm_inputs((const bf16_t*)wt->embed, bt->token_ids, B, T, Nv, S, Sp, H, escale, c->pad_token_id,
                             bt->x, w.key_valid, st));
  w.x[0] = bt->x;
  CK(launch_rmsnorm_fwd(w.x[0], H, ident, wt->layers[0].ln_in, train ? w.L[0].xn_in : w.xn, w.L[0].rstd_in, M, H,
                        eps, st));

  // position Nv-1+t predicts text token t: the only rows the loss reads from the last layer are those of
  // the targets t >= label_offset
  const RowMap lossmap{Tl, 0, Sp, Nv - 1 + lo};

  // ---------------- forward
  for (int l = 0; l < nl; ++l) {
    const ptk_gemma3_layer& L = wt->layers[l];
    GemmaLayerSave& sv = w.L[l];
    const bool sliding = (l + 1) % c->sliding_pattern != 0;
    const float* cs = sliding ? wt->rope_cos_local : wt->rope_cos_global;
    const float* sn = sliding ? wt->rope_sin_local : wt->rope_sin_global;
    bf16_t* xin = train ? sv.xn_in : w.xn;
    bf16_t* xff = train ? sv.xn_ff : w.xn;
    bf16_t* hh = train ? sv.h : w.h;
    sq.next("gemma.fwd.attn");
    CK(gemm_split(gemm(xin, H, L.wqkv, H, sv.qkv, Dqkv, M, Dqkv, H), OUT_BF16, w.skpart, w.sk_floats, st));
    CK(launch_qknorm_rope_fwd(sv.qkv, L.q_norm, L.k_norm, cs, sn, ash, eps, sv.Q, sv.K, sv.V, sv.rstd_q, sv.rstd_k,
                              st));
    {  // causal / sliding-window GQA attention, flash; O token-major, LSE kept for the backward
      FlashArgs fa;
      fa.Q = sv.Q; fa.K = sv.K; fa.V = sv.V; fa.O = sv.O; fa.lse = sv.lse;
      fa.rows = SG; fa.nkeys = Sp; fa.D = D;
      fa.ldq = D; fa.ldk = D; fa.ldo = D;
      fa.zin = Hkv; fa.zdiv = Hkv;
      fa.sQ0 = (long)Hkv * SG * D; fa.sQ1 = (long)SG * D;
      fa.sK0 = (long)Hkv * Sp * D; fa.sK1 = (long)Sp * D;
      fa.sO0 = (long)Sp * Hq * D; fa.sO1 = (long)G * D;
      fa.omap = RowMap{G, 0, Hq, 0};
      fa.qdiv = G; fa.causal = 1; fa.window = sliding ? c->sliding_window : 0;
      fa.key_valid = w.key_valid;
      fa.scale = scale;
      StageScope sf("gemma.fwd.flash", st);
      CK(launch_attn_fwd(fa, Z, st));
    }
    CK(gemm_split(gemm(sv.O, Dq, L.wo, Dq, sv.ao, H, M, H, Dq), OUT_BF16, w.skpart, w.sk_floats, st));
    CK(launch_residual_norm_fwd(sv.ao, w.x[l], L.ln_post_attn, L.ln_pre_ff, sv.x2, xff, sv.rstd_ao, sv.rstd_pre, M,
                                H, eps, st));
    sq.next("gemma.fwd.mlp");
    if (l + 1 < nl) {
      GemmArgs g = gemm(xff, H, L.wgu, H, hh, I, M, 2 * I, H);
      g.aux = sv.glu_a; g.aux2 = sv.glu_b; g.ld_aux = I;
      CK(launch_gemm(g, ACT_GEGLU, OUT_BF16, 1, st));
      CK(gemm_split(gemm(hh, I, L.wd, I, sv.dn, H, M, H, I), OUT_BF16, w.skpart, w.sk_floats, st));
    } else {
      // last layer: only the loss rows reach the loss, so its MLP runs on those R rows (h, glu_a, glu_b compact);
      // the other rows of dn are zero (their residual output is never read, their gradient is zero)
      GemmArgs g = gemm(xff, H, L.wgu, H, hh, I, R, 2 * I, H);
      g.amap = lossmap;
      g.aux = sv.glu_a; g.aux2 = sv.glu_b; g.ld_aux = I;
      CK(launch_gemm(g, ACT_GEGLU, OUT_BF16, 1, st));
      CK(launch_zero(sv.dn, (size_t)M * H * sizeof(bf16_t), st));
      GemmArgs g2 = gemm(hh, I, L.wd, I, sv.dn, H, R, H, I);
      g2.cmap = lossmap;
      CK(launch_gemm(g2, ACT_NONE, OUT_BF16, 1, st));
    }
    const float* wnext = (l + 1 < nl) ? wt->layers[l + 1].ln_in : nullptr;
    float* rnext = (l + 1 < nl) ? w.L[l + 1].rstd_in : nullptr;
    bf16_t* xnext = (train && l + 1 < nl) ? w.L[l + 1].xn_in : w.xn;
    CK(launch_residual_norm_fwd(sv.dn, sv.x2, L.ln_post_ff, wnext, w.x[l + 1], xnext, sv.rstd_dn, rnext, M, H, eps,
                                st));
  }

  // ---------------- loss (text-predicting rows only)
  sq.next("gemma.lm_head_ce");
  CK(launch_rmsnorm_fwd(w.x[nl], H, lossmap, wt->final_norm, w.xf, w.rstd_f, R, H, eps, st));
  {
    // lm_head: logits (bf16) plus, from the GEMM epilogue, each row's softmax statistics per 64 columns, so
    // the cross-entropy pass reads the 2 GB of logits once (loss_utils.py:49-67)
    GemmArgs g = gemm(w.xf, H, wt->embed, H, w.logits, V, R, V, H);
    if (w.ce_stats && !ce_two_pass()) {
      g.row_stats = w.ce_stats;
      g.ld_stats = (V / 64) * 2;
      g.stats_only = lm_stats_only() ? 1 : 0;
    }
    CK(launch_gemm(g, ACT_NONE, OUT_BF16, 1, st));
    CK(launch_count_valid(bt->labels, R, bt->loss_scale, w.gscale, w.count, st));
    if (g.row_stats)
      CK(launch_ce_stats_fwd_bwd(w.logits, V, R, V, w.ce_stats, g.ld_stats, bt->labels, w.row_loss, w.gscale, st));
    else
      CK(launch_ce_fwd_bwd(w.logits, V, R, V, bt->labels, w.row_loss, w.gscale, st));
  }
  CK(launch_loss_reduce(w.row_loss, R, w.count, bt->loss, st));
  if (fwd_only) return 0;   // validation loss (no_grad): the CE pass's d(logits) is left unused
  sq.next("gemma.lm_head_bwd");
  // tied lm_head weight grad: dE += dlogits^T . xf (the logits rows outside the loss rows have zero grad)
  if (train) CK(weight_grad(w.logits, V, ident, V, w.xf, H, ident, H, R, w.TL, w.TX, gr->embed, w.skpart, w.sk_floats, st));
  // (the K-sliced kernel addresses d(logits) with 32-bit buffer offsets: R x V bf16 must stay under 4 GiB -- at the
  // reference's default caption length T = 512, bs 32 puts 8.6 GB there, which the split-K path below takes)
  const bool ks_fits = (double)R * V * 2 + (double)LM_KSLICES * (V / LM_KSLICES) * 2 < 4293918720.0;
  if (R % 256 == 0 && V % (64 * LM_KSLICES) == 0 && ks_fits) {
    // d(xf) = dlogits . E, K = vocab, as LM_KSLICES K slices of 256x256 tiles on the 8-wave kernel: 80 tiles x 16
    // slices = 5 lock-step rounds at cfg2 (the 128x128 8-slice split ran 2.8 ms); fp32 partials, ordered sum
    GemmArgs g = gemm(w.logits, V, wt->embed_t, V, w.dxf_part, H, R, H, V / LM_KSLICES);
    CK(gemm_p8_kslices(g, LM_KSLICES, st));
    CK(launch_sum_partials(w.dxf_part, LM_KSLICES, (long)R * H, w.dxf, st));
  } else {  // d(xf) = dlogits . E, K = vocab: split-K over LM_SPLITK equal slices (fp32 partials, ordered sum);
     // a vocab that is not a multiple of 64 * LM_SPLITK (Gemma3-4B: 262 208 = 4 097 x 64) leaves a
     // remainder slice, computed into one more partial
    const int kc = V / (64 * LM_SPLITK) * 64, rem = V - LM_SPLITK * kc;
    GemmArgs g = gemm(w.logits, V, wt->embed_t, V, w.dxf_part, H, R, H, kc);
    g.sA0 = kc; g.sB0 = kc; g.sC0 = (long)R * H;
    CK(launch_gemm(g, ACT_NONE, OUT_F32, LM_SPLITK, st));
    if (rem) {
      const long o = (long)LM_SPLITK * kc;
      CK(launch_gemm(gemm(w.logits + o, V, (const bf16_t*)wt->embed_t + o, V, w.dxf_part + (long)LM_SPLITK * R * H, H, R, H, rem),
                     ACT_NONE, OUT_F32, 1, st));
    }
    CK(launch_sum_partials(w.dxf_part, LM_SPLITK + (rem ? 1 : 0), (long)R * H, w.dxf, st));
  }
  float* dR = bt->dx;
  CK(launch_zero(dR, (size_t)M * H * 4, st));
  CK(launch_rmsnorm_bwd_scatter(w.x[nl], lossmap, wt->final_norm, w.rstd_f, w.dxf, dR, R, H, st));
  if (train)
    CK(launch_rms_wgrad(w.x[nl], H, lossmap, w.rstd_f, w.dxf, H, 1, R, H, (bf16_t*)gr->final_norm, w.wpart, st));

  // ---------------- backward (dX; with gr, also every weight grad)
  for (int l = nl - 1; l >= 0; --l) {
    const ptk_gemma3_layer& L = wt->layers[l];
    const ptk_gemma3_layer_grads* GL = train ? &gr->layers[l] : nullptr;
    GemmaLayerSave& sv = w.L[l];
    const bool sliding = (l + 1) % c->sliding_pattern != 0;
    const float* cs = sliding ? wt->rope_cos_local : wt->rope_cos_global;
    const float* sn = sliding ? wt->rope_sin_local : wt->rope_sin_global;
    const bool last = l == nl - 1;
    sq.next("gemma.bwd.mlp");
    // MLP half
    // post-ff norm backward: for layers below the last it ran fused into the previous iteration's
    // input-norm backward (one pass over dR instead of two)
    if (last) {
      CK(launch_post_norm_bwd(dR, sv.dn, L.ln_post_ff, sv.rstd_dn, w.dao, M, H, st));
      if (train)
        CK(launch_rms_wgrad_bx(sv.dn, H, ident, sv.rstd_dn, dR, H, 1, M, H, (bf16_t*)GL->ln_post_ff, w.wpart, st));
    }
    // down projection weight grad: d(dn)^T . h (last layer: the loss rows and the compact h)
    if (train)
      CK(last ? weight_grad(w.dao, H, lossmap, H, sv.h, I, ident, I, R, w.TA, w.TB, GL->wd, w.skpart, w.sk_floats, st)
              : weight_grad(w.dao, H, ident, H, sv.h, I, ident, I, M, w.TA, w.TB, GL->wd, w.skpart, w.sk_floats, st));
    // d(gate|up) = GEGLU backward of dh = dd . Wd, fused into the persistent 4-wave GEMM's register
    // epilogue (the saved factors loaded one row block ahead: dg = dh * b, du = dh * a; dh never reaches HBM).  PTK_GEGLU_SPLIT=1: the plain
    // GEMM + one streaming geglu_bwd pass instead (A/B)
    if (!last) {
      if (geglu_split()) {
        CK(launch_gemm(gemm(w.dao, H, L.wd_t, H, w.h, I, M, I, H), ACT_NONE, OUT_BF16, 1, st));
        CK(launch_geglu_bwd(w.h, sv.glu_a, sv.glu_b, w.dgu, M, I, st));
      } else {
        GemmArgs g = gemm(w.dao, H, L.wd_t, H, w.dgu, 2 * I, M, I, H);
        g.aux_in = sv.glu_a;
        g.aux_in2 = sv.glu_b;
        g.ld_aux_in = I;
        CK(launch_gemm(g, ACT_GEGLU_BWD, OUT_BF16, 1, st));
      }
      if (train) CK(weight_grad(w.dgu, 2 * I, ident, 2 * I, sv.xn_ff, H, ident, H, M, w.TA, w.TB, GL->wgu, w.skpart, w.sk_floats, st));
      CK(gemm_split(gemm(w.dgu, 2 * I, L.wgu_t, 2 * I, w.dtmp, H, M, H, 2 * I), OUT_BF16, w.skpart, w.sk_floats, st));
    } else {   // last layer: MLP gradient is non-zero on the loss rows only (compact h, glu_a, glu_b, dgu)
      GemmArgs g = gemm(w.dao, H, L.wd_t, H, w.h, I, R, I, H);
      g.amap = lossmap;
      CK(launch_gemm(g, ACT_NONE, OUT_BF16, 1, st));
      CK(launch_geglu_bwd(w.h, sv.glu_a, sv.glu_b, w.dgu, R, I, st));
      if (train) CK(weight_grad(w.dgu, 2 * I, ident, 2 * I, sv.xn_ff, H, lossmap, H, R, w.TA, w.TB, GL->wgu, w.skpart, w.sk_floats, st));
      CK(launch_zero(w.dtmp, (size_t)M * H * sizeof(bf16_t), st));
      GemmArgs g2 = gemm(w.dgu, 2 * I, L.wgu_t, 2 * I, w.dtmp, H, R, H, 2 * I);
      g2.cmap = lossmap;
      CK(launch_gemm(g2, ACT_NONE, OUT_BF16, 1, st));
    }
    sq.next("gemma.bwd.attn");
    CK(residual_norm_bwd_grads(sv.x2, L.ln_pre_ff, sv.rstd_pre, w.dtmp, dR, sv.ao, L.ln_post_attn, sv.rstd_ao, w.dao,
                               M, H, train ? (bf16_t*)GL->ln_pre_ff : nullptr,
                               train ? (bf16_t*)GL->ln_post_attn : nullptr, w.wpart, st));
    if (train)
      CK(weight_grad(w.dao, H, ident, H, sv.O, Dq, ident, Dq, M, w.TA, w.TB, GL->wo, w.skpart, w.sk_floats, st));
    {  // dO (Q layout) = dao . Wo, one GEMM per kv head group of output columns
      GemmArgs g = gemm(w.dao, H, L.wo_t, H, w.dO, (long)G * D, M, G * D, H);
      g.sB0 = (long)G * D * H; g.sC0 = (long)Sp * G * D;
      g.cmap = RowMap{Sp, 0, (long)Hkv * Sp, 0};
      CK(launch_gemm(g, ACT_NONE, OUT_BF16, Hkv, st));
    }
    FlashBwdArgs dkv_plan;   // split-slab dK/dV partials finished by qknorm_rope_bwd
    dkv_plan.dkv_deferred = 0;
    {  // flash attention backward: delta = rowsum(dO*O), dK/dV per key block, dQ per query block
      FlashBwdArgs fb;
      fb.Q = sv.Q; fb.K = sv.K; fb.V = sv.V; fb.O = sv.O; fb.dO = w.dO; fb.lse = sv.lse; fb.delta = w.delta;
      fb.dQ = w.dQ; fb.dK = w.dK; fb.dV = w.dV;
      fb.rows = SG; fb.nkeys = Sp; fb.D = D;
      fb.zin = Hkv; fb.zdiv = Hkv;
      fb.ldo = D; fb.sO0 = (long)Sp * Hq * D; fb.sO1 = (long)G * D;
      fb.omap = RowMap{G, 0, Hq, 0};
      fb.qdiv = G; fb.causal = 1; fb.window = sliding ? c->sliding_window : 0;
      fb.key_valid = w.key_valid;
      fb.scale = scale;
      fb.dkv_part = w.dkv_part; fb.dkv_part_bytes = w.dkv_part_bytes;
      StageScope sf("gemma.bwd.flash", st);
      // the k_norm weight grad reads the complete dK: the unfrozen path reduces split slabs in attn_bwd
      CK(launch_attn_bwd(fb, Z, st, (dkv_reduce_split() || train) ? nullptr : &dkv_plan));
    }
    CK(launch_qknorm_rope_bwd(sv.qkv, L.q_norm, L.k_norm, cs, sn, ash, sv.rstd_q, sv.rstd_k, w.dQ, w.dK, w.dV, w.dqkv,
                              st, &dkv_plan));
    if (train) {
      CK(launch_qknorm_wgrad(sv.qkv, cs, sn, ash, sv.rstd_q, sv.rstd_k, w.dQ, w.dK, (bf16_t*)GL->q_norm,
                             (bf16_t*)GL->k_norm, w.wpart, st));
      CK(weight_grad(w.dqkv, Dqkv, ident, Dqkv, sv.xn_in, H, ident, H, M, w.TA, w.TB, GL->wqkv, w.skpart, w.sk_floats, st));
    }
    CK(gemm_split(gemm(w.dqkv, Dqkv, L.wqkv_t, Dqkv, w.dtmp, H, M, H, Dqkv), OUT_BF16, w.skpart, w.sk_floats, st));
    if (l > 0) {
      // dR += rms_bwd(x_l, ln_in, dtmp), then layer l-1's post-ff norm backward on the new dR -> dao
      const ptk_gemma3_layer& Lp = wt->layers[l - 1];
      const GemmaLayerSave& sp = w.L[l - 1];
      CK(residual_norm_bwd_grads(w.x[l], L.ln_in, sv.rstd_in, w.dtmp, dR, sp.dn, Lp.ln_post_ff, sp.rstd_dn, w.dao,
                                 M, H, train ? (bf16_t*)GL->ln_in : nullptr,
                                 train ? (bf16_t*)gr->layers[l - 1].ln_post_ff : nullptr, w.wpart, st));
    } else {
      if (train)
        CK(launch_rms_wgrad_bdy(w.x[l], H, ident, sv.rstd_in, w.dtmp, H, M, H, (bf16_t*)GL->ln_in, w.wpart, st));
      CK(launch_rmsnorm_bwd_bdn(w.x[l], L.ln_in, sv.rstd_in, w.dtmp, dR, dR, M, H, st));
    }
  }
  // input-embedding grads of every text token (tied with the lm_head grad above)
  if (train) sq.next("gemma.embed_grad");
  if (train) CK(launch_embed_grad(bt->token_ids, B, T, Nv, Sp, H, escale, dR, (bf16_t*)gr->embed, w.eg_keys, st));
  return 0;
}

}  // namespace

namespace {

// ------------------------------------------------------------------ Gemma3 KV-cache decode (generate)
// Stage1/projector_trainer.py:386-393 -> GenerationMixin._sample over Gemma3ForCausalLM with a cache: a prefill of
// the prompt embeddings, then one position per step.  Each layer is the training forward's launch sequence (same
// kernels, same fp32 residual stream and bf16 GEMM operands) on the rows of the pass; the step's attention reads
// the layer's K / V cache [B, Hkv, Smax, D] (the prefill writes its rows, each step appends one), over keys
// [0, p] on full layers and the last `sliding_window` of them on sliding layers (TF/masking_utils.py:92-101:
// key > p - W).
struct GenPass {            // per-pass activations (rows = B * S)
  float *xa, *xb, *x2, *rs1, *rs2, *rq, *rk;
  bf16_t *xn, *qkv, *Q, *K, *V, *O, *ao, *h, *dn;
  int32_t* kv;
  float* skp = nullptr;     // decode passes: the skinny GEMM's K-split partials
  size_t skp_bytes = 0;
};
// the partial buffer the skinny GEMM needs for the decode projections and the lm_head at `rows` rows
size_t gen_skinny_bytes(const ptk_gemma3_config* c, long rows) {
  if (rows > 256) return 0;   // (decode passes up to 256 rows run as 64-row chunks)
  rows = std::min<long>(rows, 64);
  const int H = c->hidden, I = c->inter, D = c->head_dim, Dq = c->heads * D, Dqkv = (c->heads + 2 * c->kv_heads) * D;
  const int M = (int)rows;
  const int shapes[5][2] = {{Dqkv, H}, {H, Dq}, {2 * I, H}, {H, I}, {c->vocab, H}};   // (N, K)
  size_t b = 0;
  for (const auto& nk : shapes) b = std::max(b, skinny_part_bytes(M, nk[0], nk[1]));
  return b;
}
// a decode-pass GEMM (bf16 out): the skinny kernel where it applies, else the general dispatch
int gen_gemm(const GenPass& g, const bf16_t* A, long lda, const void* B, long ldb, bf16_t* C, long ldc, int M, int N,
             int K, int act, hipStream_t st) {
  if (g.skp_bytes > 0 && skinny_supported(std::min(M, 64), N, K, lda, ldb, ldc, act)) {
    for (int r0 = 0; r0 < M; r0 += 64)   // (each 64-row chunk streams the weights once more)
      CK(launch_gemm_skinny(A + (long)r0 * lda, lda, (const bf16_t*)B, ldb, C + (long)r0 * ldc, ldc, std::min(64, M - r0),
                            N, K, act, g.skp, g.skp_bytes, st));
    return 0;
  }
  return launch_gemm(gemm(A, lda, B, ldb, C, ldc, M, N, K), act, OUT_BF16, 1, st);
}
struct GenWs {
  GenPass pre, dec;
  std::vector<bf16_t*> kc, vc;     // per layer [B, Hkv, Smax, D]
  bf16_t *xf, *logits;
  float* rstd_f;
  int32_t* finished;
  int64_t *next, *feed;
  void* tail;
};
GenPass gen_pass(Bump& bp, const ptk_gemma3_config* c, long M) {
  const long H = c->hidden, I = c->inter, D = c->head_dim, Hq = c->heads, Hkv = c->kv_heads;
  const long Dq = Hq * D, Dqkv = (Hq + 2 * Hkv) * D;
  GenPass g;
  g.xa = bp.take<float>(M * H);
  g.xb = bp.take<float>(M * H);
  g.x2 = bp.take<float>(M * H);
  g.rs1 = bp.take<float>(M);
  g.rs2 = bp.take<float>(M);
  g.rq = bp.take<float>(M * Hq);
  g.rk = bp.take<float>(M * Hkv);
  g.xn = bp.take<bf16_t>(M * H);
  g.qkv = bp.take<bf16_t>(M * Dqkv);
  g.Q = bp.take<bf16_t>(M * Dq);
  g.K = bp.take<bf16_t>(M * Hkv * D);
  g.V = bp.take<bf16_t>(M * Hkv * D);
  g.O = bp.take<bf16_t>(M * Dq);
  g.ao = bp.take<bf16_t>(M * H);
  g.h = bp.take<bf16_t>(M * I);
  g.dn = bp.take<bf16_t>(M * H);
  g.kv = bp.take<int32_t>(M);
  g.skp_bytes = gen_skinny_bytes(c, M);
  g.skp = g.skp_bytes ? bp.take<float>(g.skp_bytes / 4) : nullptr;
  return g;
}
GenWs gen_layout(Bump& bp, const ptk_gemma3_config* c, int B, int P, int max_new) {
  const long Pp = (P + 63) / 64 * 64, Smax = (P + max_new + 63) / 64 * 64;
  const long Z = (long)B * c->kv_heads, D = c->head_dim;
  GenWs w;
  w.pre = gen_pass(bp, c, (long)B * Pp);
  w.dec = gen_pass(bp, c, B);
  for (int l = 0; l < c->layers; ++l) {
    w.kc.push_back(bp.take<bf16_t>(Z * Smax * D));
    w.vc.push_back(bp.take<bf16_t>(Z * Smax * D));
  }
  w.xf = bp.take<bf16_t>((long)B * c->hidden);
  w.logits = bp.take<bf16_t>((long)B * c->vocab);
  w.rstd_f = bp.take<float>(B);
  w.finished = bp.take<int32_t>(B);
  w.next = bp.take<int64_t>(B);
  w.feed = bp.take<int64_t>(B);
  w.tail = bp.take<char>(p8_tail_scratch_bytes_models());
  return w;
}

// one decoder layer over the S positions of each of B rows of pass g (Sp = S rounded the pass's way: the prefill's
// padded prompt, 1 for a decode step): x_in -> x_out (fp32), the layer's K / V appended to the cache at p0, the
// queries attending cache keys [k_lo, p0 + S) (prefill: causal + window over its own rows, decode: the window
// start k_lo); xn holds the layer's input norm on entry and the next layer's on exit (w_next: none -> untouched)
// The stepwise decode's extras (DecMasks, null for ptk_gemma3_generate): RoPE positions per token (pos: the prefill's
// cumsum positions, a decode step's per-row position) and the decode step's key flags over cache slots
// [k_lo, k_lo + nk) for sliding (0) and full (1) layers.
struct DecMasks {
  const int32_t* pos;
  const int32_t* kmask[2];
  int k_lo[2], nk[2];
};
int gen_layer(const ptk_gemma3_config* c, const ptk_gemma3_weights* wt, int l, GenPass& g, const float* x_in,
              float* x_out, int B, int S, int Sp, int p0, bool prefill, int Smax, bf16_t* kc, bf16_t* vc,
              hipStream_t st, const DecMasks* dm = nullptr) {
  const ptk_gemma3_layer& L = wt->layers[l];
  const int H = c->hidden, I = c->inter, D = c->head_dim, Hq = c->heads, Hkv = c->kv_heads, G = Hq / Hkv;
  const int M = B * Sp, Dq = Hq * D, Dqkv = (Hq + 2 * Hkv) * D, Z = B * Hkv;
  const bool sliding = (l + 1) % c->sliding_pattern != 0;
  const long pofs = (dm && dm->pos) ? 0 : (long)p0 * (D / 2);   // per-token positions index the whole table
  const float* cs = (sliding ? wt->rope_cos_local : wt->rope_cos_global) + pofs;
  const float* sn = (sliding ? wt->rope_sin_local : wt->rope_sin_global) + pofs;
  CK(gen_gemm(g, g.xn, H, L.wqkv, H, g.qkv, Dqkv, M, Dqkv, H, ACT_NONE, st));
  AttnShape ash{B, Sp, Hq, Hkv, D};
  if (dm) ash.pos = dm->pos;
  CK(launch_qknorm_rope_fwd(g.qkv, L.q_norm, L.k_norm, cs, sn, ash, c->eps, g.Q, g.K, g.V, g.rq, g.rk, st));
  CK(launch_kv_append(g.K, (long)Sp * D, kc, (long)Smax * D, Z, p0, S, D, st));
  CK(launch_kv_append(g.V, (long)Sp * D, vc, (long)Smax * D, Z, p0, S, D, st));
  {
    FlashArgs fa;
    fa.Q = g.Q; fa.O = g.O; fa.lse = nullptr;
    fa.rows = Sp * G; fa.D = D;
    fa.ldq = D; fa.ldk = D; fa.ldo = D;
    fa.zin = Hkv; fa.zdiv = Hkv;
    fa.sQ0 = (long)Hkv * Sp * G * D; fa.sQ1 = (long)Sp * G * D;
    fa.sK0 = (long)Hkv * Smax * D; fa.sK1 = (long)Smax * D;
    fa.sO0 = (long)Sp * Hq * D; fa.sO1 = (long)G * D;
    fa.omap = RowMap{G, 0, Hq, 0};
    fa.qdiv = G;
    fa.scale = 1.0f / sqrtf(c->query_pre_attn_scalar);
    if (prefill) {   // the prompt's own keys: causal, the window on sliding layers, padded rows masked
      fa.K = g.K; fa.V = g.V;
      fa.sK0 = (long)Hkv * Sp * D; fa.sK1 = (long)Sp * D;
      fa.nkeys = Sp; fa.causal = 1; fa.window = sliding ? c->sliding_window : 0;
      fa.key_valid = g.kv;
    } else if (dm) {  // one query per row against cache slots [k_lo, k_lo + nk), the row's key flags
      const int w = sliding ? 0 : 1;
      fa.K = kc + (long)dm->k_lo[w] * D; fa.V = vc + (long)dm->k_lo[w] * D;
      fa.nkeys = dm->nk[w]; fa.causal = 0; fa.window = 0;
      fa.key_valid = dm->kmask[w];
    } else {         // one query position p0 against cache keys [k_lo, p0]
      const int k_lo = (sliding && c->sliding_window > 0) ? std::max(0, p0 - c->sliding_window + 1) : 0;
      fa.K = kc + (long)k_lo * D; fa.V = vc + (long)k_lo * D;
      fa.nkeys = p0 + 1 - k_lo; fa.causal = 0; fa.window = 0;
      fa.key_valid = nullptr;
    }
    CK(launch_attn_fwd(fa, Z, st));
  }
  CK(gen_gemm(g, g.O, Dq, L.wo, Dq, g.ao, H, M, H, Dq, ACT_NONE, st));
  CK(launch_residual_norm_fwd(g.ao, x_in, L.ln_post_attn, L.ln_pre_ff, g.x2, g.xn, g.rs1, g.rs2, M, H, c->eps, st));
  CK(gen_gemm(g, g.xn, H, L.wgu, H, g.h, I, M, 2 * I, H, ACT_GEGLU, st));   // (no saved GEGLU factors: no backward)
  CK(gen_gemm(g, g.h, I, L.wd, I, g.dn, H, M, H, I, ACT_NONE, st));
  const float* wnext = (l + 1 < c->layers) ? wt->layers[l + 1].ln_in : nullptr;
  CK(launch_residual_norm_fwd(g.dn, g.x2, L.ln_post_ff, wnext, x_out, g.xn, g.rs1, g.rs2, M, H, c->eps, st));
  return 0;
}

int gemma_generate(const ptk_gemma3_config* c, const ptk_gemma3_weights* wt, const ptk_gemma3_generate_desc* gd,
                   const float* prompt, const int64_t* force, int64_t* out_ids, bf16_t* step_logits, void* ws,
                   size_t ws_bytes, hipStream_t st) {
  const int B = gd->batch, P = gd->prompt_len, NT = gd->max_new_tokens;
  if (B <= 0 || P < 4 || NT <= 0) return set_error("generate: batch %d, prompt_len %d (>= 4), max_new_tokens %d", B, P, NT);
  if (gd->prompt_batch_stride < P) return set_error("generate: prompt_batch_stride %ld < prompt_len %d",
                                                    (long)gd->prompt_batch_stride, P);
  if (P + NT > wt->rope_max_pos || (P + 63) / 64 * 64 > wt->rope_max_pos)
    return set_error("generate: %d positions exceed the rope tables (%d)", P + NT, wt->rope_max_pos);
  if (c->heads % c->kv_heads) return set_error("generate: heads %% kv_heads");
  if (ws_bytes < ptk_gemma3_generate_workspace_bytes(c, B, P, NT)) return set_error("generate: workspace too small");
  const int H = c->hidden, V = c->vocab, Pp = (P + 63) / 64 * 64, Smax = (P + NT + 63) / 64 * 64;
  Bump bp(ws);
  GenWs w = gen_layout(bp, c, B, P, NT);
  TailScratchScope tail(w.tail, st);
  CK(tail.status);
  const float escale = bfround_host(sqrtf((float)H));
  CK(launch_zero(w.finished, ((size_t)B * 4 + 15) / 16 * 16, st));
  // logits row b -> sampled token, into out_ids[:, t]
  auto head = [&](const float* x, RowMap map, int t) -> int {
    CK(launch_rmsnorm_fwd(x, H, map, wt->final_norm, w.xf, w.rstd_f, B, H, c->eps, st));
    CK(gen_gemm(w.dec, w.xf, H, wt->embed, H, w.logits, V, B, V, H, ACT_NONE, st));
    if (step_logits)
      CKH(hipMemcpyAsync(step_logits + (long)t * B * V, w.logits, (size_t)B * V * 2, hipMemcpyDeviceToDevice, st));
    return launch_gen_sample(w.logits, V, B, V, gd->do_sample, gd->top_k, gd->temperature,
                             gd->top_p > 0.f ? gd->top_p : 1.f, gd->seed, t,
                             (long)gd->eos_token_id, (long)gd->pad_token_id, w.finished, out_ids + t, NT, w.next, st);
  };
  // prefill: the prompt rows, padded per sample to Pp (masked keys), every layer's K / V into the cache
  {
    GenPass& g = w.pre;
    CK(launch_gen_prompt(prompt, (long)gd->prompt_batch_stride, B, P, Pp, H, g.xa, g.kv, st));
    CK(launch_rmsnorm_fwd(g.xa, H, RowMap{0, 0, 0, 0}, wt->layers[0].ln_in, g.xn, g.rs1, B * Pp, H, c->eps, st));
    float *xi = g.xa, *xo = g.xb;
    for (int l = 0; l < c->layers; ++l) {
      CK(gen_layer(c, wt, l, g, xi, xo, B, P, Pp, 0, true, Smax, w.kc[l], w.vc[l], st));
      std::swap(xi, xo);
    }
    CK(head(xi, RowMap{1, 0, Pp, P - 1}, 0));   // the last prompt position of each sample
  }
  // decode: step t feeds the token drawn at t - 1 (or force[:, t - 1]) at position P + t - 1
  for (int t = 1; t < NT; ++t) {
    GenPass& g = w.dec;
    const int p = P + t - 1;
    const int64_t* ids = w.next;
    if (force) {
      CKH(hipMemcpy2DAsync(w.feed, 8, force + (t - 1), (size_t)NT * 8, 8, B, hipMemcpyDeviceToDevice, st));
      ids = w.feed;
    }
    CK(launch_build_llm_inputs((const bf16_t*)wt->embed, ids, B, 1, 0, 1, 1, H, escale, -1, g.xa, g.kv, st));
    CK(launch_rmsnorm_fwd(g.xa, H, RowMap{0, 0, 0, 0}, wt->layers[0].ln_in, g.xn, g.rs1, B, H, c->eps, st));
    float *xi = g.xa, *xo = g.xb;
    for (int l = 0; l < c->layers; ++l) {
      CK(gen_layer(c, wt, l, g, xi, xo, B, 1, 1, p, false, Smax, w.kc[l], w.vc[l], st));
      std::swap(xi, xo);
    }
    CK(head(xi, RowMap{0, 0, 0, 0}, t));
  }
  return 0;
}

// ------------------------------------------------------------------ stepwise decode (beam search)
// The stepwise form of the decode: ptk_gemma3_decode_prefill once, then ptk_gemma3_decode_step per token, the
// caller choosing the tokens and (beam search) the cache rows each step takes from.  The workspace carries the
// caches and per-row state between calls.  Rows = prompts x repeat (beams): the prefill runs on the prompts and
// copies each one's caches, flags and logits to its `repeat` rows (GenerationMixin._expand_inputs_for_generation).
struct DecWs {
  GenPass pre, dec;
  std::vector<bf16_t*> kc, vc;     // per layer [rows, Hkv, Smax, D]
  bf16_t *tmp, *xf, *logits_pre;   // tmp: one cache tensor (row gathers)
  float* rstd_f;
  int32_t *pos_pre, *pos_dec, *slot_ok, *slot_tmp, *nvalid, *nvalid_tmp, *kmask[2], *rep_src;
  void* tail;
  int Pp, Smax, prompts;
};
DecWs dec_layout(Bump& bp, const ptk_gemma3_config* c, const ptk_gemma3_decode_desc* d) {
  DecWs w;
  const int rows = d->rows, P = d->prompt_len, R = d->prompt_repeat;
  w.prompts = R > 0 ? rows / R : rows;
  w.Pp = (P + 63) / 64 * 64;
  w.Smax = (P + d->max_new_tokens + 4 + 63) / 64 * 64;   // + 4: a step's key window rounds up to 4 slots
  const long Z = (long)rows * c->kv_heads, D = c->head_dim, cache = Z * w.Smax * D;
  w.pre = gen_pass(bp, c, (long)w.prompts * w.Pp);
  w.dec = gen_pass(bp, c, rows);
  for (int l = 0; l < c->layers; ++l) {
    w.kc.push_back(bp.take<bf16_t>(cache));
    w.vc.push_back(bp.take<bf16_t>(cache));
  }
  w.tmp = bp.take<bf16_t>(cache);
  w.xf = bp.take<bf16_t>((long)rows * c->hidden);
  w.logits_pre = bp.take<bf16_t>((long)w.prompts * c->vocab);
  w.rstd_f = bp.take<float>(rows);
  w.pos_pre = bp.take<int32_t>((long)w.prompts * w.Pp);
  w.pos_dec = bp.take<int32_t>(rows);
  w.slot_ok = bp.take<int32_t>((long)rows * w.Smax);
  w.slot_tmp = bp.take<int32_t>((long)rows * w.Smax);
  w.nvalid = bp.take<int32_t>(rows + 4);
  w.nvalid_tmp = bp.take<int32_t>(rows + 4);
  w.kmask[0] = bp.take<int32_t>((long)rows * w.Smax);
  w.kmask[1] = bp.take<int32_t>((long)rows * w.Smax);
  w.rep_src = bp.take<int32_t>(rows);
  w.tail = bp.take<char>(p8_tail_scratch_bytes_models());
  return w;
}
int dec_check(const ptk_gemma3_config* c, const ptk_gemma3_weights* wt, const ptk_gemma3_decode_desc* d, size_t ws_bytes) {
  if (!c || !wt || !d) return set_error("decode: NULL argument");
  const int rows = d->rows, P = d->prompt_len, NT = d->max_new_tokens, R = d->prompt_repeat;
  if (rows <= 0 || R <= 0 || rows % R || P < 4 || NT <= 0)
    return set_error("decode: rows %d, prompt_repeat %d (divides rows), prompt_len %d (>= 4), max_new_tokens %d", rows,
                     R, P, NT);
  if (d->prompt_batch_stride < P) return set_error("decode: prompt_batch_stride %ld < prompt_len %d",
                                                   (long)d->prompt_batch_stride, P);
  if (P + NT > wt->rope_max_pos || (P + 63) / 64 * 64 > wt->rope_max_pos)
    return set_error("decode: %d positions exceed the rope tables (%d)", P + NT, wt->rope_max_pos);
  if (c->heads % c->kv_heads) return set_error("decode: heads %% kv_heads");
  if (ws_bytes < ptk_gemma3_decode_workspace_bytes(c, d)) return set_error("decode: workspace too small");
  return 0;
}
// every cache row r <- row src[r] (through tmp), and the rows' slot flags and valid counts
int dec_gather(const ptk_gemma3_config* c, DecWs& w, const int32_t* src, int rows, hipStream_t st) {
  const long row_bytes = (long)c->kv_heads * w.Smax * c->head_dim * 2;
  for (int l = 0; l < c->layers; ++l)
    for (bf16_t* t : {w.kc[l], w.vc[l]}) {
      CK(launch_dec_gather_rows(t, w.tmp, src, rows, row_bytes, st));
      CKH(hipMemcpyAsync(t, w.tmp, (size_t)rows * row_bytes, hipMemcpyDeviceToDevice, st));
    }
  CK(launch_dec_gather_rows(w.slot_ok, w.slot_tmp, src, rows, (long)w.Smax * 4, st));
  CKH(hipMemcpyAsync(w.slot_ok, w.slot_tmp, (size_t)rows * w.Smax * 4, hipMemcpyDeviceToDevice, st));
  CK(launch_dec_gather_i32(w.nvalid, w.nvalid_tmp, src, rows, st));
  CKH(hipMemcpyAsync(w.nvalid, w.nvalid_tmp, (size_t)rows * 4, hipMemcpyDeviceToDevice, st));
  return 0;
}
int gemma_decode_prefill(const ptk_gemma3_config* c, const ptk_gemma3_weights* wt, const ptk_gemma3_decode_desc* d,
                         const float* prompt, const int32_t* mask, long mask_ld, bf16_t* logits, void* ws,
                         size_t ws_bytes, hipStream_t st) {
  CK(dec_check(c, wt, d, ws_bytes));
  const int rows = d->rows, P = d->prompt_len, R = d->prompt_repeat, H = c->hidden, V = c->vocab;
  Bump bp(ws);
  DecWs w = dec_layout(bp, c, d);
  const int Bp = w.prompts, Pp = w.Pp, Smax = w.Smax;
  TailScratchScope tail(w.tail, st);
  CK(tail.status);
  const long cache_bytes = (long)rows * c->kv_heads * Smax * c->head_dim * 2;
  for (int l = 0; l < c->layers; ++l) {   // slots past a step's position are read (masked) by the key window
    CK(launch_zero(w.kc[l], (size_t)cache_bytes, st));
    CK(launch_zero(w.vc[l], (size_t)cache_bytes, st));
  }
  GenPass& g = w.pre;
  CK(launch_dec_prompt(prompt, (long)d->prompt_batch_stride, mask, mask_ld, 1, Bp, P, Pp, H, g.xa, g.kv, st));
  CK(launch_dec_positions(g.kv, Bp, P, Pp, Smax, w.pos_pre, w.slot_ok, w.nvalid, st));
  CK(launch_rmsnorm_fwd(g.xa, H, RowMap{0, 0, 0, 0}, wt->layers[0].ln_in, g.xn, g.rs1, Bp * Pp, H, c->eps, st));
  DecMasks dm{};
  dm.pos = w.pos_pre;
  float *xi = g.xa, *xo = g.xb;
  for (int l = 0; l < c->layers; ++l) {
    CK(gen_layer(c, wt, l, g, xi, xo, Bp, P, Pp, 0, true, Smax, w.kc[l], w.vc[l], st, &dm));
    std::swap(xi, xo);
  }
  CK(launch_rmsnorm_fwd(xi, H, RowMap{1, 0, Pp, P - 1}, wt->final_norm, w.xf, w.rstd_f, Bp, H, c->eps, st));
  bf16_t* lg = R == 1 ? logits : w.logits_pre;
  CK(launch_gemm(gemm(w.xf, H, wt->embed, H, lg, V, Bp, V, H), ACT_NONE, OUT_BF16, 1, st));
  if (R > 1) {   // prompt b -> rows b*R .. b*R + R - 1
    CK(launch_dec_repeat_index(w.rep_src, rows, R, st));
    CK(launch_dec_gather_rows(w.logits_pre, logits, w.rep_src, rows, (long)V * 2, st));
    CK(dec_gather(c, w, w.rep_src, rows, st));
  }
  return 0;
}
int gemma_decode_step(const ptk_gemma3_config* c, const ptk_gemma3_weights* wt, const ptk_gemma3_decode_desc* d,
                      int t, const int64_t* ids, const int32_t* src_rows, bf16_t* logits, void* ws, size_t ws_bytes,
                      hipStream_t st) {
  CK(dec_check(c, wt, d, ws_bytes));
  const int rows = d->rows, P = d->prompt_len, H = c->hidden, V = c->vocab;
  if (t < 1 || t >= d->max_new_tokens) return set_error("decode: step %d outside 1..%d", t, d->max_new_tokens - 1);
  if (!ids) return set_error("decode: ids is NULL");
  Bump bp(ws);
  DecWs w = dec_layout(bp, c, d);
  TailScratchScope tail(w.tail, st);
  CK(tail.status);
  if (src_rows) CK(dec_gather(c, w, src_rows, rows, st));
  const int p0 = P + t - 1;
  DecMasks dm{};
  dm.pos = w.pos_dec;
  for (int k = 0; k < 2; ++k) {   // 0: sliding layers (the last `sliding_window` slots), 1: full layers
    const int lo = (k == 0 && c->sliding_window > 0) ? std::max(0, p0 - c->sliding_window + 1) : 0;
    dm.k_lo[k] = lo;
    dm.nk[k] = (p0 + 1 - lo + 3) / 4 * 4;
    dm.kmask[k] = w.kmask[k];
    CK(launch_dec_step_prep(w.slot_ok, w.nvalid, rows, w.Smax, p0, t, lo, dm.nk[k], w.pos_dec, w.kmask[k], st));
  }
  GenPass& g = w.dec;
  const float escale = bfround_host(sqrtf((float)H));
  CK(launch_build_llm_inputs((const bf16_t*)wt->embed, ids, rows, 1, 0, 1, 1, H, escale, -1, g.xa, g.kv, st));
  CK(launch_rmsnorm_fwd(g.xa, H, RowMap{0, 0, 0, 0}, wt->layers[0].ln_in, g.xn, g.rs1, rows, H, c->eps, st));
  float *xi = g.xa, *xo = g.xb;
  for (int l = 0; l < c->layers; ++l) {
    CK(gen_layer(c, wt, l, g, xi, xo, rows, 1, 1, p0, false, w.Smax, w.kc[l], w.vc[l], st, &dm));
    std::swap(xi, xo);
  }
  CK(launch_rmsnorm_fwd(xi, H, RowMap{0, 0, 0, 0}, wt->final_norm, w.xf, w.rstd_f, rows, H, c->eps, st));
  CK(gen_gemm(w.dec, w.xf, H, wt->embed, H, logits, V, rows, V, H, ACT_NONE, st));
  return 0;
}

}  // namespace

extern "C" {

size_t ptk_gemma3_decode_workspace_bytes(const ptk_gemma3_config* c, const ptk_gemma3_decode_desc* d) {
  if (!c || !d || d->rows <= 0 || d->prompt_repeat <= 0) return 0;
  Bump bp(nullptr);
  dec_layout(bp, c, d);
  return bp.off + 256;
}

int ptk_gemma3_decode_prefill(const ptk_gemma3_config* c, const ptk_gemma3_weights* w, const ptk_gemma3_decode_desc* d,
                              const float* prompt_embeds, const int32_t* prompt_mask, int64_t prompt_mask_ld,
                              void* logits, void* ws, size_t ws_bytes, void* stream) {
  if (!prompt_embeds || !logits || !ws) return set_error("decode_prefill: NULL argument");
  if (prompt_mask && d && prompt_mask_ld < d->prompt_len) return set_error("decode_prefill: prompt_mask_ld < prompt_len");
  return gemma_decode_prefill(c, w, d, prompt_embeds, prompt_mask, (long)prompt_mask_ld, (bf16_t*)logits, ws, ws_bytes,
                              (hipStream_t)stream);
}

int ptk_gemma3_decode_step(const ptk_gemma3_config* c, const ptk_gemma3_weights* w, const ptk_gemma3_decode_desc* d,
                           int step, const int64_t* ids, const int32_t* src_rows, void* logits, void* ws,
                           size_t ws_bytes, void* stream) {
  if (!logits || !ws) return set_error("decode_step: NULL argument");
  return gemma_decode_step(c, w, d, step, ids, src_rows, (bf16_t*)logits, ws, ws_bytes, (hipStream_t)stream);
}

size_t ptk_beam_candidates_workspace_bytes(int batch, int beams, int n_cand) {
  return beam_candidates_ws_bytes(batch, beams, n_cand);
}

int ptk_beam_candidates(const void* logits, int64_t ld, const float* beam_scores, int batch, int beams, int vocab,
                        int do_sample, int top_k, float top_p, float temperature, int min_tokens_to_keep,
                        uint64_t seed, int step, int n_cand, int64_t* tokens, int32_t* beam_idx, float* scores,
                        void* ws, size_t ws_bytes, void* stream) {
  if (!logits || !beam_scores || !tokens || !beam_idx || !scores) return set_error("beam_candidates: NULL argument");
  if (ld < vocab) return set_error("beam_candidates: ld < vocab");
  return launch_beam_candidates((const bf16_t*)logits, (long)ld, beam_scores, batch, beams, vocab, do_sample, top_k,
                                top_p, temperature, min_tokens_to_keep, seed, step, n_cand, tokens, beam_idx, scores,
                                ws, ws_bytes, (hipStream_t)stream);
}

int ptk_gemma3_loss_fwd_bwd(const ptk_gemma3_config* c, const ptk_gemma3_weights* wt, const ptk_gemma3_batch* bt,
                            void* ws, size_t ws_bytes, void* stream) {
  return gemma_run(c, wt, bt, nullptr, ws, ws_bytes, (hipStream_t)stream);
}

int ptk_gemma3_loss_fwd(const ptk_gemma3_config* c, const ptk_gemma3_weights* wt, const ptk_gemma3_batch* bt,
                        void* ws, size_t ws_bytes, void* stream) {
  return gemma_run(c, wt, bt, nullptr, ws, ws_bytes, (hipStream_t)stream, true);
}

int ptk_gemma3_train_fwd_bwd(const ptk_gemma3_config* c, const ptk_gemma3_weights* wt, const ptk_gemma3_batch* bt,
                             const ptk_gemma3_grads* g, void* ws, size_t ws_bytes, void* stream) {
  if (!g) return set_error("gemma3 train: grads is NULL");
  return gemma_run(c, wt, bt, g, ws, ws_bytes, (hipStream_t)stream);
}

size_t ptk_gemma3_generate_workspace_bytes(const ptk_gemma3_config* c, int batch, int prompt_len, int max_new_tokens) {
  Bump bp(nullptr);
  gen_layout(bp, c, batch, prompt_len, max_new_tokens);
  return bp.off + 256;
}

int ptk_gemma3_generate(const ptk_gemma3_config* c, const ptk_gemma3_weights* w, const ptk_gemma3_generate_desc* g,
                        const float* prompt_embeds, const int64_t* force_ids, int64_t* out_ids, void* step_logits,
                        void* ws, size_t ws_bytes, void* stream) {
  if (!c || !w || !g || !prompt_embeds || !out_ids) return set_error("generate: NULL argument");
  return gemma_generate(c, w, g, prompt_embeds, force_ids, out_ids, (bf16_t*)step_logits, ws, ws_bytes,
                        (hipStream_t)stream);
}

int ptk_bf16_sumsq_partial_floats(void) { return scale_sumsq_partial_floats(); }

int ptk_bf16_grad_scale_sumsq(void* g, int64_t n, float scale, float* partial, float* out, void* stream) {
  return launch_scale_sumsq_bf16((bf16_t*)g, n, scale, partial, out, (hipStream_t)stream);
}

int ptk_adamw_bf16(void* params, void* grads, void* exp_avg, void* exp_avg_sq, int64_t n, const float* sumsq_total,
                   float max_norm, double lr, double beta1, double beta2, double eps, double weight_decay, int step,
                   float* norm_out, void* stream) {
  return launch_adamw_bf16((bf16_t*)params, (bf16_t*)grads, (bf16_t*)exp_avg, (bf16_t*)exp_avg_sq, n, sumsq_total,
                           max_norm, lr, beta1, beta2, eps, weight_decay, step, norm_out, (hipStream_t)stream);
}

}  // extern "C"
