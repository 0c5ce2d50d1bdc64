// Internal (C++) interface between the HIP kernels and the C-ABI layer.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "common.h"

namespace ptk {

int set_error(const char* fmt, ...);   // records the thread-local message, returns -1

// A/B switches (same-box measurements of a kernel choice): in the product library each is its compile-time default
// -- no environment read, nothing for `strings libptk.so` to find.  A diagnostic build of one source with
// -DPTK_AB_ENV (`make ablib AB_NAME=.. AB_SRC=gemm.hip AB_DEFS=-DPTK_AB_ENV`, `make diag`) reads the named variable
// once instead (an integer; unset or empty keeps the default)
#ifdef PTK_AB_ENV
}  // namespace ptk
#include <cstdlib>
namespace ptk {
inline int ab_env(const char* name, int dflt) { const char* e = getenv(name); return e && *e ? atoi(e) : dflt; }
#define PTK_AB(NAME, DFLT) ([] { static const int v_ = ::ptk::ab_env(NAME, DFLT); return v_; }())
#else
#define PTK_AB(NAME, DFLT) (DFLT)
#endif

enum Act { ACT_NONE = 0, ACT_GELU_TANH = 1, ACT_GELU_ERF = 2, ACT_GEGLU = 3,
           ACT_GELU_ERF_BWD = 4, ACT_GEGLU_BWD = 5 };
enum Out { OUT_BF16 = 0, OUT_F32 = 1, OUT_F32_BFR = 2 };

struct GemmArgs {
  const bf16_t* A = nullptr;
  const bf16_t* B = nullptr;
  void* C = nullptr;
  int M = 0, N = 0, K = 0;
  long lda = 0, ldb = 0, ldc = 0;
  int zin = 1;                                   // batch z -> (z / zin, z % zin)
  long sA0 = 0, sA1 = 0, sB0 = 0, sB1 = 0, sC0 = 0, sC1 = 0;   // element strides
  float alpha = 1.f;
  const float* bias = nullptr;                   // [N]
  const float* rowadd = nullptr;                 // rowadd[(r % period) * ld + c]
  int rowadd_period = 1;
  long ld_rowadd = 0;
  const float* resid = nullptr;                  // resid[mapped r * ld + c] (may alias C)
  long ld_resid = 0;
  // bf16 residual stream (SigLIP runs in pure bf16): the linear output (alpha*acc + bias)
  // is rounded to bf16 first, then row-add / resid16 are added and the sum is rounded again
  const bf16_t* resid16 = nullptr;               // resid16[mapped r * ld + c] (may alias C), OUT_BF16 only
  long ld_resid16 = 0;
  int bf16_linear = 0;                           // round alpha*acc + bias to bf16 before row-add / resid16
  bf16_t* aux = nullptr;                         // activation side outputs [M, *]
  bf16_t* aux2 = nullptr;
  long ld_aux = 0;
  const bf16_t* aux_in = nullptr;                // saved activations for backward epilogues
  const bf16_t* aux_in2 = nullptr;
  long ld_aux_in = 0;
  RowMap amap{0, 0, 0, 0};                       // A row remap (gather)
  RowMap cmap{0, 0, 0, 0};                       // C row remap (scatter / skip)
  // optional (256x256 8-wave kernel, ACT_NONE, bf16 out, N % 64 == 0): per (row, 64-column chunk) the max and
  // the sum of exp(x - max) of the bf16-rounded outputs, float2 at row_stats[r * ld_stats + 2 * (c / 64)]
  // (the lm_head's softmax statistics: the cross-entropy pass then reads the logits once)
  float* row_stats = nullptr;
  long ld_stats = 0;
  int stats_only = 0;   // diagnostic (PTK_LM_STATS_ONLY=1): the row statistics without the logits store
  // stream-K tail scratch of the persistent 8-wave kernel (gemm_w4.hip P8Tail, p8_tail_scratch_bytes); nullptr:
  // the calling thread's TailScratchScope, if any
  void* tail_ws = nullptr;
};

int launch_gemm(const GemmArgs& a, int act, int out, int batch, hipStream_t st);
// kernel families launch_gemm dispatches to (census: path_counts, ptk_gemm_path_counts)
enum GemmPath { GEMM_PATH_NT = 0, GEMM_PATH_BIG = 1, GEMM_PATH_BIG2 = 2, GEMM_PATH_W4 = 3, GEMM_PATH_NTB = 4,
                GEMM_PATH_P8SK = 5, GEMM_PATH_P8 = 6, GEMM_PATH_TN = 7, GEMM_NPATH = 9 };   // (8: unused since r06)
int path_counts(int64_t* out, int reset);   // out [GEMM_NPATH][8] launches per (path, act class)
// persistent 256x256 4-wave GEMM (gemm_w4.hip): batch 1 only; w4_supported says whether a shape qualifies
bool w4_supported(const GemmArgs& a, int act, int out);
int launch_gemm_w4(const GemmArgs& a, int act, int out, hipStream_t st, int max_grid);
// fraction of the persistent grid's tile rounds that hold work: ntile / (ceil(ntile / CUs) * CUs)
double w4_round_fill(long M, long N);
int device_cus();   // compute units of the current device (cached)
// persistent 8-wave variant (gemm_w4.hip): the w4 tiles and ring with two waves per SIMD
bool p8_supported(const GemmArgs& a, int act, int out);
int launch_gemm_p8(const GemmArgs& a, int act, int out, hipStream_t st, bool sk, int tm = 256);
int p8_tile_height(const GemmArgs& a, int act, int out);   // 256, or 224 / 192 where shorter tiles fill the rounds
int launch_gemm_p8_kslices(const GemmArgs& a, int slices, hipStream_t st);   // K slices as row tiles (fp32 partials)
int gemm_p8_kslices(const GemmArgs& a, int slices, hipStream_t st);          // + census / timers (gemm.hip)
// the persistent kernels would take their lean bf16 epilogue for this plain bf16 GEMM (gemm_w4.hip lean_epilogue_ok)
bool lean_epilogue_candidate(const GemmArgs& a);
bool lean_epilogue_ok(const GemmArgs& a, int act, int out, uint32_t& c_bytes);   // + c_bytes: C's extent (store rsrc)
// persistent TN GEMM (gemm_tn.hip): C[M,N] = A[K,M]^T B[K,N] on the token-major operands of a weight grad, lda / ldb
// their row strides.  OUT_BF16: slices == 1 and the weight-grad accumulate (bf16_linear + resid16 == C), with the
// stream-K tail of the 8-wave kernel when `slab` (tn_slab_bytes() bytes) is given and the plan splits; OUT_F32:
// fp32 partials of `slices` equal K slices at C + z M ldc.  tn_slices: the slice count the cost model picks for
// the weight-grad form without a slab (partials within part_floats), 0 when the TN path does not take the shape.
// gemm_tn (gemm.hip) launches with the census (GEMM_PATH_TN) and live timers
bool tn_supported(const GemmArgs& a, int out, int slices);
int tn_slices(const GemmArgs& a, long part_floats);
size_t tn_slab_bytes();
// k_rows (>= 0): the operands' real row count when K is padded up to a multiple of 64 (rows k_rows .. K - 1 are
// past the buffer ranges and read as zero)
int launch_gemm_tn(const GemmArgs& a, int out, int slices, void* slab, hipStream_t st, long k_rows = -1);
int gemm_tn(const GemmArgs& a, int out, int slices, void* slab, hipStream_t st, long k_rows = -1);
int wgrad_tn_enabled();   // the TN weight-grad path is on (models.cpp; A/B switch PTK_WGRAD_TN)
// stream-K tail of the persistent 8-wave kernel: scratch bytes (arrival counters, then partial slabs), the
// workgroups its plan spreads a GEMM's tail over (0: no split), and the thread-local scratch a model-level
// call lends to every GEMM it launches (the counters are zeroed when the scope opens)
size_t p8_tail_scratch_bytes();
size_t p8_tail_scratch_bytes_models();   // 0 when the A/B build turns the tail off (PTK_STREAMK=0)
bool streamk_enabled();                  // the stream-K tail is on (the product library: always)
int p8_tail_split(const GemmArgs& a, int act, int out);
void* tail_scope();
struct TailScratchScope {
  void* prev;
  int status = 0;   // launch status of the counter zero-fill
  TailScratchScope(void* ws, hipStream_t st);
  ~TailScratchScope();
};
// per-stage device timers (stages.cpp; PTK_STAGE_TIMERS=1): spans of one stream, nested per thread
bool stage_timers_on();
void stage_begin(const char* name, hipStream_t st);
int stage_end(hipStream_t st);
struct StageScope {
  hipStream_t st;
  bool on;
  StageScope(const char* name, hipStream_t s) : st(s), on(stage_timers_on()) { if (on) stage_begin(name, s); }
  ~StageScope() { if (on) (void)stage_end(st); }
};
// consecutive stages of one stream: next(name) ends the previous one and begins `name`
struct StageSeq {
  hipStream_t st;
  bool on, open = false;
  explicit StageSeq(hipStream_t s) : st(s), on(stage_timers_on()) {}
  void next(const char* name) {
    if (!on) return;
    if (open) (void)stage_end(st);
    stage_begin(name, st);
    open = true;
  }
  ~StageSeq() { if (on && open) (void)stage_end(st); }
};
// live GEMM timing per activation class (events recorded around each launch when enabled)
void timer_enable(int on);
void force_small_tiles(int mode);
int timer_read(int cls, double* total_ms, int* count);

// ---- row-wise normalisation (norm.hip) ----
// SigLIP LayerNorm: y(bf16) = LN(x) * w + b, fp32 statistics (x f32 or bf16)
int launch_layernorm(const float* x, const float* w, const float* b, bf16_t* y, int rows, int cols,
                     float eps, hipStream_t st);
int launch_layernorm_bf16(const bf16_t* x, const float* w, const float* b, bf16_t* y, int rows, int cols,
                          float eps, hipStream_t st);
// RMSNorm (Gemma3, scale 1+w) of x (f32) -> y bf16, rstd f32; optional row gather map
int launch_rmsnorm_fwd(const float* x, long ldx, RowMap xmap, const float* w, bf16_t* y, float* rstd,
                       int rows, int cols, float eps, hipStream_t st);
// Fused sandwich-norm residual step:
//   y = bf16(rms(t)(1+w_post)); xo = xi + y; n = bf16(rms(xo)(1+w_next))  (w_next may be null)
int launch_residual_norm_fwd(const bf16_t* t, const float* xi, const float* w_post, const float* w_next,
                             float* xo, bf16_t* n, float* rstd_t, float* rstd_x, int rows, int cols,
                             float eps, hipStream_t st);
// dxi_out = dacc + rms_bwd(x (f32), w, rstd, dn)     (dn f32);  optional row scatter of the result
int launch_rmsnorm_bwd_f32(const float* x, const float* w, const float* rstd, const float* dn,
                           const float* dacc, float* dx, int rows, int cols, hipStream_t st);
// Fused: dR += rms_bwd(x2, w_pre, rstd_pre, dn);  dt = bf16(rms_bwd(t bf16, w_post, rstd_t, bf16(dR)))
int launch_residual_norm_bwd(const float* x2, const float* w_pre, const float* rstd_pre, const float* dn,
                             float* dR, const bf16_t* t, const float* w_post, const float* rstd_t,
                             bf16_t* dt, int rows, int cols, hipStream_t st);
// dt = bf16(rms_bwd(t bf16, w, rstd_t, bf16(dR)))
int launch_post_norm_bwd(const float* dR, const bf16_t* t, const float* w, const float* rstd_t, bf16_t* dt,
                         int rows, int cols, hipStream_t st);
// final norm backward on gathered rows, scatter-add into dR rows given by map
// the same two backward passes reading a bf16 dn (the bf16 output grad of the dX GEMMs)
int launch_rmsnorm_bwd_bdn(const float* x, const float* w, const float* rstd, const bf16_t* dn, const float* dacc,
                           float* dx, int rows, int cols, hipStream_t st);
int launch_residual_norm_bwd_bdn(const float* x2, const float* w_pre, const float* rstd_pre, const bf16_t* dn,
                                 float* dR, const bf16_t* t, const float* w_post, const float* rstd_t, bf16_t* dt,
                                 int rows, int cols, hipStream_t st);
// residual_norm_bwd_bdn that also writes both norms' weight-grad partials ([blocks][cols] each, blocks =
// residual_norm_bwd_wg_blocks(rows)) for launch_rms_wgrad_finish: pre = dn * x2 * rstd_pre, post = bf16(dR) * t
// * rstd_t summed over each block's rows
int residual_norm_bwd_wg_blocks(int rows);
int launch_residual_norm_bwd_wg(const float* x2, const float* w_pre, const float* rstd_pre, const bf16_t* dn,
                                float* dR, const bf16_t* t, const float* w_post, const float* rstd_t, bf16_t* dt,
                                int rows, int cols, float* part_pre, float* part_post, hipStream_t st);
int launch_rmsnorm_bwd_scatter(const float* x, RowMap xmap, const float* w, const float* rstd,
                               const float* dn, float* dR, int rows, int cols, hipStream_t st);

// ---- attention helpers (attn.hip) ----
struct AttnShape {
  int B, S, Hq, Hkv, D;     // S = padded sequence length (multiple of 64)
  const int32_t* pos = nullptr;   // forward only: RoPE position of token b*S + s ([B*S]); null: s
};
int launch_qknorm_rope_fwd(const bf16_t* qkv, const float* qw, const float* kw, const float* cos_t,
                           const float* sin_t, AttnShape s, float eps, bf16_t* Q, bf16_t* K, bf16_t* V,
                           float* rstd_q, float* rstd_k, hipStream_t st);
int launch_qknorm_rope_bwd(const bf16_t* qkv, const float* qw, const float* kw, const float* cos_t,
                           const float* sin_t, AttnShape s, const float* rstd_q, const float* rstd_k,
                           const bf16_t* dQ, const bf16_t* dK, const bf16_t* dV, bf16_t* dqkv,
                           hipStream_t st, const struct FlashBwdArgs* dkv = nullptr);
// masked softmax over score rows: P = softmax(S) (bf16), masked entries 0.
struct MaskSpec {
  int rows_per_batch;   // score rows per z
  int qdiv;             // query position = (row % rows_per_batch) / qdiv
  int zdiv;             // sample index b = z / zdiv
  int causal;
  int window;           // 0 = none; else key must satisfy k > q - window
  const int32_t* key_valid;   // [B, cols] or null
  int key_len;          // keys >= key_len are masked (when key_valid is null)
};
int launch_softmax_fwd(const float* S, bf16_t* P, int nz, int rows, int cols, long ld, MaskSpec m,
                       hipStream_t st);
// dS = P * (dP - rowsum(P*dP)) * scale  (bf16 out)
int launch_softmax_bwd(const bf16_t* P, const float* dP, bf16_t* dS, int nrows, int cols, long ld,
                       float scale, hipStream_t st);

// ---- flash attention (flash.hip) ----
struct FlashArgs {
  const bf16_t* Q = nullptr;
  const bf16_t* K = nullptr;
  const bf16_t* V = nullptr;
  bf16_t* O = nullptr;
  float* lse = nullptr;          // [nz][rows] (optional)
  int rows = 0, nkeys = 0, D = 0;
  long ldq = 0, ldk = 0, ldo = 0;  // V shares K's strides
  int zin = 1, zdiv = 1;         // z -> (z / zin, z % zin); sample b = z / zdiv (key_valid row)
  long sQ0 = 0, sQ1 = 0, sK0 = 0, sK1 = 0, sO0 = 0, sO1 = 0;
  RowMap qmap{0, 0, 0, 0}, omap{0, 0, 0, 0};
  int qdiv = 1, causal = 0, window = 0;
  const int32_t* key_valid = nullptr;   // [B][nkeys]
  float scale = 1.f;
  int variant = 0;   // set by launch_attn_fwd (A/B switches)
};
int launch_attn_fwd(const FlashArgs& a, int nz, hipStream_t st);
// backward; Q, dO, dQ: [nz][rows][D]; K, V, dK, dV: [nz][nkeys][D]; lse, delta: [nz][rows];
// O (forward output) addressed like FlashArgs::O (z split by zin, row map omap, stride ldo).
struct FlashBwdArgs {
  const bf16_t* Q = nullptr;
  const bf16_t* K = nullptr;
  const bf16_t* V = nullptr;
  const bf16_t* O = nullptr;
  const bf16_t* dO = nullptr;
  const float* lse = nullptr;
  float* delta = nullptr;          // workspace [nz][rows]
  bf16_t* dQ = nullptr;
  bf16_t* dK = nullptr;
  bf16_t* dV = nullptr;
  int rows = 0, nkeys = 0, D = 0;
  int zin = 1, zdiv = 1;
  long ldo = 0, sO0 = 0, sO1 = 0;
  RowMap omap{0, 0, 0, 0};
  int qdiv = 1, causal = 0, window = 0;
  const int32_t* key_valid = nullptr;
  float scale = 1.f;
  // D = 256 dK/dV split-query workspace (fp32 partials); null -> no split (correct, less balanced)
  float* dkv_part = nullptr;
  size_t dkv_part_bytes = 0;
  // set by launch_attn_bwd
  int dkv_target = 0, nz = 1;
  // dK/dV work items (slab, query piece) in dispatch order, heaviest first (LPT): block b runs item
  // b / nz for z = b % nz
  int dkv_items = 0;
  unsigned char dkv_item_slab[128], dkv_item_piece[128];
  // set in the plan launch_attn_bwd hands back through `defer`: 1 = split slabs still hold fp32
  // partials in dkv_part and the consumer (qknorm_rope_bwd) sums them instead of attn_dkv_reduce_kernel
  int dkv_deferred = 0;
};

// dK/dV key slabs (flash.hip): slab s covers keys [s*DKV_KEYS, s*DKV_KEYS + DKV_KEYS), its query rows
// are walked in DKV_CH-row chunks; a slab of more than dkv_target chunks is cut into pieces
constexpr int DKV_KEYS = 128, DKV_CH = 32;
__host__ __device__ inline void dkv_slab_chunks(const FlashBwdArgs& a, int s, int& c_lo, int& c_hi) {
  int r_lo = 0, r_hi = a.rows;
  if (a.causal) {
    r_lo = min(a.rows, s * DKV_KEYS * a.qdiv);
    if (a.window > 0) r_hi = min(a.rows, (s * DKV_KEYS + DKV_KEYS + a.window - 1) * a.qdiv);
  }
  c_lo = r_lo / DKV_CH;
  c_hi = max(c_lo, (r_hi + DKV_CH - 1) / DKV_CH);
}
__host__ __device__ inline int dkv_pieces(const FlashBwdArgs& a, int s) {
  int lo, hi;
  dkv_slab_chunks(a, s, lo, hi);
  const int n = hi - lo;
  return (a.dkv_target <= 0 || n <= a.dkv_target) ? 1 : (n + a.dkv_target - 1) / a.dkv_target;
}
// first partial slot of slab s (slots are numbered slab-major over the split slabs)
__host__ __device__ inline int dkv_part_base(const FlashBwdArgs& a, int s) {
  int base = 0;
  for (int t = 0; t < s; ++t) {
    const int pt = dkv_pieces(a, t);
    if (pt > 1) base += pt;
  }
  return base;
}

// defer != null: the D = 256 split-slab reduce is not launched; *defer receives the plan (with
// dkv_deferred set when partials are pending) for launch_qknorm_rope_bwd to finish dK/dV
int launch_attn_bwd(const FlashBwdArgs& a, int nz, hipStream_t st, FlashBwdArgs* defer = nullptr);
// bytes of dkv_part for which launch_attn_bwd splits every heavy key slab (0 when it never splits)
size_t attn_bwd_workspace_bytes(const FlashBwdArgs& a, int nz);

// ---- misc (misc.hip) ----
// batched 2-D transpose of bf16 [nz][rows][cols] (ld_in) -> [nz][cols][rows] (ld_out); zero-fills
// output columns in [rows, rows_pad)
int launch_transpose(const bf16_t* in, long ld_in, long sin0, long sin1, int zin, bf16_t* out, long ld_out,
                     long sout0, long sout1, int nz, int rows, int cols, int rows_pad, hipStream_t st);
int launch_im2col(const bf16_t* px, bf16_t* out, int B, int C, int H, int W, int P, hipStream_t st);
int launch_cast_f32_bf16(const float* in, bf16_t* out, long n, hipStream_t st);
int launch_build_llm_inputs(const bf16_t* embed, const int64_t* ids, int B, int T, int Nv, int S, int Spad,
                            int H, float scale_bf16, int pad_id, float* x, int32_t* key_valid,
                            hipStream_t st);
int launch_ce_fwd_bwd(bf16_t* logits, long ld, int R, int V, const int64_t* targets, float* row_loss,
                      const float* gscale, hipStream_t st);
int launch_ce_stats_fwd_bwd(bf16_t* logits, long ld, int R, int V, const float* stats, long ld_stats,
                            const int64_t* targets, float* row_loss, const float* gscale, hipStream_t st);
int launch_count_valid(const int64_t* labels, int n, float loss_scale, float* gscale, float* count,
                       hipStream_t st);
int launch_loss_reduce(const float* row_loss, int R, const float* count, float* loss, hipStream_t st);
int launch_gather_dy(const float* dx, int B, int N, int Spad, int H, bf16_t* dy, hipStream_t st);
int launch_colsum_bf16(const bf16_t* x, int rows, int cols, float* out, float* partial, long part_floats,
                       hipStream_t st);
int launch_sumsq_partial(const float* x, long n, float* partial, int nparts, hipStream_t st);
int launch_clip_adamw(float* p, const float* g, float* m, float* v, long n, const float* partial,
                      int nparts, float grad_scale, float max_norm, float lr, float b1, float b2,
                      float eps, float wd, int step, float* norm_out, hipStream_t st);
int launch_sum_partials(const float* part, int nsplit, long n, float* out, hipStream_t st);
// zero-fill (16-B aligned pointer and size) by a kernel, not hipMemsetAsync
int launch_zero(void* p, size_t bytes, hipStream_t st);
int launch_geglu_bwd(const bf16_t* dh, const bf16_t* g, const bf16_t* u, bf16_t* dgu, long M, int I, hipStream_t st);
int launch_fill_normal_bf16(bf16_t* out, long n, uint64_t seed, float std, float mean, hipStream_t st);

// ---- KV-cache decode (generate.hip) ----
int launch_gen_prompt(const float* src, long ld_b, int B, int P, int Pp, int H, float* x, int32_t* kv, hipStream_t st);
int launch_kv_append(const bf16_t* src, long src_z, bf16_t* dst, long dst_z, int Z, int p0, int n, int D,
                     hipStream_t st);
int launch_gen_sample(const bf16_t* logits, long ld, int B, int V, int do_sample, int top_k, float temperature,
                      float top_p, uint64_t seed, int step, long eos_id, long pad_id, int32_t* finished, int64_t* out,
                      long ld_out, int64_t* next, hipStream_t st);
// skinny GEMM of the decode steps (gemm_skinny.hip): M <= 64 rows, N % 64, K % 32; ACT_NONE / ACT_GEGLU, bf16 out
bool skinny_supported(int M, int N, int K, long lda, long ldb, long ldc, int act);
size_t skinny_part_bytes(int M, int N, int K);
int launch_gemm_skinny(const bf16_t* A, long lda, const bf16_t* B, long ldb, bf16_t* C, long ldc, int M, int N,
                       int K, int act, float* part, size_t part_bytes, hipStream_t st);
// stepwise decode (ptk_gemma3_decode_prefill / _step) and beam candidates (ptk_beam_candidates)
int launch_dec_prompt(const float* src, long ld_b, const int32_t* mask, long mask_ld, int repeat, int rows, int P,
                      int Pp, int H, float* x, int32_t* kv, hipStream_t st);
int launch_dec_positions(const int32_t* kv, int rows, int P, int Pp, int Smax, int32_t* pos, int32_t* slot_ok,
                         int32_t* nvalid, hipStream_t st);
int launch_dec_step_prep(int32_t* slot_ok, const int32_t* nvalid, int rows, int Smax, int p0, int t, int k_lo, int nk,
                         int32_t* pos, int32_t* kmask, hipStream_t st);
int launch_dec_gather_rows(const void* in, void* out, const int32_t* src, int rows, long row_bytes, hipStream_t st);
int launch_dec_gather_i32(const int32_t* in, int32_t* out, const int32_t* src, int rows, hipStream_t st);
int launch_dec_repeat_index(int32_t* src, int rows, int repeat, hipStream_t st);
size_t beam_candidates_ws_bytes(int batch, int K, int n_cand);
int launch_beam_candidates(const bf16_t* logits, long ld, const float* beam_scores, int batch, int K, int V,
                           int do_sample, int top_k, float top_p, float temperature, int min_keep, uint64_t seed,
                           int step, int n_cand, int64_t* tok, int32_t* beam, float* score, void* ws,
                           size_t ws_bytes, hipStream_t st);

// ---- unfrozen-LLM step (train.hip) ----
// out [cols][rows_pad] bf16 = in[map(r)][c] (r < rows), zero for rows <= r < rows_pad
int launch_transpose_rows(const bf16_t* in, long ld_in, RowMap map, int rows, int cols, bf16_t* out, long ld_out,
                          int rows_pad, hipStream_t st);
// RMSNorm weight grad: grad[c] = bf16(grad[c] + bf16(sum_r dy'[r,c] * x[map(r),c] * rstd[r])), dy' = dy or bf16(dy);
// partial >= rms_wgrad_partial_floats(rows, cols) floats
int rms_wgrad_partial_floats(int rows, int cols);
int launch_rms_wgrad(const float* x, long ldx, RowMap xmap, const float* rstd, const float* dy, long lddy,
                     int dy_round, int rows, int cols, bf16_t* grad, float* partial, hipStream_t st);
int launch_rms_wgrad_bx(const bf16_t* x, long ldx, RowMap xmap, const float* rstd, const float* dy, long lddy,
                        int dy_round, int rows, int cols, bf16_t* grad, float* partial, hipStream_t st);
int launch_rms_wgrad_bdy(const float* x, long ldx, RowMap xmap, const float* rstd, const bf16_t* dy, long lddy,
                         int rows, int cols, bf16_t* grad, float* partial, hipStream_t st);
// the fixed-order finish alone: partial [nblk][cols] (followed by ceil(nblk/16) * cols floats of scratch)
// -> grad = bf16(grad + bf16(sum)); partial + scratch = rms_wgrad_finish_floats(nblk, cols)
int rms_wgrad_finish_floats(int nblk, int cols);
int launch_rms_wgrad_finish(float* partial, int nblk, int cols, bf16_t* grad, hipStream_t st);
// q_norm / k_norm weight grads from the attention-layout dQ / dK (partial >= 2 * ceil(B*S/64) * D floats)
int launch_qknorm_wgrad(const bf16_t* qkv, const float* cos_t, const float* sin_t, AttnShape s, const float* rstd_q,
                        const float* rstd_k, const bf16_t* dQ, const bf16_t* dK, bf16_t* gq, bf16_t* gk,
                        float* partial, hipStream_t st);
int qknorm_wgrad_partial_floats(long M, int D);
// split-K partial reduce: C = sum_s part[s] (fp32) or bf16(resid + bf16(sum)) (bf16; resid may be null / alias C)
int launch_splitk_reduce(const float* part, int S, int M, int N, void* C, long ldc, int out_bf16, const bf16_t* resid,
                         long ldr, hipStream_t st);
// ws: embed_grad_ws_bytes(B, T) bytes (the sorted (id, position) keys)
size_t embed_grad_ws_bytes(int B, int T);
int launch_embed_grad(const int64_t* ids, int B, int T, int Nv, int Spad, int H, float escale, const float* dx,
                      bf16_t* dE, void* ws, hipStream_t st);
int scale_sumsq_partial_floats();
int launch_scale_sumsq_bf16(bf16_t* g, long n, float scale, float* partial, float* out, hipStream_t st);
int launch_adamw_bf16(bf16_t* p, bf16_t* g, bf16_t* m, bf16_t* v, long n, const float* sumsq, float max_norm,
                      double lr, double b1, double b2, double eps, double wd, int step, float* norm_out,
                      hipStream_t st);

}  // namespace ptk
#include "../../include/ptk.h"
namespace ptk {
// projector backward in two stages (capi.cpp): 0 = db2, dW2; 1 = dA, db1, dW1 (comm.cpp overlaps the DDP exchange)
int projector_bwd_stage(const ptk_projector* p, int rows, const void* x, const void* a, const void* h, const void* dy,
                        float* dw1, float* db1, float* dw2, float* db2, void* ws, size_t ws_bytes, int stage,
                        hipStream_t st);
}  // namespace ptk
