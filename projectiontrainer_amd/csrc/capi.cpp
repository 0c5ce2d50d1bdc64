// C-ABI entry points: error reporting, primitive ops, projector, optimizer.
// Model-level orchestration (SigLIP, Gemma3) lives in models.cpp.
#include <stdarg.h>
#include <stdio.h>

#include "../../include/ptk.h"
#include "ptk_internal.h"

namespace ptk {

static thread_local char g_err[512] = "";

int set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
  return -1;
}

RowMap to_map(ptk_rowmap m) { return RowMap{m.g, m.skip, (long)m.gs, (long)m.off}; }

GemmArgs to_args(const ptk_gemm_desc* d) {
  GemmArgs a;
  a.A = (const bf16_t*)d->A; a.B = (const bf16_t*)d->B; a.C = d->C;
  a.M = d->M; a.N = d->N; a.K = d->K;
  a.lda = d->lda; a.ldb = d->ldb; a.ldc = d->ldc;
  a.zin = d->batch_inner > 0 ? d->batch_inner : 1;
  a.sA0 = d->sA0; a.sA1 = d->sA1; a.sB0 = d->sB0; a.sB1 = d->sB1; a.sC0 = d->sC0; a.sC1 = d->sC1;
  a.alpha = d->alpha;
  a.bias = d->bias; a.rowadd = d->rowadd; a.rowadd_period = d->rowadd_period > 0 ? d->rowadd_period : 1;
  a.ld_rowadd = d->ld_rowadd; a.resid = d->resid; a.ld_resid = d->ld_resid;
  a.aux = (bf16_t*)d->aux; a.aux2 = (bf16_t*)d->aux2; a.ld_aux = d->ld_aux;
  a.aux_in = (const bf16_t*)d->aux_in; a.aux_in2 = (const bf16_t*)d->aux_in2; a.ld_aux_in = d->ld_aux_in;
  a.amap = to_map(d->amap); a.cmap = to_map(d->cmap);
  a.resid16 = (const bf16_t*)d->resid16; a.ld_resid16 = d->ld_resid16; a.bf16_linear = d->bf16_linear;
  a.tail_ws = d->tail_ws;
  return a;
}

}  // namespace ptk

using namespace ptk;
#define ST ((hipStream_t)stream)

extern "C" {

int ptk_abi_version(void) { return PTK_ABI_VERSION; }
const char* ptk_last_error(void) { return g_err; }

int ptk_gemm(const ptk_gemm_desc* d, void* stream) {
  if (!d) return set_error("ptk_gemm: null desc");
  if (d->act == PTK_ACT_GEGLU && (d->N % 32)) return set_error("ptk_gemm: GEGLU needs N %% 32 == 0");
  return launch_gemm(to_args(d), d->act, d->out, d->batch > 0 ? d->batch : 1, ST);
}

size_t ptk_gemm_tail_scratch_bytes(void) { return p8_tail_scratch_bytes(); }
int ptk_gemm_tail_split(const ptk_gemm_desc* d) {
  if (!d) return set_error("ptk_gemm_tail_split: null desc");
  return p8_tail_split(to_args(d), d->act, d->out);
}

size_t ptk_gemm_skinny_part_bytes(int M, int N, int K) { return skinny_part_bytes(M, N, K); }
int ptk_gemm_skinny(const void* A, int64_t lda, const void* B, int64_t ldb, void* C, int64_t ldc, int M, int N, int K,
                    int act, void* part, size_t part_bytes, void* stream) {
  if (!A || !B || !C) return set_error("ptk_gemm_skinny: NULL operand");
  return launch_gemm_skinny((const bf16_t*)A, (long)lda, (const bf16_t*)B, (long)ldb, (bf16_t*)C, (long)ldc, M, N, K,
                            act, (float*)part, part_bytes, (hipStream_t)stream);
}

int ptk_layernorm(const float* x, const float* w, const float* b, void* y, int rows, int cols, float eps,
                  void* stream) {
  return launch_layernorm(x, w, b, (bf16_t*)y, rows, cols, eps, ST);
}

int ptk_rmsnorm(const float* x, const float* w, void* y, float* rstd, int rows, int cols, float eps, void* stream) {
  return launch_rmsnorm_fwd(x, cols, RowMap{0, 0, 0, 0}, w, (bf16_t*)y, rstd, rows, cols, eps, ST);
}

int ptk_rmsnorm_bwd(const float* x, const float* w, const float* rstd, const float* dn, const float* dacc, float* dx,
                    int rows, int cols, void* stream) {
  return launch_rmsnorm_bwd_f32(x, w, rstd, dn, dacc, dx, rows, cols, ST);
}

int ptk_qknorm_rope_fwd(const void* qkv, const float* q_norm_w, const float* k_norm_w, const float* cos_t,
                        const float* sin_t, int batch, int seq, int heads, int kv_heads, int head_dim, float eps,
                        void* Q, void* K, void* V, float* rstd_q, float* rstd_k, void* stream) {
  const AttnShape sh{batch, seq, heads, kv_heads, head_dim};
  return launch_qknorm_rope_fwd((const bf16_t*)qkv, q_norm_w, k_norm_w, cos_t, sin_t, sh, eps, (bf16_t*)Q,
                                (bf16_t*)K, (bf16_t*)V, rstd_q, rstd_k, ST);
}
int ptk_qknorm_rope_bwd(const void* qkv, const float* q_norm_w, const float* k_norm_w, const float* cos_t,
                        const float* sin_t, int batch, int seq, int heads, int kv_heads, int head_dim,
                        const float* rstd_q, const float* rstd_k, const void* dQ, const void* dK, const void* dV,
                        void* dqkv, void* stream) {
  const AttnShape sh{batch, seq, heads, kv_heads, head_dim};
  return launch_qknorm_rope_bwd((const bf16_t*)qkv, q_norm_w, k_norm_w, cos_t, sin_t, sh, rstd_q, rstd_k,
                                (const bf16_t*)dQ, (const bf16_t*)dK, (const bf16_t*)dV, (bf16_t*)dqkv, ST);
}
int ptk_softmax(const float* S, void* P, int nz, int rows, int cols, int64_t ld, int rows_per_batch, int qdiv,
                int zdiv, int causal, int window, const int32_t* key_valid, int key_len, void* stream) {
  MaskSpec m{rows_per_batch > 0 ? rows_per_batch : rows, qdiv > 0 ? qdiv : 1, zdiv > 0 ? zdiv : 1, causal, window,
             key_valid, key_len};
  return launch_softmax_fwd(S, (bf16_t*)P, nz, rows, cols, ld, m, ST);
}

int ptk_cross_entropy(void* logits, int64_t ld, int rows, int vocab, const int64_t* targets, float* row_loss,
                      const float* gscale, void* stream) {
  return launch_ce_fwd_bwd((bf16_t*)logits, ld, rows, vocab, targets, row_loss, gscale, ST);
}

int ptk_transpose_bf16(const void* in, int64_t ld_in, void* out, int64_t ld_out, int nz, int64_t s_in, int64_t s_out,
                       int rows, int cols, int rows_pad, void* stream) {
  return launch_transpose((const bf16_t*)in, ld_in, s_in, 0, 1, (bf16_t*)out, ld_out, s_out, 0, nz, rows, cols,
                          rows_pad, ST);
}

int ptk_transpose_rows_bf16(const void* in, int64_t ld_in, int map_g, int64_t map_gs, int64_t map_off, int rows,
                            int cols, void* out, int64_t ld_out, int rows_pad, void* stream) {
  const RowMap m{map_g, 0, map_gs, map_off};
  return launch_transpose_rows((const bf16_t*)in, ld_in, m, rows, cols, (bf16_t*)out, ld_out, rows_pad, ST);
}

int ptk_cast_f32_bf16(const float* in, void* out, int64_t n, void* stream) {
  return launch_cast_f32_bf16(in, (bf16_t*)out, n, ST);
}

int ptk_gemm_force_small_tiles(int mode) {
  if (mode != 0 && mode != 1 && mode != 2 && mode != 4 && mode != 8 && mode != 32 && mode != 512 && mode != 1024 &&
      mode != 4096)
    return set_error("gemm tile mode %d not in {0, 1, 2, 4, 8, 32, 512, 1024, 4096}", mode);
  force_small_tiles(mode);
  return 0;
}
int ptk_gemm_timer_enable(int on) {
  timer_enable(on);
  return 0;
}
int ptk_gemm_timer_read(int act_class, double* total_ms, int* count) { return timer_read(act_class, total_ms, count); }
int ptk_gemm_path_counts(int64_t* counts, int reset) { return path_counts(counts, reset); }

int ptk_fill_normal_bf16(void* out, int64_t n, uint64_t seed, float std, float mean, void* stream) {
  return launch_fill_normal_bf16((bf16_t*)out, n, seed, std, mean, ST);
}

int ptk_flash_attn_fwd(const ptk_flash_desc* d, void* stream) {
  if (!d) return set_error("flash: null desc");
  FlashArgs a;
  a.Q = (const bf16_t*)d->Q; a.K = (const bf16_t*)d->K; a.V = (const bf16_t*)d->V; a.O = (bf16_t*)d->O;
  a.lse = d->lse; a.rows = d->rows; a.nkeys = d->nkeys; a.D = d->head_dim;
  a.ldq = d->ldq; a.ldk = d->ldk; a.ldo = d->ldo;
  a.zin = d->batch_inner > 0 ? d->batch_inner : 1; a.zdiv = d->zdiv > 0 ? d->zdiv : 1;
  a.sQ0 = d->sQ0; a.sQ1 = d->sQ1; a.sK0 = d->sK0; a.sK1 = d->sK1; a.sO0 = d->sO0; a.sO1 = d->sO1;
  a.qmap = to_map(d->qmap); a.omap = to_map(d->omap);
  a.qdiv = d->qdiv > 0 ? d->qdiv : 1; a.causal = d->causal; a.window = d->window;
  a.key_valid = d->key_valid; a.scale = d->scale;
  return launch_attn_fwd(a, d->batch > 0 ? d->batch : 1, ST);
}

static FlashBwdArgs to_bwd_args(const ptk_flash_bwd_desc* d) {
  FlashBwdArgs a;
  a.Q = (const bf16_t*)d->Q; a.K = (const bf16_t*)d->K; a.V = (const bf16_t*)d->V; a.O = (const bf16_t*)d->O;
  a.dO = (const bf16_t*)d->dO; a.lse = d->lse; a.delta = d->delta;
  a.dQ = (bf16_t*)d->dQ; a.dK = (bf16_t*)d->dK; a.dV = (bf16_t*)d->dV;
  a.rows = d->rows; a.nkeys = d->nkeys; a.D = d->head_dim;
  a.zin = d->batch_inner > 0 ? d->batch_inner : 1; a.zdiv = d->zdiv > 0 ? d->zdiv : 1;
  a.ldo = d->ldo; a.sO0 = d->sO0; a.sO1 = d->sO1; a.omap = to_map(d->omap);
  a.qdiv = d->qdiv > 0 ? d->qdiv : 1; a.causal = d->causal; a.window = d->window;
  a.key_valid = d->key_valid; a.scale = d->scale;
  a.dkv_part = (float*)d->workspace;
  a.dkv_part_bytes = d->workspace && d->workspace_bytes > 0 ? (size_t)d->workspace_bytes : 0;
  return a;
}

size_t ptk_flash_bwd_workspace_bytes(const ptk_flash_bwd_desc* d) {
  if (!d) return 0;
  return attn_bwd_workspace_bytes(to_bwd_args(d), d->batch > 0 ? d->batch : 1);
}

int ptk_flash_attn_bwd(const ptk_flash_bwd_desc* d, void* stream) {
  if (!d) return set_error("flash_bwd: null desc");
  return launch_attn_bwd(to_bwd_args(d), d->batch > 0 ? d->batch : 1, ST);
}

// ---------------------------------------------------------------- projector
int ptk_projector_fwd(const ptk_projector* p, int rows, const void* x, void* a, void* h, float* out,
                      ptk_rowmap out_map, int64_t ld_out, int round_bf16, void* stream) {
  const int Dv = p->vision_dim, I = p->inter_dim, Dl = p->llm_dim;
  TailScratchScope tail(p->tail_ws, ST);
  if (tail.status) return -1;
  StageScope stage("projector.fwd", ST);
  GemmArgs g1;
  g1.A = (const bf16_t*)x; g1.B = (const bf16_t*)p->w1; g1.C = h;
  g1.M = rows; g1.N = I; g1.K = Dv; g1.lda = Dv; g1.ldb = Dv; g1.ldc = I;
  g1.bias = p->b1; g1.aux = (bf16_t*)a; g1.ld_aux = I;
  if (launch_gemm(g1, ACT_GELU_ERF, OUT_BF16, 1, ST)) return -1;
  GemmArgs g2;
  g2.A = (const bf16_t*)h; g2.B = (const bf16_t*)p->w2; g2.C = out;
  g2.M = rows; g2.N = Dl; g2.K = I; g2.lda = I; g2.ldb = I; g2.ldc = ld_out;
  g2.bias = p->b2; g2.cmap = to_map(out_map);
  return launch_gemm(g2, ACT_NONE, round_bf16 ? OUT_F32_BFR : OUT_F32, 1, ST);
}

}  // extern "C"
static size_t align256(size_t v) { return (v + 255) & ~(size_t)255; }
extern "C" {

size_t ptk_projector_workspace_bytes(const ptk_projector* p, int rows) {
  const size_t Dv = p->vision_dim, I = p->inter_dim, Dl = p->llm_dim, R = ((size_t)rows + 63) / 64 * 64;
  size_t s = 0;
  s += align256(Dl * R * 2);      // dy^T
  s += align256(I * R * 2);       // h^T, later dA^T
  s += align256(R * I * 2);       // dA
  s += align256(Dv * R * 2);      // x^T
  s += align256(64 * (I > Dl ? I : Dl) * 4);   // colsum partials
  return s;
}

}  // extern "C"

namespace ptk {
// stage 0: db2 = colsum(dy), dW2 = dy^T . h;  stage 1: dA = (dy . W2) * gelu'(a), db1 = colsum(dA), dW1 = dA^T . x
// (the projector backward in the order comm.cpp overlaps with the DDP exchange)
int projector_bwd_stage(const ptk_projector* p, int rows, const void* x, const void* a, const void* h, const void* dy,
                        float* dw1, float* db1, float* dw2, float* db2, void* ws, size_t ws_bytes, int stage,
                        hipStream_t st) {
  // weight grads contract over tokens: transposed operands are zero-padded to Rp = roundup(R, 64)
  const int Dv = p->vision_dim, I = p->inter_dim, Dl = p->llm_dim, R = rows, Rp = (rows + 63) / 64 * 64;
  if (ws_bytes < ptk_projector_workspace_bytes(p, rows)) return set_error("projector_bwd: workspace too small");
  char* w = (char*)ws;
  bf16_t* dyT = (bf16_t*)w; w += align256((size_t)Dl * Rp * 2);
  bf16_t* T = (bf16_t*)w; w += align256((size_t)I * Rp * 2);
  bf16_t* dA = (bf16_t*)w; w += align256((size_t)Rp * I * 2);
  bf16_t* xT = (bf16_t*)w; w += align256((size_t)Dv * Rp * 2);
  float* part = (float*)w;
  const long part_floats = 64L * (I > Dl ? I : Dl);   // the colsum partials of ptk_projector_workspace_bytes
  // the weight grads on the TN GEMM (gemm_tn.hip), which reads the token-major operands where they lie: K = Rp,
  // the rows R .. Rp - 1 past the operands' buffer ranges read as zero.  PTK_WGRAD_TN=0 (or operands the TN path
  // does not take): transposed copies for the NT GEMMs
  auto tn_wgrad = [&](const void* A, int lda, const void* B, int ldb, float* C, int M, int N) -> int {
    if (!wgrad_tn_enabled()) return 1;
    GemmArgs g;
    g.A = (const bf16_t*)A; g.B = (const bf16_t*)B; g.C = C; g.M = M; g.N = N; g.K = Rp;
    g.lda = lda; g.ldb = ldb; g.ldc = N;
    if (!tn_supported(g, OUT_F32, 1)) return 1;
    return gemm_tn(g, OUT_F32, 1, nullptr, st, R) ? -1 : 0;
  };
  if (stage == 0) {
    // db2 = colsum(dy); dW2 = dy^T . h  (contraction over tokens)
    if (launch_colsum_bf16((const bf16_t*)dy, R, Dl, db2, part, part_floats, st)) return -1;
    const int tn = tn_wgrad(dy, Dl, h, I, dw2, Dl, I);
    if (tn <= 0) return tn;
    if (launch_transpose((const bf16_t*)dy, Dl, 0, 0, 1, dyT, Rp, 0, 0, 1, R, Dl, Rp, st)) return -1;
    if (launch_transpose((const bf16_t*)h, I, 0, 0, 1, T, Rp, 0, 0, 1, R, I, Rp, st)) return -1;
    GemmArgs g;
    g.A = dyT; g.B = T; g.C = dw2; g.M = Dl; g.N = I; g.K = Rp; g.lda = Rp; g.ldb = Rp; g.ldc = I;
    return launch_gemm(g, ACT_NONE, OUT_F32, 1, st);
  }
  // dA = (dy . W2) * gelu'(a)
  GemmArgs g2;
  g2.A = (const bf16_t*)dy; g2.B = (const bf16_t*)p->w2t; g2.C = dA; g2.M = R; g2.N = I; g2.K = Dl;
  g2.lda = Dl; g2.ldb = Dl; g2.ldc = I; g2.aux_in = (const bf16_t*)a; g2.ld_aux_in = I;
  if (launch_gemm(g2, ACT_GELU_ERF_BWD, OUT_BF16, 1, st)) return -1;
  // db1 = colsum(dA); dW1 = dA^T . x
  if (launch_colsum_bf16(dA, R, I, db1, part, part_floats, st)) return -1;
  const int tn = tn_wgrad(dA, I, x, Dv, dw1, I, Dv);
  if (tn <= 0) return tn;
  if (launch_transpose(dA, I, 0, 0, 1, T, Rp, 0, 0, 1, R, I, Rp, st)) return -1;
  if (launch_transpose((const bf16_t*)x, Dv, 0, 0, 1, xT, Rp, 0, 0, 1, R, Dv, Rp, st)) return -1;
  GemmArgs g3;
  g3.A = T; g3.B = xT; g3.C = dw1; g3.M = I; g3.N = Dv; g3.K = Rp; g3.lda = Rp; g3.ldb = Rp; g3.ldc = Dv;
  return launch_gemm(g3, ACT_NONE, OUT_F32, 1, st);
}
}  // namespace ptk

extern "C" {

int ptk_projector_bwd(const ptk_projector* p, int rows, const void* x, const void* a, const void* h, const void* dy,
                      float* dw1, float* db1, float* dw2, float* db2, void* ws, size_t ws_bytes, void* stream) {
  TailScratchScope tail(p->tail_ws, ST);
  if (tail.status) return -1;
  StageScope stage("projector.bwd", ST);
  if (projector_bwd_stage(p, rows, x, a, h, dy, dw1, db1, dw2, db2, ws, ws_bytes, 0, ST)) return -1;
  return projector_bwd_stage(p, rows, x, a, h, dy, dw1, db1, dw2, db2, ws, ws_bytes, 1, ST);
}

int ptk_gather_vision_grad(const float* dx_llm, int batch, int num_patches, int seq_pad, int llm_dim, void* dy,
                           void* stream) {
  return launch_gather_dy(dx_llm, batch, num_patches, seq_pad, llm_dim, (bf16_t*)dy, ST);
}

// ---------------------------------------------------------------- optimizer
int ptk_clip_adamw(float* params, const float* grads, float* exp_avg, float* exp_avg_sq, int64_t n, float grad_scale,
                   float max_norm, float lr, float beta1, float beta2, float eps, float weight_decay, int step,
                   float* partial, float* norm_out, void* stream) {
  if (step < 1) return set_error("clip_adamw: step must be >= 1");
  const int nparts = 1024;
  if (launch_sumsq_partial(grads, n, partial, nparts, ST)) return -1;
  return launch_clip_adamw(params, grads, exp_avg, exp_avg_sq, n, partial, nparts, grad_scale, max_norm, lr, beta1,
                           beta2, eps, weight_decay, step, norm_out, ST);
}

}  // extern "C"
