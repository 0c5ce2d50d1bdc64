/* libptk — MI355X (gfx950) Stage-1 projector-training hot path, C ABI.
 *
 * The reference (SabaPivot/ProjectionTrainer) is pure Python: its Stage-1 step
 * (Stage1/projector_trainer.py:152-245) calls HF transformers modules and
 * torch ops.  This header is the boundary that replaces those calls: every
 * entry point takes caller-owned device pointers (from torch tensors'
 * data_ptr()), explicit sizes and a hipStream_t passed as void*.  Nothing here
 * allocates, synchronises the host, or references torch types.  Every function
 * returns 0 on success and <0 on error; ptk_last_error() returns a
 * thread-local description of the last failure.
 *
 * Dtypes: "bf16" buffers hold raw bfloat16 bits (uint16), "f32" are float.
 * Layouts are row-major; row strides are in elements.
 */
#ifndef PTK_H
#define PTK_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PTK_ABI_VERSION 8

int ptk_abi_version(void);
const char* ptk_last_error(void);

/* ------------------------------------------------------------------------ *
 * Primitive ops (unit-test surface; each replaces one torch/HF op family).  *
 * ------------------------------------------------------------------------ */

/* Row remap r -> (r / g) * gs + (r % g) + off, rows with (r % g) < skip are
 * dropped (g == 0: r + off). */
typedef struct {
  int g;
  int skip;
  int64_t gs;
  int64_t off;
} ptk_rowmap;

enum { PTK_ACT_NONE = 0, PTK_ACT_GELU_TANH = 1, PTK_ACT_GELU_ERF = 2, PTK_ACT_GEGLU = 3,
       PTK_ACT_GELU_ERF_BWD = 4, PTK_ACT_GEGLU_BWD = 5 };
enum { PTK_OUT_BF16 = 0, PTK_OUT_F32 = 1, PTK_OUT_F32_BF16ROUND = 2 };

/* C[z] = epi(alpha * A[z] . B[z]^T); A [M,K] bf16, B [N,K] bf16 (both
 * K-contiguous), K % 64 == 0.  Replaces nn.Linear / torch.matmul / the
 * attention contractions (TF gemma3 :352-382, siglip :280-303,
 * Stage1/projectors.py:17-19).  Epilogue order: +bias[c], +rowadd[r % period],
 * activation, +resid (at the remapped row), store. */
typedef struct {
  const void* A;
  const void* B;
  void* C;
  int M, N, K;
  int64_t lda, ldb, ldc;
  int batch;                 /* number of z */
  int batch_inner;           /* z -> (z / batch_inner, z % batch_inner) */
  int64_t sA0, sA1, sB0, sB1, sC0, sC1;
  float alpha;
  int act;                   /* PTK_ACT_* */
  int out;                   /* PTK_OUT_* */
  const float* bias;
  const float* rowadd;
  int rowadd_period;
  int64_t ld_rowadd;
  const float* resid;
  int64_t ld_resid;
  void* aux;                 /* GELU_ERF: pre-activation out; GEGLU: a = bf16(gelu_tanh(gate)) out */
  void* aux2;                /* GEGLU: b = bf16(gelu_tanh'(gate) * up) out (h = bf16(a * up) is C) */
  int64_t ld_aux;
  const void* aux_in;        /* GELU_ERF_BWD: pre-activation; GEGLU_BWD: the forward's a (du = bf16(dh) * a) */
  const void* aux_in2;       /* GEGLU_BWD: the forward's b (dg = bf16(dh) * b) */
  int64_t ld_aux_in;
  ptk_rowmap amap;
  ptk_rowmap cmap;
  /* bf16 residual (SigLIP's pure-bf16 tower, PTK_OUT_BF16 only): out = bf16(resid16 + bf16(linear)) when
   * bf16_linear != 0 rounds alpha*acc + bias to bf16 first (may alias C) */
  const void* resid16;
  int64_t ld_resid16;
  int bf16_linear;
  /* Optional stream-K tail scratch (NULL = off) of ptk_gemm_tail_scratch_bytes() bytes whose first
   * PTK_GEMM_TAIL_COUNTER_BYTES are zero before its first use (every GEMM leaves them zero again).  With it a
   * plain (PTK_ACT_NONE) GEMM on the persistent 8-wave kernel whose 256x256 tiles fill the last round of the
   * CUs badly spreads that round's K-tiles evenly over the CUs (fp32 partials of the tiles cut in pieces,
   * summed in K order: deterministic).  One GEMM at a time per scratch (stream order). */
  void* tail_ws;
} ptk_gemm_desc;
int ptk_gemm(const ptk_gemm_desc* d, void* stream);
#define PTK_GEMM_TAIL_COUNTER_BYTES 16384
size_t ptk_gemm_tail_scratch_bytes(void);
/* Workgroups the stream-K plan spreads this GEMM's last tile round over (0: no split), for tests. */
int ptk_gemm_tail_split(const ptk_gemm_desc* d);

/* LayerNorm (SigLIP, modeling_siglip.py:329): x f32 [rows,cols] -> y bf16. */
int ptk_layernorm(const float* x, const float* w, const float* b, void* y, int rows, int cols, float eps,
                  void* stream);
/* Gemma3RMSNorm (modeling_gemma3.py:136-150): y bf16 = x * rstd * (1 + w). */
int ptk_rmsnorm(const float* x, const float* w, void* y, float* rstd, int rows, int cols, float eps,
                void* stream);
/* dx = dacc + d/dx RMSNorm(x; w) applied to dn (f32), dacc may be NULL or == dx. */
int ptk_rmsnorm_bwd(const float* x, const float* w, const float* rstd, const float* dn, const float* dacc,
                    float* dx, int rows, int cols, void* stream);
/* Masked softmax over the last dim (scores f32 -> P bf16), see ptk_internal MaskSpec. */
/* Gemma3 q/k RMSNorm (scale 1+w) + RoPE (rotate-half) of the fused qkv projection rows, scattered to the
 * attention layouts Q [B,Hkv,S,G,D], K/V [B,Hkv,S,D]; rstd per (row, q head) / (row, kv head).
 * Replaces modeling_gemma3.py:356-360 (q_norm / k_norm / apply_rotary_pos_emb). qkv: bf16 [B*S, (Hq+2Hkv)*D],
 * cos/sin: f32 [S, D/2]. */
int ptk_qknorm_rope_fwd(const void* qkv, const float* q_norm_w, const float* k_norm_w, const float* cos_t,
                        const float* sin_t, int batch, int seq, int heads, int kv_heads, int head_dim, float eps,
                        void* Q, void* K, void* V, float* rstd_q, float* rstd_k, void* stream);
/* Backward of ptk_qknorm_rope_fwd: d(qkv) bf16 [B*S, (Hq+2Hkv)*D] from dQ, dK, dV (attention layouts). */
int ptk_qknorm_rope_bwd(const void* qkv, const float* q_norm_w, const float* k_norm_w, const float* cos_t,
                        const float* sin_t, int batch, int seq, int heads, int kv_heads, int head_dim,
                        const float* rstd_q, const float* rstd_k, const void* dQ, const void* dK, const void* dV,
                        void* dqkv, void* stream);
int ptk_softmax(const float* S, void* P, int nz, int rows, int cols, int64_t ld, int rows_per_batch, int qdiv,
                int zdiv, int causal, int window, const int32_t* key_valid, int key_len, void* stream);
/* Fused cross-entropy forward+backward on bf16 logits (TF/loss/loss_utils.py:49-67):
 * row_loss[r] = lse - logit[t]; logits overwritten with (softmax - onehot) * gscale[0]. */
int ptk_cross_entropy(void* logits, int64_t ld, int rows, int vocab, const int64_t* targets, float* row_loss,
                      const float* gscale, void* stream);
int ptk_transpose_bf16(const void* in, int64_t ld_in, void* out, int64_t ld_out, int nz, int64_t s_in,
                       int64_t s_out, int rows, int cols, int rows_pad, void* stream);
/* Stage-2 weight-grad operand transpose with a row gather: out[c][r] = in[map(r)][c] for r < rows, 0 for
 * rows <= r < rows_pad; map(r) = (r / g) * gs + (r % g) + off (g = 0: r + off).  The token-major dY / X of
 * dW = dY^T X (Stage2/trainer.py:400-441 autograd) become K-contiguous operands of the library's GEMMs. */
int ptk_transpose_rows_bf16(const void* in, int64_t ld_in, int map_g, int64_t map_gs, int64_t map_off, int rows,
                            int cols, void* out, int64_t ld_out, int rows_pad, void* stream);
/* Stage-2 weight grad of one nn.Linear (the autograd accumulate of Stage2/trainer.py:420-423 into a bf16 .grad):
 * grad [Ny, Nx] = bf16(grad + bf16(dY^T X)) over `rows` token rows, dY [.., Ny] / X [.., Nx] token-major with row
 * maps as ptk_transpose_rows_bf16's.  Identity maps and rows % 64 == 0: the persistent TN GEMM reads both where
 * they lie (K slices as fp32 partials in `part` [slices][Ny][Nx], summed in slice order; part may be NULL: one
 * slice); otherwise both are transposed into ta [Ny][Kp] / tb [Nx][Kp] (Kp = rows rounded up to 64) for the NT
 * GEMMs.  mode: 0 auto, 1 the transpose path, 2 the TN path only (error where it does not apply). */
int ptk_weight_grad_bf16(const void* dy, int64_t lddy, int y_map_g, int64_t y_map_gs, int64_t y_map_off, int Ny,
                         const void* x, int64_t ldx, int x_map_g, int64_t x_map_gs, int64_t x_map_off, int Nx, int rows,
                         void* grad, void* ta, void* tb, float* part, int64_t part_floats, int mode, void* stream);
int ptk_cast_f32_bf16(const float* in, void* out, int64_t n, void* stream);
int ptk_fill_normal_bf16(void* out, int64_t n, uint64_t seed, float std, float mean, void* stream);
/* Live GEMM timing: when enabled, HIP events are recorded on the launch stream
 * around every GEMM launch, grouped by epilogue class (PTK_ACT_*).  read()
 * synchronises those events and returns the summed kernel time and count. */
int ptk_gemm_timer_enable(int on);   /* 0 off, 1 every class, (1 << 8) | class mask: only those classes */
/* Tile-path test hook: 0 = shape heuristic, 1 = every GEMM on the 128x128 kernel,
   2 / 4 = every single-batch GEMM on the 256x256 / barrier-staggered 256x256 kernel,
   8 / 32 = every single-batch GEMM the persistent 4-wave / 8-wave (two waves per SIMD) 256x256 kernel
   supports on it, 512 / 1024 / 4096 = every plain / GELU-tanh single-batch GEMM on the 8-wave kernel with
   224- / 192- / 160-row tiles.  Any other mode is an error (64 / 128, the two-group 256x128 kernel, left the
   library in round 6). */
int ptk_gemm_force_small_tiles(int mode);
int ptk_gemm_timer_read(int act_class, double* total_ms, int* count);
/* Dispatch census (tests): counts[path * 8 + act] = GEMM launches since the last reset per kernel family
 * (0 128x128, 1 256x256 8-wave, 2 staggered 256x256 8-wave, 3 persistent 4-wave, 4 128x128 batched (split-K
 * slices, batch > 1), 5 persistent 8-wave with a stream-K tail round, 6 persistent 8-wave, 7 token-major weight
 * grad, 8 unused since round 6) and epilogue class (PTK_ACT_*): PTK_GEMM_NPATHS * 8 counts (ABI 5: 9 paths)
 * class (PTK_ACT_*); counts may be
 * NULL; reset != 0 zeroes them afterwards.  Host-side counters, no GPU work. */
#define PTK_GEMM_NPATHS 9
int ptk_gemm_path_counts(int64_t* counts, int reset);

/* Per-stage device timers (SURVEY §5 tracing; the reference has none).  Off unless PTK_STAGE_TIMERS=1 or
 * ptk_stage_timers_enable(1).  The model entry points mark their pieces (siglip.fwd.*, gemma.fwd.*,
 * gemma.lm_head_ce, gemma.bwd.*, projector.*); host code brackets its own with ptk_stage_begin / ptk_stage_end
 * on a stream (spans nest per thread; a span begun while its stream is captured into a graph records
 * nothing).  ptk_stage_timers_read waits for the recorded spans and writes "name\tms\tcount\n" per stage in
 * first-seen order into buf (NUL-terminated, truncated to cap - 1); it returns the full report's length, or -1
 * with ptk_last_error set; reset != 0 clears the totals afterwards. */
int ptk_stage_timers_enable(int on);
int ptk_stage_begin(const char* name, void* stream);
int ptk_stage_end(void* stream);
int64_t ptk_stage_timers_read(char* buf, size_t cap, int reset);

/* Flash attention forward: O = softmax(scale * Q K^T + mask) V per z, bf16 in/out,
 * LSE (natural log) per query row.  z -> (z0, z1) = (z / batch_inner, z % batch_inner);
 * Q row r of z at Q + z0*sQ0 + z1*sQ1 + qmap(r)*ldq; keys/values at K/V + ... + k*ldk;
 * query position = r / qdiv (causal, window); key_valid[(z / zdiv) * nkeys + k] (or NULL).
 * Replaces sdpa in modeling_siglip.py:289-300 and modeling_gemma3.py:365-379. */
typedef struct {
  const void* Q; const void* K; const void* V; void* O; float* lse;
  int rows, nkeys, head_dim;
  int64_t ldq, ldk, ldo;
  int batch, batch_inner, zdiv;
  int64_t sQ0, sQ1, sK0, sK1, sO0, sO1;
  ptk_rowmap qmap, omap;
  int qdiv, causal, window;
  const int32_t* key_valid;
  float scale;
} ptk_flash_desc;
int ptk_flash_attn_fwd(const ptk_flash_desc* d, void* stream);

/* Flash attention backward (dQ, dK, dV; bf16).  Q/dO/dQ [batch][rows][hd], K/V/dK/dV
 * [batch][nkeys][hd], lse/delta [batch][rows] (delta is scratch); O = forward output
 * addressed like ptk_flash_desc.O (batch_inner split, omap, ldo).  rows, nkeys % 64 == 0. */
typedef struct {
  const void* Q; const void* K; const void* V; const void* O; const void* dO;
  const float* lse; float* delta;
  void* dQ; void* dK; void* dV;
  int rows, nkeys, head_dim;
  int batch, batch_inner, zdiv;
  int64_t ldo, sO0, sO1;
  ptk_rowmap omap;
  int qdiv, causal, window;
  const int32_t* key_valid;
  float scale;
  /* optional scratch for head_dim 256: heavy causal key slabs are split over query pieces whose
   * fp32 dK/dV partials live here (size: ptk_flash_bwd_workspace_bytes); NULL = no split. */
  void* workspace;
  int64_t workspace_bytes;
} ptk_flash_bwd_desc;
size_t ptk_flash_bwd_workspace_bytes(const ptk_flash_bwd_desc* d);
int ptk_flash_attn_bwd(const ptk_flash_bwd_desc* d, void* stream);

/* ------------------------------------------------------------------------ *
 * SigLIP vision tower, frozen forward                                      *
 * replaces vision_tower(pixel_values=...).last_hidden_state                *
 * (Stage1/projector_trainer.py:158-171 -> modeling_siglip.py:576-619;      *
 * the unused MAP head is skipped: its output is discarded at :173).        *
 * ------------------------------------------------------------------------ */
typedef struct {
  int image_size, patch_size, channels, hidden, heads, intermediate, layers;
  float eps;
} ptk_siglip_config;

typedef struct {
  const void* wqkv;  const float* bqkv;   /* bf16 [3D, D] rows q|k|v, f32 [3D] */
  const void* wo;    const float* bo;     /* bf16 [D, D], f32 [D] */
  const void* w1;    const float* b1;     /* bf16 [I, D], f32 [I] */
  const void* w2;    const float* b2;     /* bf16 [D, I], f32 [D] */
  const float* ln1_w; const float* ln1_b;
  const float* ln2_w; const float* ln2_b;
} ptk_siglip_layer;

typedef struct {
  const void* patch_w;          /* bf16 [D, C*P*P] (conv weight flattened c,ky,kx) */
  const float* patch_b;         /* f32 [D] */
  const float* pos;             /* f32 [N, D] */
  const float* post_w; const float* post_b;
  const ptk_siglip_layer* layers;   /* HOST array [layers] */
} ptk_siglip_weights;

size_t ptk_siglip_workspace_bytes(const ptk_siglip_config* c, int batch);
/* pixels bf16 [B, C, H, W]; out bf16 [B*N, D] = last_hidden_state (all N patches). */
int ptk_siglip_fwd(const ptk_siglip_config* c, const ptk_siglip_weights* w, int batch, const void* pixels,
                   void* out, void* ws, size_t ws_bytes, void* stream);

/* ------------------------------------------------------------------------ *
 * MLPProjector (Stage1/projectors.py:13-29): Linear -> GELU(erf) -> Linear  *
 * ------------------------------------------------------------------------ */
typedef struct {
  int vision_dim, inter_dim, llm_dim;
  const void* w1;   const float* b1;    /* bf16 [I, Dv], f32 [I] */
  const void* w2;   const float* b2;    /* bf16 [Dl, I], f32 [Dl] */
  const void* w2t;                      /* bf16 [I, Dl] (backward) */
  void* tail_ws;                        /* optional stream-K tail scratch of the projector's GEMMs (see
                                           ptk_gemm_desc.tail_ws; zeroed by every projector call; NULL = off) */
} ptk_projector;

/* x bf16 [rows, Dv] -> a (pre-activation, bf16 [rows, I]), h (bf16 [rows, I]),
 * out f32 [*, Dl] at rows remapped by out_map (the LLM input slots);
 * round_bf16 != 0 stores the bf16-rounded value (autocast output semantics). */
int ptk_projector_fwd(const ptk_projector* p, int rows, const void* x, void* a, void* h, float* out,
                      ptk_rowmap out_map, int64_t ld_out, int round_bf16, void* stream);
size_t ptk_projector_workspace_bytes(const ptk_projector* p, int rows);
/* dy bf16 [rows, Dl] -> dw1 [I, Dv], db1 [I], dw2 [Dl, I], db2 [Dl] (f32, overwritten). */
int ptk_projector_bwd(const ptk_projector* p, int rows, const void* x, const void* a, const void* h,
                      const void* dy, float* dw1, float* db1, float* dw2, float* db2, void* ws, size_t ws_bytes,
                      void* stream);
/* dy[(b,i)] = bf16(dx_llm[b*seq_pad + i - 1]) (i >= 1), 0 for i == 0 (the dropped patch). */
int ptk_gather_vision_grad(const float* dx_llm, int batch, int num_patches, int seq_pad, int llm_dim, void* dy,
                           void* stream);

/* ------------------------------------------------------------------------ *
 * Gemma3 frozen forward + dX backward with causal-LM loss                   *
 * replaces language_model(inputs_embeds, attention_mask, labels).loss and   *
 * accelerator.backward(loss) down to d(inputs_embeds)                       *
 * (Stage1/projector_trainer.py:183-237 -> modeling_gemma3.py:511-659).      *
 * ------------------------------------------------------------------------ */
typedef struct {
  int vocab, hidden, inter, layers, heads, kv_heads, head_dim;
  int sliding_window, sliding_pattern;     /* layer i full iff (i+1) % pattern == 0 */
  int pad_token_id;
  float query_pre_attn_scalar, eps;
} ptk_gemma3_config;

typedef struct {
  const void* wqkv;  const void* wqkv_t;  /* bf16 [Dq+2Dkv, H], [H, Dq+2Dkv] */
  const void* wo;    const void* wo_t;    /* bf16 [H, Dq], [Dq, H] */
  const void* wgu;   const void* wgu_t;   /* bf16 [2I, H] gate/up interleaved per 16 rows, [H, 2I] */
  const void* wd;    const void* wd_t;    /* bf16 [H, I], [I, H] */
  const float* ln_in; const float* ln_post_attn; const float* ln_pre_ff; const float* ln_post_ff;  /* [H] */
  const float* q_norm; const float* k_norm;                                                        /* [hd] */
} ptk_gemma3_layer;

typedef struct {
  const void* embed;      /* bf16 [V, H] (tied lm_head) */
  const void* embed_t;    /* bf16 [H, V] */
  const float* final_norm;
  const float* rope_cos_local; const float* rope_sin_local;    /* f32 [max_pos, hd/2] */
  const float* rope_cos_global; const float* rope_sin_global;
  int rope_max_pos;
  const ptk_gemma3_layer* layers;    /* HOST array [layers] */
} ptk_gemma3_weights;

typedef struct {
  int batch, text_len, num_vision, seq_pad;   /* S = num_vision + text_len <= seq_pad, seq_pad % 64 == 0 */
  const int64_t* token_ids;                   /* [B, T] */
  const int64_t* labels;                      /* [B, T - label_offset] (pad -> -100): targets of text positions
                                                 label_offset .. T-1 */
  float* x;        /* f32 [B*seq_pad, H]: vision rows pre-filled; text/pad rows written here */
  float* dx;       /* f32 [B*seq_pad, H]: out, d(loss*loss_scale)/dx */
  float loss_scale;
  float* loss;     /* device f32 [1]: mean CE over valid targets */
  /* text positions before label_offset carry no target (Stage 1: 0; Stage 2: the question length, whose
   * labels are -100 at Stage2/trainer.py:390-396): their logits are never computed */
  int label_offset;
} ptk_gemma3_batch;

size_t ptk_gemma3_workspace_bytes(const ptk_gemma3_config* c, int batch, int text_len, int seq_pad);
int ptk_gemma3_loss_fwd_bwd(const ptk_gemma3_config* c, const ptk_gemma3_weights* w, const ptk_gemma3_batch* b,
                            void* ws, size_t ws_bytes, void* stream);
/* Forward + loss only (validation under torch.no_grad, Stage2/trainer.py:518-591): b->loss is written, b->dx
 * is not touched; same workspace as ptk_gemma3_loss_fwd_bwd. */
int ptk_gemma3_loss_fwd(const ptk_gemma3_config* c, const ptk_gemma3_weights* w, const ptk_gemma3_batch* b,
                        void* ws, size_t ws_bytes, void* stream);

/* ------------------------------------------------------------------------ *
 * Gemma3 forward + loss + FULL backward (unfrozen LLM, Stage 2, cfg4)       *
 * replaces language_model(inputs_embeds, attention_mask) + the manual CE   *
 * + accelerator.backward(loss) of VQATrainerStage2.train                  *
 * (Stage2/trainer.py:339-423): d(inputs_embeds) as the frozen path, plus   *
 * every parameter's gradient ACCUMULATED into caller-owned bf16 .grad      *
 * buffers (bf16(grad + bf16(g)), autograd's accumulation into bf16 params, *
 * train_vqa_stage2.py:180-187 loads the LLM in bf16).  The tied embedding  *
 * receives the lm_head term and the question/answer-embedding term         *
 * (trainer.py:351-360).  Grads must be zeroed by the caller (zero_grad).   *
 * ------------------------------------------------------------------------ */
typedef struct {
  void* wqkv; void* wo; void* wgu; void* wd;    /* bf16, the layouts of ptk_gemma3_layer (wgu interleaved) */
  void* ln_in; void* ln_post_attn; void* ln_pre_ff; void* ln_post_ff;   /* bf16 [H] */
  void* q_norm; void* k_norm;                                           /* bf16 [hd] */
} ptk_gemma3_layer_grads;

typedef struct {
  void* embed;        /* bf16 [V, H] (tied lm_head + input embedding) */
  void* final_norm;   /* bf16 [H] */
  const ptk_gemma3_layer_grads* layers;   /* HOST array [layers] */
} ptk_gemma3_grads;

size_t ptk_gemma3_train_workspace_bytes(const ptk_gemma3_config* c, int batch, int text_len, int seq_pad);
int ptk_gemma3_train_fwd_bwd(const ptk_gemma3_config* c, const ptk_gemma3_weights* w, const ptk_gemma3_batch* b,
                             const ptk_gemma3_grads* g, void* ws, size_t ws_bytes, void* stream);

/* ------------------------------------------------------------------------ *
 * KV-cache decode: the validation `generate` of Stage1/projector_trainer.py:386-393                       *
 * (unwrapped_llm.generate(inputs_embeds=projected_embeds, attention_mask=ones, max_new_tokens=64,          *
 * do_sample=True, pad_token_id, eos_token_id) -> GenerationMixin._sample with a cache).  Prefill of the    *
 * prompt embeddings (all positions valid) into a per-layer K / V cache, then one token per step:           *
 * embedding x bf16(sqrt H), the 26 layers on the training path's kernels with the step's query against     *
 * the cache (sliding layers: the last `sliding_window` keys), final norm, tied lm_head (bf16 logits), and  *
 * the sampling step (temperature, top-k with ties kept, a softmax draw; or greedy argmax).  A row that      *
 * produced eos_token_id emits pad_token_id from then on.                                                    *
 * ------------------------------------------------------------------------ */
typedef struct {
  int batch, prompt_len, max_new_tokens;
  int do_sample;             /* 0: greedy argmax (first maximal index) */
  int top_k;                 /* <= 0 or >= vocab: no top-k (HF GenerationConfig default: 50) */
  float temperature;         /* > 0 when sampling (default 1) */
  uint64_t seed;             /* the draw of step t, row b: a counter-based uniform of (seed, t, b) */
  int64_t eos_token_id, pad_token_id;
  int64_t prompt_batch_stride;   /* rows of prompt_embeds between consecutive samples (>= prompt_len) */
  float top_p;               /* (0, 1]; < 1: TopPLogitsWarper after top-k (needs 0 < top_k <= 512); 0 reads as 1 */
} ptk_gemma3_generate_desc;

size_t ptk_gemma3_generate_workspace_bytes(const ptk_gemma3_config* c, int batch, int prompt_len, int max_new_tokens);
/* prompt_embeds: f32 rows [b * prompt_batch_stride + i], i < prompt_len, width hidden (the projector output as the
 * Stage-1 engine lays it out in the LLM input).  out_ids: int64 [batch, max_new_tokens].  force_ids (optional,
 * int64 [batch, max_new_tokens]): teacher forcing -- step t > 0 feeds force_ids[:, t-1] instead of the token drawn
 * at t-1 (out_ids still records the draws).  step_logits (optional, bf16 [max_new_tokens][batch][vocab]): every
 * step's logits.  Needs rope tables of prompt_len + max_new_tokens positions. */
int ptk_gemma3_generate(const ptk_gemma3_config* c, const ptk_gemma3_weights* w, const ptk_gemma3_generate_desc* g,
                        const float* prompt_embeds, const int64_t* force_ids, int64_t* out_ids, void* step_logits,
                        void* ws, size_t ws_bytes, void* stream);

/* ------------------------------------------------------------------------ *
 * Stepwise KV-cache decode (ABI 8): Stage 2's validation generate (Stage2/trainer.py:596-626:            *
 * generate(inputs_embeds=[projected image tokens | question], attention_mask with the padded question      *
 * tokens 0, max_new_tokens=512, do_sample=True, num_beams=3, top_p=0.9, top_k=50) -> GenerationMixin.       *
 * _beam_search).  The prefill runs the prompts once and gives each of its `prompt_repeat` rows (the beams)  *
 * the prompt's cache and logits; each step feeds one token per row, after re-ordering the cache rows by    *
 * src_rows (the beams the caller kept: _reorder_cache).  Masked prompt tokens are masked keys and position  *
 * ids follow HF: cumsum(mask) - 1 over the prompt, then the row's valid count + step - 1.  The workspace    *
 * holds the caches and the per-row state from the prefill to the last step.                               *
 * ------------------------------------------------------------------------ */
typedef struct {
  int rows;                     /* decode rows = prompts x prompt_repeat */
  int prompt_len, max_new_tokens;
  int prompt_repeat;            /* consecutive rows sharing one prompt (num_beams) */
  int64_t prompt_batch_stride;  /* rows of prompt_embeds between consecutive prompts (>= prompt_len) */
} ptk_gemma3_decode_desc;

size_t ptk_gemma3_decode_workspace_bytes(const ptk_gemma3_config* c, const ptk_gemma3_decode_desc* d);
/* prompt_embeds f32 [prompts][prompt_batch_stride][hidden]; prompt_mask int32 [prompts][prompt_mask_ld] (1 = token,
 * 0 = padding) or NULL (all valid); logits out: bf16 [rows][vocab], the last prompt position of each row's prompt */
int ptk_gemma3_decode_prefill(const ptk_gemma3_config* c, const ptk_gemma3_weights* w, const ptk_gemma3_decode_desc* d,
                              const float* prompt_embeds, const int32_t* prompt_mask, int64_t prompt_mask_ld,
                              void* logits, void* ws, size_t ws_bytes, void* stream);
/* step 1 .. max_new_tokens - 1: ids int64 [rows] (the token each row appends), src_rows int32 [rows] or NULL (row r
 * continues from row src_rows[r]'s cache before the token is appended); logits out: bf16 [rows][vocab] */
int ptk_gemma3_decode_step(const ptk_gemma3_config* c, const ptk_gemma3_weights* w, const ptk_gemma3_decode_desc* d,
                           int step, const int64_t* ids, const int32_t* src_rows, void* logits, void* ws,
                           size_t ws_bytes, void* stream);
/* One beam-search selection (transformers GenerationMixin._get_top_k_continuations) for `batch` items of `beams`
 * rows: log_softmax of the bf16 logits [batch * beams][ld]; with do_sample the warpers on the log probs in HF's
 * order (temperature, top-k keeping ties and at least min_tokens_to_keep, top-p keeping min_tokens_to_keep; top_k
 * in 1..512 when sampling), + beam_scores[row]; then per item n_cand (<= 32) candidates over beams x vocab:
 * do_sample -> drawn without replacement from softmax(accumulated) (the n_cand largest accumulated + Gumbel noise
 * of (seed, step, row, token): torch.multinomial's distribution; order = draw order), else the n_cand largest
 * (descending).  Out [batch][n_cand]: token, beam (0..beams-1) and accumulated log prob; fewer candidates than
 * n_cand with a finite score leave token -1.  beams <= 8; ws: ptk_beam_candidates_workspace_bytes(batch, beams,
 * n_cand) bytes (one workgroup per row writes its best n_cand there, a second pass merges each item's rows). */
size_t ptk_beam_candidates_workspace_bytes(int batch, int beams, int n_cand);
int ptk_beam_candidates(const void* logits, int64_t ld, const float* beam_scores, int batch, int beams, int vocab,
                        int do_sample, int top_k, float top_p, float temperature, int min_tokens_to_keep,
                        uint64_t seed, int step, int n_cand, int64_t* tokens, int32_t* beam_idx, float* scores,
                        void* ws, size_t ws_bytes, void* stream);

/* The decode steps' skinny GEMM (unit-test surface; the decode calls it internally): C[M][N] bf16 =
 * A[M][K] . B[N][K]^T for M <= 64, N % 128 == 0, K % 32 == 0 (K >= 64), act PTK_ACT_NONE or PTK_ACT_GEGLU
 * (interleaved gate|up columns -> N / 2 output columns); part: fp32 K-split partials of
 * ptk_gemm_skinny_part_bytes(M, N, K) bytes (0: none needed). */
size_t ptk_gemm_skinny_part_bytes(int M, int N, int K);
int ptk_gemm_skinny(const void* A, int64_t lda, const void* B, int64_t ldb, void* C, int64_t ldc, int M, int N, int K,
                    int act, void* part, size_t part_bytes, void* stream);

/* clip_grad_norm_ + AdamW over bf16 parameters (Stage2/trainer.py:426-443, optimizer :145-149).
 * ptk_bf16_grad_scale_sumsq: g = bf16(g * scale) in place (scale 1: untouched), *out = sum g^2 (fp32,
 * deterministic; partial: >= ptk_bf16_sumsq_partial_floats() floats).  Sum the *out of every shard / rank
 * first (all-reduce), then ptk_adamw_bf16 clips by max_norm (<= 0: no clip) with that total and applies
 * AdamW with every tensor op rounded to bf16, as torch's single-tensor AdamW on bf16 parameters. */
int ptk_bf16_sumsq_partial_floats(void);
int ptk_bf16_grad_scale_sumsq(void* g, int64_t n, float scale, float* partial, float* out, void* stream);
int ptk_adamw_bf16(void* params, void* grads, void* exp_avg, void* exp_avg_sq, int64_t n, const float* sumsq_total,
                   float max_norm, double lr, double beta1, double beta2, double eps, double weight_decay, int step,
                   float* norm_out, void* stream);

/* ------------------------------------------------------------------------ *
 * clip_grad_norm_(max_norm) + AdamW over a flat f32 parameter buffer        *
 * (Stage1/projector_trainer.py:75-79, :240-242).  grad_scale multiplies g   *
 * first (DDP 1/world).  partial: >= 1024 floats scratch.  norm_out: [1].    *
 * ------------------------------------------------------------------------ */
int ptk_clip_adamw(float* params, const float* grads, float* exp_avg, float* exp_avg_sq, int64_t n,
                   float grad_scale, float max_norm, float lr, float beta1, float beta2, float eps,
                   float weight_decay, int step, float* partial, float* norm_out, void* stream);

/* ------------------------------------------------------------------------ *
 * Data-parallel exchange over RCCL (SURVEY §8(b) ptk_comm_init /            *
 * allreduce_avg, §8(e)): replaces the DDP reducer behind                    *
 * accelerator.backward (Stage1/projector_trainer.py:237,                    *
 * Stage1/accelerator_setup.py:12-16).  One process per GPU; RCCL is loaded  *
 * at the first call (no link-time dependency).                              *
 * ------------------------------------------------------------------------ */
typedef struct ptk_comm ptk_comm;
int ptk_comm_unique_id_bytes(void);              /* 128 */
/* rank 0 creates the id; the caller hands the bytes to every rank (e.g. through torch.distributed) */
int ptk_comm_get_unique_id(void* unique_id);
/* collective over `world` ranks on the current HIP device */
int ptk_comm_init(ptk_comm** comm, const void* unique_id, int world, int rank);
int ptk_comm_destroy(ptk_comm* comm);
int ptk_comm_world(const ptk_comm* comm);
/* in place over ranks, n f32, on `stream`: the sum, or the average (DDP's gradient average) */
int ptk_comm_allreduce_sum(ptk_comm* comm, float* buf, int64_t n, void* stream);
int ptk_comm_allreduce_avg(ptk_comm* comm, float* buf, int64_t n, void* stream);
/* ptk_projector_bwd into the flat grad buffer [dW1 | db1 | dW2 | db2] (the MLPProjector parameter order) with
 * the ranks' SUM of it exchanged on comm_stream, overlapped: dW2 | db2 are computed first and all-reduced while
 * the dA and dW1 GEMMs run on `stream`, then dW1 | db1; `stream` waits for the exchange before returning
 * control to its next work.  The 1/world of DDP's average is folded into ptk_clip_adamw's grad_scale. */
int ptk_projector_bwd_allreduce(const ptk_projector* p, int rows, const void* x, const void* a, const void* h,
                                const void* dy, float* flat_grad, void* ws, size_t ws_bytes, ptk_comm* comm,
                                void* comm_stream, void* stream);

/* ------------------------------------------------------------------------ *
 * Host data step: image resize + normalise.              *
 * Replaces, per image, `Image.open(p).convert('RGB').resize((S, S))` and    *
 * `processor(images=image).pixel_values` of XrayTextPairDataset.__getitem__ *
 * (Stage1/train_projection_stage1.py:97-99) plus the trainer's cast to the  *
 * tower dtype (Stage1/projector_trainer.py:158-171): JPEG decode stays on   *
 * the host, the bicubic resample (Pillow Resample.c semantics, bit-exact)   *
 * and the rescale/normalise run on the GPU.                                 *
 * ------------------------------------------------------------------------ */

/* Host-only (no GPU): taps per output of a Pillow-compatible antialiased bicubic resample
 * in_size -> out_size (Resample.c precompute_coeffs: ceil(2 * max(in/out, 1)) * 2 + 1). */
int ptk_resize_ksize(int in_size, int out_size);
/* Host-only: fixed-point weights (Resample.c precompute_coeffs + normalize_coeffs_8bpc):
 * bounds [out][2] = (first source index, tap count), coeffs [out][ksize] int32 at 22 fraction bits.
 * Returns ksize, or < 0 on error. */
int ptk_resize_coeffs(int in_size, int out_size, int32_t* bounds, int32_t* coeffs);

typedef struct ptk_image_desc {
  int64_t src_off;    /* byte offset of the image in src: h rows of w * c bytes, packed */
  int32_t h, w, c;    /* source size; c = 1 (greyscale: .convert('RGB') replicates it) or 3 */
  int32_t kh, kv;     /* taps of the horizontal / vertical pass (ptk_resize_ksize) */
  int32_t pad_;
  int64_t coef_off;   /* int32 offset in coefs: bounds_h [S][2], k_h [S][kh], bounds_v [S][2], k_v [S][kv] */
  int64_t tmp_off;    /* byte offset of the image's [h][S][c] uint8 intermediate in tmp */
} ptk_image_desc;

/* Every image i of n: out[i][ch] = lut[ch][resize_v(resize_h(src_i))] as [3][S][S] planar, bf16
 * (out_f32 = 0) or f32 (out_f32 = 1); lut: [3][256] of the output type in device memory.  desc, coefs, src, tmp
 * are device pointers; max_h / max_row_bytes bound every image's h / w * c (grid and LDS sizing,
 * max_row_bytes <= 65536). */
int ptk_image_preprocess(const uint8_t* src, const int32_t* coefs, const ptk_image_desc* desc, int n, int max_h,
                         int max_row_bytes, int out_size, const void* lut, int out_f32, uint8_t* tmp, void* out,
                         void* stream);

#ifdef __cplusplus
}
#endif
#endif /* PTK_H */
