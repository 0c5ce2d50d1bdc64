// Kernels of the KV-cache decode (ptk_gemma3_generate, models.cpp): the validation `generate` of the Stage-1
// trainer (Stage1/projector_trainer.py:386-393: unwrapped_llm.generate(inputs_embeds=projected_embeds,
// attention_mask=ones, max_new_tokens=64, do_sample=True, pad_token_id, eos_token_id)) and of Stage 2
// (Stage2/trainer.py:626).  The layers themselves run on the training path's kernels; what is new here is
//   * the prompt copy into the padded prefill layout (+ its key-valid mask),
//   * the K / V cache append (the prefill's rows, then one row per decode step),
//   * the per-row sampling step: HF generate's logits processors for do_sample (temperature, then top-k: every
//     logit below the k-th largest dropped, ties kept -- TF/generation/logits_process.py TopKLogitsWarper), a
//     softmax draw over what is left, or greedy argmax (first index of the maximum, as torch.argmax), and the
//     finished-sequence rule of GenerationMixin._sample (a row that produced eos_token_id emits pad_token_id).
#include "common.h"
#include "ptk_internal.h"

namespace ptk {

// prompt rows b*ld_b + i (i < P, fp32 [.., H]) -> x rows b*Pp + i; rows P..Pp-1 zero; key_valid = (i < P)
__global__ void __launch_bounds__(256) gen_prompt_kernel(const float* __restrict__ src, long ld_b, int P, int Pp,
                                                         int H, float* __restrict__ x, int32_t* __restrict__ kv) {
  const long row = blockIdx.x;
  const int b = (int)(row / Pp), i = (int)(row - (long)b * Pp);
  if (threadIdx.x == 0) kv[row] = i < P;
  float* xr = x + row * H;
  const float* sr = src + ((long)b * ld_b + i) * H;
  for (int c = threadIdx.x * 4; c < H; c += 1024)
    *reinterpret_cast<float4*>(xr + c) = i < P ? *reinterpret_cast<const float4*>(sr + c) : make_float4(0, 0, 0, 0);
}
int launch_gen_prompt(const float* src, long ld_b, int B, int P, int Pp, int H, float* x, int32_t* kv,
                      hipStream_t st) {
  if (H % 4 || P > Pp) return set_error("generate: prompt layout (H %% 4, P <= Pp)");
  hipLaunchKernelGGL(gen_prompt_kernel, dim3((unsigned)((long)B * Pp)), dim3(256), 0, st, src, ld_b, P, Pp, H, x, kv);
  return hipGetLastError() == hipSuccess ? 0 : set_error("gen_prompt launch failed");
}

// rows [0, n) of each z of src [Z][src_z / D][D] -> rows p0 .. p0 + n - 1 of dst [Z][dst_z / D][D] (bf16, D % 8 == 0)
__global__ void __launch_bounds__(256) kv_append_kernel(const bf16_t* __restrict__ src, long src_z,
                                                        bf16_t* __restrict__ dst, long dst_z, int p0, int n, int D,
                                                        long total) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;   // one 16-B chunk
  if (i >= total) return;
  const int per = D / 8;
  const long z = i / ((long)n * per);
  const long r = i - z * n * per;
  const int s = (int)(r / per), c = (int)(r - (long)s * per);
  *reinterpret_cast<uint4*>(dst + z * dst_z + (long)(p0 + s) * D + 8 * c) =
      *reinterpret_cast<const uint4*>(src + z * src_z + (long)s * D + 8 * c);
}
int launch_kv_append(const bf16_t* src, long src_z, bf16_t* dst, long dst_z, int Z, int p0, int n, int D,
                     hipStream_t st) {
  if (D % 8) return set_error("kv_append: head_dim %% 8");
  const long total = (long)Z * n * (D / 8);
  if (total <= 0) return 0;
  hipLaunchKernelGGL(kv_append_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, src, src_z, dst,
                     dst_z, p0, n, D, total);
  return hipGetLastError() == hipSuccess ? 0 : set_error("kv_append launch failed");
}

// bf16 bits -> unsigned key with the order of the values (NaNs are not expected in logits)
PTK_DEV uint32_t bf_key(uint16_t u) { return (u & 0x8000u) ? (uint32_t)(~u & 0xffffu) : (uint32_t)(u | 0x8000u); }

// counter-based uniform in [0, 1) (splitmix64 of seed, step, row; 24 random bits)
PTK_DEV float gen_uniform(uint64_t seed, int step, int row) {
  uint64_t z = seed + 0x9e3779b97f4a7c15ull * (uint64_t)(1 + step) + 0xbf58476d1ce4e5b9ull * (uint64_t)(1 + row);
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  z ^= z >> 31;
  return (float)(z >> 40) * (1.0f / 16777216.0f);
}

constexpr int GS_T = 1024;   // threads per row

// f(i, u) for every element i < V of a bf16 row (u: the raw bits), each thread over elements in increasing index
// order: 16-B loads, four in flight per thread (the decode's per-token row passes are latency-bound otherwise:
// 2-byte loads one at a time measured ~0.8 ms per item at V = 262 144); the row must be 16-B aligned for the
// vector part (else everything goes through the scalar tail)
template <int NT, class F>
PTK_DEV void scan_row(const uint16_t* row, int V, F&& f) {
  const int tid = threadIdx.x;
  const int n8 = ((uintptr_t)row & 15) ? 0 : V / 8;
  const uint4* r4 = reinterpret_cast<const uint4*>(row);
  for (int c0 = tid; c0 < n8; c0 += 4 * NT) {
    uint4 q[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int c = c0 + j * NT;
      q[j] = c < n8 ? r4[c] : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int c = c0 + j * NT;
      if (c < n8) {
        const uint32_t w[4] = {q[j].x, q[j].y, q[j].z, q[j].w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          f(8 * c + 2 * e, (uint16_t)(w[e] & 0xffffu));
          f(8 * c + 2 * e + 1, (uint16_t)(w[e] >> 16));
        }
      }
    }
  }
  for (int i = 8 * n8 + tid; i < V; i += NT) f(i, row[i]);
}

// One workgroup per batch row b: the next token from logits row b (bf16 [V]).
//   greedy (do_sample == 0): argmax, the first index among equal maxima;
//   sampling: z_i = x_i / temperature; keep every i with x_i >= the top_k-th largest x (top_k <= 0 or >= V: all);
//   draw i with probability exp(z_i - z_max) / sum over the kept (inverse CDF in index order of one uniform).
// finished[b] != 0: the token is pad_id; a row whose token is eos_id becomes finished.  tok -> out[b * ld_out]
// and next[b].
constexpr int GS_LIST = 1024;   // kept entries sorted for top-p
__global__ void __launch_bounds__(GS_T) gen_sample_kernel(const bf16_t* __restrict__ logits, long ld, int V,
                                                          int do_sample, int top_k, float temperature, float top_p,
                                                          uint64_t seed, int step, long eos_id, long pad_id,
                                                          int32_t* __restrict__ finished, int64_t* __restrict__ out,
                                                          long ld_out, int64_t* __restrict__ next) {
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  constexpr int NW = GS_T / 64;
  const uint16_t* row = reinterpret_cast<const uint16_t*>(logits) + (long)b * ld;
  __shared__ uint32_t hist[256];
  __shared__ float redf[NW];
  __shared__ int redi[NW];
  __shared__ uint32_t sel[4];
  __shared__ float prefix[GS_T];
  const bool fin = finished[b] != 0;
  long tok = pad_id;
  if (!fin) {
    // max (and its first index) over the row
    float mx = -INFINITY;
    int mi = 0x7fffffff;
    scan_row<GS_T>(row, V, [&](int i, uint16_t u) {
      const float v = bf2f(u);
      if (v > mx) { mx = v; mi = i; }
    });
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
      const float ov = __shfl_xor(mx, o, 64);
      const int oi = __shfl_xor(mi, o, 64);
      if (ov > mx || (ov == mx && oi < mi)) { mx = ov; mi = oi; }
    }
    if (lane == 0) { redf[wave] = mx; redi[wave] = mi; }
    __syncthreads();
    mx = redf[0];
    mi = redi[0];
    for (int w = 1; w < NW; ++w)
      if (redf[w] > mx || (redf[w] == mx && redi[w] < mi)) { mx = redf[w]; mi = redi[w]; }
    __syncthreads();
    if (!do_sample) {
      tok = mi;
    } else {
      // top-k threshold key by a two-pass radix select over the 16-bit keys (high byte, then low byte)
      uint32_t thr = 0;
      if (top_k > 0 && top_k < V) {
        uint32_t need = (uint32_t)top_k, hi = 0;
        for (int pass = 0; pass < 2; ++pass) {
          for (int i = tid; i < 256; i += GS_T) hist[i] = 0;
          __syncthreads();
          scan_row<GS_T>(row, V, [&](int, uint16_t u) {
            const uint32_t k = bf_key(u);
            if (pass == 0) atomicAdd(&hist[k >> 8], 1u);
            else if ((k >> 8) == hi) atomicAdd(&hist[k & 255u], 1u);
          });
          __syncthreads();
          if (tid == 0) {
            uint32_t acc = 0;
            int bin = 255;
            for (; bin > 0; --bin) {
              if (acc + hist[bin] >= need) break;
              acc += hist[bin];
            }
            sel[0] = (uint32_t)bin;
            sel[1] = need - acc;   // how many of this bin's keys are still needed
          }
          __syncthreads();
          if (pass == 0) { hi = sel[0]; need = sel[1]; }
          else thr = (hi << 8) | sel[0];
          __syncthreads();
        }
      }
      const float inv_t = 1.f / temperature;
      if (top_p < 1.f || (top_k > 0 && top_k <= GS_LIST / 2) || V <= GS_LIST) {
        // the kept set (top-k, ties kept) sorted ascending by logit in LDS (bitonic), the cumulative softmax of
        // z = x / T; TopPLogitsWarper (min_tokens_to_keep 1) drops entries with cumulative mass <= 1 - top_p; then
        // the draw by inverse CDF over what is left (sorted order: the same law as a draw in index order)
        __shared__ float ls[GS_LIST];
        __shared__ int lt[GS_LIST];
        __shared__ int cnt;
        if (tid == 0) cnt = 0;
        __syncthreads();
        scan_row<GS_T>(row, V, [&](int i, uint16_t u) {
          if (bf_key(u) >= thr) {
            const int slot = atomicAdd(&cnt, 1);
            if (slot < GS_LIST) { ls[slot] = (bf2f(u) - mx) * inv_t; lt[slot] = i; }
          }
        });
        __syncthreads();
        const int n = min(cnt, GS_LIST);
        int np2 = 1;
        while (np2 < n) np2 <<= 1;
        for (int i = n + tid; i < np2; i += GS_T) { ls[i] = INFINITY; lt[i] = 0x7fffffff; }
        __syncthreads();
        for (int size = 2; size <= np2; size <<= 1)
          for (int stride = size >> 1; stride > 0; stride >>= 1) {
            for (int i = tid; i < np2; i += GS_T) {
              const int j = i ^ stride;
              if (j > i) {
                const bool up = (i & size) == 0;
                const float a = ls[i], c = ls[j];
                const bool gt = a > c || (a == c && lt[i] > lt[j]);
                if (gt == up) { ls[i] = c; ls[j] = a; const int tt = lt[i]; lt[i] = lt[j]; lt[j] = tt; }
              }
            }
            __syncthreads();
          }
        if (tid == 0) {   // (<= 1024 entries, once per row and token)
          float tot = 0.f;
          for (int i = 0; i < n; ++i) tot += __expf(ls[i]);   // z <= 0 (the row max at 0)
          float cum = 0.f;
          int first = 0;
          for (int i = 0; i < n; ++i) {
            cum += __expf(ls[i]);
            if (cum / tot <= 1.f - top_p) first = i + 1;
          }
          first = min(first, n - 1);
          float kept = 0.f;
          for (int i = first; i < n; ++i) kept += __expf(ls[i]);
          const float target = gen_uniform(seed, step, b) * kept;
          float s = 0.f;
          int pick = lt[n - 1];
          for (int i = first; i < n; ++i) {
            s += __expf(ls[i]);
            if (target < s) { pick = lt[i]; break; }
          }
          redi[0] = cnt > GS_LIST ? -1 : pick;
        }
        __syncthreads();
        tok = redi[0] >= 0 ? redi[0] : mi;
      } else {
      // the kept mass over a contiguous chunk per thread, in index order
      const int chunk = (V + GS_T - 1) / GS_T, c0 = tid * chunk, c1 = min(V, c0 + chunk);
      float part = 0.f;
      for (int i = c0; i < c1; ++i) {
        const uint16_t u = row[i];
        if (bf_key(u) >= thr) part += __expf((bf2f(u) - mx) * inv_t);
      }
      prefix[tid] = part;
      __syncthreads();
      if (tid == 0) {   // exclusive scan (1024 floats, once per token)
        float s = 0.f;
        for (int t = 0; t < GS_T; ++t) { const float v = prefix[t]; prefix[t] = s; s += v; }
        redf[0] = s;
        redi[0] = -1;
      }
      __syncthreads();
      const float target = gen_uniform(seed, step, b) * redf[0];
      const float lo = prefix[tid];
      if (lo <= target && target < lo + part) {
        float s = lo;
        int pick = -1, last = -1;
        for (int i = c0; i < c1; ++i) {
          const uint16_t u = row[i];
          if (bf_key(u) < thr) continue;
          last = i;
          s += __expf((bf2f(u) - mx) * inv_t);
          if (target < s) { pick = i; break; }
        }
        redi[0] = pick >= 0 ? pick : last;
      }
      __syncthreads();
      tok = redi[0] >= 0 ? redi[0] : mi;   // (rounding left the target past the total: the maximum)
      }
    }
  }
  if (tid == 0) {
    out[(long)b * ld_out] = tok;
    next[b] = tok;
    if (!fin && tok == eos_id) finished[b] = 1;
  }
}
int launch_gen_sample(const bf16_t* logits, long ld, int B, int V, int do_sample, int top_k, float temperature,
                      float top_p, uint64_t seed, int step, long eos_id, long pad_id, int32_t* finished, int64_t* out,
                      long ld_out, int64_t* next, hipStream_t st) {
  if (do_sample && !(temperature > 0.f)) return set_error("generate: temperature must be > 0 when sampling");
  if (do_sample && !(top_p > 0.f && top_p <= 1.f)) return set_error("generate: top_p must be in (0, 1]");
  if (do_sample && top_p < 1.f && !(top_k > 0 && top_k <= GS_LIST / 2) && V > GS_LIST / 2)
    return set_error("generate: top_p < 1 needs 0 < top_k <= %d (the kept set is sorted in LDS)", GS_LIST / 2);
  hipLaunchKernelGGL(gen_sample_kernel, dim3((unsigned)B), dim3(GS_T), 0, st, logits, ld, V, do_sample, top_k,
                     temperature, do_sample ? top_p : 1.f, seed, step, eos_id, pad_id, finished, out, ld_out, next);
  return hipGetLastError() == hipSuccess ? 0 : set_error("gen_sample launch failed");
}

}  // namespace ptk

// ================================================================== stepwise decode (beam search)
// The pieces of ptk_gemma3_decode_prefill / _step (models.cpp): Stage 2's validation generate
// (Stage2/trainer.py:596-626: inputs_embeds = [projected image tokens | question], attention_mask with the padded
// question tokens 0, num_beams 3, do_sample, top_k 50, top_p 0.9) needs per-row prompt masks, the position ids HF
// derives from them (GenerationMixin._prepare_position_ids_for_generation: cumsum(mask) - 1, masked -> 0), and the
// cache rows re-ordered by the selected beams every step.

namespace ptk {

// prompt p = r / repeat -> decode row r: x rows r*Pp + i (i < P from src, else 0); key flag = (i < P) & mask[p][i]
__global__ void __launch_bounds__(256) dec_prompt_kernel(const float* __restrict__ src, long ld_b,
                                                         const int32_t* __restrict__ mask, long mask_ld, int repeat,
                                                         int P, int Pp, int H, float* __restrict__ x,
                                                         int32_t* __restrict__ kv) {
  const long row = blockIdx.x;
  const int r = (int)(row / Pp), i = (int)(row - (long)r * Pp), pr = r / repeat;
  const bool in = i < P;
  if (threadIdx.x == 0) kv[row] = in && (!mask || mask[(long)pr * mask_ld + i] != 0);
  float* xr = x + row * H;
  const float* sr = src + ((long)pr * ld_b + (in ? i : 0)) * H;
  for (int c = threadIdx.x * 4; c < H; c += 1024)
    *reinterpret_cast<float4*>(xr + c) = in ? *reinterpret_cast<const float4*>(sr + c) : make_float4(0, 0, 0, 0);
}

// one wave per decode row: position ids of the prompt slots (cumsum of the key flags - 1, 0 where masked), the
// row's slot-valid flags for the cache (slots < P), its valid count (the next position)
__global__ void __launch_bounds__(64) dec_positions_kernel(const int32_t* __restrict__ kv, int P, int Pp, int Smax,
                                                           int32_t* __restrict__ pos, int32_t* __restrict__ slot_ok,
                                                           int32_t* __restrict__ nvalid) {
  const int r = blockIdx.x, lane = threadIdx.x;
  int base = 0;
  for (int i0 = 0; i0 < Pp; i0 += 64) {
    const int i = i0 + lane;
    const int v = i < Pp ? kv[(long)r * Pp + i] : 0;
    const uint64_t m = __ballot(v != 0);
    const int before = __popcll(m & ((1ull << lane) - 1ull));
    if (i < Pp) pos[(long)r * Pp + i] = v ? base + before : 0;
    if (i < P) slot_ok[(long)r * Smax + i] = v;
    base += __popcll(m);
  }
  for (int i = P + lane; i < Smax; i += 64) slot_ok[(long)r * Smax + i] = 0;
  if (lane == 0) nvalid[r] = base;
}

// decode step t (slot p0 = P + t - 1): the new token's slot becomes valid, its position is the row's valid count
// + t - 1, and the key flags of cache slots [k_lo, k_lo + nk) (nk a multiple of 4, slots past p0 masked) are
// copied out contiguous for the attention call
__global__ void __launch_bounds__(256) dec_step_prep_kernel(int32_t* __restrict__ slot_ok, const int32_t* __restrict__ nvalid,
                                                            int Smax, int p0, int t, int k_lo, int nk,
                                                            int32_t* __restrict__ pos, int32_t* __restrict__ kmask) {
  const int r = blockIdx.x;
  const int32_t* so = slot_ok + (long)r * Smax;
  for (int j = threadIdx.x; j < nk; j += 256) {
    const int s = k_lo + j;
    kmask[(long)r * nk + j] = s < p0 ? so[s] : (s == p0 ? 1 : 0);
  }
  if (threadIdx.x == 0) {
    slot_ok[(long)r * Smax + p0] = 1;
    pos[r] = nvalid[r] + t - 1;
  }
}

// out row r = in row src[r] (16-B chunks; rows of `row_bytes`, a multiple of 16)
__global__ void __launch_bounds__(256) dec_gather_rows_kernel(const uint4* __restrict__ in, uint4* __restrict__ out,
                                                              const int32_t* __restrict__ src, long chunks_per_row,
                                                              long total) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= total) return;
  const long r = i / chunks_per_row, c = i - r * chunks_per_row;
  out[i] = in[(long)src[r] * chunks_per_row + c];
}

int launch_dec_prompt(const float* src, long ld_b, const int32_t* mask, long mask_ld, int repeat, int rows, int P,
                      int Pp, int H, float* x, int32_t* kv, hipStream_t st) {
  if (H % 4 || P > Pp || repeat < 1) return set_error("decode: prompt layout (H %% 4, P <= Pp, repeat >= 1)");
  hipLaunchKernelGGL(dec_prompt_kernel, dim3((unsigned)((long)rows * Pp)), dim3(256), 0, st, src, ld_b, mask, mask_ld,
                     repeat, P, Pp, H, x, kv);
  return hipGetLastError() == hipSuccess ? 0 : set_error("dec_prompt launch failed");
}
int launch_dec_positions(const int32_t* kv, int rows, int P, int Pp, int Smax, int32_t* pos, int32_t* slot_ok,
                         int32_t* nvalid, hipStream_t st) {
  hipLaunchKernelGGL(dec_positions_kernel, dim3((unsigned)rows), dim3(64), 0, st, kv, P, Pp, Smax, pos, slot_ok, nvalid);
  return hipGetLastError() == hipSuccess ? 0 : set_error("dec_positions launch failed");
}
int launch_dec_step_prep(int32_t* slot_ok, const int32_t* nvalid, int rows, int Smax, int p0, int t, int k_lo, int nk,
                         int32_t* pos, int32_t* kmask, hipStream_t st) {
  if (nk % 4 || k_lo + nk > Smax || p0 >= Smax) return set_error("decode: step layout (nk %d, k_lo %d, p0 %d)", nk, k_lo, p0);
  hipLaunchKernelGGL(dec_step_prep_kernel, dim3((unsigned)rows), dim3(256), 0, st, slot_ok, nvalid, Smax, p0, t, k_lo,
                     nk, pos, kmask);
  return hipGetLastError() == hipSuccess ? 0 : set_error("dec_step_prep launch failed");
}
int launch_dec_gather_rows(const void* in, void* out, const int32_t* src, int rows, long row_bytes, hipStream_t st) {
  if (row_bytes % 16) return set_error("decode: gathered rows must be multiples of 16 B");
  const long cpr = row_bytes / 16, total = cpr * rows;
  if (total <= 0) return 0;
  hipLaunchKernelGGL(dec_gather_rows_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st,
                     (const uint4*)in, (uint4*)out, src, cpr, total);
  return hipGetLastError() == hipSuccess ? 0 : set_error("dec_gather_rows launch failed");
}

__global__ void __launch_bounds__(256) dec_gather_i32_kernel(const int32_t* __restrict__ in, int32_t* __restrict__ out,
                                                              const int32_t* __restrict__ src, int rows) {
  const int r = blockIdx.x * 256 + threadIdx.x;
  if (r < rows) out[r] = in[src[r]];
}
__global__ void __launch_bounds__(256) dec_repeat_index_kernel(int32_t* __restrict__ src, int rows, int repeat) {
  const int r = blockIdx.x * 256 + threadIdx.x;
  if (r < rows) src[r] = r / repeat;
}
int launch_dec_gather_i32(const int32_t* in, int32_t* out, const int32_t* src, int rows, hipStream_t st) {
  hipLaunchKernelGGL(dec_gather_i32_kernel, dim3((unsigned)((rows + 255) / 256)), dim3(256), 0, st, in, out, src, rows);
  return hipGetLastError() == hipSuccess ? 0 : set_error("dec_gather_i32 launch failed");
}
int launch_dec_repeat_index(int32_t* src, int rows, int repeat, hipStream_t st) {
  hipLaunchKernelGGL(dec_repeat_index_kernel, dim3((unsigned)((rows + 255) / 256)), dim3(256), 0, st, src, rows, repeat);
  return hipGetLastError() == hipSuccess ? 0 : set_error("dec_repeat_index launch failed");
}

// ------------------------------------------------------------------ beam candidates
// GenerationMixin._beam_search, one step (b, c of its loop: transformers/generation/utils.py _get_top_k_continuations):
// per decode row (batch item b, beam k) log_probs = log_softmax(fp32 logits); with do_sample the warpers act on
// them in HF's order -- temperature (/T), top-k (keep >= the k-th largest, k = max(top_k, min_keep)), top-p (sort
// ascending, cumulative softmax, drop where <= 1 - top_p, keep the last min_keep) -- the rest -inf; + the beam's
// running score; then over the beams x vocab of item b:
//   do_sample: n_cand draws without replacement from softmax(accumulated) (torch.multinomial), taken as the
//              n_cand largest accumulated + Gumbel noise (the same distribution; order = draw order);
//   greedy:    the n_cand largest accumulated (torch.topk, descending).
// Out per item: tokens, beam (0..K-1) and the accumulated log prob (without the noise) of each candidate.
constexpr int BC_T = 1024;     // threads per item
constexpr int BC_LIST = 1024;  // kept entries per row (top-k with ties); more -> error flag (token -1)

PTK_DEV float bc_gumbel(uint64_t seed, int step, int row, int tok) {
  uint64_t z = seed ^ (0x9e3779b97f4a7c15ull * (uint64_t)(1 + step));
  z += 0xbf58476d1ce4e5b9ull * (uint64_t)(1 + row) + 0x94d049bb133111ebull * (uint64_t)(1 + tok);
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  z ^= z >> 31;
  const float u = ((float)(z >> 40) + 0.5f) * (1.0f / 16777216.0f);   // (0, 1)
  return -__logf(-__logf(u));
}

// One workgroup per decode row (item b = blockIdx / K, beam k = blockIdx % K): the row's best n_cand candidates
// (selection key, accumulated score, token) into the scratch; beam_merge_kernel then takes each item's best n_cand
// over its K rows.
__global__ void __launch_bounds__(BC_T) beam_cand_kernel(const bf16_t* __restrict__ logits, long ld,
                                                         const float* __restrict__ beam_scores, int K, int V,
                                                         int do_sample, int top_k, float top_p, float temperature,
                                                         int min_keep, uint64_t seed, int step, int n_cand,
                                                         float* __restrict__ sc_key, float* __restrict__ sc_acc,
                                                         int32_t* __restrict__ sc_tok) {
  const int rowi = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  constexpr int NW = BC_T / 64;
  __shared__ uint32_t hist[256];
  __shared__ float redf[NW];
  __shared__ int redi[NW];
  __shared__ uint32_t sel[2];
  __shared__ int cnt;
  __shared__ float ls[BC_LIST];      // kept entries of the row: log prob (processed), then accumulated
  __shared__ int lt[BC_LIST];        //                              token
  __shared__ float best_key[32], best_acc[32];
  __shared__ int best_tok[32];
  __shared__ int nbest;
  if (tid == 0) nbest = 0;
  const float inv_t = (do_sample && temperature > 0.f) ? 1.f / temperature : 1.f;
  const uint16_t* row = reinterpret_cast<const uint16_t*>(logits) + (long)rowi * ld;
  // log_softmax statistics (fp32 over the bf16 logits)
  float mx = -INFINITY;
  scan_row<BC_T>(row, V, [&](int, uint16_t u) { mx = fmaxf(mx, bf2f(u)); });
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o, 64));
  if (lane == 0) redf[wave] = mx;
  __syncthreads();
  mx = redf[0];
  for (int w = 1; w < NW; ++w) mx = fmaxf(mx, redf[w]);
  __syncthreads();
  float se = 0.f;
  scan_row<BC_T>(row, V, [&](int, uint16_t u) { se += __expf(bf2f(u) - mx); });
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) se += __shfl_xor(se, o, 64);
  if (lane == 0) redf[wave] = se;
  __syncthreads();
  se = 0.f;
  for (int w = 0; w < NW; ++w) se += redf[w];
  const float lse = mx + __logf(se);
  __syncthreads();
  // the row's kept set: the kk largest logits (ties kept) -- log_softmax and /T preserve the order
  const int kk = do_sample ? (top_k > 0 ? max(top_k, min_keep) : V) : n_cand;
  uint32_t thr = 0;
  if (kk < V) {
    uint32_t need = (uint32_t)kk, hi = 0;
    for (int pass = 0; pass < 2; ++pass) {
      for (int i = tid; i < 256; i += BC_T) hist[i] = 0;
      __syncthreads();
      scan_row<BC_T>(row, V, [&](int, uint16_t u) {
        const uint32_t key = bf_key(u);
        if (pass == 0) atomicAdd(&hist[key >> 8], 1u);
        else if ((key >> 8) == hi) atomicAdd(&hist[key & 255u], 1u);
      });
      __syncthreads();
      if (tid == 0) {
        uint32_t acc = 0;
        int bin = 255;
        for (; bin > 0; --bin) {
          if (acc + hist[bin] >= need) break;
          acc += hist[bin];
        }
        sel[0] = (uint32_t)bin;
        sel[1] = need - acc;
      }
      __syncthreads();
      if (pass == 0) { hi = sel[0]; need = sel[1]; }
      else thr = (hi << 8) | sel[0];
      __syncthreads();
    }
  }
  if (tid == 0) cnt = 0;
  __syncthreads();
  scan_row<BC_T>(row, V, [&](int i, uint16_t u) {
    if (bf_key(u) >= thr) {
      const int slot = atomicAdd(&cnt, 1);
      if (slot < BC_LIST) { ls[slot] = (bf2f(u) - lse) * inv_t; lt[slot] = i; }
    }
  });
  __syncthreads();
  const bool bad = cnt > BC_LIST;
  const int n = min(cnt, BC_LIST);
  // top-p over the kept entries: bitonic sort ascending by score (then token), cumulative softmax
  if (do_sample && top_p < 1.f) {
    int np2 = 1;
    while (np2 < n) np2 <<= 1;
    for (int i = n + tid; i < np2; i += BC_T) { ls[i] = INFINITY; lt[i] = 0x7fffffff; }
    __syncthreads();
    for (int size = 2; size <= np2; size <<= 1)
      for (int stride = size >> 1; stride > 0; stride >>= 1) {
        for (int i = tid; i < np2; i += BC_T) {
          const int j = i ^ stride;
          if (j > i) {
            const bool up = (i & size) == 0;
            const float a = ls[i], c = ls[j];
            const bool gt = a > c || (a == c && lt[i] > lt[j]);
            if (gt == up) { ls[i] = c; ls[j] = a; const int tt = lt[i]; lt[i] = lt[j]; lt[j] = tt; }
          }
        }
        __syncthreads();
      }
    if (tid == 0) {   // (n <= 1024 entries, once per row and step)
      const float top = ls[n - 1];
      float tot = 0.f;
      for (int i = 0; i < n; ++i) tot += __expf(ls[i] - top);
      float cum = 0.f;
      int first = 0;
      for (int i = 0; i < n; ++i) {
        cum += __expf(ls[i] - top);
        if (cum / tot <= 1.f - top_p) first = i + 1;
      }
      cnt = min(first, max(0, n - min_keep));   // kept: [first, n)
    }
    __syncthreads();
  } else if (tid == 0) {
    cnt = 0;
  }
  __syncthreads();
  const int first = cnt;
  const float bs = beam_scores[rowi];
  for (int i = first + tid; i < n; i += BC_T) ls[i] += bs;   // accumulated = processed log prob + beam score
  __syncthreads();
  // the row's best n_cand by selection key (accumulated, + Gumbel noise when sampling): n_cand rounds of a block
  // arg-max (ties: the lower token)
  for (int rnd = 0; rnd < n_cand; ++rnd) {
    float bk = -INFINITY;
    int bi = -1;
    for (int i = first + tid; i < n; i += BC_T) {
      if (lt[i] < 0) continue;   // taken
      const float key = do_sample ? ls[i] + bc_gumbel(seed, step, rowi, lt[i]) : ls[i];
      if (key > bk || (key == bk && (bi < 0 || lt[i] < lt[bi]))) { bk = key; bi = i; }
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
      const float ok = __shfl_xor(bk, o, 64);
      const int oi = __shfl_xor(bi, o, 64);
      if (ok > bk || (ok == bk && oi >= 0 && (bi < 0 || lt[oi] < lt[bi]))) { bk = ok; bi = oi; }
    }
    if (lane == 0) { redf[wave] = bk; redi[wave] = bi; }
    __syncthreads();
    if (tid == 0) {
      float k0 = redf[0];
      int i0 = redi[0];
      for (int w = 1; w < NW; ++w)
        if (redf[w] > k0 || (redf[w] == k0 && redi[w] >= 0 && (i0 < 0 || lt[redi[w]] < lt[i0]))) { k0 = redf[w]; i0 = redi[w]; }
      if (i0 >= 0 && k0 > -INFINITY) {
        best_key[nbest] = k0; best_acc[nbest] = ls[i0]; best_tok[nbest] = lt[i0];
        ++nbest;
        lt[i0] = -1;
      }
    }
    __syncthreads();
  }
  if (tid < n_cand) {
    const long o = (long)rowi * n_cand + tid;
    const bool ok = tid < nbest;
    sc_key[o] = ok ? best_key[tid] : -INFINITY;
    sc_acc[o] = ok ? best_acc[tid] : -INFINITY;
    sc_tok[o] = bad ? -2 : (ok ? best_tok[tid] : -1);
  }
}

// item b: the best n_cand over its K rows' lists (descending key; ties: the lower beam, then the lower token)
__global__ void __launch_bounds__(64) beam_merge_kernel(const float* __restrict__ sc_key,
                                                        const float* __restrict__ sc_acc,
                                                        const int32_t* __restrict__ sc_tok, int K, int n_cand,
                                                        int64_t* __restrict__ out_tok, int32_t* __restrict__ out_beam,
                                                        float* __restrict__ out_score) {
  const int b = blockIdx.x, lane = threadIdx.x;
  if (lane != 0) return;   // (K x n_cand <= 256 entries, once per item and step)
  const long base = (long)b * K * n_cand;
  bool bad = false;
  for (int i = 0; i < K * n_cand; ++i) bad |= sc_tok[base + i] == -2;
  int taken[8] = {0, 0, 0, 0, 0, 0, 0, 0};   // next unread entry of each row's (descending) list
  for (int c = 0; c < n_cand; ++c) {
    int best = -1;
    float bk = -INFINITY;
    for (int k = 0; k < K; ++k) {
      if (taken[k] >= n_cand) continue;
      const long o = base + (long)k * n_cand + taken[k];
      if (sc_tok[o] < 0) continue;
      const float key = sc_key[o];
      if (best < 0 || key > bk) { bk = key; best = k; }   // (a tie keeps the lower beam)
    }
    const long out = (long)b * n_cand + c;
    if (best < 0 || bad) {
      out_tok[out] = -1; out_beam[out] = -1; out_score[out] = -INFINITY;
      continue;
    }
    const long o = base + (long)best * n_cand + taken[best];
    out_tok[out] = sc_tok[o]; out_beam[out] = best; out_score[out] = sc_acc[o];
    ++taken[best];
  }
}

size_t beam_candidates_ws_bytes(int batch, int K, int n_cand) {
  return (size_t)batch * K * n_cand * 12 + 256;
}

int launch_beam_candidates(const bf16_t* logits, long ld, const float* beam_scores, int batch, int K, int V,
                           int do_sample, int top_k, float top_p, float temperature, int min_keep, uint64_t seed,
                           int step, int n_cand, int64_t* tok, int32_t* beam, float* score, void* ws,
                           size_t ws_bytes, hipStream_t st) {
  if (batch <= 0 || K <= 0 || K > 8 || V <= 0 || n_cand <= 0 || n_cand > 32)
    return set_error("beam_candidates: batch %d, beams %d (1..8), vocab %d, n_cand %d (1..32)", batch, K, V, n_cand);
  if (do_sample && !(temperature > 0.f)) return set_error("beam_candidates: temperature must be > 0 when sampling");
  if (do_sample && !(top_p > 0.f && top_p <= 1.f)) return set_error("beam_candidates: top_p must be in (0, 1]");
  if (do_sample && !(top_k > 0 && top_k <= BC_LIST / 2) && V > BC_LIST / 2)
    return set_error("beam_candidates: sampling needs 0 < top_k <= %d (the kept set lives in LDS)", BC_LIST / 2);
  if (!ws || ws_bytes < beam_candidates_ws_bytes(batch, K, n_cand))
    return set_error("beam_candidates: workspace too small (%zu bytes needed)", beam_candidates_ws_bytes(batch, K, n_cand));
  const long nr = (long)batch * K * n_cand;
  float* sk = (float*)ws;
  float* sa = sk + nr;
  int32_t* stok = (int32_t*)(sa + nr);
  hipLaunchKernelGGL(beam_cand_kernel, dim3((unsigned)(batch * K)), dim3(BC_T), 0, st, logits, ld, beam_scores, K, V,
                     do_sample, top_k, top_p, temperature, min_keep, seed, step, n_cand, sk, sa, stok);
  if (hipGetLastError() != hipSuccess) return set_error("beam_candidates launch failed");
  hipLaunchKernelGGL(beam_merge_kernel, dim3((unsigned)batch), dim3(64), 0, st, sk, sa, stok, K, n_cand, tok, beam,
                     score);
  return hipGetLastError() == hipSuccess ? 0 : set_error("beam_merge launch failed");
}

}  // namespace ptk
