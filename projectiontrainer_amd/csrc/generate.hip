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

// One workgroup per batch row b: the next token from logits row b (bf16 [V]).
//   greedy (do_sample == 0): argmax, the first index among equal maxima;
//   sampling: z_i = x_i / temperature; keep every i with x_i >= the top_k-th largest x (top_k <= 0 or >= V: all);
//   draw i with probability exp(z_i - z_max) / sum over the kept (inverse CDF in index order of one uniform).
// finished[b] != 0: the token is pad_id; a row whose token is eos_id becomes finished.  tok -> out[b * ld_out]
// and next[b].
__global__ void __launch_bounds__(GS_T) gen_sample_kernel(const bf16_t* __restrict__ logits, long ld, int V,
                                                          int do_sample, int top_k, float temperature, uint64_t seed,
                                                          int step, long eos_id, long pad_id,
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
    for (int i = tid; i < V; i += GS_T) {
      const float v = bf2f(row[i]);
      if (v > mx) { mx = v; mi = i; }
    }
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
          for (int i = tid; i < V; i += GS_T) {
            const uint32_t k = bf_key(row[i]);
            if (pass == 0) atomicAdd(&hist[k >> 8], 1u);
            else if ((k >> 8) == hi) atomicAdd(&hist[k & 255u], 1u);
          }
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
      // the kept mass over a contiguous chunk per thread, in index order
      const float inv_t = 1.f / temperature;
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
  if (tid == 0) {
    out[(long)b * ld_out] = tok;
    next[b] = tok;
    if (!fin && tok == eos_id) finished[b] = 1;
  }
}
int launch_gen_sample(const bf16_t* logits, long ld, int B, int V, int do_sample, int top_k, float temperature,
                      uint64_t seed, int step, long eos_id, long pad_id, int32_t* finished, int64_t* out, long ld_out,
                      int64_t* next, hipStream_t st) {
  if (do_sample && !(temperature > 0.f)) return set_error("generate: temperature must be > 0 when sampling");
  hipLaunchKernelGGL(gen_sample_kernel, dim3((unsigned)B), dim3(GS_T), 0, st, logits, ld, V, do_sample, top_k,
                     temperature, seed, step, eos_id, pad_id, finished, out, ld_out, next);
  return hipGetLastError() == hipSuccess ? 0 : set_error("gen_sample launch failed");
}

}  // namespace ptk
