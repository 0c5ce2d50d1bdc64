// Host-side ASan driver for libptk's C ABI ("a debug build with -fsanitize=address for host code").
// Built by `make -C projectiontrainer_amd/csrc asan` from the product sources compiled host-only with
// -fsanitize=address (no device code, no GPU needed) and run by tests/test_host_asan.py.  It drives the entry
// points whose work is host code: the workspace layouts of the model entry points (bump allocation over every
// tensor of SigLIP / Gemma3 / the projector at the benchmarked and edge shapes), the resize-coefficient
// precompute of the image pipeline into exactly-sized heap buffers, argument validation that must fail before
// any launch, the dispatch census, the stage timers and the error strings.  Any out-of-bounds access,
// use-after-free or double free aborts the run with an AddressSanitizer report.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../include/ptk.h"

static int g_fail = 0;
#define EXPECT(c)                                                         \
  do {                                                                    \
    if (!(c)) {                                                           \
      fprintf(stderr, "%s:%d: expected %s\n", __FILE__, __LINE__, #c);    \
      ++g_fail;                                                           \
    }                                                                     \
  } while (0)

int main(int argc, char** argv) {
  EXPECT(ptk_abi_version() == PTK_ABI_VERSION);
  if (argc > 1 && strcmp(argv[1], "--overflow-probe") == 0) {
    // negative control: a coefficient buffer one row short; the instrumented image.hip host code must trip ASan
    const int k = ptk_resize_ksize(500, 224);
    int32_t* bounds = (int32_t*)malloc(sizeof(int32_t) * 2 * 224);
    int32_t* coeffs = (int32_t*)malloc(sizeof(int32_t) * 223 * k);
    ptk_resize_coeffs(500, 224, bounds, coeffs);
    free(coeffs);
    free(bounds);
    printf("host_abi_check: overflow not detected\n");
    return 0;
  }

  // image pipeline: PIL-style resize coefficients, every (in, out) pair of a sweep, exactly-sized buffers
  for (int in = 1; in <= 700; in += (in < 64 ? 1 : 37))
    for (int out : {1, 2, 7, 224, 384, 448}) {
      const int k = ptk_resize_ksize(in, out);
      EXPECT(k > 0);
      int32_t* bounds = (int32_t*)malloc(sizeof(int32_t) * 2 * out);
      int32_t* coeffs = (int32_t*)malloc(sizeof(int32_t) * (size_t)out * k);
      EXPECT(ptk_resize_coeffs(in, out, bounds, coeffs) == k);
      for (int o = 0; o < out; ++o) {
        EXPECT(bounds[2 * o] >= 0 && bounds[2 * o + 1] >= 1 && bounds[2 * o + 1] <= k);
        EXPECT(bounds[2 * o] + bounds[2 * o + 1] <= in);
      }
      free(bounds);
      free(coeffs);
    }
  EXPECT(ptk_resize_ksize(0, 10) < 0);

  // workspace layouts (host bump allocation over every tensor; the model entry points size their own)
  ptk_siglip_config sl{384, 16, 3, 1024, 16, 4096, 24, 1e-6f};
  ptk_siglip_config sb{224, 16, 3, 768, 12, 3072, 12, 1e-6f};
  for (int b : {1, 2, 16, 32}) {
    EXPECT(ptk_siglip_workspace_bytes(&sl, b) > ptk_siglip_workspace_bytes(&sl, 1) / 2);
    EXPECT(ptk_siglip_workspace_bytes(&sb, b) > 0);
  }
  ptk_gemma3_config g1{262144, 1152, 6912, 26, 4, 1, 256, 512, 6, 0, 256.f, 1e-6f};
  ptk_gemma3_config g4{262208, 2560, 10240, 34, 8, 4, 256, 1024, 6, 0, 256.f, 1e-6f};
  for (const ptk_gemma3_config* c : {&g1, &g4})
    for (int b : {1, 2, 16, 32})
      for (int t : {64, 128, 256}) {
        const int sp = (576 + t + 63) / 64 * 64;
        const size_t f = ptk_gemma3_workspace_bytes(c, b, t, sp), tr = ptk_gemma3_train_workspace_bytes(c, b, t, sp);
        EXPECT(f > 0 && tr >= f);
      }
  // the KV-cache decode's layout (prefill rows, per-layer K / V caches, decode rows) and its host-side refusals
  for (const ptk_gemma3_config* c : {&g1, &g4})
    for (int b : {1, 32})
      for (int nt : {1, 64}) {
        const size_t a = ptk_gemma3_generate_workspace_bytes(c, b, 575, nt);
        EXPECT(a > 0 && ptk_gemma3_generate_workspace_bytes(c, b, 575, nt + 64) > a);
      }
  {
    ptk_gemma3_generate_desc gd{};
    gd.batch = 2; gd.prompt_len = 575; gd.max_new_tokens = 64; gd.prompt_batch_stride = 100;   // stride < prompt
    ptk_gemma3_weights gw{};
    gw.rope_max_pos = 704;
    int64_t dummy = 0;
    EXPECT(ptk_gemma3_generate(&g1, &gw, &gd, (const float*)&dummy, nullptr, &dummy, nullptr, nullptr, 0, nullptr) < 0);
    gd.prompt_batch_stride = 704; gd.max_new_tokens = 200;                                      // past the rope tables
    EXPECT(ptk_gemma3_generate(&g1, &gw, &gd, (const float*)&dummy, nullptr, &dummy, nullptr, nullptr, 0, nullptr) < 0);
    EXPECT(ptk_gemma3_generate(&g1, &gw, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, 0, nullptr) < 0);
  }
  // the stepwise decode (beam search): layout monotone in rows and new tokens, host-side refusals before any launch
  for (const ptk_gemma3_config* c : {&g1, &g4})
    for (int rows : {3, 48})
      for (int nt : {2, 512}) {
        ptk_gemma3_decode_desc dd{rows, 639, nt, 3, 704};
        const size_t a = ptk_gemma3_decode_workspace_bytes(c, &dd);
        dd.max_new_tokens = nt + 64;
        EXPECT(a > 0 && ptk_gemma3_decode_workspace_bytes(c, &dd) > a);
      }
  {
    ptk_gemma3_weights gw{};
    gw.rope_max_pos = 4096;
    ptk_gemma3_decode_desc dd{4, 639, 8, 3, 704};   // rows not a multiple of prompt_repeat
    int64_t dummy = 0;
    EXPECT(ptk_gemma3_decode_prefill(&g1, &gw, &dd, (const float*)&dummy, nullptr, 0, &dummy, &dummy, 1 << 20, nullptr) < 0);
    dd.rows = 6; dd.prompt_batch_stride = 100;      // stride < prompt
    EXPECT(ptk_gemma3_decode_prefill(&g1, &gw, &dd, (const float*)&dummy, nullptr, 0, &dummy, &dummy, 1 << 20, nullptr) < 0);
    dd.prompt_batch_stride = 704;                   // workspace too small
    EXPECT(ptk_gemma3_decode_prefill(&g1, &gw, &dd, (const float*)&dummy, nullptr, 0, &dummy, &dummy, 1 << 20, nullptr) < 0);
    EXPECT(ptk_gemma3_decode_step(&g1, &gw, &dd, 0, &dummy, nullptr, &dummy, &dummy, (size_t)1 << 40, nullptr) < 0);  // step 0
    EXPECT(ptk_gemma3_decode_step(&g1, &gw, &dd, 8, &dummy, nullptr, &dummy, &dummy, (size_t)1 << 40, nullptr) < 0);  // past the last
    float sc = 0.f;
    int32_t bi = 0;
    EXPECT(ptk_beam_candidates(&dummy, 512, &sc, 1, 3, 512, 0, 0, 1.f, 1.f, 1, 0, 0, 64, &dummy, &bi, &sc, nullptr, 0, nullptr) < 0);  // n_cand > 32
    EXPECT(ptk_beam_candidates(&dummy, 262144, &sc, 1, 3, 262144, 1, 0, 0.9f, 1.f, 2, 0, 0, 6, &dummy, &bi, &sc, nullptr, 0, nullptr) < 0);  // no top-k
    EXPECT(ptk_beam_candidates(&dummy, 512, &sc, 1, 3, 512, 1, 50, 0.9f, 0.f, 2, 0, 0, 6, &dummy, &bi, &sc, nullptr, 0, nullptr) < 0);  // T = 0
    EXPECT(ptk_beam_candidates(&dummy, 512, &sc, 1, 3, 512, 0, 0, 1.f, 1.f, 1, 0, 0, 6, &dummy, &bi, &sc, &dummy, 8, nullptr) < 0);  // ws too small
    EXPECT(ptk_beam_candidates_workspace_bytes(16, 3, 6) >= 16 * 3 * 6 * 12);
  }
  ptk_projector pj{};
  pj.vision_dim = 1024; pj.inter_dim = 4096; pj.llm_dim = 1152;
  for (int rows : {1, 576, 18432}) EXPECT(ptk_projector_workspace_bytes(&pj, rows) > 0);
  EXPECT(ptk_gemm_tail_scratch_bytes() >= PTK_GEMM_TAIL_COUNTER_BYTES);

  // validation paths: errors before any launch, with a message
  ptk_gemma3_batch bt{};
  bt.batch = 1; bt.text_len = 8; bt.num_vision = 4; bt.seq_pad = 30;   // not a multiple of 64
  ptk_gemma3_weights wt{};
  EXPECT(ptk_gemma3_loss_fwd_bwd(&g1, &wt, &bt, nullptr, 0, nullptr) != 0);
  EXPECT(strstr(ptk_last_error(), "seq_pad") != nullptr);
  EXPECT(ptk_siglip_fwd(&sl, nullptr, 1, nullptr, nullptr, nullptr, 0, nullptr) != 0);
  EXPECT(strstr(ptk_last_error(), "workspace") != nullptr);
  ptk_comm* comm = nullptr;
  EXPECT(ptk_comm_unique_id_bytes() == 128);
  EXPECT(ptk_projector_bwd_allreduce(&pj, 1, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, 0, comm, nullptr,
                                     nullptr) != 0);

  // dispatch census and stage timers (timers off: begin / end pair up without recording)
  std::vector<int64_t> counts(PTK_GEMM_NPATHS * 8, -1);
  EXPECT(ptk_gemm_path_counts(counts.data(), 1) == 0);
  for (int64_t v : counts) EXPECT(v == 0);
  EXPECT(ptk_stage_begin("outer", nullptr) == 0);
  EXPECT(ptk_stage_begin("inner", nullptr) == 0);
  EXPECT(ptk_stage_end(nullptr) == 0);
  EXPECT(ptk_stage_end(nullptr) == 0);
  EXPECT(ptk_stage_end(nullptr) != 0);    // unpaired end
  char rep[64];
  EXPECT(ptk_stage_timers_read(rep, sizeof rep, 1) == 0 && rep[0] == 0);

  if (g_fail) {
    fprintf(stderr, "host_abi_check: %d failed expectations\n", g_fail);
    return 1;
  }
  printf("host_abi_check: ok\n");
  return 0;
}
