// Plain library GEMMs on hipBLASLt (no epilogue beyond the output cast): the frozen Gemma3 projections
// and dX products whose outputs need nothing fused (bf16 or fp32 C = A . B^T).  Every GEMM with a fused
// epilogue (bias, GELU / GEGLU and their backward, residual adds, row maps) stays on the hand-written
// MFMA kernels (gemm.hip, gemm_w4.hip).
//
// Row-major C[M,N] (ldc) = A[M,K] (lda) . B[N,K]^T (ldb) is, column-major, C' (N x M) = B'^T . A' with
// B' = B as a K x N column-major matrix (ld ldb, op T) and A' = A as K x M (ld lda, op N).
// One handle and one 64 MiB workspace per process (created on the first call), the algorithm of each
// shape chosen once by hipBLASLt's heuristic and cached.
#include <hipblaslt/hipblaslt.h>

#include <map>
#include <mutex>
#include <tuple>

#include "ptk_internal.h"

namespace ptk {

namespace {

struct Plan {
  hipblasLtMatmulDesc_t desc = nullptr;
  hipblasLtMatrixLayout_t la = nullptr, lb = nullptr, lc = nullptr;
  hipblasLtMatmulAlgo_t algo;
  bool ok = false;
};

constexpr size_t WS_BYTES = 64ull << 20;
hipblasLtHandle_t g_handle = nullptr;
void* g_ws = nullptr;
std::mutex g_mu;
std::map<std::tuple<int, int, int, long, long, long, int>, Plan> g_plans;

bool init() {
  if (g_handle) return true;
  if (hipblasLtCreate(&g_handle) != HIPBLAS_STATUS_SUCCESS) return false;
  if (hipMalloc(&g_ws, WS_BYTES) != hipSuccess) return false;
  return true;
}

Plan* plan_for(const GemmArgs& a, int out) {
  const auto key = std::make_tuple(a.M, a.N, a.K, a.lda, a.ldb, a.ldc, out);
  auto it = g_plans.find(key);
  if (it != g_plans.end()) return it->second.ok ? &it->second : nullptr;
  Plan& p = g_plans[key];
  const hipDataType ct = out == OUT_F32 ? HIP_R_32F : HIP_R_16BF;
  if (hipblasLtMatmulDescCreate(&p.desc, HIPBLAS_COMPUTE_32F, HIP_R_32F) != HIPBLAS_STATUS_SUCCESS) return nullptr;
  const int32_t opT = HIPBLAS_OP_T, opN = HIPBLAS_OP_N;
  hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_TRANSA, &opT, sizeof(opT));
  hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_TRANSB, &opN, sizeof(opN));
  if (hipblasLtMatrixLayoutCreate(&p.la, HIP_R_16BF, a.K, a.N, a.ldb) != HIPBLAS_STATUS_SUCCESS ||
      hipblasLtMatrixLayoutCreate(&p.lb, HIP_R_16BF, a.K, a.M, a.lda) != HIPBLAS_STATUS_SUCCESS ||
      hipblasLtMatrixLayoutCreate(&p.lc, ct, a.N, a.M, a.ldc) != HIPBLAS_STATUS_SUCCESS)
    return nullptr;
  hipblasLtMatmulPreference_t pref;
  hipblasLtMatmulPreferenceCreate(&pref);
  uint64_t ws = WS_BYTES;
  hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &ws, sizeof(ws));
  hipblasLtMatmulHeuristicResult_t res[8];
  int n = 0;
  const hipblasStatus_t st = hipblasLtMatmulAlgoGetHeuristic(g_handle, p.desc, p.la, p.lb, p.lc, p.lc, pref, 8, res, &n);
  hipblasLtMatmulPreferenceDestroy(pref);
  for (int i = 0; st == HIPBLAS_STATUS_SUCCESS && i < n; ++i)
    if (res[i].state == HIPBLAS_STATUS_SUCCESS && res[i].workspaceSize <= WS_BYTES) {
      p.algo = res[i].algo;
      p.ok = true;
      break;
    }
  return p.ok ? &p : nullptr;
}

// dW[Ny, Nx] = dY^T . X over K token rows, both operands token-major (ld lddy / ldx): column-major
// dW' (Nx x Ny) = X' (Nx x K, op N) . dY'^T (op T on Ny x K).  fp32 out (the accumulate is the caller's).
Plan* plan_tn(int Ny, int Nx, int K, long lddy, long ldx, long ldc) {
  const auto key = std::make_tuple(-Ny, Nx, K, lddy, ldx, ldc, 99);
  auto it = g_plans.find(key);
  if (it != g_plans.end()) return it->second.ok ? &it->second : nullptr;
  Plan& p = g_plans[key];
  if (hipblasLtMatmulDescCreate(&p.desc, HIPBLAS_COMPUTE_32F, HIP_R_32F) != HIPBLAS_STATUS_SUCCESS) return nullptr;
  const int32_t opT = HIPBLAS_OP_T, opN = HIPBLAS_OP_N;
  hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_TRANSA, &opN, sizeof(opN));
  hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_TRANSB, &opT, sizeof(opT));
  if (hipblasLtMatrixLayoutCreate(&p.la, HIP_R_16BF, Nx, K, ldx) != HIPBLAS_STATUS_SUCCESS ||
      hipblasLtMatrixLayoutCreate(&p.lb, HIP_R_16BF, Ny, K, lddy) != HIPBLAS_STATUS_SUCCESS ||
      hipblasLtMatrixLayoutCreate(&p.lc, HIP_R_32F, Nx, Ny, ldc) != HIPBLAS_STATUS_SUCCESS)
    return nullptr;
  hipblasLtMatmulPreference_t pref;
  hipblasLtMatmulPreferenceCreate(&pref);
  uint64_t ws = WS_BYTES;
  hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &ws, sizeof(ws));
  hipblasLtMatmulHeuristicResult_t res[8];
  int n = 0;
  const hipblasStatus_t st = hipblasLtMatmulAlgoGetHeuristic(g_handle, p.desc, p.la, p.lb, p.lc, p.lc, pref, 8, res, &n);
  hipblasLtMatmulPreferenceDestroy(pref);
  for (int i = 0; st == HIPBLAS_STATUS_SUCCESS && i < n; ++i)
    if (res[i].state == HIPBLAS_STATUS_SUCCESS && res[i].workspaceSize <= WS_BYTES) {
      p.algo = res[i].algo;
      p.ok = true;
      break;
    }
  return p.ok ? &p : nullptr;
}

}  // namespace

int launch_gemm_blaslt_tn(const bf16_t* dy, long lddy, int Ny, const bf16_t* x, long ldx, int Nx, int K, float* C,
                          long ldc, hipStream_t st) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (!init()) return 0;
  Plan* p = plan_tn(Ny, Nx, K, lddy, ldx, ldc);
  if (!p) return 0;
  const float alpha = 1.f, beta = 0.f;
  const hipblasStatus_t s = hipblasLtMatmul(g_handle, p->desc, &alpha, x, p->la, dy, p->lb, &beta, C, p->lc, C, p->lc,
                                            &p->algo, g_ws, WS_BYTES, st);
  if (s != HIPBLAS_STATUS_SUCCESS) return set_error("hipblasLtMatmul (dY^T X) failed (%d)", (int)s);
  return 1;
}

bool blaslt_supported(const GemmArgs& a, int act, int out) {
  return act == ACT_NONE && (out == OUT_BF16 || out == OUT_F32) && !a.bias && !a.rowadd && !a.resid && !a.resid16 &&
         !a.bf16_linear && !a.aux && !a.aux2 && !a.aux_in && a.alpha == 1.f && a.amap.g == 0 && a.amap.off == 0 &&
         a.cmap.g == 0 && a.cmap.off == 0 && a.zin == 1;
}

// 1 = launched, 0 = not available for this shape (caller falls back to the MFMA kernels), < 0 = error
int launch_gemm_blaslt(const GemmArgs& a, int out, hipStream_t st) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (!init()) return 0;
  Plan* p = plan_for(a, out);
  if (!p) return 0;
  const float alpha = 1.f, beta = 0.f;
  const hipblasStatus_t s = hipblasLtMatmul(g_handle, p->desc, &alpha, a.B, p->la, a.A, p->lb, &beta, a.C, p->lc, a.C,
                                            p->lc, &p->algo, g_ws, WS_BYTES, st);
  if (s != HIPBLAS_STATUS_SUCCESS) return set_error("hipblasLtMatmul failed (%d)", (int)s);
  return 1;
}

}  // namespace ptk
