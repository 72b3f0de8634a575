// hipBLASLt for plain library GEMMs: out[M,N] (bf16 / fp16) = A[M,K]·B[N,K]ᵀ (+ fp32 bias per column) (+ bf16 residual),
// fp32 accumulation.  Used where the vendor's stream-K kernel beats the hand-written 8-phase one — the N = 768,
// K = 768 shapes (VideoMAE attention output projection forward and its input gradient on Wᵀ), where 588 tiles of
// 256² fall on 256 CUs as 2.3 rounds and the vendor kernel runs 196 workgroups of exactly 3 tiles (DESIGN.md,
// round 6).  Host code only: descriptor / layout / heuristic setup, cached per shape and epilogue.
#include "common.h"
#include <hipblaslt/hipblaslt.h>
#include <map>
#include <mutex>
#include <tuple>

namespace {

constexpr size_t LT_WS_BYTES = 128ull << 20;

struct LtPlan {
  hipblasLtMatmulDesc_t desc = nullptr;
  hipblasLtMatrixLayout_t la = nullptr, lb = nullptr, lc = nullptr, ld = nullptr;
  hipblasLtMatmulAlgo_t algo;
  size_t ws = 0;
};

struct LtDev {
  hipblasLtHandle_t handle = nullptr;
  size_t ws_bytes = LT_WS_BYTES;
  std::map<hipStream_t, void*> ws;   // one workspace per stream: launches on two streams may run concurrently
  std::map<std::tuple<int, int, int, long, long, long, long, int, int>, LtPlan> plans;
};

std::mutex g_lt_mu;
std::map<int, LtDev> g_lt;


LtDev* lt_dev() {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return nullptr;
  LtDev& d = g_lt[dev];
  if (!d.handle && hipblasLtCreate(&d.handle) != HIPBLAS_STATUS_SUCCESS) {
    d.handle = nullptr;
    return nullptr;
  }
  return &d;
}

void* lt_ws(LtDev* d, hipStream_t st) {
  auto it = d->ws.find(st);
  if (it != d->ws.end()) return it->second;
  void* p = nullptr;
  if (hipMalloc(&p, d->ws_bytes) != hipSuccess) return nullptr;
  d->ws[st] = p;
  return p;
}

// Column-major view: Dᵀ[N, M] = op_T(B as col-major [K, N]) · (A as col-major [K, M]); the bias (length N = rows of
// Dᵀ) is the per-output-feature bias of the row-major product.
LtPlan* lt_plan(LtDev* d, int dtype, int M, int N, int K, long lda, long ldb, long ldr, long ldo, int epi) {
  const auto key = std::make_tuple(M, N, K, lda, ldb, ldr, ldo, epi, dtype);
  const hipDataType dt = dtype == CMHAR_F16 ? HIP_R_16F : HIP_R_16BF;
  auto it = d->plans.find(key);
  if (it != d->plans.end()) return &it->second;
  LtPlan p;
  const hipblasOperation_t ta = HIPBLAS_OP_T, tb = HIPBLAS_OP_N;
  bool ok = hipblasLtMatmulDescCreate(&p.desc, HIPBLAS_COMPUTE_32F, HIP_R_32F) == HIPBLAS_STATUS_SUCCESS;
  ok = ok && hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_TRANSA, &ta, sizeof(ta)) == HIPBLAS_STATUS_SUCCESS;
  ok = ok && hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_TRANSB, &tb, sizeof(tb)) == HIPBLAS_STATUS_SUCCESS;
  if (ok && (epi & 1)) {
    const hipblasLtEpilogue_t e = HIPBLASLT_EPILOGUE_BIAS;
    const hipDataType bt = HIP_R_32F;
    ok = hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_EPILOGUE, &e, sizeof(e)) == HIPBLAS_STATUS_SUCCESS &&
         hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_BIAS_DATA_TYPE, &bt, sizeof(bt)) == HIPBLAS_STATUS_SUCCESS;
  }
  ok = ok && hipblasLtMatrixLayoutCreate(&p.la, dt, K, N, ldb) == HIPBLAS_STATUS_SUCCESS;
  ok = ok && hipblasLtMatrixLayoutCreate(&p.lb, dt, K, M, lda) == HIPBLAS_STATUS_SUCCESS;
  ok = ok && hipblasLtMatrixLayoutCreate(&p.lc, dt, N, M, (epi & 2) ? ldr : ldo) == HIPBLAS_STATUS_SUCCESS;
  ok = ok && hipblasLtMatrixLayoutCreate(&p.ld, dt, N, M, ldo) == HIPBLAS_STATUS_SUCCESS;
  hipblasLtMatmulPreference_t pref = nullptr;
  ok = ok && hipblasLtMatmulPreferenceCreate(&pref) == HIPBLAS_STATUS_SUCCESS;
  const uint64_t wsb = d->ws_bytes;
  ok = ok && hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &wsb, sizeof(wsb)) ==
                 HIPBLAS_STATUS_SUCCESS;
  hipblasLtMatmulHeuristicResult_t res[1];
  int got = 0;
  ok = ok && hipblasLtMatmulAlgoGetHeuristic(d->handle, p.desc, p.la, p.lb, p.lc, p.ld, pref, 1, res, &got) ==
                 HIPBLAS_STATUS_SUCCESS && got > 0 && res[0].workspaceSize <= d->ws_bytes;
  if (pref) hipblasLtMatmulPreferenceDestroy(pref);
  if (!ok) {
    if (p.desc) hipblasLtMatmulDescDestroy(p.desc);
    for (auto l : {p.la, p.lb, p.lc, p.ld}) if (l) hipblasLtMatrixLayoutDestroy(l);
    return nullptr;
  }
  p.algo = res[0].algo;
  p.ws = res[0].workspaceSize;
  return &d->plans.emplace(key, p).first->second;
}

}  // namespace

extern "C" int cmhar_blaslt_linear(int dtype, int M, int N, int K, const void* A, long lda, const void* B, long ldb, void* out,
                                   long ldo, const float* bias, const void* residual, long ldr, hipStream_t st) {
  if (dtype != CMHAR_BF16 && dtype != CMHAR_F16) return 7;
  if (M <= 0 || N <= 0 || K <= 0) return 0;
  if (!A || !B || !out || lda < K || ldb < K || ldo < N || (residual && ldr < N)) return 1;
  std::lock_guard<std::mutex> lock(g_lt_mu);
  LtDev* d = lt_dev();
  if (!d) return 2;
  const int epi = (bias ? 1 : 0) | (residual ? 2 : 0);
  LtPlan* p = lt_plan(d, dtype, M, N, K, lda, ldb, residual ? ldr : 0, ldo, epi);
  if (!p) return 3;
  void* ws = p->ws ? lt_ws(d, st) : nullptr;
  if (p->ws && !ws) return 6;
  if (bias && hipblasLtMatmulDescSetAttribute(p->desc, HIPBLASLT_MATMUL_DESC_BIAS_POINTER, &bias, sizeof(bias)) !=
                  HIPBLAS_STATUS_SUCCESS)
    return 4;
  const float alpha = 1.f, beta = residual ? 1.f : 0.f;
  const void* C = residual ? residual : out;
  if (hipblasLtMatmul(d->handle, p->desc, &alpha, B, p->la, A, p->lb, &beta, C, p->lc, out, p->ld, &p->algo, ws,
                      p->ws, st) != HIPBLAS_STATUS_SUCCESS)
    return 5;
  return 0;
}

// 1 when the library finds an algorithm for this shape / epilogue (plans it on the current device), else 0.
extern "C" int cmhar_blaslt_linear_ok(int dtype, int M, int N, int K, long lda, long ldb, long ldo, int has_bias, int has_residual,
                                      long ldr) {
  std::lock_guard<std::mutex> lock(g_lt_mu);
  LtDev* d = lt_dev();
  if (!d) return 0;
  if (dtype != CMHAR_BF16 && dtype != CMHAR_F16) return 0;
  return lt_plan(d, dtype, M, N, K, lda, ldb, has_residual ? ldr : 0, ldo, (has_bias ? 1 : 0) | (has_residual ? 2 : 0)) ? 1 : 0;
}
