// Plain bf16 GEMMs through hipBLASLt (the library GEMM for the products with no fused epilogue:
// the QKV projection, the dgrads whose output is a plain store, and train_mode='full''s weight
// gradients). Row-major NT convention of ltx_gemm_bf16_nt:
//   C[M, N] (+)= A[M, K] . W[N, K]^T (+ bias[N])
// a_kmajor / w_kmajor = 1: the operand is stored K-major ([K, M] / [K, N] row-major), which is how
// the token-major activations and gradients sit in HBM for a weight gradient (K = tokens) -- the
// library reads them transposed, so no transpose pass is needed.
// hipBLASLt is column-major: the row-major C[M, N] is D[N, M] = W . A^T with m = N, n = M, k = K.
// One handle, one workspace and one cached algorithm per (device, shape, layout) key.
#include <hipblaslt/hipblaslt.h>

#include <map>
#include <mutex>
#include <tuple>

#include "common.h"
#include "ltx_hip.h"

namespace ltx {
namespace {

constexpr size_t kBlasltWs = 64u << 20;

struct BlasltDev {
  hipblasLtHandle_t handle = nullptr;
  std::map<hipStream_t, void*> ws;  // one workspace per stream: concurrent streams never share it
};

struct BlasltPlan {
  hipblasLtMatmulDesc_t desc = nullptr;
  hipblasLtMatrixLayout_t a = nullptr, b = nullptr, c = nullptr;
  hipblasLtMatmulAlgo_t algo;
  size_t ws = 0;
};

using PlanKey = std::tuple<int, int, int, int, int64_t, int64_t, int64_t, int64_t, int64_t, int64_t, int, int>;

std::mutex g_mu;
std::map<int, BlasltDev> g_dev;
std::map<PlanKey, BlasltPlan> g_plans;

int blas_fail(hipblasStatus_t st, const char* what) {
  return fail(LTX_ERR_UNSUPPORTED, std::string("hipBLASLt ") + what + " failed: status " + std::to_string((int)st));
}

}  // namespace
}  // namespace ltx

using namespace ltx;

extern "C" int ltx_gemm_blaslt_bf16(int a_kmajor, int w_kmajor, const void* A, int64_t lda, const void* W,
                                    int64_t ldw, void* C, int64_t ldc, int64_t M, int64_t N, int64_t K,
                                    const void* bias, int accumulate, void* stream) {
  LTX_CHECK_ARG(A && W && C && M > 0 && N > 0 && K > 0, "gemm_blaslt: null operand or empty shape");
  LTX_CHECK_ARG(lda >= (a_kmajor ? M : K) && ldw >= (w_kmajor ? N : K) && ldc >= N,
                "gemm_blaslt: leading dim smaller than the row");
  LTX_CHECK_ARG(!(bias && accumulate), "gemm_blaslt: bias with accumulate is not supported");
  int dev = 0;
  hipError_t he = hipGetDevice(&dev);
  if (he != hipSuccess) return fail((int)he, hipGetErrorString(he));
  std::lock_guard<std::mutex> lock(g_mu);
  BlasltDev& d = g_dev[dev];
  if (!d.handle) {
    hipblasStatus_t st = hipblasLtCreate(&d.handle);
    if (st != HIPBLAS_STATUS_SUCCESS) return blas_fail(st, "create");
  }
  void*& ws = d.ws[(hipStream_t)stream];
  if (!ws) {
    he = hipMalloc(&ws, kBlasltWs);
    if (he != hipSuccess) return fail((int)he, hipGetErrorString(he));
  }
  const PlanKey key{dev, a_kmajor, w_kmajor, bias != nullptr, M, N, K, lda, ldw, ldc, accumulate, 0};
  auto it = g_plans.find(key);
  if (it == g_plans.end()) {
    BlasltPlan pl;
    hipblasStatus_t st = hipblasLtMatmulDescCreate(&pl.desc, HIPBLAS_COMPUTE_32F, HIP_R_32F);
    if (st != HIPBLAS_STATUS_SUCCESS) return blas_fail(st, "desc");
    // A_bl = W: [N, K] row-major = col-major [K, N] -> op T; K-major [K, N] = col-major [N, K] -> op N
    const hipblasOperation_t ta = w_kmajor ? HIPBLAS_OP_N : HIPBLAS_OP_T;
    // B_bl = A^T: [M, K] row-major = col-major [K, M] -> op N; K-major [K, M] = col-major [M, K] -> op T
    const hipblasOperation_t tb = a_kmajor ? HIPBLAS_OP_T : HIPBLAS_OP_N;
    hipblasLtMatmulDescSetAttribute(pl.desc, HIPBLASLT_MATMUL_DESC_TRANSA, &ta, sizeof(ta));
    hipblasLtMatmulDescSetAttribute(pl.desc, HIPBLASLT_MATMUL_DESC_TRANSB, &tb, sizeof(tb));
    if (bias) {
      const hipblasLtEpilogue_t epi = HIPBLASLT_EPILOGUE_BIAS;
      const hipDataType bt = HIP_R_16BF;
      hipblasLtMatmulDescSetAttribute(pl.desc, HIPBLASLT_MATMUL_DESC_EPILOGUE, &epi, sizeof(epi));
      hipblasLtMatmulDescSetAttribute(pl.desc, HIPBLASLT_MATMUL_DESC_BIAS_DATA_TYPE, &bt, sizeof(bt));
    }
    st = w_kmajor ? hipblasLtMatrixLayoutCreate(&pl.a, HIP_R_16BF, N, K, ldw)
                  : hipblasLtMatrixLayoutCreate(&pl.a, HIP_R_16BF, K, N, ldw);
    if (st != HIPBLAS_STATUS_SUCCESS) return blas_fail(st, "layout A");
    st = a_kmajor ? hipblasLtMatrixLayoutCreate(&pl.b, HIP_R_16BF, M, K, lda)
                  : hipblasLtMatrixLayoutCreate(&pl.b, HIP_R_16BF, K, M, lda);
    if (st != HIPBLAS_STATUS_SUCCESS) return blas_fail(st, "layout B");
    st = hipblasLtMatrixLayoutCreate(&pl.c, HIP_R_16BF, N, M, ldc);
    if (st != HIPBLAS_STATUS_SUCCESS) return blas_fail(st, "layout C");
    hipblasLtMatmulPreference_t pref;
    st = hipblasLtMatmulPreferenceCreate(&pref);
    if (st != HIPBLAS_STATUS_SUCCESS) return blas_fail(st, "preference");
    const uint64_t wsb = kBlasltWs;
    hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &wsb, sizeof(wsb));
    hipblasLtMatmulHeuristicResult_t res[1];
    int got = 0;
    st = hipblasLtMatmulAlgoGetHeuristic(d.handle, pl.desc, pl.a, pl.b, pl.c, pl.c, pref, 1, res, &got);
    hipblasLtMatmulPreferenceDestroy(pref);
    if (st != HIPBLAS_STATUS_SUCCESS || got < 1) return blas_fail(st, "heuristic (no algorithm)");
    pl.algo = res[0].algo;
    pl.ws = res[0].workspaceSize;
    it = g_plans.emplace(key, pl).first;
  }
  BlasltPlan& pl = it->second;
  if (bias) {
    hipblasStatus_t st = hipblasLtMatmulDescSetAttribute(pl.desc, HIPBLASLT_MATMUL_DESC_BIAS_POINTER, &bias,
                                                         sizeof(bias));
    if (st != HIPBLAS_STATUS_SUCCESS) return blas_fail(st, "bias pointer");
  }
  const float alpha = 1.0f, beta = accumulate ? 1.0f : 0.0f;
  hipblasStatus_t st = hipblasLtMatmul(d.handle, pl.desc, &alpha, W, pl.a, A, pl.b, &beta, C, pl.c, C, pl.c,
                                       &pl.algo, ws, pl.ws, (hipStream_t)stream);
  if (st != HIPBLAS_STATUS_SUCCESS) return blas_fail(st, "matmul");
  return LTX_OK;
}
