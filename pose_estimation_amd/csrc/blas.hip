// Plain f32 GEMMs on hipBLASLt: the GCN `feature_map @ weights + bias` of Conv_layer /
// Conv_fuse_layer (lib/network/point/gcn3d.py:136-216) and the TBase Conv1d
// chain (lib/network/pose/posenet.py:51-81, P1). These are library-shaped GEMMs (short K 128-1024,
// long M, bias / ReLU epilogue, no fusion beyond it), where hipBLASLt's f32 kernels measured 90-128
// TF/s against 62-99 for this library's own implicit-GEMM tiles (profiles/bench_gemm.py); the fused
// hot ops stay hand-written.
//
// Row-major problem, expressed in hipBLASLt's column-major terms:
//   out[m*ldo + n] = act( sum_k A[m*lda + k] W[n*K + k] + bias[n] + beta * res[m*ldr + n] )
//   D (N x M, ld ldo) = op_T(W as K x N, ld K) * (A as K x M, ld lda) (+ beta C, C = res)
// in `batch` strided groups (A / D / C advance a_grp / o_grp / r_grp floats per group, W shared):
// a row subset of every crop (TBase's P1 over the first N1 of each crop's N rows).
//
// A plan is created once (heuristic query, algorithm chosen) and owned by the caller; running it is
// one hipblasLtMatmul enqueue on the caller's stream (graph-capturable), with a caller-owned
// workspace. Nothing is allocated per call.
#include <hipblaslt/hipblaslt.h>

#include <new>

#include "krrn_common.h"

struct krrn_blas_gemm {
  hipblasLtHandle_t handle = nullptr;
  hipblasLtMatmulDesc_t desc = nullptr;
  hipblasLtMatrixLayout_t la = nullptr, lb = nullptr, lc = nullptr, ld = nullptr;
  hipblasLtMatmulAlgo_t algo;
  size_t ws = 0;
  int has_bias = 0, has_res = 0;
  float beta = 0.f;
};

namespace {

void destroy(krrn_blas_gemm* g) {
  if (!g) return;
  if (g->la) hipblasLtMatrixLayoutDestroy(g->la);
  if (g->lb) hipblasLtMatrixLayoutDestroy(g->lb);
  if (g->lc) hipblasLtMatrixLayoutDestroy(g->lc);
  if (g->ld) hipblasLtMatrixLayoutDestroy(g->ld);
  if (g->desc) hipblasLtMatmulDescDestroy(g->desc);
  if (g->handle) hipblasLtDestroy(g->handle);
  delete g;
}

bool batched(hipblasLtMatrixLayout_t l, int batch, long long stride) {
  if (batch <= 1) return true;
  const int32_t b = batch;
  const int64_t s = stride;
  return hipblasLtMatrixLayoutSetAttribute(l, HIPBLASLT_MATRIX_LAYOUT_BATCH_COUNT, &b, sizeof(b)) ==
             HIPBLAS_STATUS_SUCCESS &&
         hipblasLtMatrixLayoutSetAttribute(l, HIPBLASLT_MATRIX_LAYOUT_STRIDED_BATCH_OFFSET, &s, sizeof(s)) ==
             HIPBLAS_STATUS_SUCCESS;
}

}  // namespace

KRRN_API int krrn_blas_gemm_create(int M, int N, int K, int lda, int ldo, int batch, long long a_grp,
                                   long long o_grp, int has_bias, int relu, int has_res, int ldr, long long r_grp,
                                   long long max_ws, krrn_blas_gemm** out_plan, long long* ws_bytes) {
  if (!out_plan || !ws_bytes) return KRRN_EARG;
  *out_plan = nullptr;
  if (M < 1 || N < 1 || K < 1 || batch < 1 || lda < K || ldo < N || (has_res && ldr < N) || max_ws < 0)
    return KRRN_ESHAPE;
  krrn_blas_gemm* g = new (std::nothrow) krrn_blas_gemm();
  if (!g) return KRRN_EARG;
  g->has_bias = has_bias;
  g->has_res = has_res;
  g->beta = has_res ? 1.f : 0.f;
  bool ok = hipblasLtCreate(&g->handle) == HIPBLAS_STATUS_SUCCESS;
  ok = ok && hipblasLtMatmulDescCreate(&g->desc, HIPBLAS_COMPUTE_32F, HIP_R_32F) == HIPBLAS_STATUS_SUCCESS;
  const int32_t opT = HIPBLAS_OP_T, opN = HIPBLAS_OP_N;
  ok = ok && hipblasLtMatmulDescSetAttribute(g->desc, HIPBLASLT_MATMUL_DESC_TRANSA, &opT, sizeof(opT)) ==
                 HIPBLAS_STATUS_SUCCESS;
  ok = ok && hipblasLtMatmulDescSetAttribute(g->desc, HIPBLASLT_MATMUL_DESC_TRANSB, &opN, sizeof(opN)) ==
                 HIPBLAS_STATUS_SUCCESS;
  const uint32_t epi = has_bias ? (relu ? HIPBLASLT_EPILOGUE_RELU_BIAS : HIPBLASLT_EPILOGUE_BIAS)
                                : (relu ? HIPBLASLT_EPILOGUE_RELU : HIPBLASLT_EPILOGUE_DEFAULT);
  ok = ok && hipblasLtMatmulDescSetAttribute(g->desc, HIPBLASLT_MATMUL_DESC_EPILOGUE, &epi, sizeof(epi)) ==
                 HIPBLAS_STATUS_SUCCESS;
  if (has_bias) {
    const int32_t bt = HIP_R_32F;
    ok = ok && hipblasLtMatmulDescSetAttribute(g->desc, HIPBLASLT_MATMUL_DESC_BIAS_DATA_TYPE, &bt, sizeof(bt)) ==
                   HIPBLAS_STATUS_SUCCESS;
  }
  // A := W (K x N col-major, ld K, transposed), B := A rows (K x M, ld lda), C / D: N x M
  ok = ok && hipblasLtMatrixLayoutCreate(&g->la, HIP_R_32F, K, N, K) == HIPBLAS_STATUS_SUCCESS;
  ok = ok && hipblasLtMatrixLayoutCreate(&g->lb, HIP_R_32F, K, M, lda) == HIPBLAS_STATUS_SUCCESS;
  ok = ok && hipblasLtMatrixLayoutCreate(&g->lc, HIP_R_32F, N, M, has_res ? ldr : ldo) == HIPBLAS_STATUS_SUCCESS;
  ok = ok && hipblasLtMatrixLayoutCreate(&g->ld, HIP_R_32F, N, M, ldo) == HIPBLAS_STATUS_SUCCESS;
  ok = ok && batched(g->la, batch, 0) && batched(g->lb, batch, a_grp) &&
       batched(g->lc, batch, has_res ? r_grp : o_grp) && batched(g->ld, batch, o_grp);
  if (ok) {
    hipblasLtMatmulPreference_t pref = nullptr;
    ok = hipblasLtMatmulPreferenceCreate(&pref) == HIPBLAS_STATUS_SUCCESS;
    const uint64_t mw = (uint64_t)max_ws;
    ok = ok && hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &mw,
                                                     sizeof(mw)) == HIPBLAS_STATUS_SUCCESS;
    hipblasLtMatmulHeuristicResult_t res[1];
    int n = 0;
    ok = ok && hipblasLtMatmulAlgoGetHeuristic(g->handle, g->desc, g->la, g->lb, g->lc, g->ld, pref, 1, res, &n) ==
                   HIPBLAS_STATUS_SUCCESS &&
         n > 0 && res[0].state == HIPBLAS_STATUS_SUCCESS;
    if (ok) {
      g->algo = res[0].algo;
      g->ws = res[0].workspaceSize;
    }
    if (pref) hipblasLtMatmulPreferenceDestroy(pref);
  }
  if (!ok) {
    destroy(g);
    return KRRN_EUNSUPPORTED;
  }
  *out_plan = g;
  *ws_bytes = (long long)g->ws;
  return KRRN_OK;
}

KRRN_API int krrn_blas_gemm_run(const krrn_blas_gemm* g, const float* a, const float* w, const float* bias,
                                const float* res, float* out, void* workspace, long long ws_bytes, void* stream) {
  if (!g || !a || !w || !out) return KRRN_EARG;
  if ((g->has_bias && !bias) || (g->has_res && !res) || (g->ws && (!workspace || ws_bytes < (long long)g->ws)))
    return KRRN_EARG;
  if (g->has_bias &&
      hipblasLtMatmulDescSetAttribute(g->desc, HIPBLASLT_MATMUL_DESC_BIAS_POINTER, &bias, sizeof(bias)) !=
          HIPBLAS_STATUS_SUCCESS)
    return KRRN_EUNSUPPORTED;
  const float alpha = 1.f;
  const hipblasStatus_t st =
      hipblasLtMatmul(g->handle, g->desc, &alpha, w, g->la, a, g->lb, &g->beta, g->has_res ? res : out, g->lc, out,
                      g->ld, &g->algo, workspace, g->ws, (hipStream_t)stream);
  return st == HIPBLAS_STATUS_SUCCESS ? KRRN_OK : KRRN_EUNSUPPORTED;
}

KRRN_API int krrn_blas_gemm_destroy(krrn_blas_gemm* g) {
  destroy(g);
  return KRRN_OK;
}
