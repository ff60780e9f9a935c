// Dense GEMM C entry points (nn.Linear forward / dX / dW); the kernels are instantiated in
// gemm_dense_{bf16,bf16f,f16,f16f,f32}.hip (gemm_dense.h).
#include "gemm_dense.h"

using namespace mmdx;

extern "C" size_t mmdx_gemm_bias_grad_workspace_size(int dtype, int M, int N, int K) {
  const SplitPlan p = plan_dense(dtype, M, N, K);
  const size_t fused = p.splits > 1 ? (size_t)p.splits * ((size_t)M * N + M) * sizeof(float) : 0;
  const size_t plain = std::max(mmdx_gemm_workspace_size(dtype, M, N, K),
                                mmdx_bias_grad_workspace_size(K, M));
  return std::max(fused, plain);
}

extern "C" int mmdx_gemm_bias_grad(int dtype, int M, int N, int K, const void* A, long lda,
                                   const void* B, long ldb, void* C, long ldc, int c_dtype,
                                   float* db, void* ws, size_t ws_bytes, void* stream) {
  MMDX_CHECK_ARG(lda >= M && ldb >= N && ldc >= N && db, "gemm bias grad: bad arguments");
  MMDX_CHECK_ARG(ws && ws_bytes >= mmdx_gemm_bias_grad_workspace_size(dtype, M, N, K),
                 "gemm bias grad: workspace too small");
  hipStream_t st = (hipStream_t)stream;
  const SplitPlan p = plan_dense(dtype, M, N, K);
  const long abytes = (long)K * lda * 2, bbytes = (long)K * ldb * 2;
  const bool fused = wgrad_bias_fused_on() && dtype != F32 && p.splits > 1 && p.bm == 128 &&
                     M % 8 == 0 && N % 8 == 0 && lda % 8 == 0 && ldb % 8 == 0 &&
                     ((uintptr_t)A & 15) == 0 && ((uintptr_t)B & 15) == 0 &&
                     abytes < (1L << 31) && bbytes < (1L << 31);
  if (fused) {
    if (dtype == F16) {
      if (c_dtype == F32)
        return gemm_wgrad_bias_f16f(p, M, N, K, A, lda, B, ldb, C, ldc, db, ws, st);
      return gemm_wgrad_bias_f16(p, M, N, K, A, lda, B, ldb, C, ldc, db, ws, st);
    }
    if (c_dtype == F32)
      return gemm_wgrad_bias_bf16f(p, M, N, K, A, lda, B, ldb, C, ldc, db, ws, st);
    return gemm_wgrad_bias_bf16(p, M, N, K, A, lda, B, ldb, C, ldc, db, ws, st);
  }
  // the GEMM, then the column sums of dY = A^T ([K][lda], M columns)
  MMDX_CHECK_ARG(lda == M, "gemm bias grad: unfused path needs lda == M");
  int rc = mmdx_gemm(dtype, M, N, K, A, lda, 0, B, ldb, 0, C, ldc, c_dtype, nullptr, nullptr,
                     ACT_NONE, 1.f, 0.f, nullptr, ws, ws_bytes, stream);
  if (rc) return rc;
  return mmdx_bias_grad(dtype, A, K, M, db, 0.f, ws, ws_bytes, stream);
}

extern "C" size_t mmdx_gemm_workspace_size(int dtype, int M, int N, int K) {
  const SplitPlan p = plan_dense(dtype, M, N, K);
  return p.splits > 1 ? (size_t)p.splits * M * N * sizeof(float) : 0;
}

static int gemm_entry(int dtype, int M, int N, int K, const void* A, long lda, int a_kmajor,
                         const void* B, long ldb, int b_kmajor, void* C, long ldc, int c_dtype,
                         const float* bias, const float* addend, int act, float alpha,
                         float beta, void* preact, void* workspace, size_t ws_bytes,
                         void* stream, const void* res) {
  MMDX_CHECK_ARG(M > 0 && N > 0 && K > 0, "mmdx_gemm: empty problem M=%d N=%d K=%d", M, N, K);
  hipStream_t st = (hipStream_t)stream;
  if (dtype == F32) {
    MMDX_CHECK_ARG(c_dtype == F32, "mmdx_gemm: fp32 compute needs fp32 output");
    return gemm_typed_f32(M, N, K, A, lda, a_kmajor, B, ldb, b_kmajor, C, ldc, bias,
                                    addend, act, alpha, beta, preact, workspace, ws_bytes, st, res);
  }
  if (dtype == F16) {
    if (c_dtype == F32)
      return gemm_typed_f16f(M, N, K, A, lda, a_kmajor, B, ldb, b_kmajor, C, ldc, bias,
                                    addend, act, alpha, beta, preact, workspace, ws_bytes, st, res);
    MMDX_CHECK_ARG(c_dtype == F16, "mmdx_gemm: fp16 compute writes fp16 or fp32");
    return gemm_typed_f16(M, N, K, A, lda, a_kmajor, B, ldb, b_kmajor, C, ldc, bias,
                                addend, act, alpha, beta, preact, workspace, ws_bytes, st, res);
  }
  MMDX_CHECK_ARG(dtype == BF16, "mmdx_gemm: bad dtype %d", dtype);
  MMDX_CHECK_ARG(c_dtype == F32 || c_dtype == BF16, "mmdx_gemm: bf16 compute writes bf16/fp32");
  if (c_dtype == F32)
    return gemm_typed_bf16f(M, N, K, A, lda, a_kmajor, B, ldb, b_kmajor, C, ldc, bias,
                                   addend, act, alpha, beta, preact, workspace, ws_bytes, st, res);
  return gemm_typed_bf16(M, N, K, A, lda, a_kmajor, B, ldb, b_kmajor, C, ldc, bias, addend, act,
                                alpha, beta, preact, workspace, ws_bytes, st, res);
}

extern "C" int mmdx_gemm(int dtype, int M, int N, int K, const void* A, long lda, int a_kmajor,
                         const void* B, long ldb, int b_kmajor, void* C, long ldc, int c_dtype,
                         const float* bias, const float* addend, int act, float alpha,
                         float beta, void* preact, void* workspace, size_t ws_bytes,
                         void* stream) {
  return gemm_entry(dtype, M, N, K, A, lda, a_kmajor, B, ldb, b_kmajor, C, ldc, c_dtype, bias,
                    addend, act, alpha, beta, preact, workspace, ws_bytes, stream, nullptr);
}

extern "C" int mmdx_gemm_res(int dtype, int M, int N, int K, const void* A, long lda,
                             int a_kmajor, const void* B, long ldb, int b_kmajor, void* C,
                             long ldc, int c_dtype, const float* bias, const float* addend,
                             int act, float alpha, float beta, void* preact,
                             const void* residual, void* workspace, size_t ws_bytes,
                             void* stream) {
  MMDX_CHECK_ARG(residual != C, "mmdx_gemm_res: the residual must not alias C");
  return gemm_entry(dtype, M, N, K, A, lda, a_kmajor, B, ldb, b_kmajor, C, ldc, c_dtype, bias,
                    addend, act, alpha, beta, preact, workspace, ws_bytes, stream, residual);
}
