// Lab build of tools/lab/gemm8ph.h (the 8-wave ping-pong 256 x 256 GEMM; not on the product
// path until it is dispatched by mmdx_gemm) with a C entry point, timed by tools/gemm8ph_lab.py.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -shared -fPIC -I include \
//     -o tools/lab/libgemm8ph_lab.so tools/lab/gemm8ph_lab.hip
#include "gemm8ph.h"

using namespace mmdx;

template <typename T, typename OutT, bool AK, bool BK, int SCHED>
static int launch1(int M, int N, int K, const void* A, long lda, const void* B, long ldb, void* C,
                  long ldc, int splits, void* ws, hipStream_t st) {
  typedef typename std::conditional<AK, HalfK<T>, HalfR<T>>::type OA;
  typedef typename std::conditional<BK, HalfK<T>, HalfR<T>>::type OB;
  typename OA::Src sa{};
  typename OB::Src sb{};
  sa.base = (const T*)A; sa.ld = lda; sa.R = M; sa.vec = true;
  sb.base = (const T*)B; sb.ld = ldb; sb.R = N; sb.vec = true;
  if constexpr (!AK) sa.vrows = K;
  if constexpr (!BK) sb.vrows = K;
  const int nwg = ((M + 255) / 256) * ((N + 255) / 256);
  const int kper = ((K + 64 * splits - 1) / (64 * splits)) * 64;
  if (splits > 1) {
    EpiPartial epi{(float*)ws, M, N};
    hipLaunchKernelGGL((gemm8ph_kernel<OA, OB, EpiPartial, T, SCHED>), dim3(nwg, 1, splits), dim3(512),
                       0, st, sa, sb, epi, M, N, K, kper);
  } else {
    EpiStore<OutT> epi{(OutT*)C, ldc, M, N, nullptr, nullptr, ACT_NONE, 1.f, 0.f, nullptr};
    hipLaunchKernelGGL((gemm8ph_kernel<OA, OB, EpiStore<OutT>, T, SCHED>), dim3(nwg, 1, 1), dim3(512), 0,
                       st, sa, sb, epi, M, N, K, kper);
  }
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

static int g_sched = 1;
template <typename T, typename OutT, bool AK, bool BK>
static int launch(int M, int N, int K, const void* A, long lda, const void* B, long ldb, void* C,
                  long ldc, int splits, void* ws, hipStream_t st) {
  if (g_sched == 0)
    return launch1<T, OutT, AK, BK, 0>(M, N, K, A, lda, B, ldb, C, ldc, splits, ws, st);
  return launch1<T, OutT, AK, BK, 1>(M, N, K, A, lda, B, ldb, C, ldc, splits, ws, st);
}

extern "C" void lab_gemm8ph_sched(int s) { g_sched = s; }

template <typename T, typename OutT>
static int by_major(int ak, int bk, int M, int N, int K, const void* A, long lda, const void* B,
                    long ldb, void* C, long ldc, int splits, void* ws, hipStream_t st) {
  if (ak && bk) return launch<T, OutT, true, true>(M, N, K, A, lda, B, ldb, C, ldc, splits, ws, st);
  if (ak) return launch<T, OutT, true, false>(M, N, K, A, lda, B, ldb, C, ldc, splits, ws, st);
  if (bk) return launch<T, OutT, false, true>(M, N, K, A, lda, B, ldb, C, ldc, splits, ws, st);
  return launch<T, OutT, false, false>(M, N, K, A, lda, B, ldb, C, ldc, splits, ws, st);
}

// dtype 1 = bf16, 2 = f16; out_f32: C in fp32 (else the operand dtype)
extern "C" int lab_gemm8ph(int dtype, int out_f32, int ak, int bk, int M, int N, int K,
                           const void* A, long lda, const void* B, long ldb, void* C, long ldc,
                           int splits, void* ws, hipStream_t st) {
  if (K % 8 || (!ak && M % 8) || (!bk && N % 8)) return 2;
  if (dtype == 2)
    return out_f32 ? by_major<f16, float>(ak, bk, M, N, K, A, lda, B, ldb, C, ldc, splits, ws, st)
                   : by_major<f16, f16>(ak, bk, M, N, K, A, lda, B, ldb, C, ldc, splits, ws, st);
  return out_f32 ? by_major<bf16, float>(ak, bk, M, N, K, A, lda, B, ldb, C, ldc, splits, ws, st)
                 : by_major<bf16, bf16>(ak, bk, M, N, K, A, lda, B, ldb, C, ldc, splits, ws, st);
}
