// Dense GEMM (nn.Linear forward / dX / dW) on the implicit-GEMM core: the templates.  The
// instantiations are spread over one translation unit per (compute, output) dtype pair
// (gemm_dense_{bf16,bf16f,f16,f16f,f32}.hip) so the library builds them in parallel; the
// C entry points live in gemm_dense.hip.
#pragma once
#include <type_traits>

#include "igemm.h"
#include "../../include/mmdx.h"

namespace mmdx {

struct SplitPlan { int bm, bn, splits, kper; };

// Split-K target: about this many (tile, split) blocks for grids of < 256 tiles (read once;
// MMDX_SPLITK_TARGET for A/B runs).  Every split writes an fp32 M x N slab that the reduce
// reads back, so the target trades slab traffic against idle CUs: C5 (paired, two boxes)
// 128 / 192 / 256 / 512 / 1024 -> 2379 / 2539 / 2587-2656 / 2609 / 2529 samples/s, C4
// neutral (tools/lab_splitk{,2}.sh, profiles/r04_splitk_sweep.txt).
static long splitk_target() { return knobs().splitk_target; }

// Tile + split-K choice; shared by the workspace query and the launch so both agree.
static SplitPlan plan_dense(int dtype, int M, int N, int K) {
  SplitPlan p;
  const int BK = dtype == F32 ? KTile<float>::BK : KTile<bf16>::BK;
  p.bm = M <= 64 ? 64 : 128;
  p.bn = N <= 64 ? 64 : 128;
  const long tiles = (long)((M + p.bm - 1) / p.bm) * ((N + p.bn - 1) / p.bn);
  const int ktiles = (K + BK - 1) / BK;
  int s = 1;
  if (tiles < 256 && ktiles >= 8) {
    s = (int)((splitk_target() + tiles - 1) / tiles);
    s = std::min(s, ktiles / 4);
    s = std::max(s, 1);
  }
  const int kt_per = (ktiles + s - 1) / s;
  p.kper = kt_per * BK;
  p.splits = (K + p.kper - 1) / p.kper;
  if (p.splits < 1) p.splits = 1;
  return p;
}

template <typename OutT>
__global__ void splitk_reduce_kernel(const float* __restrict__ ws, int splits, int M, int N,
                                     EpiStore<OutT, true> epi) {
  const long total = (long)M * N;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total;
       i += (long)gridDim.x * blockDim.x) {
    float v = 0.f;
    for (int z = 0; z < splits; ++z) v += ws[(long)z * total + i];
    epi.apply((int)(i / N), (int)(i % N), v);
  }
}

// The same for N % 4 == 0 and M * N < 2^31: 4 consecutive columns per thread (16-B partial
// loads, 4 splits' loads in flight, 32-bit index math — the scalar kernel's 64-bit divisions
// and one-load-at-a-time split loop made it ~12 us per C5 weight gradient); the sum over the
// splits keeps the order z = 0, 1, ..., so the result is the scalar kernel's bit for bit.
template <typename OutT>
__global__ __launch_bounds__(256) void splitk_reduce4_kernel(const float* __restrict__ ws,
                                                             int splits, int M, int N,
                                                             EpiStore<OutT, true> epi,
                                                             const float* __restrict__ bpart =
                                                                 nullptr,
                                                             float* __restrict__ db = nullptr) {
  // fused wgrad + bias (gemm_wgrad_bias_typed): the bias partials [splits][M] are reduced by
  // the same launch, in split order
  if (db)
    for (int m = blockIdx.x * blockDim.x + threadIdx.x; m < M; m += gridDim.x * blockDim.x) {
      float sb = 0.f;
      for (int z = 0; z < splits; ++z) sb += bpart[(long)z * M + m];
      db[m] = sb;
    }
  const int total4 = M * N / 4, n4 = N / 4;
  const f32x4* w = (const f32x4*)ws;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total4; i += gridDim.x * blockDim.x) {
    f32x4 v = f32x4{0.f, 0.f, 0.f, 0.f};
    int z = 0;
    for (; z + 4 <= splits; z += 4) {
      const f32x4 a = w[(long)z * total4 + i], b = w[(long)(z + 1) * total4 + i];
      const f32x4 c = w[(long)(z + 2) * total4 + i], d = w[(long)(z + 3) * total4 + i];
      v += a;
      v += b;
      v += c;
      v += d;
    }
    for (; z < splits; ++z) v += w[(long)z * total4 + i];
    const int m = i / n4;
    epi.apply4(m, (i - m * n4) * 4, v);
  }
}

// Retired (round 6, tools/lab/RETIRED.md): 8-wave 256 x 128 tiles (MMDX_GEMM8_MIN: 2-20 %
// slower on every C5 Linear shape, profiles/r03_gemm8_ab.txt), 256 x 256 tiles for the backward
// orientations (MMDX_GEMM256_MIN) and 32-deep K stages for them (MMDX_GEMM256_NS).

// 8-wave 256 x 256 tiles (waves 2 x 4 of 128 x 64, two 64 KB stages, one block per CU: a
// quarter of the LDS-DMA and half the fragment reads per MFMA of the 64 x 64-per-wave tiles)
// for the forward orientation only (both operands k-major: x W^T), where the isolated C5 table has the 256 x 256 tiles 3-8 % ahead on the ViT-B shapes while the
// backward orientations and the BERT-base shapes lose (profiles/r03n_gemm_bench_f16.txt).
// Default 90 tiles: every C5 encoder forward GEMM (ViT-B QKV / FFN-up 450 / 600 tiles, ViT-B
// N = 768 150, BERT-base QKV / FFN-up 288 / 384, BERT-base N = 768 96).  Round 3 set 400 (the
// ViT-B QKV / FFN-up only; profiles/r03u_c5_ab_gemm256fwd.txt); on the round-4 kernels (vector
// epilogue, residual input) 400 / 300 / 200 / 140 / 90 / 60 / 30 / 1 gave C5 2772 / 2781 / 2797
// / 2831 / 2863-2876 / 2877 / 2877 / 2871 samples/s, C4 neutral
// (profiles/r04_gemm256_fwd_sweep.txt); 0 disables (knobs(): a test pins the 128 x 128 kernel
// as its baseline).
static long gemm256_fwd_min_tiles() { return knobs().gemm256_fwd_min; }

// The 128 x 128 tiles as 8 waves of 64 x 32 (two 512-thread blocks per CU) instead of 4 waves
// of 64 x 64, as conv.hip's k-major conv tiles.  Default on: C5 2870 / 2865 -> 2910 / 2896
// samples/s paired; isolated C5 dgrad / wgrad shapes 1-8 % faster, the forward ones (mostly
// 256 x 256 tiles) equal; the one loss in tools/gemm_bench.py is the 4096^3 weight gradient
// (156 -> 216 us), which no config runs (r05 s24).  MMDX_GEMM_8W128=0 restores the 4-wave
// tiles.
static bool gemm_8w128_on() { return knobs().gemm_8w128; }

template <typename T, int BM, int BN, bool AK, bool BKm, class Epi>
static int launch_dense(const void* A, long lda, const void* B, long ldb, const Epi& epi,
                        int M, int N, int K, int splits, int kper, hipStream_t st) {
  typedef typename std::conditional<AK, DenseK<T>, DenseR<T>>::type SA;
  typedef typename std::conditional<BKm, DenseK<T>, DenseR<T>>::type SB;
  typedef typename std::conditional<AK, KLoad<T, BM, SA>, RLoad<T, BM, SA>>::type LA;
  typedef typename std::conditional<BKm, KLoad<T, BN, SB>, RLoad<T, BN, SB>>::type LB;
  constexpr int VEC = Vec16<T>::N;
  const bool va = lda % VEC == 0 && ((uintptr_t)A & 15) == 0;
  const bool vb = ldb % VEC == 0 && ((uintptr_t)B & 15) == 0;
  SA sa{(const T*)A, lda, M, va};
  SB sb{(const T*)B, ldb, N, vb};
  if constexpr (!AK) sa.vrows = K;  // R-major: k runs over the leading-dimension rows
  if constexpr (!BKm) sb.vrows = K;
  const int nwg = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  if constexpr (sizeof(T) == 2) {
    // LDS-DMA kernel when every 16-B chunk is either wholly inside or wholly outside the
    // operand: k-major needs K % 8 == 0, row-major needs its row count % 8 == 0
    const long abytes = (long)(AK ? M : K) * lda * 2, bbytes = (long)(BKm ? N : K) * ldb * 2;
    const bool oka = va && (AK ? K % 8 == 0 : M % 8 == 0) && abytes < (1L << 31);
    const bool okb = vb && (BKm ? K % 8 == 0 : N % 8 == 0) && bbytes < (1L << 31);
    if (oka && okb) {
      if constexpr (BM == 128 && BN == 128 && AK && BKm && !HasBiasSum<Epi>::value) {
        const long t256 = (long)((M + 255) / 256) * ((N + 255) / 256);
        const long lim256 = gemm256_fwd_min_tiles();
        if (splits == 1 && lim256 > 0 && t256 >= lim256 && K >= 128) {
          typedef DmaK<256, SA, 64, 8> OA8;
          typedef DmaK<256, SB, 64, 8> OB8;
          hipLaunchKernelGGL((igemm_dma_kernel<256, 256, OA8, OB8, Epi, 2, T, 512, 2, 4>),
                             dim3((unsigned)t256, 1, 1), dim3(512), 0, st, sa, sb, epi, M, N, K,
                             kper);
          MMDX_LAUNCH_CHECK();
          return 0;
        }
      }
      if constexpr (BM == 128 && BN == 128) {
        if (gemm_8w128_on()) {  // 8 waves of 64 x 32
          typedef typename std::conditional<AK, DmaK<128, SA, 64, 8>,
                                            DmaR<128, SA, 64, 8>>::type OA8;
          typedef typename std::conditional<BKm, DmaK<128, SB, 64, 8>,
                                            DmaR<128, SB, 64, 8>>::type OB8;
          if ((long)nwg * splits <= 256 && kper >= 256)
            hipLaunchKernelGGL((igemm_dma_kernel<128, 128, OA8, OB8, Epi, 3, T, 512, 2, 4>),
                               dim3(nwg, 1, splits), dim3(512), 0, st, sa, sb, epi, M, N, K, kper);
          else
            hipLaunchKernelGGL((igemm_dma_kernel<128, 128, OA8, OB8, Epi, 2, T, 512, 2, 4>),
                               dim3(nwg, 1, splits), dim3(512), 0, st, sa, sb, epi, M, N, K, kper);
          MMDX_LAUNCH_CHECK();
          return 0;
        }
      }
      typedef typename std::conditional<AK, DmaK<BM, SA>, DmaR<BM, SA>>::type OA;
      typedef typename std::conditional<BKm, DmaK<BN, SB>, DmaR<BN, SB>>::type OB;
      // three operand stages where the grid leaves one block per CU and K is long
      if ((long)nwg * splits <= 256 && kper >= 256)
        hipLaunchKernelGGL((igemm_dma_kernel<BM, BN, OA, OB, Epi, 3, T>),
                           dim3(nwg, 1, splits), dim3(NT), 0, st, sa, sb, epi, M, N, K, kper);
      else
        hipLaunchKernelGGL((igemm_dma_kernel<BM, BN, OA, OB, Epi, 2, T>),
                           dim3(nwg, 1, splits), dim3(NT), 0, st, sa, sb, epi, M, N, K, kper);
      MMDX_LAUNCH_CHECK();
      return 0;
    }
  }
  hipLaunchKernelGGL((igemm_kernel<T, BM, BN, 2, 2, LA, LB, Epi>), dim3(nwg, 1, splits),
                     dim3(NT), 0, st, sa, sb, epi, M, N, K, kper);
  MMDX_LAUNCH_CHECK();
  return 0;
}

template <typename T, bool AK, bool BKm, class Epi>
static int dispatch_tile(const SplitPlan& p, const void* A, long lda, const void* B, long ldb,
                         const Epi& epi, int M, int N, int K, hipStream_t st) {
  if (p.bm == 128 && p.bn == 128)
    return launch_dense<T, 128, 128, AK, BKm>(A, lda, B, ldb, epi, M, N, K, p.splits, p.kper, st);
  if (p.bm == 128)
    return launch_dense<T, 128, 64, AK, BKm>(A, lda, B, ldb, epi, M, N, K, p.splits, p.kper, st);
  if (p.bn == 128)
    return launch_dense<T, 64, 128, AK, BKm>(A, lda, B, ldb, epi, M, N, K, p.splits, p.kper, st);
  return launch_dense<T, 64, 64, AK, BKm>(A, lda, B, ldb, epi, M, N, K, p.splits, p.kper, st);
}

template <typename T, class Epi>
static int dispatch_major(const SplitPlan& p, const void* A, long lda, int ak, const void* B,
                          long ldb, int bk, const Epi& epi, int M, int N, int K,
                          hipStream_t st) {
  if (ak && bk) return dispatch_tile<T, true, true>(p, A, lda, B, ldb, epi, M, N, K, st);
  if (ak && !bk) return dispatch_tile<T, true, false>(p, A, lda, B, ldb, epi, M, N, K, st);
  if (!ak && !bk) return dispatch_tile<T, false, false>(p, A, lda, B, ldb, epi, M, N, K, st);
  return dispatch_tile<T, false, true>(p, A, lda, B, ldb, epi, M, N, K, st);
}

template <typename T, typename OutT>
static int gemm_typed(int M, int N, int K, const void* A, long lda, int ak, const void* B,
                      long ldb, int bk, void* C, long ldc, const float* bias,
                      const float* addend, int act,
                      float alpha, float beta, void* preact, void* ws, size_t ws_bytes,
                      hipStream_t st, const void* res = nullptr) {
  const SplitPlan p = plan_dense(sizeof(T) == 2 ? BF16 : F32, M, N, K);  // BF16 = any 16-bit
  MMDX_CHECK_ARG(lda >= (ak ? K : M) && ldb >= (bk ? K : N) && ldc >= N,
                 "mmdx_gemm: leading dimension too small");
  EpiStore<OutT, true> epi{(OutT*)C, ldc, M, N, bias, addend, act, alpha, beta, (OutT*)preact};
  epi.res = (const OutT*)res;
  if (p.splits == 1) return dispatch_major<T>(p, A, lda, ak, B, ldb, bk, epi, M, N, K, st);
  const size_t need = (size_t)p.splits * M * N * sizeof(float);
  MMDX_CHECK_ARG(ws && ws_bytes >= need, "mmdx_gemm: workspace %zu < %zu", ws_bytes, need);
  EpiPartial part{(float*)ws, M, N};
  int rc = dispatch_major<T>(p, A, lda, ak, B, ldb, bk, part, M, N, K, st);
  if (rc) return rc;
  const long total = (long)M * N;
  const bool vec_reduce = knobs().splitk_vec;   // MMDX_SPLITK_VEC=0: the scalar reduce (A/B)
  if (vec_reduce && N % 4 == 0 && total < (1L << 31) && ((uintptr_t)ws & 15) == 0) {
    const int blocks = (int)std::min<long>((total / 4 + 255) / 256, 8192);
    hipLaunchKernelGGL(splitk_reduce4_kernel<OutT>, dim3(blocks), dim3(256), 0, st,
                       (const float*)ws, p.splits, M, N, epi);
  } else {
    const int blocks = (int)std::min<long>((total + 255) / 256, 4096);
    hipLaunchKernelGGL(splitk_reduce_kernel<OutT>, dim3(blocks), dim3(256), 0, st,
                       (const float*)ws, p.splits, M, N, epi);
  }
  MMDX_LAUNCH_CHECK();
  return 0;
}

// dW = A B with A = dY^T and B = X both R-major (the weight gradient of a Linear layer), plus
// its bias gradient db = row sums of A, fused into the split-K GEMM (EpiPartialBias) and
// reduced over the splits by the split-K reduce launch; bias partials follow the fp32 slabs
// in the workspace.

// MMDX_WGRAD_BIAS_FUSED=0: GEMM + column-sum kernels
static bool wgrad_bias_fused_on() { return knobs().wgrad_bias_fused; }

template <typename T, typename OutT>
static int gemm_wgrad_bias_typed(const SplitPlan& p, int M, int N, int K, const void* A, long lda,
                                 const void* B, long ldb, void* C, long ldc, float* db,
                                 void* ws, hipStream_t st) {
  EpiPartialBias part{};
  part.ws = (float*)ws;
  part.M = M;
  part.N = N;
  part.bpart = (float*)ws + (size_t)p.splits * M * N;
  int rc = dispatch_tile<T, false, false>(p, A, lda, B, ldb, part, M, N, K, st);
  if (rc) return rc;
  EpiStore<OutT, true> epi{(OutT*)C, ldc, M, N, nullptr, nullptr, ACT_NONE, 1.f, 0.f, nullptr};
  const long total = (long)M * N;
  const int blocks = (int)std::min<long>((total / 4 + 255) / 256, 8192);
  hipLaunchKernelGGL(splitk_reduce4_kernel<OutT>, dim3(blocks), dim3(256), 0, st,
                     (const float*)ws, p.splits, M, N, epi, (const float*)part.bpart, db);
  MMDX_LAUNCH_CHECK();
  return 0;
}


// One instantiation set per (T, OutT), defined in its own translation unit (gemm_dense_<tag>.hip).
#define MMDX_GEMM_TU_DECL(TAG, T, OUT)                                                       \
  int gemm_typed_##TAG(int M, int N, int K, const void* A, long lda, int ak, const void* B,  \
                       long ldb, int bk, void* C, long ldc, const float* bias,               \
                       const float* addend, int act, float alpha, float beta, void* preact,  \
                       void* ws, size_t ws_bytes, hipStream_t st, const void* res);          \
  int gemm_wgrad_bias_##TAG(const SplitPlan& p, int M, int N, int K, const void* A,          \
                            long lda, const void* B, long ldb, void* C, long ldc, float* db, \
                            void* ws, hipStream_t st);
MMDX_GEMM_TU_DECL(bf16, bf16, bf16)
MMDX_GEMM_TU_DECL(bf16f, bf16, float)
MMDX_GEMM_TU_DECL(f16, f16, f16)
MMDX_GEMM_TU_DECL(f16f, f16, float)
MMDX_GEMM_TU_DECL(f32, float, float)

#define MMDX_GEMM_TU_DEF(TAG, T, OUT)                                                        \
  int gemm_typed_##TAG(int M, int N, int K, const void* A, long lda, int ak, const void* B,  \
                       long ldb, int bk, void* C, long ldc, const float* bias,               \
                       const float* addend, int act, float alpha, float beta, void* preact,  \
                       void* ws, size_t ws_bytes, hipStream_t st, const void* res) {         \
    return gemm_typed<T, OUT>(M, N, K, A, lda, ak, B, ldb, bk, C, ldc, bias, addend, act,    \
                              alpha, beta, preact, ws, ws_bytes, st, res);                   \
  }
// the fused weight + bias gradient (16-bit compute only)
#define MMDX_GEMM_TU_DEF_WB(TAG, T, OUT)                                                     \
  int gemm_wgrad_bias_##TAG(const SplitPlan& p, int M, int N, int K, const void* A,          \
                            long lda, const void* B, long ldb, void* C, long ldc, float* db, \
                            void* ws, hipStream_t st) {                                      \
    return gemm_wgrad_bias_typed<T, OUT>(p, M, N, K, A, lda, B, ldb, C, ldc, db, ws, st);    \
  }

}  // namespace mmdx
