// NHWC convolution on the implicit-GEMM core: fwd, dgrad, wgrad (+ weight packing).
// Replaces every nn.Conv2d of the torchvision ResNet trunk that ImageEncoderCNN wraps
// (training_pipeline.py:178-183, run through _backbone_forward_grad TP:285-289).
#include <algorithm>
#include <cstdlib>

#include "igemm.h"
#include "../../include/mmdx.h"

namespace mmdx {

static ConvGeom geom(const mmdx_conv_desc* d) {
  ConvGeom g;
  g.N = d->N; g.H = d->H; g.W = d->W; g.C = d->C; g.K = d->K; g.R = d->R; g.S = d->S;
  g.sh = d->stride_h; g.sw = d->stride_w; g.ph = d->pad_h; g.pw = d->pad_w;
  g.P = d->P; g.Q = d->Q;
  return g;
}

static int check_desc(const mmdx_conv_desc* d, int vec) {
  MMDX_CHECK_ARG(d && d->N > 0 && d->H > 0 && d->W > 0 && d->C > 0 && d->K > 0 && d->R > 0 &&
                     d->S > 0 && d->stride_h > 0 && d->stride_w > 0,
                 "conv: bad descriptor");
  MMDX_CHECK_ARG(d->P == (d->H + 2 * d->pad_h - d->R) / d->stride_h + 1 &&
                     d->Q == (d->W + 2 * d->pad_w - d->S) / d->stride_w + 1,
                 "conv: output size P=%d Q=%d inconsistent with input", d->P, d->Q);
  MMDX_CHECK_ARG(d->C % vec == 0 && d->K % vec == 0,
                 "conv: channels C=%d K=%d must be multiples of %d", d->C, d->K, vec);
  return 0;
}

template <typename T>
__global__ void pack_weight_kernel(const float* __restrict__ w, int K, int Cm, int C, int RS,
                                   T* __restrict__ krsc, T* __restrict__ crsk) {
  const long total = (long)K * RS * C;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total;
       i += (long)gridDim.x * blockDim.x) {
    // i indexes KRSC order
    const int c = (int)(i % C);
    const long t = i / C;
    const int rs = (int)(t % RS);
    const int k = (int)(t / RS);
    const float v = c < Cm ? w[((long)k * Cm + c) * RS + rs] : 0.f;
    if (krsc) krsc[i] = from_f<T>(v);
    if (crsk) crsk[((long)c * RS + rs) * K + k] = from_f<T>(v);
  }
}

// All conv weights of a trunk in ONE launch (mmdx_conv_pack_multi).  The master weight is a
// matrix Wm[K][C*RS] (col j = c*RS + rs); CRSK is exactly Wm^T and KRSC permutes each row
// (c, rs) -> (rs, c).  A block moves one 64 x 64 tile of Wm through LDS: coalesced fp32
// reads along j, coalesced bf16 writes along j (KRSC, per-row permutation) and along k (CRSK,
// transposed).  Block b belongs to the item whose [first_block, next first_block) holds it;
// 32-bit index math (every weight < 2^31 elements).  Channel-padded weights (C > c_master)
// keep mmdx_conv_pack_weight.
constexpr int PACK_T = 64;

template <typename T>
__global__ __launch_bounds__(256) void pack_multi_kernel(const mmdx_pack_item* __restrict__ it,
                                                         int n) {
  __shared__ float tile[PACK_T][PACK_T + 1];
  const long b = blockIdx.x;
  int lo = 0, hi = n - 1;  // last item with first_block <= b
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (it[mid].first_block <= b) lo = mid; else hi = mid - 1;
  }
  const mmdx_pack_item t = it[lo];
  const int K = t.K, RS = t.RS, J = t.C * RS;
  const int tj = (J + PACK_T - 1) / PACK_T;
  const int local = (int)(b - t.first_block);
  const int k0 = (local / tj) * PACK_T, j0 = (local % tj) * PACK_T;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;  // 64 x 4
  for (int r = ty; r < PACK_T; r += 4) {
    const int k = k0 + r, j = j0 + tx;
    tile[r][tx] = k < K && j < J ? t.w[(long)k * J + j] : 0.f;
  }
  __syncthreads();
  if (t.krsc) {  // row k: element j = c*RS + rs -> (rs*C + c)
    T* krsc = (T*)t.krsc;
    for (int r = ty; r < PACK_T; r += 4) {
      const int k = k0 + r, j = j0 + tx;
      if (k < K && j < J) {
        const int c = j / RS, rs = j - c * RS;
        krsc[(long)k * J + rs * t.C + c] = from_f<T>(tile[r][tx]);
      }
    }
  }
  if (t.crsk) {  // CRSK[j][k] = Wm[k][j]
    T* crsk = (T*)t.crsk;
    for (int r = ty; r < PACK_T; r += 4) {
      const int j = j0 + r, k = k0 + tx;
      if (j < J && k < K) crsk[(long)j * K + k] = from_f<T>(tile[tx][r]);
    }
  }
}

// partial[z][k][(r*S+s)*C + c] summed over z -> dw[k][c][r][s] (c < Cm), dw = beta*dw + sum
__global__ void wgrad_reduce_kernel(const float* __restrict__ ws, int splits, int K, int C,
                                    int Cm, int RS, float* __restrict__ dw, float beta) {
  // iterate in the slab's KRSC order (coalesced reads of every split), scatter to KCRS
  const long slab = (long)K * RS * C;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < slab;
       i += (long)gridDim.x * blockDim.x) {
    // 32-bit decode (slab < 2^31, checked by the launcher): 64-bit division is slow
    const unsigned ui = (unsigned)i;
    const int c = (int)(ui % (unsigned)C);
    if (c >= Cm) continue;
    const unsigned t = ui / (unsigned)C;
    const int rs = (int)(t % (unsigned)RS);
    const int k = (int)(t / (unsigned)RS);
    // 8 independent partial sums keep 8 slab loads in flight (fixed order: deterministic)
    float a[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    int z = 0;
    for (; z + 8 <= splits; z += 8) {
#pragma unroll
      for (int j = 0; j < 8; ++j) a[j] += ws[(long)(z + j) * slab + i];
    }
    for (int j = 0; z < splits; ++z, ++j) a[j] += ws[(long)z * slab + i];
    const float v = ((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7]));
    const long o = ((long)k * Cm + c) * RS + rs;
    dw[o] = beta != 0.f ? beta * dw[o] + v : v;
  }
}

// The same reduction with the splits themselves spread over Z thread groups of the block
// (Z = 1..16 by split count): a thread sums only ~splits/Z float4 partials with four
// independent accumulators, the Z group sums meet in LDS in a fixed order (deterministic).
// The one-thread-per-element loop above is latency-bound at high split counts (the layer1/2
// weight gradients split 50-256 ways: 20-54 us per launch at 0.5 TB/s).  slab % 4 == 0.
template <int Z>
__global__ __launch_bounds__(256) void wgrad_reduce_z_kernel(const float* __restrict__ ws,
                                                             int splits, int K, int C, int Cm,
                                                             int RS, float* __restrict__ dw,
                                                             float beta) {
  constexpr int E = 256 / Z;  // float4 columns per block
  __shared__ f32x4 red[256];
  const long n4 = (long)K * RS * C / 4;
  const int e = threadIdx.x % E, zg = threadIdx.x / E;
  const int per = (splits + Z - 1) / Z;
  const int z0 = min(splits, zg * per), z1 = min(splits, z0 + per);
  const f32x4* w4 = (const f32x4*)ws;
  for (long base = (long)blockIdx.x * E; base < n4; base += (long)gridDim.x * E) {
    const long i4 = base + e;
    f32x4 a0 = {0.f, 0.f, 0.f, 0.f}, a1 = a0, a2 = a0, a3 = a0;
    if (i4 < n4) {
      int z = z0;
      for (; z + 4 <= z1; z += 4) {
        a0 += w4[(long)z * n4 + i4];
        a1 += w4[(long)(z + 1) * n4 + i4];
        a2 += w4[(long)(z + 2) * n4 + i4];
        a3 += w4[(long)(z + 3) * n4 + i4];
      }
      for (; z < z1; ++z) a0 += w4[(long)z * n4 + i4];
    }
    red[threadIdx.x] = (a0 + a1) + (a2 + a3);
    __syncthreads();
    if (zg == 0 && i4 < n4) {
      f32x4 v = red[e];
#pragma unroll
      for (int q = 1; q < Z; ++q) v += red[q * E + e];
      const unsigned i = (unsigned)(i4 * 4);  // 32-bit decode (slab < 2^31)
      const int c = (int)(i % (unsigned)C);
      const unsigned t = i / (unsigned)C;
      const int rs = (int)(t % (unsigned)RS), k = (int)(t / (unsigned)RS);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (c + j >= Cm) break;
        const long o = ((long)k * Cm + c + j) * RS + rs;
        dw[o] = beta != 0.f ? beta * dw[o] + v[j] : v[j];
      }
    }
    __syncthreads();
  }
}

static void wgrad_reduce(const float* ws, int splits, int K, int C, int Cm, int RS, float* dw,
                         float beta, hipStream_t st) {
  const long total = (long)K * C * RS;  // < 2^31: checked by the wgrad entry point
  // split groups only for the deep splits (>= 128: the stem's and layer1's weight gradients,
  // at the end of the backward where little else runs); elsewhere the per-element loop, whose
  // lower memory-level parallelism disturbs the concurrent dgrad/BN chain less (all-split:
  // 0.6 % slower train step despite 2 % less isolated wgrad time).
  const bool per_element = splits < 128;
  if (total % 4 != 0 || per_element) {
    const int blocks = (int)std::min<long>((total + 255) / 256, 8192);
    hipLaunchKernelGGL(wgrad_reduce_kernel, dim3(blocks), dim3(256), 0, st, ws, splits, K, C,
                       Cm, RS, dw, beta);
    return;
  }
  const int Z = splits < 4 ? 1 : splits < 8 ? 2 : splits < 16 ? 4 : splits < 32 ? 8 : 16;
  const long cols = total / 4;
  const int blocks = (int)std::min<long>((cols + 256 / Z - 1) / (256 / Z), 8192);
#define MMDX_WRZ(z)                                                                          \
  hipLaunchKernelGGL(wgrad_reduce_z_kernel<z>, dim3(blocks), dim3(256), 0, st, ws, splits, K, \
                     C, Cm, RS, dw, beta)
  switch (Z) {
    case 1: MMDX_WRZ(1); break;
    case 2: MMDX_WRZ(2); break;
    case 4: MMDX_WRZ(4); break;
    case 8: MMDX_WRZ(8); break;
    default: MMDX_WRZ(16); break;
  }
#undef MMDX_WRZ
}

template <typename T, int BM, int BN, class LA, class LB, class Epi>
static int launch(const typename LA::SrcT& sa, const typename LB::SrcT& sb, const Epi& epi,
                  int M, int N, int K, int splits, int kper, hipStream_t st) {
  const int nwg = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  hipLaunchKernelGGL((igemm_kernel<T, BM, BN, 2, 2, LA, LB, Epi>), dim3(nwg, 1, splits),
                     dim3(NT), 0, st, sa, sb, epi, M, N, K, kper);
  MMDX_LAUNCH_CHECK();
  return 0;
}

// Three operand stages when the grid gives at most one block per CU anyway (the third
// stage costs occupancy only where there would be a second block to lose) and the K loop
// is long enough to keep two tiles in flight.
static bool use_three_stages(long blocks, int ktiles_per_block) {
  // grid limit measured in the C4 step: 0 and 256 tie, 512 is 3.5 % slower
  return blocks <= 256 && ktiles_per_block >= 4;
}

template <int BM, int BN, class OA, class OB, class Epi, int NS>
static void launch_dma_ns(const typename OA::SrcT& sa, const typename OB::SrcT& sb,
                          const Epi& epi, int M, int N, int K, int splits, int kper, int nwg,
                          hipStream_t st) {
  hipLaunchKernelGGL((igemm_dma_kernel<BM, BN, OA, OB, Epi, NS>), dim3(nwg, 1, splits),
                     dim3(NT), 0, st, sa, sb, epi, M, N, K, kper);
}

template <int BM, int BN, class OA, class OB, class Epi>
static int launch_dma_ops(const typename OA::SrcT& sa, const typename OB::SrcT& sb,
                          const Epi& epi, int M, int N, int K, int splits, int kper,
                          hipStream_t st) {
  const int nwg = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  if (use_three_stages((long)nwg * splits, (kper + 63) / 64)) {
    launch_dma_ns<BM, BN, OA, OB, Epi, 3>(sa, sb, epi, M, N, K, splits, kper, nwg, st);
  } else {
    launch_dma_ns<BM, BN, OA, OB, Epi, 2>(sa, sb, epi, M, N, K, splits, kper, nwg, st);
  }
  MMDX_LAUNCH_CHECK();
  return 0;
}

// both operands k-major
template <int BM, int BN, class SA, class SB, class Epi>
static int launch_dma(const SA& sa, const SB& sb, const Epi& epi, int M, int N, int K,
                      int splits, int kper, hipStream_t st) {
  return launch_dma_ops<BM, BN, DmaK<BM, SA>, DmaK<BN, SB>>(sa, sb, epi, M, N, K, splits, kper,
                                                            st);
}

// bf16 gathers whose K tiles are whole filter taps (C % 64 == 0) take the LDS-DMA kernel
template <class S> struct DmaOk { static constexpr bool value = false; };
template <> struct DmaOk<Im2colK<bf16, true>> { static constexpr bool value = true; };
template <> struct DmaOk<DgradK<bf16, true>> { static constexpr bool value = true; };
template <> struct DmaOk<Im2colK<bf16, false>> { static constexpr bool value = true; };
template <> struct DmaOk<DenseK<bf16>> { static constexpr bool value = true; };
template <> struct DmaOk<PointFwdK<bf16>> { static constexpr bool value = true; };
template <> struct DmaOk<PointDgradK<bf16>> { static constexpr bool value = true; };

// buffer-DMA preconditions: 32-bit byte offsets (< 2 GiB) and a 32-bit tap-validity mask
static bool dma_geom_ok(const ConvGeom& g, bool dgrad, int max_taps = 32, long rows = 0) {
  const long xb = (long)g.N * g.H * g.W * g.C * 2, yb = (long)g.N * g.P * g.Q * g.K * 2;
  if (xb >= (1L << 31) || yb >= (1L << 31) || g.R * g.S > max_taps) return false;
  // the k-major gathers decode their rows by float reciprocal (fdivu): rows < 2^22
  if (rows >= (1L << 22) - 256) return false;
  return !dgrad || (g.sh == 1 && g.sw == 1);
}

// 1x1, stride 1, no padding: the implicit GEMM's gathers are plain dense matrices over NHWC
static bool is_pointwise(const ConvGeom& g) {
  return g.R == 1 && g.S == 1 && g.sh == 1 && g.sw == 1 && g.ph == 0 && g.pw == 0;
}

// 128x64 tiles when 128x128 would give fewer tiles than this (< 1.5 per CU); measured in the
// C4 step: 256 and 384 tie, 640 is 1.5 % slower
constexpr long kNarrowBelow = 384;

// 8-wave 256 x 128 tiles (one 512-thread block per CU, three 48 KB operand stages): for the
// k-major conv GEMMs with N >= 128 and at least this many tiles (MMDX_CONV8_MIN; 0 = off).
// Off by default: at threshold 160 the isolated C4 forward convs took 2.51 vs 2.41 ms and the
// dgrads 2.22 vs 2.11 ms, the train step 9001 / 8999 vs 9089 / 9059 samples/s (paired in one
// call, profiles/r03_conv8_ab.txt) — one block per CU leaves no second block to cover a
// block's barrier waits and epilogue
static long conv8_min_tiles() {
  const char* e = getenv("MMDX_CONV8_MIN");  // read per launch: tests / A-B runs switch it
  return e ? atol(e) : 0L;
}

template <class SA, class SB, class Epi>
static bool try_conv8(const SA& sa, const SB& sb, const Epi& epi, int M, int N, int K,
                      hipStream_t st) {
  const long tiles = (long)((M + 255) / 256) * ((N + 127) / 128);
  const long lim = conv8_min_tiles();
  if (lim <= 0 || N < 128 || tiles < lim || K < 128) return false;
  hipLaunchKernelGGL((igemm_dma_kernel<256, 128, DmaK<256, SA, 64, 8>, DmaK<128, SB, 64, 8>, Epi,
                                       3, bf16, 512, 4, 2>),
                     dim3((unsigned)tiles, 1, 1), dim3(512), 0, st, sa, sb, epi, M, N, K, K);
  return true;
}

template <typename T, class SA, class Epi>
static int conv_gemm_epi(const SA& sa, const void* w, const Epi& epi, int M, int N, int K,
                         hipStream_t st, bool dma_ok) {
  DenseK<T> sb{(const T*)w, K, N, true};
  if constexpr (DmaOk<SA>::value) {
    if (dma_ok) {
      if (try_conv8(sa, sb, epi, M, N, K, st)) {
        MMDX_LAUNCH_CHECK();
        return 0;
      }
      // 128x64 tiles when N is narrow or 128x128 tiles would leave CUs idle (< 1.5 per CU)
      const long tiles128 = (long)((M + 127) / 128) * ((N + 127) / 128);
      if (N <= 64 || tiles128 < kNarrowBelow)
        return launch_dma<128, 64>(sa, sb, epi, M, N, K, 1, K, st);
      return launch_dma<128, 128>(sa, sb, epi, M, N, K, 1, K, st);
    }
  }
  if (N <= 64)
    return launch<T, 128, 64, KLoad<T, 128, SA>, KLoad<T, 64, DenseK<T>>>(sa, sb, epi, M, N, K,
                                                                            1, K, st);
  return launch<T, 128, 128, KLoad<T, 128, SA>, KLoad<T, 128, DenseK<T>>>(sa, sb, epi, M, N, K,
                                                                            1, K, st);
}

template <typename T, class SA>
static int conv_gemm(const SA& sa, const void* w, void* out, int M, int N, int K, float beta,
                     hipStream_t st, float* stats = nullptr, bool dma_ok = false,
                     const BnStat& bs = BnStat{}, const void* acc_src = nullptr,
                     const uint8_t* acc_mask = nullptr) {
  EpiStore<T> epi{(T*)out, N, M, N, nullptr, nullptr, ACT_NONE, 1.f, beta, nullptr,
                  (float2*)stats};
  epi.bs = bs;  // only the LDS-DMA kernel's epilogue honours it (see dgrad_bnstat_ok)
  epi.acc_src = (const T*)acc_src;
  epi.acc_mask = acc_mask;
  return conv_gemm_epi<T>(sa, w, epi, M, N, K, st, dma_ok);
}

template <typename T>
static int conv_fwd_t(const mmdx_conv_desc* d, const void* x, const void* w, void* y,
                      float* stats, hipStream_t st) {
  const ConvGeom g = geom(d);
  const int M = g.N * g.P * g.Q, N = g.K, K = g.R * g.S * g.C;
  if (g.C % KTile<T>::BK == 0 && is_pointwise(g))  // x itself is the [M][C] A operand
    return conv_gemm<T>(PointFwdK<T>{{(const T*)x, g.C, M, true}}, w, y, M, N, K, 0.f, st,
                        stats, dma_geom_ok(g, false, 32, M));
  if (g.C % KTile<T>::BK == 0)
    return conv_gemm<T>(Im2colK<T, true>{(const T*)x, g, M}, w, y, M, N, K, 0.f, st, stats,
                        dma_geom_ok(g, false, 32, M));
  // channel count a power of two: the LDS-DMA kernel decodes each lane's tap itself
  const bool pow2 = g.C >= 8 && (g.C & (g.C - 1)) == 0 && g.R * g.S <= 64;
  Im2colK<T, false> sa{(const T*)x, g, M, pow2 ? __builtin_ctz(g.C) : 0, 1.f / (float)g.S};
  return conv_gemm<T>(sa, w, y, M, N, K, 0.f, st, stats, pow2 && dma_geom_ok(g, false, 64, M));
}

template <typename T>
static int conv_fwd_bn_eval_t(const mmdx_conv_desc* d, const void* x, const void* w, void* y,
                              const float* gamma, const float* beta, const float* rmean,
                              const float* rvar, float eps, const void* res, int relu,
                              hipStream_t st) {
  const ConvGeom g = geom(d);
  const int M = g.N * g.P * g.Q, N = g.K, K = g.R * g.S * g.C;
  EpiBnEval<T> epi;
  static_cast<EpiStore<T>&>(epi) =
      EpiStore<T>{(T*)y, N, M, N, nullptr, nullptr, ACT_NONE, 1.f, 0.f, nullptr, nullptr};
  epi.gamma = gamma; epi.beta_bn = beta; epi.rmean = rmean; epi.rvar = rvar; epi.eps = eps;
  epi.res = (const T*)res; epi.relu = relu != 0;
  if (g.C % KTile<T>::BK == 0 && is_pointwise(g))
    return conv_gemm_epi<T>(PointFwdK<T>{{(const T*)x, g.C, M, true}}, w, epi, M, N, K, st,
                            dma_geom_ok(g, false, 32, M));
  if (g.C % KTile<T>::BK == 0)
    return conv_gemm_epi<T>(Im2colK<T, true>{(const T*)x, g, M}, w, epi, M, N, K, st,
                            dma_geom_ok(g, false, 32, M));
  const bool pow2 = g.C >= 8 && (g.C & (g.C - 1)) == 0 && g.R * g.S <= 64;
  Im2colK<T, false> sa{(const T*)x, g, M, pow2 ? __builtin_ctz(g.C) : 0, 1.f / (float)g.S};
  return conv_gemm_epi<T>(sa, w, epi, M, N, K, st, pow2 && dma_geom_ok(g, false, 64, M));
}

// Strided dgrad as sh*sw phase GEMMs (see DgradPhaseK); phases no tap reaches are written
// as zeros (beta = 0) or left untouched (beta != 0).
template <typename T>
static int conv_dgrad_phases(const ConvGeom& g, const void* dy, const void* w_crsk, void* dx,
                             float beta, hipStream_t st, BnStat bs = BnStat{}) {
  for (int a = 0; a < g.sh; ++a) {
    for (int b = 0; b < g.sw; ++b) {
      PhaseGeom ph;
      ph.Hp = g.H > a ? (g.H - a + g.sh - 1) / g.sh : 0;
      ph.Wp = g.W > b ? (g.W - b + g.sw - 1) / g.sw : 0;
      if (ph.Hp == 0 || ph.Wp == 0) continue;
      ph.r0 = (a + g.ph) % g.sh;
      ph.s0 = (b + g.pw) % g.sw;
      ph.ntr = ph.r0 < g.R ? (g.R - 1 - ph.r0) / g.sh + 1 : 0;
      ph.nts = ph.s0 < g.S ? (g.S - 1 - ph.s0) / g.sw + 1 : 0;
      ph.dr0 = (a + g.ph - ph.r0) / g.sh;
      ph.ds0 = (b + g.pw - ph.s0) / g.sw;
      const int K = ph.ntr * ph.nts * g.K;
      if (K == 0 && beta != 0.f) continue;
      const int M = g.N * ph.Hp * ph.Wp, N = g.C;
      DgradPhaseK<T> sa{(const T*)dy, g, ph, M};
      PhaseTapK<T> sb{(const T*)w_crsk, (long)g.R * g.S * g.K, g.C, g.K, g.S, g.sh, g.sw, ph};
      EpiPhase<T> epi{(T*)dx, g.C, M, N, beta, ph.Hp, ph.Wp, g.H, g.W, a, b, g.sh, g.sw};
      epi.bs = bs;
      bs.tile0 += (M + 127) / 128;  // the next phase's tiles follow this phase's
      int rc = -1;
      if constexpr (sizeof(T) == 2) {
        if (dma_geom_ok(g, false, 32, M)) {
          const long tiles128 = (long)((M + 127) / 128) * ((N + 127) / 128);
          if (try_conv8(sa, sb, epi, M, N, K, st)) {
            MMDX_LAUNCH_CHECK();
            continue;
          }
          if (N <= 64 || tiles128 < kNarrowBelow)
            rc = launch_dma<128, 64>(sa, sb, epi, M, N, K, 1, K, st);
          else
            rc = launch_dma<128, 128>(sa, sb, epi, M, N, K, 1, K, st);
          if (rc) return rc;
          continue;
        }
      }
      if (N <= 64) {
        rc = launch<T, 128, 64, KLoad<T, 128, DgradPhaseK<T>>, KLoad<T, 64, PhaseTapK<T>>>(
            sa, sb, epi, M, N, K, 1, K, st);
      } else {
        rc = launch<T, 128, 128, KLoad<T, 128, DgradPhaseK<T>>, KLoad<T, 128, PhaseTapK<T>>>(
            sa, sb, epi, M, N, K, 1, K, st);
      }
      if (rc) return rc;
    }
  }
  return 0;
}

template <typename T>
static int conv_dgrad_t(const mmdx_conv_desc* d, const void* dy, const void* w_crsk, void* dx,
                        float beta, hipStream_t st, const BnStat& bs = BnStat{},
                        const void* acc_src = nullptr, const uint8_t* acc_mask = nullptr) {
  const ConvGeom g = geom(d);
  if ((g.sh > 1 || g.sw > 1) && g.K % KTile<T>::BK == 0)
    return conv_dgrad_phases<T>(g, dy, w_crsk, dx, beta, st, bs);
  const int M = g.N * g.H * g.W, N = g.C, K = g.R * g.S * g.K;
  if (g.K % KTile<T>::BK == 0 && is_pointwise(g))  // dY itself is the [M][K] A operand
    return conv_gemm<T>(PointDgradK<T>{{(const T*)dy, g.K, M, true}}, w_crsk, dx, M, N, K,
                        beta, st, nullptr, dma_geom_ok(g, true, 32, M), bs, acc_src, acc_mask);
  if (g.K % KTile<T>::BK == 0)
    return conv_gemm<T>(DgradK<T, true>{(const T*)dy, g, M}, w_crsk, dx, M, N, K, beta, st,
                        nullptr, dma_geom_ok(g, true, 32, M), bs, acc_src, acc_mask);
  return conv_gemm<T>(DgradK<T, false>{(const T*)dy, g, M}, w_crsk, dx, M, N, K, beta, st,
                      nullptr, false, BnStat{}, acc_src, acc_mask);
}

struct WgradPlan { int bm, bn, splits, kper; };
// 8-wave 256 x 128 weight-gradient tiles (one block per CU, three stages) for Kout >= 256
// and C*R*S >= 128 (MMDX_WGRAD8=0: off); their splits target one block per CU
// 8-wave 256 x 128 weight-gradient tiles (MMDX_WGRAD8=1; off by default: isolated C4 wgrads
// 2.78 vs 2.51 ms, train step 8967 vs 9050 samples/s, profiles/r03_wgrad8_ab.txt)
static bool wgrad8_on() {
  const char* e = getenv("MMDX_WGRAD8");
  return e && atoi(e) != 0;
}

static WgradPlan plan_wgrad(int dtype, const mmdx_conv_desc* d) {
  WgradPlan p;
  const int BK = dtype == BF16 ? KTile<bf16>::BK : KTile<float>::BK;
  const int M = d->K, N = d->R * d->S * d->C;
  const long K = (long)d->N * d->P * d->Q;
  if (dtype == BF16 && M >= 256 && N >= 128 && wgrad8_on()) {
    p.bm = 256;
    p.bn = 128;
    const long tiles = (long)((M + 255) / 256) * ((N + 127) / 128);
    const long ktiles = (K + BK - 1) / BK;
    long s = (256L + tiles - 1) / tiles;
    s = std::max(1L, std::min(s, ktiles / 16L));
    const long kt_per = (ktiles + s - 1) / s;
    p.kper = (int)(kt_per * BK);
    p.splits = (int)((K + p.kper - 1) / p.kper);
    return p;
  }
  p.bm = M <= 64 ? 64 : 128;
  p.bn = N <= 64 ? 64 : 128;
  const long tiles = (long)((M + p.bm - 1) / p.bm) * ((N + p.bn - 1) / p.bn);
  const long ktiles = (K + BK - 1) / BK;
  // ~2 blocks per CU, each split at least 16 K tiles deep (keeps the partial slabs small).
  // Measured: 256 / 384 / 768 / 1024-block targets lose to 512 in the C4 step; ~4 per CU for
  // the 3x3 convs of layer3/4 ran 4-12 % faster in isolation but 0.2 % slower in the train
  // step (more blocks contending with the dgrad chain); 8 / 16 / 32 least K tiles tie.
  const long target = 512L;
  const long min_kt = 16L;
  long s = (target + tiles - 1) / tiles;
  s = std::max(1L, std::min(s, ktiles / min_kt));
  const long kt_per = (ktiles + s - 1) / s;
  p.kper = (int)(kt_per * BK);
  p.splits = (int)((K + p.kper - 1) / p.kper);
  return p;
}

template <typename T, class SB>
static int wgrad_dma(const WgradPlan& p, const DenseR<T>& sa, const SB& sb, const EpiPartial& epi,
                     int M, int N, int K, hipStream_t st) {
  if (p.bm == 256) {
    const int nwg = ((M + 255) / 256) * ((N + 127) / 128);
    hipLaunchKernelGGL((igemm_dma_kernel<256, 128, DmaR<256, DenseR<T>, 64, 8>, DmaR<128, SB, 64, 8>,
                                         EpiPartial, 3, bf16, 512, 4, 2>),
                       dim3(nwg, 1, p.splits), dim3(512), 0, st, sa, sb, epi, M, N, K, p.kper);
    MMDX_LAUNCH_CHECK();
    return 0;
  }
  if (p.bm == 128 && p.bn == 128)
    return launch_dma_ops<128, 128, DmaR<128, DenseR<T>>, DmaR<128, SB>>(sa, sb, epi, M, N, K,
                                                                        p.splits, p.kper, st);
  if (p.bm == 128)
    return launch_dma_ops<128, 64, DmaR<128, DenseR<T>>, DmaR<64, SB>>(sa, sb, epi, M, N, K,
                                                                      p.splits, p.kper, st);
  if (p.bn == 128)
    return launch_dma_ops<64, 128, DmaR<64, DenseR<T>>, DmaR<128, SB>>(sa, sb, epi, M, N, K,
                                                                      p.splits, p.kper, st);
  return launch_dma_ops<64, 64, DmaR<64, DenseR<T>>, DmaR<64, SB>>(sa, sb, epi, M, N, K,
                                                                  p.splits, p.kper, st);
}

template <typename T>
static int conv_wgrad_t(const mmdx_conv_desc* d, int cm, const void* x, const void* dy,
                        float* dw, float beta, void* ws, size_t ws_bytes, hipStream_t st) {
  const ConvGeom g = geom(d);
  const WgradPlan p = plan_wgrad(sizeof(T) == 2 ? BF16 : F32, d);
  const int M = g.K, N = g.R * g.S * g.C;
  const long Kl = (long)g.N * g.P * g.Q;
  MMDX_CHECK_ARG(Kl < (1L << 31), "conv wgrad: N*P*Q too large");
  MMDX_CHECK_ARG((long)M * N < (1L << 31), "conv wgrad: K*C*R*S too large");
  const int K = (int)Kl;
  const size_t need = (size_t)p.splits * M * N * sizeof(float);
  MMDX_CHECK_ARG(ws && ws_bytes >= need, "conv wgrad: workspace %zu < %zu", ws_bytes, need);
  DenseR<T> sa{(const T*)dy, g.K, M, true, K};
  const Im2colR<T> sb = make_im2colr<T>((const T*)x, g, N);  // one 64-pixel K tile per issue
  EpiPartial epi{(float*)ws, M, N};
  int rc;
  if constexpr (sizeof(T) == 2) {
   if (dma_geom_ok(g, false, 1 << 30) && K < (1 << 23)) {
    // LDS-DMA wgrad: both operands R-major (M = Kout and N = R*S*C are multiples of 8).  A
    // 1x1 / stride-1 / unpadded conv's im2col^T is x^T itself: a dense R-major operand
    // (no window decode or tap tests)
    if (is_pointwise(g))
      rc = wgrad_dma<T>(p, sa, PointWgradR<T>{{(const T*)x, g.C, N, true, K}}, epi, M, N, K,
                        st);
    else
      rc = wgrad_dma<T>(p, sa, sb, epi, M, N, K, st);
    if (rc) return rc;
    wgrad_reduce((const float*)ws, p.splits, g.K, g.C, cm, g.R * g.S, dw, beta, st);
    MMDX_LAUNCH_CHECK();
    return 0;
   }
  }
  typedef RLoad<T, 128, DenseR<T>> A128;
  typedef RLoad<T, 64, DenseR<T>> A64;
  typedef RLoad<T, 128, Im2colR<T>> B128;
  typedef RLoad<T, 64, Im2colR<T>> B64;
  if (p.bm == 128 && p.bn == 128)
    rc = launch<T, 128, 128, A128, B128>(sa, sb, epi, M, N, K, p.splits, p.kper, st);
  else if (p.bm == 128)
    rc = launch<T, 128, 64, A128, B64>(sa, sb, epi, M, N, K, p.splits, p.kper, st);
  else if (p.bn == 128)
    rc = launch<T, 64, 128, A64, B128>(sa, sb, epi, M, N, K, p.splits, p.kper, st);
  else
    rc = launch<T, 64, 64, A64, B64>(sa, sb, epi, M, N, K, p.splits, p.kper, st);
  if (rc) return rc;
  wgrad_reduce((const float*)ws, p.splits, g.K, g.C, cm, g.R * g.S, dw, beta, st);
  MMDX_LAUNCH_CHECK();
  return 0;
}

}  // namespace mmdx

using namespace mmdx;

extern "C" int mmdx_conv_pack_weight(int dtype, const mmdx_conv_desc* d, int c_master,
                                     const float* w, void* krsc, void* crsk, void* stream) {
  MMDX_CHECK_ARG(dtype != F16, "mmdx_conv_pack_weight: fp16 is the C5 path only");
  MMDX_CHECK_ARG(d && c_master > 0 && c_master <= d->C, "conv pack: bad channels");
  const long total = (long)d->K * d->R * d->S * d->C;
  const int blocks = (int)std::min<long>((total + 255) / 256, 4096);
  hipStream_t st = (hipStream_t)stream;
  if (dtype == BF16)
    hipLaunchKernelGGL(pack_weight_kernel<bf16>, dim3(blocks), dim3(256), 0, st, w, d->K,
                       c_master, d->C, d->R * d->S, (bf16*)krsc, (bf16*)crsk);
  else
    hipLaunchKernelGGL(pack_weight_kernel<float>, dim3(blocks), dim3(256), 0, st, w, d->K,
                       c_master, d->C, d->R * d->S, (float*)krsc, (float*)crsk);
  MMDX_LAUNCH_CHECK();
  return 0;
}

extern "C" long mmdx_conv_pack_blocks(int K, int C, int RS) {
  return (long)((K + PACK_T - 1) / PACK_T) * ((C * RS + PACK_T - 1) / PACK_T);
}

extern "C" int mmdx_conv_pack_multi(int dtype, const mmdx_pack_item* items, int n_items,
                                    long total_blocks, void* stream) {
  MMDX_CHECK_ARG(dtype != F16, "mmdx_conv_pack_multi: fp16 is the C5 path only");
  MMDX_CHECK_ARG(items && n_items > 0 && total_blocks > 0 && total_blocks < (1L << 31),
                 "conv pack multi: bad item table");
  hipStream_t st = (hipStream_t)stream;
  if (dtype == BF16)
    hipLaunchKernelGGL(pack_multi_kernel<bf16>, dim3((unsigned)total_blocks), dim3(256), 0, st,
                       items, n_items);
  else
    hipLaunchKernelGGL(pack_multi_kernel<float>, dim3((unsigned)total_blocks), dim3(256), 0, st,
                       items, n_items);
  MMDX_LAUNCH_CHECK();
  return 0;
}

extern "C" int mmdx_conv_fwd_stat_blocks(const mmdx_conv_desc* d) {
  return (int)(((long)d->N * d->P * d->Q + 127) / 128);
}

extern "C" int mmdx_conv_fwd(int dtype, const mmdx_conv_desc* d, const void* x,
                             const void* w, void* y, float* stat_part, void* stream) {
  MMDX_CHECK_ARG(dtype != F16, "mmdx_conv_fwd: fp16 is the C5 path only");
  int rc = check_desc(d, dtype == BF16 ? 8 : 4);
  if (rc) return rc;
  MMDX_CHECK_ARG((long)d->N * d->P * d->Q < (1L << 31), "conv fwd: too many pixels");
  if (dtype == BF16) return conv_fwd_t<bf16>(d, x, w, y, stat_part, (hipStream_t)stream);
  return conv_fwd_t<float>(d, x, w, y, stat_part, (hipStream_t)stream);
}

extern "C" int mmdx_conv_fwd_bn_eval(int dtype, const mmdx_conv_desc* d, const void* x,
                                     const void* w, void* y, const float* gamma,
                                     const float* beta, const float* running_mean,
                                     const float* running_var, float eps, const void* residual,
                                     int relu, void* stream) {
  MMDX_CHECK_ARG(dtype != F16, "mmdx_conv_fwd_bn_eval: fp16 is the C5 path only");
  int rc = check_desc(d, dtype == BF16 ? 8 : 4);
  if (rc) return rc;
  MMDX_CHECK_ARG(gamma && beta && running_mean && running_var, "conv fwd bn-eval: null BN");
  MMDX_CHECK_ARG((long)d->N * d->P * d->Q < (1L << 31), "conv fwd: too many pixels");
  if (dtype == BF16)
    return conv_fwd_bn_eval_t<bf16>(d, x, w, y, gamma, beta, running_mean, running_var, eps,
                                    residual, relu, (hipStream_t)stream);
  return conv_fwd_bn_eval_t<float>(d, x, w, y, gamma, beta, running_mean, running_var, eps,
                                   residual, relu, (hipStream_t)stream);
}

extern "C" int mmdx_conv_dgrad(int dtype, const mmdx_conv_desc* d, const void* dy,
                               const void* w_crsk, void* dx, float beta, void* stream) {
  MMDX_CHECK_ARG(dtype != F16, "mmdx_conv_dgrad: fp16 is the C5 path only");
  int rc = check_desc(d, dtype == BF16 ? 8 : 4);
  if (rc) return rc;
  if (dtype == BF16) return conv_dgrad_t<bf16>(d, dy, w_crsk, dx, beta, (hipStream_t)stream);
  return conv_dgrad_t<float>(d, dy, w_crsk, dx, beta, (hipStream_t)stream);
}

extern "C" int mmdx_conv_dgrad_accmask(int dtype, const mmdx_conv_desc* d, const void* dy,
                                       const void* w_crsk, void* dx, const void* acc_src,
                                       const uint8_t* acc_mask, void* stream) {
  MMDX_CHECK_ARG(dtype != F16, "mmdx_conv_dgrad_accmask: fp16 is the C5 path only");
  int rc = check_desc(d, dtype == BF16 ? 8 : 4);
  if (rc) return rc;
  MMDX_CHECK_ARG(acc_src && acc_mask && d->stride_h == 1 && d->stride_w == 1,
                 "conv dgrad accmask: needs a stride-1 conv and both accumulation operands");
  MMDX_CHECK_ARG(((uintptr_t)acc_src & 15) == 0 && ((uintptr_t)dx & 15) == 0,
                 "conv dgrad accmask: dx / acc_src must be 16-B aligned");
  hipStream_t st = (hipStream_t)stream;
  if (dtype == BF16)
    return conv_dgrad_t<bf16>(d, dy, w_crsk, dx, 0.f, st, BnStat{}, acc_src, acc_mask);
  return conv_dgrad_t<float>(d, dy, w_crsk, dx, 0.f, st, BnStat{}, acc_src, acc_mask);
}

extern "C" size_t mmdx_conv_wgrad_workspace_size(int dtype, const mmdx_conv_desc* d) {
  const WgradPlan p = plan_wgrad(dtype, d);
  return (size_t)p.splits * d->K * d->R * d->S * d->C * sizeof(float);
}

extern "C" int mmdx_conv_wgrad(int dtype, const mmdx_conv_desc* d, int c_master,
                               const void* x, const void* dy, float* dw, float beta,
                               void* ws, size_t ws_bytes, void* stream) {
  MMDX_CHECK_ARG(dtype != F16, "mmdx_conv_wgrad: fp16 is the C5 path only");
  int rc = check_desc(d, dtype == BF16 ? 8 : 4);
  if (rc) return rc;
  MMDX_CHECK_ARG(c_master > 0 && c_master <= d->C, "conv wgrad: bad c_master");
  if (dtype == BF16)
    return conv_wgrad_t<bf16>(d, c_master, x, dy, dw, beta, ws, ws_bytes, (hipStream_t)stream);
  return conv_wgrad_t<float>(d, c_master, x, dy, dw, beta, ws, ws_bytes, (hipStream_t)stream);
}

// Fused consumer-BN backward statistics are produced by the LDS-DMA dgrad kernels only
// (bf16, Kout % 64 == 0, 32-bit offsets; strided convs need every output phase reached).
// Returns the number of 128-row partial slots, or 0 when the fusion does not apply.
extern "C" int mmdx_conv_dgrad_stat_blocks(int dtype, const mmdx_conv_desc* d) {
  if (dtype != BF16 || !d || d->K % 64 != 0 || d->C % 8 != 0) return 0;
  const ConvGeom g = geom(d);
  if (g.sh == 1 && g.sw == 1) {
    if (!dma_geom_ok(g, true, 32, (long)g.N * g.H * g.W)) return 0;
    return (int)(((long)g.N * g.H * g.W + 127) / 128);
  }
  // every phase has at most N*H*W rows: this check passing implies each phase's launch passes
  if (!dma_geom_ok(g, false, 32, (long)g.N * g.H * g.W)) return 0;
  long tiles = 0;
  for (int a = 0; a < g.sh; ++a)
    for (int b = 0; b < g.sw; ++b) {
      const int Hp = g.H > a ? (g.H - a + g.sh - 1) / g.sh : 0;
      const int Wp = g.W > b ? (g.W - b + g.sw - 1) / g.sw : 0;
      const int r0 = (a + g.ph) % g.sh, s0 = (b + g.pw) % g.sw;
      if (Hp == 0 || Wp == 0) continue;
      if (r0 >= g.R || s0 >= g.S) return 0;  // an unreached phase: no fused statistics
      tiles += ((long)g.N * Hp * Wp + 127) / 128;
    }
  return (int)tiles;
}

extern "C" int mmdx_conv_dgrad_bnstat(int dtype, const mmdx_conv_desc* d, const void* dy,
                                      const void* w_crsk, void* dx, float beta,
                                      const void* bn_y, const void* bn_out, const float* gamma,
                                      const float* bn_beta, const float* save_mean,
                                      const float* save_rstd, int relu, float* stat_part,
                                      void* stream) {
  MMDX_CHECK_ARG(dtype != F16, "mmdx_conv_dgrad_bnstat: fp16 is the C5 path only");
  int rc = check_desc(d, 8);
  if (rc) return rc;
  const int tiles = mmdx_conv_dgrad_stat_blocks(dtype, d);
  MMDX_CHECK_ARG(tiles > 0, "conv dgrad bnstat: fused statistics unsupported for this conv");
  MMDX_CHECK_ARG(beta == 0.f || (d->stride_h == 1 && d->stride_w == 1),
                 "conv dgrad bnstat: accumulation (beta != 0) needs a stride-1 conv");
  MMDX_CHECK_ARG(bn_y && save_mean && save_rstd && stat_part, "conv dgrad bnstat: null operand");
  MMDX_CHECK_ARG(((uintptr_t)dx & 15) == 0 && ((uintptr_t)bn_y & 15) == 0 &&
                     ((uintptr_t)bn_out & 15) == 0,
                 "conv dgrad bnstat: dx / y / out must be 16-B aligned");
  BnStat bs{bn_y, gamma, bn_beta, save_mean, save_rstd, (float2*)stat_part, relu, tiles, 0,
            bn_out};
  return conv_dgrad_t<bf16>(d, dy, w_crsk, dx, beta, (hipStream_t)stream, bs);
}

// ------------------------------------------------------------------------------ stem
// ResNet stem (backbone.0, TP:183: conv 7x7 / stride 2 / pad 3, 3 -> 64 channels) as an
// ordinary NHWC conv over PIXEL PAIRS.  The image is written once, zero-bordered, as bf16
// [N][H+2p][(W+2p)/2][8]: a "pixel" of the pair image is two adjacent padded pixels x 4
// channels (c = 3 is zero), one 16-B chunk.  Output column q reads padded columns 2q+s,
// s < S, = pairs q+j, j < ceil(S/2), both parities: a stride (2, 1), unpadded R x ceil(S/2)
// conv with 8 channels, K = 7*4*8 = 224 (vs 7*7*8 = 392 for the channel-padded image), no
// border taps, on the same implicit-GEMM kernels (fwd + BN-stat epilogue, wgrad).  The
// weight maps to w'[k][r][j][e*4+c] = w[k][c][r][2j+e] (0 where 2j+e >= S or c >= C).
namespace mmdx {

__global__ void stem_pair_input_kernel(const float* __restrict__ x, int N, int C, int H, int W,
                                       int pad, int Hp, int W2, bf16* __restrict__ out) {
  const long total = (long)N * Hp * W2;
  GRID_STRIDE(i, total) {  // 32-bit decode (total < 2^31, checked by the entry point)
    const unsigned ui = (unsigned)i;
    const int j = (int)(ui % (unsigned)W2);
    const unsigned t = ui / (unsigned)W2;
    const int hp = (int)(t % (unsigned)Hp);
    const int n = (int)(t / (unsigned)Hp);
    const int ih = hp - pad;
    bf16x8 v;
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int iw = 2 * j + e - pad;
      const bool in = (unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W;
#pragma unroll
      for (int c = 0; c < 4; ++c)
        v[e * 4 + c] = (bf16)(in && c < C ? x[(((long)n * C + c) * H + ih) * W + iw] : 0.f);
    }
    *(bf16x8*)(out + i * 8) = v;
  }
}

__global__ void stem_pair_pack_kernel(const float* __restrict__ w, int K, int C, int R, int S,
                                      int S2, bf16* __restrict__ out) {
  const long total = (long)K * R * S2 * 8;
  GRID_STRIDE(i, total) {
    const int ce = (int)(i & 7), e = ce >> 2, c = ce & 3;
    const long t = i >> 3;
    const int j = (int)(t % S2);
    const long t2 = t / S2;
    const int r = (int)(t2 % R), k = (int)(t2 / R);
    const int s = 2 * j + e;
    out[i] = (bf16)(c < C && s < S ? w[(((long)k * C + c) * R + r) * S + s] : 0.f);
  }
}

// wgrad of the pair conv (fp32, its own KCRS: [K][8][R][S2]) -> master dw [K][C][R][S]
__global__ void stem_pair_grad_kernel(const float* __restrict__ dwp, int K, int C, int R, int S,
                                      int S2, float* __restrict__ dw, float beta) {
  const long total = (long)K * C * R * S;
  GRID_STRIDE(i, total) {
    const int s = (int)(i % S);
    const long t = i / S;
    const int r = (int)(t % R);
    const long t2 = t / R;
    const int c = (int)(t2 % C), k = (int)(t2 / C);
    const float v = dwp[(((long)k * 8 + (s & 1) * 4 + c) * R + r) * S2 + (s >> 1)];
    dw[i] = beta != 0.f ? beta * dw[i] + v : v;
  }
}

}  // namespace mmdx

extern "C" int mmdx_stem_pair_desc(int N, int C, int H, int W, int K, int R, int S, int stride,
                                   int pad, mmdx_conv_desc* out) {
  MMDX_CHECK_ARG(out && N > 0 && C > 0 && C <= 4 && H > 0 && W > 0 && K > 0 && R > 0 && S > 0 &&
                     pad >= 0 && stride == 2 && (W + 2 * pad) % 2 == 0 &&
                     H + 2 * pad >= R && W + 2 * pad >= S,
                 "stem pair: needs stride 2, C <= 4, even padded width");
  const int Hp = H + 2 * pad, W2 = (W + 2 * pad) / 2, S2 = (S + 1) / 2;
  mmdx_conv_desc d;
  d.N = N; d.H = Hp; d.W = W2; d.C = 8; d.K = K; d.R = R; d.S = S2;
  d.stride_h = stride; d.stride_w = 1; d.pad_h = 0; d.pad_w = 0;
  d.P = (Hp - R) / stride + 1;
  d.Q = W2 - S2 + 1;
  MMDX_CHECK_ARG(d.Q == (W + 2 * pad - S) / stride + 1, "stem pair: output width mismatch");
  *out = d;
  return 0;
}

extern "C" int mmdx_stem_pair_input(const float* x_nchw, int N, int C, int H, int W, int pad,
                                    void* out, void* stream) {
  MMDX_CHECK_ARG(x_nchw && out && C > 0 && C <= 4 && (W + 2 * pad) % 2 == 0,
                 "stem pair input: bad args");
  const int Hp = H + 2 * pad, W2 = (W + 2 * pad) / 2;
  const long total = (long)N * Hp * W2;
  MMDX_CHECK_ARG(total < (1L << 31), "stem pair input: more than 2^31 pixel pairs");
  hipLaunchKernelGGL(stem_pair_input_kernel, dim3(grid_for(total)), dim3(256), 0,
                     (hipStream_t)stream, x_nchw, N, C, H, W, pad, Hp, W2, (bf16*)out);
  MMDX_LAUNCH_CHECK();
  return 0;
}

extern "C" int mmdx_stem_pair_pack_weight(const float* w_kcrs, int K, int C, int R, int S,
                                          void* w_packed, void* stream) {
  MMDX_CHECK_ARG(w_kcrs && w_packed && C > 0 && C <= 4, "stem pair pack: bad args");
  const int S2 = (S + 1) / 2;
  const long total = (long)K * R * S2 * 8;
  hipLaunchKernelGGL(stem_pair_pack_kernel, dim3(grid_for(total)), dim3(256), 0,
                     (hipStream_t)stream, w_kcrs, K, C, R, S, S2, (bf16*)w_packed);
  MMDX_LAUNCH_CHECK();
  return 0;
}

extern "C" int mmdx_stem_pair_grad(const float* dw_pair, int K, int C, int R, int S, float* dw,
                                   float beta, void* stream) {
  MMDX_CHECK_ARG(dw_pair && dw && C > 0 && C <= 4, "stem pair grad: bad args");
  const long total = (long)K * C * R * S;
  hipLaunchKernelGGL(stem_pair_grad_kernel, dim3(grid_for(total)), dim3(256), 0,
                     (hipStream_t)stream, dw_pair, K, C, R, S, (S + 1) / 2, dw, beta);
  MMDX_LAUNCH_CHECK();
  return 0;
}
