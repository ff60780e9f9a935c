// NHWC convolution on the implicit-GEMM core: fwd, dgrad, wgrad (+ weight packing).
// Replaces every nn.Conv2d of the torchvision ResNet trunk that ImageEncoderCNN wraps
// (training_pipeline.py:178-183, run through _backbone_forward_grad TP:285-289).
#include <algorithm>
#include <type_traits>
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

// 256-row tiles for the narrow-N k-major conv GEMMs (N <= 64: the layer1 3x3 / 1x1 C = K = 64
// convs), where a 128 x 64 block runs a short K loop (9 taps) of 16 MFMAs per wave per barrier:
// twice the rows per block halve the weight-tile DMAs per output and double the MFMAs per
// barrier.  256 x 64 in 8 waves of 64 x 32, two stages, when the grid still has >= 1024 such
// blocks: C4's layer1 (M 401408) fwd / dgrad 0.486 / 0.376 -> 0.45 / 0.33 ms isolated, C4
// 8963 / 8991 vs 8911 / 8922 samples/s paired; C2's layer1 (M 200704, 784 blocks) lost 18 %
// with it, so it keeps 128 x 64.  MMDX_CONV_N64_WIDE = 0 off / 1 on forces it (knobs()).
static bool conv_n64_wide(long M) {
  const int v = knobs().conv_n64_wide;
  return v < 0 ? (M + 255) / 256 >= 1024 : v != 0;
}

// 128 x 128 k-major conv tiles in 8 waves of 64 x 32 (two 512-thread blocks, 16 waves per CU)
// instead of 4 waves of 64 x 64: twice the waves to cover the LDS-DMA and barrier waits at
// half the accumulators per lane.  Default on: isolated C4 fwd / dgrad 2.48 / 2.25 -> 2.28 /
// 2.15 ms, C4 8957 / 8969 -> 9250 / 9271 samples/s paired (r05 s22).  MMDX_CONV_8W128=0
// restores the 4-wave tiles.
static bool conv_8w128_on() { return knobs().conv_8w128; }

// Retired variants (measured slower, removed from the library in round 6; their code and
// measurements: tools/lab/RETIRED.md): 8-wave 256 x 128 conv tiles (MMDX_CONV8_MIN), 32-deep K
// tiles (MMDX_CONV_BK32), 8-wave phase-dgrad / 128 x 64 / weight-gradient tiles
// (MMDX_DGRAD_PHASE_8W, MMDX_CONV_8W64, MMDX_WGRAD_8W), the halo-band A operand
// (MMDX_CONV_HALO), the BN-fold timing probe (MMDX_FOLD_PROBE), the other 256-row variants of
// MMDX_CONV_N64_WIDE, 256 x 128 weight-gradient tiles (MMDX_WGRAD8), tap-aligned 64-column
// weight-gradient tiles (MMDX_WGRAD_TAP_BN) and the BN finalize fused into the conv
// (MMDX_BN_FIN, mmdx_conv_fwd_bnfin).

template <typename T, class SA, class Epi>
static int conv_gemm_epi(const SA& sa, const void* w, const Epi& epi, int M, int N, int K,
                         hipStream_t st, bool dma_ok) {
  DenseK<T> sb{(const T*)w, K, N, true};
  if constexpr (DmaOk<SA>::value) {
    if (dma_ok) {
      // 128x64 tiles when N is narrow or 128x128 tiles would leave CUs idle (< 1.5 per CU)
      const long tiles128 = (long)((M + 127) / 128) * ((N + 127) / 128);
      if (N <= 64 && conv_n64_wide(M)) {
        hipLaunchKernelGGL((igemm_dma_kernel<256, 64, DmaK<256, SA, 64, 8>,
                                             DmaK<64, DenseK<T>, 64, 8>, Epi, 2, bf16, 512, 4, 2>),
                           dim3((M + 255) / 256), dim3(512), 0, st, sa, sb, epi, M, N, K, K);
        MMDX_LAUNCH_CHECK();
        return 0;
      }
      if (N <= 64 || tiles128 < kNarrowBelow)
        return launch_dma<128, 64>(sa, sb, epi, M, N, K, 1, K, st);
      if (conv_8w128_on()) {
        hipLaunchKernelGGL((igemm_dma_kernel<128, 128, DmaK<128, SA, 64, 8>,
                                             DmaK<128, DenseK<T>, 64, 8>, Epi, 2, bf16, 512, 2,
                                             4>),
                           dim3((unsigned)tiles128), dim3(512), 0, st, sa, sb, epi, M, N, K, K);
        MMDX_LAUNCH_CHECK();
        return 0;
      }
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

// ---------------------------------------------------------------------------------------
// Direct stem forward (bf16 pixel-pair stem: C = 8, S = 4 pair columns, stride (2, 1), no
// padding, K = 64 output channels).  As an implicit GEMM its A operand is a 14x re-read of
// the pair image (each input element feeds 7 filter rows x 4 pair columns at stride 2), so
// the generic kernel moves 1.1 GB through L2 -> LDS for 0.26 GB of HBM traffic and runs at
// 0.19 of the HBM roofline.  Here a block owns STEM_PB output rows of one image (all Q
// columns, all 64 channels): the 2*(STEM_PB-1)+R input rows it reads are staged in LDS once,
// and the A fragments are read straight from that image — k-step r of the MFMA loop is filter
// row r, its 32 k = the 4 pair columns s x 8 channels, which sit contiguously at pair
// q + s of input row 2p + r.  Same operand values, same k order, same MFMA sequence per output
// as the implicit-GEMM kernel (bit-identical y); the BatchNorm partials are per block
// (STEM_PB * Q rows: mmdx_conv_fwd_stat_rows).  Wave w owns output channels 16w..16w+15; its
// 7 weight fragments stay in registers.
// ---------------------------------------------------------------------------------------
constexpr int STEM_PB = 2;   // output rows per block
constexpr int STEM_LDY = 64 + 8;  // staged output row (bf16), padded

static bool stem_direct_on() { return knobs().stem_direct; }  // MMDX_STEM_DIRECT (A/B, tests)

static bool stem_direct_geom(const ConvGeom& g) {
  return g.C == 8 && g.S == 4 && (g.R == 7 || g.R == 8) && g.sh == 2 && g.sw == 1 && g.ph == 0 &&
         g.pw == 0 && g.K == 64 && g.Q % 16 == 0 && g.Q <= 256 && g.P % STEM_PB == 0 &&
         2 * (g.P - 1) + g.R <= g.H && g.Q + 3 <= g.W;
}

// NT: row tiles per block (STEM_PB * Q / 16) as a compile-time bound (14 for the 112-wide
// ResNet stem; 32 covers Q <= 256) — the accumulators of unused tiles would hold registers
template <int R, int NT>
__global__ __launch_bounds__(256, 2) void stem_direct_fwd_kernel(
    const bf16* __restrict__ x, const bf16* __restrict__ w, bf16* __restrict__ y,
    float2* __restrict__ part, int H, int W, int P, int Q) {
  constexpr int IR = 2 * (STEM_PB - 1) + R;      // staged input rows
  extern __shared__ __attribute__((aligned(16))) char stem_lds[];
  bf16* xin = (bf16*)stem_lds;                   // [IR][W][8]
  const int rows = STEM_PB * Q;                  // output rows (pixels) of this block
  bf16* ys = xin + ((IR * W * 8 + 7) & ~7);      // [rows][STEM_LDY]
  const int blocks_per_img = P / STEM_PB;
  const int n = blockIdx.x / blocks_per_img, p0 = (blockIdx.x - n * blocks_per_img) * STEM_PB;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  // the input rows 2*p0 .. 2*p0+IR-1 of image n are one contiguous span of IR*W*16 bytes
  {
    const bf16x8* src = (const bf16x8*)(x + ((long)n * H + 2 * p0) * W * 8);
    bf16x8* dst = (bf16x8*)xin;
    const int chunks = IR * W;
    for (int i = threadIdx.x; i < chunks; i += 256) dst[i] = src[i];
  }
  // weight fragments: channel 16*wid + (lane & 15), k = r*32 + (lane >> 4)*8 .. +7
  bf16x8 wf[R];
  const bf16* wrow = w + (long)(16 * wid + (lane & 15)) * (R * 32) + (lane >> 4) * 8;
#pragma unroll
  for (int r = 0; r < R; ++r) wf[r] = *(const bf16x8*)(wrow + r * 32);
  __syncthreads();
  // output row tile mt: pixel row p0 + mt / (Q/16), columns (mt % (Q/16))*16 .. +15
  constexpr int MAXT = NT;
  const int nt = rows / 16, tq = Q / 16;
  f32x4 acc[MAXT];
#pragma unroll
  for (int t = 0; t < MAXT; ++t) {
    acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
    if (t < nt) {
      const int pl = t / tq, q0 = (t - pl * tq) * 16;
      const bf16* a0 = xin + ((2 * pl) * W + q0 + (lane & 15) + (lane >> 4)) * 8;
#pragma unroll
      for (int r = 0; r < R; ++r)
        acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(*(const bf16x8*)(a0 + r * W * 8), wf[r],
                                                         acc[t], 0, 0, 0);
    }
  }
  // BatchNorm partials of this block's rows for the wave's 16 channels: (mean, M2), exact
  // two-pass over the accumulators, then merged over the four lane groups (equal counts)
  float sum = 0.f;
#pragma unroll
  for (int t = 0; t < MAXT; ++t)
    if (t < nt) sum += (acc[t][0] + acc[t][1]) + (acc[t][2] + acc[t][3]);
  sum += __shfl_xor(sum, 16, 64);
  sum += __shfl_xor(sum, 32, 64);
  const float mean = sum / (float)rows;
  float m2 = 0.f;
#pragma unroll
  for (int t = 0; t < MAXT; ++t)
    if (t < nt)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float d = acc[t][j] - mean;
        m2 += d * d;
      }
  m2 += __shfl_xor(m2, 16, 64);
  m2 += __shfl_xor(m2, 32, 64);
  if (part && lane < 16)
    part[(long)(16 * wid + lane) * gridDim.x + blockIdx.x] = make_float2(mean, m2);
  // stage bf16 rows through LDS, then the block's output (rows contiguous pixels x 64
  // channels) goes out as 16-B stores
#pragma unroll
  for (int t = 0; t < MAXT; ++t)
    if (t < nt)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        ys[(t * 16 + (lane >> 4) * 4 + j) * STEM_LDY + 16 * wid + (lane & 15)] =
            from_f<bf16>(acc[t][j]);
  __syncthreads();
  bf16x8* yo = (bf16x8*)(y + ((long)n * P + p0) * Q * 64);
  for (int i = threadIdx.x; i < rows * 8; i += 256)
    yo[i] = *(const bf16x8*)(ys + (i >> 3) * STEM_LDY + (i & 7) * 8);
}

static size_t stem_direct_lds(const ConvGeom& g) {
  const int IR = 2 * (STEM_PB - 1) + g.R;
  return (size_t)((IR * g.W * 8 + 7) & ~7) * 2 + (size_t)STEM_PB * g.Q * STEM_LDY * 2;
}

static int stem_direct_fwd(const ConvGeom& g, const void* x, const void* w, void* y,
                           float* stats, hipStream_t st) {
  const int blocks = g.N * (g.P / STEM_PB);
  const size_t lds = stem_direct_lds(g);
  MMDX_CHECK_ARG(lds <= 64 * 1024 && g.Q <= 256, "stem direct: tile does not fit");
#define STEM_LAUNCH(RR, TT)                                                                   \
  hipLaunchKernelGGL((stem_direct_fwd_kernel<RR, TT>), dim3(blocks), dim3(256), lds, st,       \
                     (const bf16*)x, (const bf16*)w, (bf16*)y, (float2*)stats, g.H, g.W, g.P, g.Q)
  const bool q112 = STEM_PB * g.Q / 16 == 14;
  if (g.R == 7) {
    if (q112) STEM_LAUNCH(7, 14); else STEM_LAUNCH(7, 32);
  } else {
    if (q112) STEM_LAUNCH(8, 14); else STEM_LAUNCH(8, 32);
  }
#undef STEM_LAUNCH
  MMDX_LAUNCH_CHECK();
  return 0;
}

// stat_rows: the rows per statistics slab the caller sized `stats` for (128; 2*Q selects the
// direct stem kernel, which writes one slab per block); without stats the knob decides
template <typename T>
static int conv_fwd_t(const mmdx_conv_desc* d, const void* x, const void* w, void* y,
                      float* stats, int stat_rows, hipStream_t st) {
  const ConvGeom g = geom(d);
  const int M = g.N * g.P * g.Q, N = g.K, K = g.R * g.S * g.C;
  const bool direct = stem_direct_geom(g) && std::is_same<T, bf16>::value &&
                      (stats ? stat_rows == STEM_PB * g.Q : stem_direct_on());
  MMDX_CHECK_ARG(!stats || direct || stat_rows == 128,
                 "conv fwd: statistics slabs of %d rows (128, or %d for the direct stem)",
                 stat_rows, STEM_PB * g.Q);
  if constexpr (std::is_same<T, bf16>::value)
    if (direct) return stem_direct_fwd(g, x, w, y, stats, st);
  if (g.C % KTile<T>::BK == 0 && is_pointwise(g))  // x itself is the [M][C] A operand
    return conv_gemm<T>(PointFwdK<T>{{(const T*)x, g.C, M, true}}, w, y, M, N, K, 0.f, st,
                        stats, dma_geom_ok(g, false, 32, M));
  if (g.C % KTile<T>::BK == 0)
    return conv_gemm<T>(Im2colK<T, true>{(const T*)x, g, M}, w, y, M, N, K, 0.f, st, stats,
                        dma_geom_ok(g, false, 32, M));
  // channel count a power of two: the LDS-DMA kernel decodes each lane's tap itself
  const bool pow2 = g.C >= 8 && (g.C & (g.C - 1)) == 0 && g.R * g.S <= 64;
  Im2colK<T, false> sa{(const T*)x, g, M, pow2 ? __builtin_ctz(g.C) : 0, 1.f / (float)g.S};
  return conv_gemm<T>(sa, w, y, M, N, K, 0.f, st, stats, pow2 && dma_geom_ok(g, false, 64, M),
                      BnStat{});
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
static bool phase_geom(const ConvGeom& g, int a, int b, PhaseGeom& ph) {
  ph.Hp = g.H > a ? (g.H - a + g.sh - 1) / g.sh : 0;
  ph.Wp = g.W > b ? (g.W - b + g.sw - 1) / g.sw : 0;
  if (ph.Hp == 0 || ph.Wp == 0) return false;
  ph.r0 = (a + g.ph) % g.sh;
  ph.s0 = (b + g.pw) % g.sw;
  ph.ntr = ph.r0 < g.R ? (g.R - 1 - ph.r0) / g.sh + 1 : 0;
  ph.nts = ph.s0 < g.S ? (g.S - 1 - ph.s0) / g.sw + 1 : 0;
  ph.dr0 = (a + g.ph - ph.r0) / g.sh;
  ph.ds0 = (b + g.pw - ph.s0) / g.sw;
  return true;
}

// bf16 LDS-DMA path: every phase in ONE launch (grid z = phase; each block selects its own
// phase's geometry, EpiPhase::select).  The sh*sw separate launches each filled a quarter of
// the chip (layer4's 3x3/2: 4 x 196 tiles of 128 x 128 on 256 CUs) and were the slowest
// C4 convs per FLOP (isolated 0.175-0.186 of their roofline).
template <typename T>
static int conv_dgrad_phases_merged(const ConvGeom& g, const void* dy, const void* w_crsk,
                                    void* dx, float beta, hipStream_t st, BnStat bs) {
  DgradPhaseK<T> sa{(const T*)dy, g, PhaseGeom{}, 0};
  PhaseTapK<T> sb{(const T*)w_crsk, (long)g.R * g.S * g.K, g.C, g.K, g.S, g.sh, g.sw,
                  PhaseGeom{}};
  EpiPhase<T> epi{(T*)dx, g.C, 0, g.C, beta, 0, 0, g.H, g.W, 0, 0, g.sh, g.sw};
  epi.bs = bs;
  const int N = g.C;
  int np = 0, mmax = 0, kmax = 0;
  long tiles128 = 0;
  for (int a = 0; a < g.sh; ++a) {
    for (int b = 0; b < g.sw; ++b) {
      PhaseGeom ph;
      if (!phase_geom(g, a, b, ph)) continue;
      const int K = ph.ntr * ph.nts * g.K;
      if (K == 0 && beta != 0.f) continue;
      MMDX_CHECK_ARG(np < MAX_PHASES, "dgrad phases: more than %d", MAX_PHASES);
      const int M = g.N * ph.Hp * ph.Wp;
      sa.phs[np] = sb.phs[np] = ph;
      sa.Ms[np] = epi.Ms[np] = M;
      epi.Ks[np] = K;
      epi.Hps[np] = ph.Hp; epi.Wps[np] = ph.Wp;
      epi.as[np] = a; epi.bs_[np] = b;
      epi.tile0s[np] = bs.tile0;
      bs.tile0 += (M + 127) / 128;  // the next phase's statistics tiles follow this phase's
      mmax = std::max(mmax, M);
      kmax = std::max(kmax, K);
      tiles128 += (long)((M + 127) / 128) * ((N + 127) / 128);
      ++np;
    }
  }
  if (np == 0) return 0;
  // the 128x64 / 128x128 choice on the whole grid's tiles
  if (N <= 64 || tiles128 < kNarrowBelow) {
    const int nwg = ((mmax + 127) / 128) * ((N + 63) / 64);
    hipLaunchKernelGGL((igemm_dma_kernel<128, 64, DmaK<128, DgradPhaseK<T>>,
                                         DmaK<64, PhaseTapK<T>>, EpiPhase<T>, 2>),
                       dim3(nwg, 1, np), dim3(NT), 0, st, sa, sb, epi, mmax, N, kmax, kmax);
  } else {
    const int nwg = ((mmax + 127) / 128) * ((N + 127) / 128);
    hipLaunchKernelGGL((igemm_dma_kernel<128, 128, DmaK<128, DgradPhaseK<T>>,
                                         DmaK<128, PhaseTapK<T>>, EpiPhase<T>, 2>),
                       dim3(nwg, 1, np), dim3(NT), 0, st, sa, sb, epi, mmax, N, kmax, kmax);
  }
  MMDX_LAUNCH_CHECK();
  return 0;
}

template <typename T>
static int conv_dgrad_phases(const ConvGeom& g, const void* dy, const void* w_crsk, void* dx,
                             float beta, hipStream_t st, BnStat bs = BnStat{}) {
  if constexpr (sizeof(T) == 2) {
    if (dma_geom_ok(g, false, 32, (long)g.N * ((g.H + g.sh - 1) / g.sh) *
                                       ((g.W + g.sw - 1) / g.sw)))
      return conv_dgrad_phases_merged<T>(g, dy, w_crsk, dx, beta, st, bs);
  }
  for (int a = 0; a < g.sh; ++a) {
    for (int b = 0; b < g.sw; ++b) {
      PhaseGeom ph;
      if (!phase_geom(g, a, b, ph)) continue;
      const int K = ph.ntr * ph.nts * g.K;
      if (K == 0 && beta != 0.f) continue;
      const int M = g.N * ph.Hp * ph.Wp, N = g.C;
      DgradPhaseK<T> sa{(const T*)dy, g, ph, M};
      PhaseTapK<T> sb{(const T*)w_crsk, (long)g.R * g.S * g.K, g.C, g.K, g.S, g.sh, g.sw, ph};
      EpiPhase<T> epi{(T*)dx, g.C, M, N, beta, ph.Hp, ph.Wp, g.H, g.W, a, b, g.sh, g.sw};
      epi.bs = bs;
      bs.tile0 += (M + 127) / 128;  // the next phase's tiles follow this phase's
      int rc = -1;
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

// split-K block target of the conv weight gradients (MMDX_WGRAD_TARGET, knobs()).  Re-swept on
// the round-5 kernels (split-major order, 8-wave fwd / dgrad tiles; tools/lab/r05_wgrad_target*):
// 256 vs 512 C4 9292 / 9305 / 9305 vs 9266 / 9293 / 9263 paired (+0.3 %), C2 +0.6 %, C3 -0.4 %,
// 768 / 1024 -0.6 / -0.8 %; conv HBM traffic 145.2 -> 137.7 MB per launch (fewer fp32 slabs)
static long wgrad_split_target() { return knobs().wgrad_target; }

static WgradPlan plan_wgrad(int dtype, const mmdx_conv_desc* d) {
  WgradPlan p;
  const int BK = dtype == BF16 ? KTile<bf16>::BK : KTile<float>::BK;
  const int M = d->K, N = d->R * d->S * d->C;
  const long K = (long)d->N * d->P * d->Q;
  p.bm = M <= 64 ? 64 : 128;
  p.bn = N <= 64 ? 64 : 128;
  if (dtype == BF16 && stem_direct_geom(geom(d)) && d->R == 7) {
    // the pixel-pair stem: K splits of whole 2-row pixel tiles (~256 splits), the layout the
    // direct kernel needs; the implicit-GEMM kernel takes the same splits (same sums)
    const long tile_px = (long)STEM_PB * d->Q, ptiles = K / tile_px;
    const long tps = (ptiles + 255) / 256;
    p.kper = (int)(tps * tile_px);
    p.splits = (int)((ptiles + tps - 1) / tps);
    return p;
  }
  const long tiles = (long)((M + p.bm - 1) / p.bm) * ((N + p.bn - 1) / p.bn);
  const long ktiles = (K + BK - 1) / BK;
  // ~1 block per CU, each split at least 16 K tiles deep (keeps the partial slabs small).
  // Rounds 2-3 measured 512 best (256 / 384 / 768 / 1024 lost); round 5 re-swept: 256 (above);
  // ~4 per CU for
  // the 3x3 convs of layer3/4 ran 4-12 % faster in isolation but 0.2 % slower in the train
  // step (more blocks contending with the dgrad chain); 8 / 16 / 32 least K tiles tie.
  const long target = wgrad_split_target();
  const long min_kt = 16L;
  long s = (target + tiles - 1) / tiles;
  s = std::max(1L, std::min(s, ktiles / min_kt));
  const long kt_per = (ktiles + s - 1) / s;
  p.kper = (int)(kt_per * BK);
  p.splits = (int)((K + p.kper - 1) / p.kper);
  return p;
}

// ---------------------------------------------------------------------------------------
// Direct stem weight gradient (the pixel-pair stem of stem_direct_fwd_kernel): dW'[k][kk] =
// sum over pixels of dy[pixel][k] * x_pair[2p + r][q + s][c], kk = (r*4 + s)*8 + c.  As an
// implicit GEMM its B operand is the same 14x re-read of the pair image; here a block owns one
// K split of the plan (plan_wgrad: whole 2-row pixel tiles), stages each tile's dy rows
// (224 pixels x 64 channels, k-lines padded to 144 B) and its input rows in LDS, and reads
// both MFMA operands k-major with ds_read_b64_tr_b16 straight from them: the x operand's
// k-line of pixel (p, q) at tap (r, s) is the 16-B pair chunk [2p + r][q + s] — consecutive
// pixels are consecutive chunks, so no im2col exists anywhere.  The next tile's rows are
// fetched into registers while the current one is multiplied.  Partials go to the plan's
// split-K workspace in its [split][k][kk] layout and are reduced by wgrad_reduce as before.
// Waves: 2 output-channel halves (2 m-tiles each) x 4 groups of tap columns (4, 4, 3, 3 of the
// 14 n-tiles).
// ---------------------------------------------------------------------------------------
constexpr int STEM_LDD = 72;  // staged dy k-line (bf16): 64 channels + pad (conflict-free tr)

__device__ __forceinline__ bf16x8 tr_frag(const bf16* lo, const bf16* hi) {
  typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
  const s16x4 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)lo);
  const s16x4 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)hi);
  return __builtin_bit_cast(bf16x8, __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7));
}

template <int R>
__global__ __launch_bounds__(512, 1) void stem_direct_wgrad_kernel(
    const bf16* __restrict__ x, const bf16* __restrict__ dy, float* __restrict__ ws, int H,
    int W, int P, int Q, int tiles_per_split, int tiles_total) {
  constexpr int IR = 2 * (STEM_PB - 1) + R;
  constexpr int M = 64, N = R * 32;                 // k_out, kk
  constexpr int NTT = N / 16;                        // n-tiles (14 for R = 7)
  extern __shared__ __attribute__((aligned(16))) char stem_lds[];
  const int rows = STEM_PB * Q;                      // pixels per tile
  bf16* dys = (bf16*)stem_lds;                       // [rows][STEM_LDD]
  bf16* xin = dys + rows * STEM_LDD;                 // [IR][W][8]
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int mh = wid & 1, ng = wid >> 1;             // m-tiles 2mh, 2mh+1; n-tile group
  static_assert(NTT >= 12 && NTT <= 16, "4 groups of 3-4 n-tiles");
  // groups of 4, 4, then the rest split evenly (R = 7: 4, 4, 3, 3 of 14)
  const int ntn = ng < 2 ? 4 : (ng == 2 ? (NTT - 8) / 2 : NTT - 8 - (NTT - 8) / 2);
  const int nt0 = ng < 3 ? ng * 4 : 8 + (NTT - 8) / 2;
  const int bpi = P / STEM_PB;
  const int t0 = blockIdx.x * tiles_per_split;
  const int nt = min(tiles_per_split, tiles_total - t0);  // the last split may be short
  // per-thread 16-B chunks of one tile: dy rows*8 chunks, x IR*W chunks
  constexpr int DYC = 4, XC = 3;                     // chunks per thread (rows <= 256, W <= 512)
  bf16x8 rdy[DYC], rx[XC];
  const int ndy = rows * 8, nx = IR * W;
  auto fetch = [&](int t) {
    const int n = t / bpi, p0 = (t - n * bpi) * STEM_PB;
    const bf16x8* sdy = (const bf16x8*)(dy + ((long)n * P + p0) * Q * 64);
    const bf16x8* sx = (const bf16x8*)(x + ((long)n * H + 2 * p0) * W * 8);
#pragma unroll
    for (int j = 0; j < DYC; ++j) {
      const int i = threadIdx.x + j * 512;
      if (i < ndy) rdy[j] = sdy[i];
    }
#pragma unroll
    for (int j = 0; j < XC; ++j) {
      const int i = threadIdx.x + j * 512;
      if (i < nx) rx[j] = sx[i];
    }
  };
  auto stage = [&]() {
#pragma unroll
    for (int j = 0; j < DYC; ++j) {
      const int i = threadIdx.x + j * 512;
      if (i < ndy) *(bf16x8*)(dys + (i >> 3) * STEM_LDD + (i & 7) * 8) = rdy[j];
    }
#pragma unroll
    for (int j = 0; j < XC; ++j) {
      const int i = threadIdx.x + j * 512;
      if (i < nx) *(bf16x8*)(xin + i * 8) = rx[j];
    }
  };
  f32x4 acc[2][4];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
  // fragment lane roles (ds_read_b64_tr_b16): group g reads k-lines 8g + qq (and + 4),
  // columns 4pp .. 4pp+3 of the 16-column tile
  const int g = lane >> 4, qq = (lane & 15) >> 2, pp = lane & 3;
  fetch(t0);
  stage();
  __syncthreads();
  for (int t = 0; t < nt; ++t) {
    if (t + 1 < nt) fetch(t0 + t + 1);  // in flight during the MFMAs
    const int ksteps = rows / 32;
    for (int ks = 0; ks < ksteps; ++ks) {
      const int k_lo = ks * 32 + 8 * g + qq, k_hi = k_lo + 4;   // this lane's two pixels
      bf16x8 af[2];
#pragma unroll
      for (int a = 0; a < 2; ++a) {
        const int col = (2 * mh + a) * 16 + 4 * pp;
        af[a] = tr_frag(dys + k_lo * STEM_LDD + col, dys + k_hi * STEM_LDD + col);
      }
      // x operand: pixel (pl, q) -> pair chunk [2 pl + r][q + s], channel 4 (pp & 1)
      const int pl_lo = k_lo >= Q, q_lo = k_lo - pl_lo * Q;
      const int pl_hi = k_hi >= Q, q_hi = k_hi - pl_hi * Q;
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        if (b < ntn) {
          const int tap = (nt0 + b) * 2 + (pp >> 1), r = tap >> 2, sx = tap & 3;
          const int cofs = (pp & 1) * 4;
          const bf16x8 bf =
              tr_frag(xin + ((2 * pl_lo + r) * W + q_lo + sx) * 8 + cofs,
                      xin + ((2 * pl_hi + r) * W + q_hi + sx) * 8 + cofs);
#pragma unroll
          for (int a = 0; a < 2; ++a)
            acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[a], bf, acc[a][b], 0, 0, 0);
        }
      }
    }
    __syncthreads();  // every wave is done with this tile's LDS rows
    if (t + 1 < nt) {
      stage();
      __syncthreads();
    }
  }
  // partial slab of this split: ws[z][k][kk]
  float* o = ws + (long)blockIdx.x * M * N;
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b)
      if (b < ntn)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          o[((2 * mh + a) * 16 + (lane >> 4) * 4 + j) * N + (nt0 + b) * 16 + (lane & 15)] =
              acc[a][b][j];
}

// The im2col^T operand of the 3x3 / strided weight gradients in the row-quartered LDS image
// (DmaRq: one pixel state per lane; MMDX_WGRAD_RQ=0 restores DmaR for A/B runs)
static bool wgrad_rq_on() { return knobs().wgrad_rq; }

template <typename T, class SB>
static int wgrad_dma(const WgradPlan& p, const DenseR<T>& sa, const SB& sb, const EpiPartial& epi,
                     int M, int N, int K, hipStream_t st) {
  if constexpr (std::is_same<SB, Im2colR<T>>::value) {
    if (wgrad_rq_on()) {
      if (p.bm == 128 && p.bn == 128)
        return launch_dma_ops<128, 128, DmaR<128, DenseR<T>>, DmaRq<128, SB>>(
            sa, sb, epi, M, N, K, p.splits, p.kper, st);
      if (p.bm == 128)
        return launch_dma_ops<128, 64, DmaR<128, DenseR<T>>, DmaRq<64, SB>>(
            sa, sb, epi, M, N, K, p.splits, p.kper, st);
      if (p.bn == 128)
        return launch_dma_ops<64, 128, DmaR<64, DenseR<T>>, DmaRq<128, SB>>(
            sa, sb, epi, M, N, K, p.splits, p.kper, st);
      return launch_dma_ops<64, 64, DmaR<64, DenseR<T>>, DmaRq<64, SB>>(sa, sb, epi, M, N, K,
                                                                       p.splits, p.kper, st);
    }
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
    // the pixel-pair stem: whole 2-row pixel tiles per split -> the direct kernel
    const int tile_px = STEM_PB * g.Q;
    if (stem_direct_geom(g) && stem_direct_on() && g.R == 7 && p.kper % tile_px == 0 &&
        K % tile_px == 0 && tile_px <= 256 && g.W * (2 * (STEM_PB - 1) + g.R) <= 3 * 512) {
      const size_t lds = (size_t)tile_px * STEM_LDD * 2 +
                         (size_t)(2 * (STEM_PB - 1) + g.R) * g.W * 16;
      hipLaunchKernelGGL(stem_direct_wgrad_kernel<7>, dim3(p.splits), dim3(512), lds, st,
                         (const bf16*)x, (const bf16*)dy, (float*)ws, g.H, g.W, g.P, g.Q,
                         p.kper / tile_px, K / tile_px);
      MMDX_LAUNCH_CHECK();
      wgrad_reduce((const float*)ws, p.splits, g.K, g.C, cm, g.R * g.S, dw, beta, st);
      MMDX_LAUNCH_CHECK();
      return 0;
    }
  }
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
  MMDX_CHECK_ARG(items && n_items > 0 && total_blocks > 0 && total_blocks < (1L << 31),
                 "conv pack multi: bad item table");
  hipStream_t st = (hipStream_t)stream;
  if (dtype == F16)  // the C5 encoder stacks' weight casts (RS = 1 items: plain [K][C] copies)
    hipLaunchKernelGGL(pack_multi_kernel<f16>, dim3((unsigned)total_blocks), dim3(256), 0, st,
                       items, n_items);
  else if (dtype == BF16)
    hipLaunchKernelGGL(pack_multi_kernel<bf16>, dim3((unsigned)total_blocks), dim3(256), 0, st,
                       items, n_items);
  else
    hipLaunchKernelGGL(pack_multi_kernel<float>, dim3((unsigned)total_blocks), dim3(256), 0, st,
                       items, n_items);
  MMDX_LAUNCH_CHECK();
  return 0;
}

extern "C" int mmdx_conv_fwd_stat_rows(const mmdx_conv_desc* d) {
  return stem_direct_geom(geom(d)) && stem_direct_on() ? STEM_PB * d->Q : 128;
}

extern "C" int mmdx_conv_fwd_stat_blocks(const mmdx_conv_desc* d) {
  const long rpb = mmdx_conv_fwd_stat_rows(d);
  return (int)(((long)d->N * d->P * d->Q + rpb - 1) / rpb);
}

extern "C" int mmdx_conv_fwd_rows(int dtype, const mmdx_conv_desc* d, const void* x,
                                  const void* w, void* y, float* stat_part, int stat_rows,
                                  void* stream) {
  MMDX_CHECK_ARG(dtype != F16, "mmdx_conv_fwd: fp16 is the C5 path only");
  int rc = check_desc(d, dtype == BF16 ? 8 : 4);
  if (rc) return rc;
  MMDX_CHECK_ARG((long)d->N * d->P * d->Q < (1L << 31), "conv fwd: too many pixels");
  if (dtype == BF16)
    return conv_fwd_t<bf16>(d, x, w, y, stat_part, stat_rows, (hipStream_t)stream);
  return conv_fwd_t<float>(d, x, w, y, stat_part, stat_rows, (hipStream_t)stream);
}

extern "C" int mmdx_conv_fwd(int dtype, const mmdx_conv_desc* d, const void* x,
                             const void* w, void* y, float* stat_part, void* stream) {
  MMDX_CHECK_ARG(d, "conv fwd: null descriptor");
  return mmdx_conv_fwd_rows(dtype, d, x, w, y, stat_part,
                            dtype == BF16 ? mmdx_conv_fwd_stat_rows(d) : 128, stream);
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
