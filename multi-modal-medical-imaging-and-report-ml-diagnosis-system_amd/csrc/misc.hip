// Pooling, layout conversion, casts, GELU backward, bias gradient, dropout, BCE-with-logits.
#include <algorithm>

#include "common.h"
#include "pool.h"
#include "../../include/mmdx.h"

namespace mmdx {

// ----------------------------------------------------------------------------- maxpool
// Semantics of PyTorch CPU max_pool2d: padded taps are skipped, the FIRST maximum in
// row-major window order wins (strict '>'), NaN propagates.
template <typename T>
__global__ void maxpool_fwd_kernel(const T* __restrict__ x, int N, int H, int W, int C, int k,
                                   int s, int p, T* __restrict__ y, uint8_t* __restrict__ am,
                                   int P, int Q) {
  typedef typename Vec16<T>::type V;
  constexpr int VEC = Vec16<T>::N;
  const int cv = C / VEC;
  const long total = (long)N * P * Q * cv;
  GRID_STRIDE(i, total) {
    const int c = (int)(i % cv) * VEC;
    long t = i / cv;
    const int q = (int)(t % Q); t /= Q;
    const int pp = (int)(t % P);
    const int n = (int)(t / P);
    float best[VEC];
    int arg[VEC];
#pragma unroll
    for (int j = 0; j < VEC; ++j) { best[j] = -INFINITY; arg[j] = -1; }
    for (int r = 0; r < k; ++r) {
      const int ih = pp * s - p + r;
      if ((unsigned)ih >= (unsigned)H) continue;
      for (int ss = 0; ss < k; ++ss) {
        const int iw = q * s - p + ss;
        if ((unsigned)iw >= (unsigned)W) continue;
        const V v = *(const V*)(x + (((long)n * H + ih) * W + iw) * C + c);
#pragma unroll
        for (int j = 0; j < VEC; ++j) {
          const float f = to_f(v[j]);
          if (arg[j] < 0 || f > best[j] || (f != f && best[j] == best[j])) {
            best[j] = f;
            arg[j] = r * k + ss;
          }
        }
      }
    }
    V o;
#pragma unroll
    for (int j = 0; j < VEC; ++j) {
      o[j] = from_f<T>(best[j]);
      am[i * VEC + j] = (uint8_t)arg[j];
    }
    *(V*)(y + i * VEC) = o;
  }
}

// Gather form: each input element sums dy of the windows whose argmax points at it.
template <typename T>
__global__ void maxpool_bwd_kernel(const uint8_t* __restrict__ am, const T* __restrict__ dy,
                                   int N, int H, int W, int C, int k, int s, int p, int P, int Q,
                                   T* __restrict__ dx) {
  typedef typename Vec16<T>::type V;
  constexpr int VEC = Vec16<T>::N;
  const int cv = C / VEC;
  const long total = (long)N * H * W * cv;
  GRID_STRIDE(i, total) {
    const int c = (int)(i % cv) * VEC;
    long t = i / cv;
    const int w = (int)(t % W); t /= W;
    const int h = (int)(t % H);
    const int n = (int)(t / H);
    float acc[VEC];
#pragma unroll
    for (int j = 0; j < VEC; ++j) acc[j] = 0.f;
    // windows (pp,q) with pp*s - p <= h <= pp*s - p + k - 1
    const int p_lo = max(0, (h + p - k + s) / s), p_hi = min(P - 1, (h + p) / s);
    const int q_lo = max(0, (w + p - k + s) / s), q_hi = min(Q - 1, (w + p) / s);
    for (int pp = p_lo; pp <= p_hi; ++pp) {
      const int r = h + p - pp * s;
      if (r < 0 || r >= k) continue;
      for (int q = q_lo; q <= q_hi; ++q) {
        const int ss = w + p - q * s;
        if (ss < 0 || ss >= k) continue;
        const long o = (((long)n * P + pp) * Q + q) * C + c;
        const V g = *(const V*)(dy + o);
#pragma unroll
        for (int j = 0; j < VEC; ++j)
          if (am[o + j] == r * k + ss) acc[j] += to_f(g[j]);
      }
    }
    V out;
#pragma unroll
    for (int j = 0; j < VEC; ++j) out[j] = from_f<T>(acc[j]);
    *(V*)(dx + i * VEC) = out;
  }
}

// The ResNet stem pool (3x3, stride 2): the nine window loads of a thread are all issued
// before the first compare (the generic loop above compiles to one load-compare round trip
// per tap) and the argmax bytes go out as one 8-byte (bf16 / fp16) or 4-byte (fp32) store.
// Same window order, tie rule and NaN rule as maxpool_fwd_kernel.

//
// BN = true: the pool reads the stem conv's RAW output and applies its train-mode BatchNorm
// + ReLU on the fly (the stem unit's post-activation tensor is never written: its backward
// recomputes the ReLU mask from the raw output, and nothing else reads it).  Each tap value
// is the bf16 the separate BN-apply pass would have stored — same scale/shift expressions
// (bn_coef_fwd), same fp32 math, rounded to T before the compare — so the pooled values and
// argmax bytes are bit-identical to BN-apply followed by the pool.
__device__ __forceinline__ void bn_coef_fwd(const float* gamma, const float* beta,
                                            const float* mean, const float* rstd, int c,
                                            float& scale, float& shift) {
  // the expressions of bn_finalize_kernel (norm.hip): scale = g*rstd, shift = b - mean*g*rstd
  const float g = gamma ? gamma[c] : 1.f;
  scale = g * rstd[c];
  shift = (beta ? beta[c] : 0.f) - mean[c] * g * rstd[c];
}

template <typename T, bool BN = false>
__global__ void maxpool3s2_fwd_kernel(const T* __restrict__ x, int N, int H, int W, int C,
                                      int p, T* __restrict__ y, uint8_t* __restrict__ am, int P,
                                      int Q, const float* __restrict__ gamma,
                                      const float* __restrict__ beta,
                                      const float* __restrict__ mean,
                                      const float* __restrict__ rstd, int relu) {
  typedef typename Vec16<T>::type V;
  constexpr int VEC = Vec16<T>::N;
  typedef typename ArgPack<VEC>::type A;
  const int cv = C / VEC;
  const long total = (long)N * P * Q * cv;
  // the grid stride is a multiple of cv when the block is: a thread's channel vector (and
  // its BN coefficients) is then fixed, computed once instead of per output
  const bool fixed_c = blockDim.x % cv == 0;
  float sc[VEC], sh[VEC];
  if constexpr (BN) {
    if (fixed_c) {
      const int c0 = (int)(threadIdx.x % cv) * VEC;
#pragma unroll
      for (int j = 0; j < VEC; ++j) bn_coef_fwd(gamma, beta, mean, rstd, c0 + j, sc[j], sh[j]);
    }
  }
  GRID_STRIDE(i, total) {
    // 32-bit index math (total < 2^31, checked by the entry point): a 64-bit division is a
    // long software sequence on the GPU
    const unsigned ui = (unsigned)i, ucv = (unsigned)cv;
    const int c = (int)(ui % ucv) * VEC;
    if constexpr (BN) {
      if (!fixed_c) {
#pragma unroll
        for (int j = 0; j < VEC; ++j) bn_coef_fwd(gamma, beta, mean, rstd, c + j, sc[j], sh[j]);
      }
    }
    unsigned t = ui / ucv;
    const int q = (int)(t % (unsigned)Q); t /= (unsigned)Q;
    const int pp = (int)(t % (unsigned)P);
    const int n = (int)(t / (unsigned)P);
    V v[9];
    bool ok[9];
#pragma unroll
    for (int r = 0; r < 3; ++r) {
      const int ih = pp * 2 - p + r;
#pragma unroll
      for (int ss = 0; ss < 3; ++ss) {
        const int iw = q * 2 - p + ss;
        ok[r * 3 + ss] = (unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W;
        v[r * 3 + ss] = ok[r * 3 + ss] ? *(const V*)(x + (((long)n * H + ih) * W + iw) * C + c)
                                       : V{};
      }
    }
    float best[VEC];
    int arg[VEC];
#pragma unroll
    for (int j = 0; j < VEC; ++j) { best[j] = -INFINITY; arg[j] = -1; }
#pragma unroll
    for (int w9 = 0; w9 < 9; ++w9) {
      if (!ok[w9]) continue;
#pragma unroll
      for (int j = 0; j < VEC; ++j) {
        float f = to_f(v[w9][j]);
        if constexpr (BN) {
          f = f * sc[j] + sh[j];
          if (relu) f = fmaxf(f, 0.f);
          f = to_f(from_f<T>(f));  // the value BN-apply would have stored
        }
        if (arg[j] < 0 || f > best[j] || (f != f && best[j] == best[j])) {
          best[j] = f;
          arg[j] = w9;
        }
      }
    }
    V o;
    A packed = 0;
#pragma unroll
    for (int j = 0; j < VEC; ++j) {
      o[j] = from_f<T>(best[j]);
      packed |= (A)(uint8_t)arg[j] << (8 * j);
    }
    *(A*)(am + i * VEC) = packed;
    *(V*)(y + i * VEC) = o;
  }
}

// Backward of the 3x3 / stride-2 pool: an input pixel lies in at most 2 x 2 windows; their
// dy vectors and packed argmax bytes are loaded together, summed in the generic kernel's
// window order.
template <typename T>
__global__ void maxpool3s2_bwd_kernel(const uint8_t* __restrict__ am, const T* __restrict__ dy,
                                      int N, int H, int W, int C, int p, int P, int Q,
                                      T* __restrict__ dx) {
  typedef typename Vec16<T>::type V;
  constexpr int VEC = Vec16<T>::N;
  const Pool3s2Grad<T> pg{am, dy, H, W, C, p, P, Q};
  const int cv = C / VEC;
  const long total = (long)N * H * W * cv;
  GRID_STRIDE(i, total) {  // 32-bit index math (total < 2^31, checked by the entry point)
    const unsigned ui = (unsigned)i, ucv = (unsigned)cv;
    const int c = (int)(ui % ucv) * VEC;
    unsigned t = ui / ucv;
    const int w = (int)(t % (unsigned)W); t /= (unsigned)W;
    const int h = (int)(t % (unsigned)H);
    const int n = (int)(t / (unsigned)H);
    *(V*)(dx + i * VEC) = pg.at(n, h, w, c);
  }
}

// ----------------------------------------------------------------------------- avgpool
template <typename T>
__global__ void avgpool_fwd_kernel(const T* __restrict__ x, int N, int HW, int C,
                                   T* __restrict__ y) {
  const long total = (long)N * C;
  GRID_STRIDE(i, total) {
    const int c = (int)(i % C);
    const long n = i / C;
    float acc = 0.f;
    for (int k = 0; k < HW; ++k) acc += to_f(x[(n * HW + k) * C + c]);
    y[i] = from_f<T>(acc / (float)HW);
  }
}

template <typename T>
__global__ void avgpool_bwd_kernel(const T* __restrict__ dy, int N, int HW, int C,
                                   T* __restrict__ dx) {
  const long total = (long)N * HW * C;
  const float inv = 1.f / (float)HW;
  GRID_STRIDE(i, total) {
    const int c = (int)(i % C);
    const long n = i / ((long)HW * C);
    dx[i] = from_f<T>(to_f(dy[n * C + c]) * inv);
  }
}

// ----------------------------------------------------------------------------- layout
template <typename T>
__global__ void nchw_to_nhwc_kernel(const float* __restrict__ x, int N, int C, int H, int W,
                                    int cp, T* __restrict__ y) {
  const long total = (long)N * H * W;
  GRID_STRIDE(i, total) {
    const long hw = i % ((long)H * W);
    const long n = i / ((long)H * W);
    for (int c = 0; c < cp; ++c)
      y[i * cp + c] = from_f<T>(c < C ? x[(n * C + c) * H * W + hw] : 0.f);
  }
}

template <typename D, typename S>
__global__ void cast_kernel(const S* __restrict__ x, long n, D* __restrict__ y) {
  GRID_STRIDE(i, n) y[i] = from_f<D>(to_f(x[i]));
}

__global__ void axpby_kernel(long n, float a, const float* __restrict__ x, float b,
                             const float* __restrict__ y, float* __restrict__ out) {
  GRID_STRIDE(i, n) out[i] = a * x[i] + (y ? b * y[i] : 0.f);
}

// ----------------------------------------------------------------------------- GELU / bias
template <typename T>
__global__ void gelu_bwd_kernel(const T* __restrict__ pre, const T* __restrict__ dy, long n,
                                T* __restrict__ dx) {
  GRID_STRIDE(i, n) dx[i] = from_f<T>(to_f(dy[i]) * gelu_erf_grad(to_f(pre[i])));
}

constexpr int BG_ROWS = 256;     // the most rows a pass-1 block takes
constexpr int BG_ROWS_MIN = 32;  // the fewest (sizes the workspace)
// rows per pass-1 block: enough blocks to cover the chip (>= 1024) at N = 768 as at 3072 —
// with a fixed 256 rows a C5 bias gradient ([8192, 768] fp16) ran as 64 blocks, 1.4 TB/s
static int bias_grad_rows(long M, int N, int vec) {
  const long nx = (N / vec + 63) / 64;
  const long nb_target = (1024 + nx - 1) / nx;
  long rows = (M + nb_target - 1) / nb_target;
  rows = (rows + 3) / 4 * 4;
  return (int)std::max<long>(BG_ROWS_MIN, std::min<long>(BG_ROWS, rows));
}
// Column sums of dY [M][N] (bias gradients) in two deterministic passes.  Pass 1: a block
// owns 64 16-B column vectors x `rows` rows; its 4 row lanes stride the rows with vector
// loads (a wave reads 1 KB of one row), then combine through LDS into one partial row.
// (The first version summed one column per thread with 2-B loads and serial adds: 63 us per
// call, 6.9 ms per C5 step.)
template <typename T>
__global__ __launch_bounds__(256) void bias_grad_partial_kernel(const T* __restrict__ dy,
                                                                long M, int N,
                                                                float* __restrict__ part,
                                                                int rows) {
  typedef typename Vec16<T>::type V;
  constexpr int VEC = Vec16<T>::N;
  __shared__ float red[4][64 * VEC];
  const int cv = threadIdx.x & 63, lane = threadIdx.x >> 6;
  const int j = blockIdx.x * 64 + cv;          // column vector
  const bool ok = j < N / VEC;
  const long r0 = (long)blockIdx.y * rows, r1 = min(M, r0 + rows);
  float acc[VEC];
#pragma unroll
  for (int e = 0; e < VEC; ++e) acc[e] = 0.f;
  if (ok) {
#pragma unroll 4
    for (long r = r0 + lane; r < r1; r += 4) {
      const V v = ((const V*)(dy + r * N))[j];
#pragma unroll
      for (int e = 0; e < VEC; ++e) acc[e] += to_f(v[e]);
    }
  }
#pragma unroll
  for (int e = 0; e < VEC; ++e) red[lane][cv * VEC + e] = acc[e];
  __syncthreads();
  if (lane == 0 && ok) {
#pragma unroll
    for (int e = 0; e < VEC; ++e) {
      const int c = cv * VEC + e;
      part[(long)blockIdx.y * N + (long)j * VEC + e] =
          (red[0][c] + red[1][c]) + (red[2][c] + red[3][c]);
    }
  }
}
// N not a multiple of the vector width: one column per thread
template <typename T>
__global__ void bias_grad_partial_scalar_kernel(const T* __restrict__ dy, long M, int N,
                                                float* __restrict__ part, int rows) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= N) return;
  const long r0 = (long)blockIdx.y * rows, r1 = min(M, r0 + rows);
  float acc = 0.f;
  for (long r = r0; r < r1; ++r) acc += to_f(dy[r * N + n]);
  part[(long)blockIdx.y * N + n] = acc;
}
// Pass 2: 64 columns x 4 lanes per block, the lanes stride the partial rows
__global__ __launch_bounds__(256) void bias_grad_finalize_kernel(const float* __restrict__ part,
                                                                 int nb, int N, float* db,
                                                                 float beta_acc) {
  __shared__ float red[4][64];
  const int cc = threadIdx.x & 63, lane = threadIdx.x >> 6;
  const int n = blockIdx.x * 64 + cc;
  float acc = 0.f;
  if (n < N) {
#pragma unroll 4
    for (int b = lane; b < nb; b += 4) acc += part[(long)b * N + n];
  }
  red[lane][cc] = acc;
  __syncthreads();
  if (lane != 0 || n >= N) return;
  const float s = (red[0][cc] + red[1][cc]) + (red[2][cc] + red[3][cc]);
  db[n] = beta_acc != 0.f ? beta_acc * db[n] + s : s;
}

// ----------------------------------------------------------------------------- dropout
__device__ __forceinline__ uint32_t hash64(uint64_t x) {
  x ^= x >> 33; x *= 0xff51afd7ed558ccdULL;
  x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ULL;
  x ^= x >> 33;
  return (uint32_t)x;
}
template <typename T>
__global__ void dropout_fwd_kernel(const T* __restrict__ x, long n, float p, uint64_t seed,
                                   uint64_t off, const uint64_t* __restrict__ ctr,
                                   T* __restrict__ y, uint8_t* __restrict__ mask) {
  const float scale = 1.f / (1.f - p);
  if (ctr) off += ctr[0] << 32;
  GRID_STRIDE(i, n) {
    const float u = (hash64(seed * 0x9E3779B97F4A7C15ULL + off + (uint64_t)i) >> 8) *
                    (1.f / 16777216.f);
    const uint8_t keep = u >= p;
    mask[i] = keep;
    y[i] = from_f<T>(keep ? to_f(x[i]) * scale : 0.f);
  }
}
__global__ void counter_incr_kernel(uint64_t* c) { c[0] += 1; }

template <typename T>
__global__ void dropout_bwd_kernel(const T* __restrict__ dy, const uint8_t* __restrict__ mask,
                                   long n, float p, T* __restrict__ dx) {
  const float scale = 1.f / (1.f - p);
  GRID_STRIDE(i, n) dx[i] = from_f<T>(mask[i] ? to_f(dy[i]) * scale : 0.f);
}

// ----------------------------------------------------------------------------- BCE
// loss = mean( (1-y)*z + log(1 + exp(-z)) ), in the max-shifted form PyTorch uses.
__global__ void bce_fwd_kernel(const float* __restrict__ z, const float* __restrict__ y, int n,
                               float* loss) {
  __shared__ float red[4];
  float acc = 0.f;
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const float zi = z[i], yi = y[i];
    const float mx = fmaxf(-zi, 0.f);
    acc += (1.f - yi) * zi + mx + logf(expf(-mx) + expf(-zi - mx));
  }
  acc = block_sum<256>(acc, red);
  if (threadIdx.x == 0) loss[0] = acc / (float)n;
}
__global__ void bce_bwd_kernel(const float* __restrict__ z, const float* __restrict__ y, int n,
                               const float* __restrict__ dloss, float* __restrict__ dz) {
  const float g = (dloss ? dloss[0] : 1.f) / (float)n;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const float s = 1.f / (1.f + expf(-z[i]));
    dz[i] = (s - y[i]) * g;
  }
}

}  // namespace mmdx

using namespace mmdx;

#define DISPATCH_T(dtype, ...) MMDX_DISPATCH(dtype, __VA_ARGS__)

extern "C" int mmdx_maxpool_fwd(int dtype, const void* x, int N, int H, int W, int C, int k,
                                int s, int p, void* y, uint8_t* argmax, int P, int Q,
                                void* stream) {
  const int VEC = dtype == F32 ? 4 : 8;
  MMDX_CHECK_ARG(C % VEC == 0 && k * k <= 255 && argmax, "maxpool: bad args");
  MMDX_CHECK_ARG(P == (H + 2 * p - k) / s + 1 && Q == (W + 2 * p - k) / s + 1,
                 "maxpool: inconsistent output size");
  const long total = (long)N * P * Q * (C / VEC);
  MMDX_CHECK_ARG((long)N * H * W * C < (1L << 31), "maxpool: more than 2^31 input elements");
  if (k == 3 && s == 2)
    DISPATCH_T(dtype, hipLaunchKernelGGL((maxpool3s2_fwd_kernel<T, false>),
                                         dim3(grid_for(total)), dim3(256), 0, (hipStream_t)stream,
                                         (const T*)x, N, H, W, C, p, (T*)y, argmax, P, Q,
                                         (const float*)nullptr, (const float*)nullptr,
                                         (const float*)nullptr, (const float*)nullptr, 0));
  else
    DISPATCH_T(dtype, hipLaunchKernelGGL(maxpool_fwd_kernel<T>, dim3(grid_for(total)),
                                         dim3(256), 0, (hipStream_t)stream, (const T*)x, N, H, W,
                                         C, k, s, p, (T*)y, argmax, P, Q));
  MMDX_LAUNCH_CHECK();
  return 0;
}

extern "C" int mmdx_maxpool_bn_fwd(int dtype, const void* x, int N, int H, int W, int C,
                                   int k, int s, int p, const float* gamma, const float* beta,
                                   const float* save_mean, const float* save_rstd, int relu,
                                   void* y, uint8_t* argmax, int P, int Q, void* stream) {
  const int VEC = dtype == F32 ? 4 : 8;
  MMDX_CHECK_ARG(C % VEC == 0 && argmax && save_mean && save_rstd, "maxpool bn: bad args");
  MMDX_CHECK_ARG(k == 3 && s == 2, "maxpool bn: only the 3x3 / stride-2 stem pool is fused");
  MMDX_CHECK_ARG(P == (H + 2 * p - k) / s + 1 && Q == (W + 2 * p - k) / s + 1,
                 "maxpool bn: inconsistent output size");
  const long total = (long)N * P * Q * (C / VEC);
  MMDX_CHECK_ARG((long)N * H * W * C < (1L << 31), "maxpool bn: more than 2^31 input elements");
  DISPATCH_T(dtype, hipLaunchKernelGGL((maxpool3s2_fwd_kernel<T, true>), dim3(grid_for(total)),
                                       dim3(256), 0, (hipStream_t)stream, (const T*)x, N, H, W, C,
                                       p, (T*)y, argmax, P, Q, gamma, beta, save_mean, save_rstd,
                                       relu));
  MMDX_LAUNCH_CHECK();
  return 0;
}

extern "C" int mmdx_maxpool_bwd(int dtype, const uint8_t* argmax, const void* dy, int N, int H,
                                int W, int C, int k, int s, int p, int P, int Q, void* dx,
                                void* stream) {
  const int VEC = dtype == F32 ? 4 : 8;
  MMDX_CHECK_ARG(C % VEC == 0, "maxpool bwd: bad C");
  const long total = (long)N * H * W * (C / VEC);
  MMDX_CHECK_ARG((long)N * H * W * C < (1L << 31), "maxpool bwd: more than 2^31 elements");
  if (k == 3 && s == 2 && p <= 1)
    DISPATCH_T(dtype, hipLaunchKernelGGL(maxpool3s2_bwd_kernel<T>, dim3(grid_for(total)),
                                         dim3(256), 0, (hipStream_t)stream, argmax,
                                         (const T*)dy, N, H, W, C, p, P, Q, (T*)dx));
  else
    DISPATCH_T(dtype, hipLaunchKernelGGL(maxpool_bwd_kernel<T>, dim3(grid_for(total)),
                                         dim3(256), 0, (hipStream_t)stream, argmax,
                                         (const T*)dy, N, H, W, C, k, s, p, P, Q, (T*)dx));
  MMDX_LAUNCH_CHECK();
  return 0;
}

extern "C" int mmdx_avgpool_fwd(int dtype, const void* x, int N, int HW, int C, void* y,
                                void* stream) {
  const long total = (long)N * C;
  DISPATCH_T(dtype, hipLaunchKernelGGL(avgpool_fwd_kernel<T>, dim3(grid_for(total)), dim3(256),
                                       0, (hipStream_t)stream, (const T*)x, N, HW, C, (T*)y));
  MMDX_LAUNCH_CHECK();
  return 0;
}

extern "C" int mmdx_avgpool_bwd(int dtype, const void* dy, int N, int HW, int C, void* dx,
                                void* stream) {
  const long total = (long)N * HW * C;
  DISPATCH_T(dtype, hipLaunchKernelGGL(avgpool_bwd_kernel<T>, dim3(grid_for(total)), dim3(256),
                                       0, (hipStream_t)stream, (const T*)dy, N, HW, C, (T*)dx));
  MMDX_LAUNCH_CHECK();
  return 0;
}

extern "C" int mmdx_nchw_to_nhwc(int dtype, const float* x, int N, int C, int H, int W,
                                 int c_pad, void* y, void* stream) {
  MMDX_CHECK_ARG(c_pad >= C, "nchw_to_nhwc: c_pad < C");
  const long total = (long)N * H * W;
  DISPATCH_T(dtype, hipLaunchKernelGGL(nchw_to_nhwc_kernel<T>, dim3(grid_for(total)), dim3(256),
                                       0, (hipStream_t)stream, x, N, C, H, W, c_pad, (T*)y));
  MMDX_LAUNCH_CHECK();
  return 0;
}

extern "C" int mmdx_cast(int dst, int src, const void* x, long n, void* y, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (dst == BF16 && src == F32)
    hipLaunchKernelGGL((cast_kernel<bf16, float>), dim3(grid_for(n)), dim3(256), 0, st,
                       (const float*)x, n, (bf16*)y);
  else if (dst == F32 && src == BF16)
    hipLaunchKernelGGL((cast_kernel<float, bf16>), dim3(grid_for(n)), dim3(256), 0, st,
                       (const bf16*)x, n, (float*)y);
  else if (dst == F32 && src == F32)
    hipLaunchKernelGGL((cast_kernel<float, float>), dim3(grid_for(n)), dim3(256), 0, st,
                       (const float*)x, n, (float*)y);
  else if (dst == F16 && src == F32)
    hipLaunchKernelGGL((cast_kernel<f16, float>), dim3(grid_for(n)), dim3(256), 0, st,
                       (const float*)x, n, (f16*)y);
  else if (dst == F32 && src == F16)
    hipLaunchKernelGGL((cast_kernel<float, f16>), dim3(grid_for(n)), dim3(256), 0, st,
                       (const f16*)x, n, (float*)y);
  else
    hipLaunchKernelGGL((cast_kernel<bf16, bf16>), dim3(grid_for(n)), dim3(256), 0, st,
                       (const bf16*)x, n, (bf16*)y);
  MMDX_LAUNCH_CHECK();
  return 0;
}

extern "C" int mmdx_gelu_bwd(int dtype, const void* pre, const void* dy, long n, void* dx,
                             void* stream) {
  DISPATCH_T(dtype, hipLaunchKernelGGL(gelu_bwd_kernel<T>, dim3(grid_for(n)), dim3(256), 0,
                                       (hipStream_t)stream, (const T*)pre, (const T*)dy, n,
                                       (T*)dx));
  MMDX_LAUNCH_CHECK();
  return 0;
}

// MMDX_BIAS_GRAD_GEMM=1 (16-bit dY with M, N multiples of 8): db = 1^T dY as a 1 x N x M
// GEMM on the MFMA core (a ones row in the workspace as A, dY read R-major as B, split-K over
// the M rows into fp32 slabs + the split-K reduce, beta = beta_acc).  Tested
// (test_kernels_gpu.py::test_bias_grad) but off: in the C5 step it ran slower than the two
// column-sum passes below (2624 / 2624 vs 2647 / 2655 samples/s, paired) — its ~200 blocks
// of mostly idle 64 x 128 MFMA tiles hold CUs the other tower's kernels want.
static bool bias_grad_gemm_ok(int dtype, long M, int N) {
  const bool on = knobs().bias_grad_gemm;
  return on && dtype != F32 && M % 8 == 0 && N % 8 == 0 && M < (1L << 30);
}
static size_t bias_grad_ones_bytes(long M) { return ((size_t)M * 2 + 255) & ~(size_t)255; }

template <typename T>
__global__ void fill_ones_kernel(T* __restrict__ p, long n) {
  GRID_STRIDE(i, n) p[i] = from_f<T>(1.f);
}

extern "C" size_t mmdx_bias_grad_workspace_size(long M, int N) {
  const size_t cs = (size_t)((M + BG_ROWS_MIN - 1) / BG_ROWS_MIN) * N * sizeof(float);
  // the GEMM form's workspace (the split plan depends on the dtype class only through the
  // K tile, the same for bf16 and f16)
  const size_t gm = M < (1L << 30) ? bias_grad_ones_bytes(M) +
                                         mmdx_gemm_workspace_size(BF16, 1, N, (int)M)
                                   : 0;
  return std::max(cs, gm);
}

extern "C" int mmdx_bias_grad(int dtype, const void* dy, long M, int N, float* db,
                              float beta_acc, void* ws, size_t ws_bytes, void* stream) {
  if (bias_grad_gemm_ok(dtype, M, N) && ((uintptr_t)dy & 15) == 0 && ws &&
      ws_bytes >= mmdx_bias_grad_workspace_size(M, N)) {
    hipStream_t st = (hipStream_t)stream;
    char* ones = (char*)ws;
    const size_t ob = bias_grad_ones_bytes(M);
    DISPATCH_T(dtype, hipLaunchKernelGGL(fill_ones_kernel<T>, dim3(grid_for(M)), dim3(256), 0,
                                         st, (T*)ones, M));
    MMDX_LAUNCH_CHECK();
    return mmdx_gemm(dtype, 1, N, (int)M, ones, M, 1, dy, N, 0, db, N, F32, nullptr, nullptr,
                     0, 1.f, beta_acc, nullptr, ones + ob, ws_bytes - ob, stream);
  }
  const int vec = dtype == F32 ? 4 : 8;
  const int rows = bias_grad_rows(M, N, vec);
  const int nb = (int)((M + rows - 1) / rows);
  MMDX_CHECK_ARG(ws && ws_bytes >= mmdx_bias_grad_workspace_size(M, N),
                 "bias_grad: workspace too small");
  hipStream_t st = (hipStream_t)stream;
  if (N % vec == 0 && ((uintptr_t)dy & 15) == 0)
    DISPATCH_T(dtype, hipLaunchKernelGGL(bias_grad_partial_kernel<T>,
                                         dim3((N / vec + 63) / 64, nb), dim3(256), 0, st,
                                         (const T*)dy, M, N, (float*)ws, rows));
  else
    DISPATCH_T(dtype, hipLaunchKernelGGL(bias_grad_partial_scalar_kernel<T>,
                                         dim3((N + 255) / 256, nb), dim3(256), 0, st,
                                         (const T*)dy, M, N, (float*)ws, rows));
  hipLaunchKernelGGL(bias_grad_finalize_kernel, dim3((N + 63) / 64), dim3(256), 0, st,
                     (const float*)ws, nb, N, db, beta_acc);
  MMDX_LAUNCH_CHECK();
  return 0;
}

extern "C" int mmdx_dropout_fwd(int dtype, const void* x, long n, float p, uint64_t seed,
                                uint64_t offset, uint64_t* counter, void* y, uint8_t* mask,
                                void* stream) {
  MMDX_CHECK_ARG(p >= 0.f && p < 1.f, "dropout: p out of range");
  DISPATCH_T(dtype, hipLaunchKernelGGL(dropout_fwd_kernel<T>, dim3(grid_for(n)), dim3(256), 0,
                                       (hipStream_t)stream, (const T*)x, n, p, seed, offset,
                                       (const uint64_t*)counter, (T*)y, mask));
  if (counter)
    hipLaunchKernelGGL(counter_incr_kernel, dim3(1), dim3(1), 0, (hipStream_t)stream, counter);
  MMDX_LAUNCH_CHECK();
  return 0;
}

extern "C" int mmdx_dropout_bwd(int dtype, const void* dy, const uint8_t* mask, long n, float p,
                                void* dx, void* stream) {
  DISPATCH_T(dtype, hipLaunchKernelGGL(dropout_bwd_kernel<T>, dim3(grid_for(n)), dim3(256), 0,
                                       (hipStream_t)stream, (const T*)dy, mask, n, p, (T*)dx));
  MMDX_LAUNCH_CHECK();
  return 0;
}

extern "C" int mmdx_bce_logits_fwd(const float* logits, const float* target, int B, int C,
                                   float* loss, void* stream) {
  MMDX_CHECK_ARG(B > 0 && C > 0, "bce: empty");
  hipLaunchKernelGGL(bce_fwd_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, logits, target,
                     B * C, loss);
  MMDX_LAUNCH_CHECK();
  return 0;
}

extern "C" int mmdx_bce_logits_bwd(const float* logits, const float* target, int B, int C,
                                   const float* dloss, float* dlogits, void* stream) {
  const int n = B * C;
  hipLaunchKernelGGL(bce_bwd_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream,
                     logits, target, n, dloss, dlogits);
  MMDX_LAUNCH_CHECK();
  return 0;
}

extern "C" int mmdx_axpby(long n, float a, const float* x, float b, const float* y, float* out,
                          void* stream) {
  hipLaunchKernelGGL(axpby_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, n, a, x,
                     b, y, out);
  MMDX_LAUNCH_CHECK();
  return 0;
}
