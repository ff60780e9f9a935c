// Shared device/host helpers for the mmdx HIP library (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <stdint.h>
#include <stddef.h>

namespace mmdx {

typedef __bf16 bf16;
typedef _Float16 f16;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(8))) _Float16 f16x8;
typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(2))) float f32x2;
typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;
typedef __attribute__((ext_vector_type(4))) short s16x4;

enum Dtype { F32 = 0, BF16 = 1, F16 = 2 };
enum Act { ACT_NONE = 0, ACT_RELU = 1, ACT_GELU = 2, ACT_GELU_BWD = 3 };

constexpr int WAVE = 64;

// Launch-heuristic knobs (MMDX_* environment variables, documented where each is used), read
// ONCE per process into this read-only struct instead of a getenv walk per launch (158 conv
// launches per C4 step used to read up to 14 of them each).  mmdx_reload_config() re-reads the
// environment: tests and A/B runs that switch a knob call it between launches, never while one
// is being issued.
struct Knobs {
  int conv_n64_wide;      // MMDX_CONV_N64_WIDE: -1 auto (>= 1024 256-row blocks), 0 off, 1 on
  bool conv_8w128;        // MMDX_CONV_8W128 (default on)
  bool stem_direct;       // MMDX_STEM_DIRECT (default on)
  long wgrad_target;      // MMDX_WGRAD_TARGET: conv weight-gradient split-K blocks (256)
  bool wgrad_rq;          // MMDX_WGRAD_RQ (default on)
  long gemm256_fwd_min;   // MMDX_GEMM256_FWD_MIN: 256 x 256 forward tiles from this many (90)
  bool gemm_8w128;        // MMDX_GEMM_8W128 (default on)
  long splitk_target;     // MMDX_SPLITK_TARGET: dense split-K blocks (256)
  bool splitk_vec;        // MMDX_SPLITK_VEC (default on)
  bool wgrad_bias_fused;  // MMDX_WGRAD_BIAS_FUSED (default on)
  bool bias_grad_gemm;    // MMDX_BIAS_GRAD_GEMM (default off)
  int ln_bwd_rpw;         // MMDX_LN_BWD_RPW: 4 | 8 (8)
  int attn_fwd_nw;        // MMDX_ATTN_FWD_NW: raw value (0 = unset)
  int attn_bwd_nw;        // MMDX_ATTN_BWD_NW: raw value (0 = unset)
  bool lstm_bwd_probe;    // MMDX_LSTM_BWD_PROBE: lab phase stamps (tools/lab/lstm_probe.py)
};
const Knobs& knobs();

__device__ __forceinline__ float to_f(float x) { return x; }
__device__ __forceinline__ float to_f(bf16 x) { return (float)x; }
__device__ __forceinline__ float to_f(f16 x) { return (float)x; }
template <typename T> __device__ __forceinline__ T from_f(float x);
template <> __device__ __forceinline__ float from_f<float>(float x) { return x; }
template <> __device__ __forceinline__ bf16 from_f<bf16>(float x) { return (bf16)x; }
template <> __device__ __forceinline__ f16 from_f<f16>(float x) { return (f16)x; }

// 16-byte vector of T: 8 bf16 or 4 f32.
template <typename T> struct Vec16;
template <> struct Vec16<bf16> { static constexpr int N = 8; typedef bf16x8 type; };
template <> struct Vec16<float> { static constexpr int N = 4; typedef f32x4 type; };
template <> struct Vec16<f16> { static constexpr int N = 8; typedef f16x8 type; };

// The element-type dispatch of every C-ABI entry: `dtype` (MMDX_F32 / _BF16 / _F16) picks T
// for the statement(s).  One macro for the whole library.
#define MMDX_DISPATCH(dtype, ...)                  \
  do {                                             \
    if ((dtype) == ::mmdx::BF16) {                 \
      typedef ::mmdx::bf16 T;                      \
      __VA_ARGS__;                                 \
    } else if ((dtype) == ::mmdx::F16) {           \
      typedef ::mmdx::f16 T;                       \
      __VA_ARGS__;                                 \
    } else {                                       \
      typedef float T;                             \
      __VA_ARGS__;                                 \
    }                                              \
  } while (0)

// exact (erf) GELU as torch.nn.GELU() default / BERT "gelu"
__device__ __forceinline__ float gelu_erf(float x) {
  return 0.5f * x * (1.0f + erff(x * 0.70710678118654752f));
}
__device__ __forceinline__ float gelu_erf_grad(float x) {
  const float cdf = 0.5f * (1.0f + erff(x * 0.70710678118654752f));
  const float pdf = 0.39894228040143268f * __expf(-0.5f * x * x);
  return cdf + x * pdf;
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Block-wide sum for blockDim.x == NT (multiple of 64); `red` needs NT/64 floats.
template <int NT>
__device__ __forceinline__ float block_sum(float v, float* red) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  if (l == 0) red[w] = v;
  __syncthreads();
  float t = 0.f;
#pragma unroll
  for (int i = 0; i < NT / 64; ++i) t += red[i];
  __syncthreads();
  return t;
}

// elementwise launch geometry: grid-stride loops over at most 8192 blocks of 256
static inline int grid_for(long n, int per = 256) {
  return (int)std::max<long>(1, std::min<long>((n + per - 1) / per, 8192));
}

#define GRID_STRIDE(i, n) \
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < (n); i += (long)gridDim.x * blockDim.x)

}  // namespace mmdx

// Error plumbing for the C ABI (defined in capi.cpp).
extern "C" void mmdx_set_error(const char* fmt, ...);

#define MMDX_CHECK_ARG(cond, ...)                     \
  do {                                               \
    if (!(cond)) {                                   \
      mmdx_set_error(__VA_ARGS__);                   \
      return -22; /* -EINVAL */                      \
    }                                                \
  } while (0)

#define MMDX_LAUNCH_CHECK()                                          \
  do {                                                               \
    hipError_t _e = hipGetLastError();                               \
    if (_e != hipSuccess) {                                          \
      mmdx_set_error("HIP launch failed: %s", hipGetErrorString(_e)); \
      return -(int)_e;                                               \
    }                                                                \
  } while (0)
