// ViT-B/16 image tower pieces (build-defined C5 backbone, SURVEY §8 a1: torchvision
// vit_b_16 semantics): patchify for the 16x16/16 patch-embedding GEMM, class-token +
// position-embedding token assembly, strided row copies (class-token rows), and a
// dtype-generic elementwise add for residual gradient sums.  The encoder blocks run on
// the GEMM / attention / LayerNorm kernels.
#include <algorithm>

#include "common.h"
#include "../../include/mmdx.h"

namespace mmdx {

static int vgrid(long n, int per = 256) {
  return (int)std::max<long>(1, std::min<long>((n + per - 1) / per, 8192));
}

// x NCHW fp32 [N][C][H][W] -> patches [N * (H/p) * (W/p)][C*p*p] in (c, ky, kx) order
// (the flattening of a Conv2d weight [D][C][p][p]); one thread per 8 consecutive kx.
template <typename T>
__global__ void patchify_kernel(const float* __restrict__ x, int N, int C, int H, int W, int p,
                                T* __restrict__ out) {
  const int gh = H / p, gw = W / p, K = C * p * p, kv = K / 8;
  const long total = (long)N * gh * gw * kv;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total;
       i += (long)gridDim.x * blockDim.x) {
    const int k8 = (int)(i % kv);
    const long row = i / kv;
    const int n = (int)(row / (gh * gw)), rem = (int)(row % (gh * gw));
    const int py = rem / gw, px = rem - py * gw;
    const int k = k8 * 8, c = k / (p * p), r = k - c * p * p, ky = r / p, kx = r - ky * p;
    const float* src = x + (((long)n * C + c) * H + py * p + ky) * W + px * p + kx;
    typename Vec16<T>::type o;
    if constexpr (sizeof(T) == 2) {
      const f32x4 a = *(const f32x4*)src, b = *(const f32x4*)(src + 4);
#pragma unroll
      for (int j = 0; j < 4; ++j) { o[j] = from_f<T>(a[j]); o[4 + j] = from_f<T>(b[j]); }
      *(typename Vec16<T>::type*)(out + row * K + k) = o;
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) out[row * K + k + j] = from_f<T>(src[j]);
    }
  }
}

// tokens[n][0] = cls + pos[0]; tokens[n][1 + q] = emb[n][q] + pos[1 + q]
template <typename T>
__global__ void vit_tokens_fwd_kernel(const T* __restrict__ emb, const float* __restrict__ cls,
                                      const float* __restrict__ pos, int N, int S, int D,
                                      T* __restrict__ tok) {
  const long total = (long)N * S * D;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total;
       i += (long)gridDim.x * blockDim.x) {
    const int d = (int)(i % D);
    const long r = i / D;
    const int s = (int)(r % S);
    const long n = r / S;
    const float v = s == 0 ? cls[d] : to_f(emb[(n * (S - 1) + s - 1) * D + d]);
    tok[i] = from_f<T>(v + pos[(long)s * D + d]);
  }
}

// demb[n][q] = dtok[n][1 + q]  (the cls / pos gradients are column sums: mmdx_bias_grad)
template <typename T>
__global__ void vit_tokens_bwd_kernel(const T* __restrict__ dtok, int N, int S, int D,
                                      T* __restrict__ demb) {
  const long total = (long)N * (S - 1) * D;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total;
       i += (long)gridDim.x * blockDim.x) {
    const int d = (int)(i % D);
    const long r = i / D;
    const long n = r / (S - 1);
    const int q = (int)(r % (S - 1));
    demb[i] = dtok[(n * S + 1 + q) * D + d];
  }
}

template <typename T>
__global__ void rows_copy_kernel(const T* __restrict__ src, long src_ld, T* __restrict__ dst,
                                 long dst_ld, long rows, int D) {
  const long total = rows * D;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total;
       i += (long)gridDim.x * blockDim.x) {
    const long r = i / D;
    const int d = (int)(i - r * D);
    dst[r * dst_ld + d] = src[r * src_ld + d];
  }
}

template <typename T>
__global__ void add_kernel(long n, const T* __restrict__ x, const T* __restrict__ y,
                           T* __restrict__ out) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n;
       i += (long)gridDim.x * blockDim.x)
    out[i] = from_f<T>(to_f(x[i]) + to_f(y[i]));
}

}  // namespace mmdx

using namespace mmdx;

#define VIT_DISPATCH(dtype, ...) MMDX_DISPATCH(dtype, __VA_ARGS__)

extern "C" int mmdx_patchify(int dtype, const float* x, int N, int C, int H, int W, int p,
                             void* out, void* stream) {
  MMDX_CHECK_ARG(N > 0 && p > 0 && H % p == 0 && W % p == 0 && (C * p * p) % 8 == 0 && p % 8 == 0,
                 "patchify: bad shape C=%d H=%d W=%d p=%d", C, H, W, p);
  const long total = (long)N * (H / p) * (W / p) * (C * p * p / 8);
  VIT_DISPATCH(dtype, hipLaunchKernelGGL(patchify_kernel<T>, dim3(vgrid(total)), dim3(256), 0,
                                         (hipStream_t)stream, x, N, C, H, W, p, (T*)out));
  MMDX_LAUNCH_CHECK();
  return 0;
}

extern "C" int mmdx_vit_tokens_fwd(int dtype, const void* emb, const float* cls,
                                   const float* pos, int N, int S, int D, void* tokens,
                                   void* stream) {
  MMDX_CHECK_ARG(N > 0 && S > 1 && D > 0, "vit tokens: bad shape");
  const long total = (long)N * S * D;
  VIT_DISPATCH(dtype, hipLaunchKernelGGL(vit_tokens_fwd_kernel<T>, dim3(vgrid(total)),
                                         dim3(256), 0, (hipStream_t)stream, (const T*)emb, cls,
                                         pos, N, S, D, (T*)tokens));
  MMDX_LAUNCH_CHECK();
  return 0;
}

extern "C" int mmdx_vit_tokens_bwd(int dtype, const void* dtokens, int N, int S, int D,
                                   void* demb, void* stream) {
  MMDX_CHECK_ARG(N > 0 && S > 1 && D > 0, "vit tokens bwd: bad shape");
  const long total = (long)N * (S - 1) * D;
  VIT_DISPATCH(dtype, hipLaunchKernelGGL(vit_tokens_bwd_kernel<T>, dim3(vgrid(total)),
                                         dim3(256), 0, (hipStream_t)stream, (const T*)dtokens,
                                         N, S, D, (T*)demb));
  MMDX_LAUNCH_CHECK();
  return 0;
}

extern "C" int mmdx_rows_copy(int dtype, const void* src, long src_ld, void* dst, long dst_ld,
                              long rows, int D, void* stream) {
  MMDX_CHECK_ARG(rows > 0 && D > 0 && src_ld >= D && dst_ld >= D, "rows_copy: bad shape");
  VIT_DISPATCH(dtype, hipLaunchKernelGGL(rows_copy_kernel<T>, dim3(vgrid(rows * D)), dim3(256),
                                         0, (hipStream_t)stream, (const T*)src, src_ld, (T*)dst,
                                         dst_ld, rows, D));
  MMDX_LAUNCH_CHECK();
  return 0;
}

extern "C" int mmdx_add(int dtype, long n, const void* x, const void* y, void* out,
                        void* stream) {
  MMDX_CHECK_ARG(n > 0, "add: empty");
  VIT_DISPATCH(dtype, hipLaunchKernelGGL(add_kernel<T>, dim3(vgrid(n)), dim3(256), 0,
                                         (hipStream_t)stream, n, (const T*)x, (const T*)y,
                                         (T*)out));
  MMDX_LAUNCH_CHECK();
  return 0;
}
