// Multi-tensor AdamW (torch.optim.AdamW semantics) and global grad-norm clipping.
//
// The host splits every parameter tensor of every group into <= 64K-element chunks and
// uploads one descriptor per chunk (pointers already offset to the chunk); the kernel
// runs one workgroup per chunk with 16-B vector loads — no per-element tensor lookup.
// The step counter is a device scalar, so the update replays inside a hipGraph.
#include <algorithm>

#include "common.h"
#include "../../include/mmdx.h"

namespace mmdx {

__global__ void step_incr_kernel(float* step) { step[0] += 1.f; }

__device__ __forceinline__ bool aligned16(const void* p) { return ((uintptr_t)p & 15) == 0; }

// p <- p*(1-lr*wd); m <- lerp(m, g, 1-b1); v <- b2*v + (1-b2) g^2;
// p <- p - lr/bc1 * m / (sqrt(v)/sqrt(bc2) + eps)
__device__ __forceinline__ void adamw_elem(float& p, float g, float& m, float& v, float decay,
                                           float b1, float b2, float step_size, float bc2s,
                                           float eps) {
  p *= decay;
  m = m + (1.f - b1) * (g - m);
  v = v * b2 + (1.f - b2) * g * g;
  p = p - step_size * (m / (sqrtf(v) / bc2s + eps));
}

__global__ __launch_bounds__(256) void adamw_kernel(const mmdx_adamw_tensor* __restrict__ tab,
                                                    float beta1, float beta2, float eps,
                                                    const float* __restrict__ step,
                                                    const float* __restrict__ gscale) {
  const mmdx_adamw_tensor d = tab[blockIdx.x];
  const double s = (double)step[0];
  const double bc1 = 1.0 - pow((double)beta1, s);
  const float bc2s = (float)sqrt(1.0 - pow((double)beta2, s));
  const float gs = gscale ? gscale[0] : 1.f;
  const float step_size = (float)(d.lr / bc1);
  const float decay = 1.f - d.lr * d.wd;
  const long n = d.n;
  long i0 = 0;
  if (aligned16(d.p) && aligned16(d.g) && aligned16(d.m) && aligned16(d.v)) {
    const long nv = n / 4;
    for (long i = threadIdx.x; i < nv; i += blockDim.x) {
      f32x4 p = ((f32x4*)d.p)[i], m = ((f32x4*)d.m)[i], v = ((f32x4*)d.v)[i];
      const f32x4 g = ((const f32x4*)d.g)[i];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float pj = p[j], mj = m[j], vj = v[j];
        adamw_elem(pj, g[j] * gs, mj, vj, decay, beta1, beta2, step_size, bc2s, eps);
        p[j] = pj;
        m[j] = mj;
        v[j] = vj;
      }
      ((f32x4*)d.p)[i] = p;
      ((f32x4*)d.m)[i] = m;
      ((f32x4*)d.v)[i] = v;
    }
    i0 = nv * 4;
  }
  for (long i = i0 + threadIdx.x; i < n; i += blockDim.x) {
    float p = d.p[i], m = d.m[i], v = d.v[i];
    adamw_elem(p, d.g[i] * gs, m, v, decay, beta1, beta2, step_size, bc2s, eps);
    d.p[i] = p;
    d.m[i] = m;
    d.v[i] = v;
  }
}

__global__ __launch_bounds__(256) void scale_grads_kernel(const mmdx_adamw_tensor* __restrict__ tab,
                                                          const float* __restrict__ scale) {
  const mmdx_adamw_tensor d = tab[blockIdx.x];
  const float s = scale[0];
  float* g = (float*)d.g;
  for (long i = threadIdx.x; i < d.n; i += blockDim.x) g[i] *= s;
}

__global__ __launch_bounds__(256) void sumsq_kernel(const mmdx_adamw_tensor* __restrict__ tab,
                                                    float* __restrict__ part) {
  __shared__ float red[4];
  const mmdx_adamw_tensor d = tab[blockIdx.x];
  float acc = 0.f;
  long i0 = 0;
  if (aligned16(d.g)) {
    const long nv = d.n / 4;
    for (long i = threadIdx.x; i < nv; i += blockDim.x) {
      const f32x4 g = ((const f32x4*)d.g)[i];
      acc += g[0] * g[0] + g[1] * g[1] + g[2] * g[2] + g[3] * g[3];
    }
    i0 = nv * 4;
  }
  for (long i = i0 + threadIdx.x; i < d.n; i += blockDim.x) acc += d.g[i] * d.g[i];
  acc = block_sum<256>(acc, red);
  if (threadIdx.x == 0) part[blockIdx.x] = acc;
}

__global__ __launch_bounds__(256) void norm_finalize_kernel(const float* __restrict__ part, int n,
                                                            float max_norm, float* norm,
                                                            float* scale) {
  __shared__ float red[4];
  float acc = 0.f;
  for (int i = threadIdx.x; i < n; i += blockDim.x) acc += part[i];
  acc = block_sum<256>(acc, red);
  if (threadIdx.x == 0) {
    const float nrm = sqrtf(acc);
    norm[0] = nrm;
    if (scale) scale[0] = max_norm > 0.f ? fminf(1.f, max_norm / (nrm + 1e-6f)) : 1.f;
  }
}

}  // namespace mmdx

using namespace mmdx;

extern "C" int mmdx_adamw_multi(int nchunks, const mmdx_adamw_tensor* table, float beta1,
                                float beta2, float eps, float* step_dev,
                                const float* grad_scale, void* stream) {
  MMDX_CHECK_ARG(nchunks > 0 && table && step_dev, "adamw: bad args");
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(step_incr_kernel, dim3(1), dim3(1), 0, st, step_dev);
  hipLaunchKernelGGL(adamw_kernel, dim3(nchunks), dim3(256), 0, st, table, beta1, beta2, eps,
                     (const float*)step_dev, grad_scale);
  MMDX_LAUNCH_CHECK();
  return 0;
}

extern "C" size_t mmdx_grad_norm_workspace_size(int nchunks) {
  return (size_t)std::max(nchunks, 1) * sizeof(float);
}

extern "C" int mmdx_grad_norm(int nchunks, const mmdx_adamw_tensor* table, float max_norm,
                              float* norm, float* scale, void* ws, size_t ws_bytes,
                              void* stream) {
  MMDX_CHECK_ARG(nchunks > 0 && table && norm, "grad_norm: bad args");
  MMDX_CHECK_ARG(ws && ws_bytes >= mmdx_grad_norm_workspace_size(nchunks),
                 "grad_norm: workspace");
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(sumsq_kernel, dim3(nchunks), dim3(256), 0, st, table, (float*)ws);
  hipLaunchKernelGGL(norm_finalize_kernel, dim3(1), dim3(256), 0, st, (const float*)ws, nchunks,
                     max_norm, norm, scale);
  MMDX_LAUNCH_CHECK();
  return 0;
}

extern "C" int mmdx_scale_grads(int nchunks, const mmdx_adamw_tensor* table, const float* scale,
                                void* stream) {
  MMDX_CHECK_ARG(nchunks > 0 && table && scale, "scale_grads: bad args");
  hipLaunchKernelGGL(scale_grads_kernel, dim3(nchunks), dim3(256), 0, (hipStream_t)stream, table,
                     scale);
  MMDX_LAUNCH_CHECK();
  return 0;
}
