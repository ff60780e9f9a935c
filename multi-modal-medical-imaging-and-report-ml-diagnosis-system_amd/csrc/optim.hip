// Multi-tensor AdamW (torch.optim.AdamW semantics) and global grad-norm clipping.
// One launch updates every parameter of every group: the per-tensor table lives in HBM
// and the step counter is a device scalar, so the update replays inside a hipGraph.
#include <algorithm>

#include "common.h"
#include "../../include/mmdx.h"

namespace mmdx {

__device__ __forceinline__ int find_tensor(const mmdx_adamw_tensor* __restrict__ tab, int nt,
                                           long e) {
  int lo = 0, hi = nt - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (tab[mid].off <= e) lo = mid; else hi = mid - 1;
  }
  return lo;
}

__global__ void step_incr_kernel(float* step) { step[0] += 1.f; }

// p <- p*(1-lr*wd); m <- lerp(m, g, 1-b1); v <- b2*v + (1-b2) g^2;
// p <- p - lr/bc1 * m / (sqrt(v)/sqrt(bc2) + eps)
__global__ void adamw_kernel(const mmdx_adamw_tensor* __restrict__ tab, int nt, long total,
                             float beta1, float beta2, float eps, const float* __restrict__ step,
                             const float* __restrict__ gscale) {
  const double s = (double)step[0];
  const double bc1 = 1.0 - pow((double)beta1, s);
  const double bc2 = 1.0 - pow((double)beta2, s);
  const float bc2_sqrt = (float)sqrt(bc2);
  const float gs = gscale ? gscale[0] : 1.f;
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < total;
       e += (long)gridDim.x * blockDim.x) {
    const int t = find_tensor(tab, nt, e);
    const mmdx_adamw_tensor d = tab[t];
    const long i = e - d.off;
    const float g = d.g[i] * gs;
    float p = d.p[i];
    p *= 1.f - d.lr * d.wd;
    float m = d.m[i];
    m = m + (1.f - beta1) * (g - m);
    float v = d.v[i];
    v = v * beta2 + (1.f - beta2) * g * g;
    const float step_size = (float)(d.lr / bc1);
    const float denom = sqrtf(v) / bc2_sqrt + eps;
    p = p - step_size * (m / denom);
    d.p[i] = p;
    d.m[i] = m;
    d.v[i] = v;
  }
}

__global__ void scale_grads_kernel(const mmdx_adamw_tensor* __restrict__ tab, int nt, long total,
                                   const float* __restrict__ scale) {
  const float s = scale[0];
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < total;
       e += (long)gridDim.x * blockDim.x) {
    const int t = find_tensor(tab, nt, e);
    float* g = (float*)tab[t].g;
    g[e - tab[t].off] *= s;
  }
}

constexpr int GN_BLOCKS = 1024;

__global__ void sumsq_kernel(const mmdx_adamw_tensor* __restrict__ tab, int nt, long total,
                             float* __restrict__ part) {
  __shared__ float red[4];
  float acc = 0.f;
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < total;
       e += (long)gridDim.x * blockDim.x) {
    const int t = find_tensor(tab, nt, e);
    const float g = tab[t].g[e - tab[t].off];
    acc += g * g;
  }
  acc = block_sum<256>(acc, red);
  if (threadIdx.x == 0) part[blockIdx.x] = acc;
}

__global__ void norm_finalize_kernel(const float* __restrict__ part, int n, float max_norm,
                                     float* norm, float* scale) {
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

extern "C" int mmdx_adamw_multi(int ntensors, const mmdx_adamw_tensor* table, long total,
                                float beta1, float beta2, float eps, float* step_dev,
                                const float* grad_scale, void* stream) {
  MMDX_CHECK_ARG(ntensors > 0 && table && step_dev && total > 0, "adamw: bad args");
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(step_incr_kernel, dim3(1), dim3(1), 0, st, step_dev);
  const int blocks = (int)std::min<long>((total + 255) / 256, 8192);
  hipLaunchKernelGGL(adamw_kernel, dim3(blocks), dim3(256), 0, st, table, ntensors, total, beta1,
                     beta2, eps, (const float*)step_dev, grad_scale);
  MMDX_LAUNCH_CHECK();
  return 0;
}

extern "C" size_t mmdx_grad_norm_workspace_size(void) { return GN_BLOCKS * sizeof(float); }

extern "C" int mmdx_grad_norm(int ntensors, const mmdx_adamw_tensor* table, long total,
                              float max_norm, float* norm, float* scale, void* ws,
                              size_t ws_bytes, void* stream) {
  MMDX_CHECK_ARG(ntensors > 0 && table && norm, "grad_norm: bad args");
  MMDX_CHECK_ARG(ws && ws_bytes >= GN_BLOCKS * sizeof(float), "grad_norm: workspace");
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(sumsq_kernel, dim3(GN_BLOCKS), dim3(256), 0, st, table, ntensors, total,
                     (float*)ws);
  hipLaunchKernelGGL(norm_finalize_kernel, dim3(1), dim3(256), 0, st, (const float*)ws,
                     GN_BLOCKS, max_norm, norm, scale);
  MMDX_LAUNCH_CHECK();
  return 0;
}

extern "C" int mmdx_scale_grads(int ntensors, const mmdx_adamw_tensor* table, long total,
                                const float* scale, void* stream) {
  MMDX_CHECK_ARG(ntensors > 0 && table && scale, "scale_grads: bad args");
  const int blocks = (int)std::min<long>((total + 255) / 256, 8192);
  hipLaunchKernelGGL(scale_grads_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, table,
                     ntensors, total, scale);
  MMDX_LAUNCH_CHECK();
  return 0;
}
