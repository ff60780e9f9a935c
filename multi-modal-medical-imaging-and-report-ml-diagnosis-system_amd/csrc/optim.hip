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

__global__ void step_incr_kernel(float* step, const float* found_inf) {
  if (found_inf && found_inf[0] != 0.f) return;  // GradScaler: an overflowed step is skipped
  step[0] += 1.f;
}

// 16-B vectors per thread per loop iteration of the AdamW update
constexpr int ADAMW_U = 4;

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
                                                    const float* __restrict__ gscale,
                                                    const float* __restrict__ found_inf) {
  if (found_inf && found_inf[0] != 0.f) return;
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
    f32x4* P = (f32x4*)d.p;
    f32x4* Mv = (f32x4*)d.m;
    f32x4* Vv = (f32x4*)d.v;
    const f32x4* G = (const f32x4*)d.g;
    // ADAMW_U vectors per thread per iteration, all loads issued before any store (the
    // stores may alias the next iteration's loads as far as the compiler knows, so a
    // one-vector loop kept one 64-B group of loads in flight per thread)
    long i = threadIdx.x;
    for (; i + (ADAMW_U - 1) * (long)blockDim.x < nv; i += ADAMW_U * (long)blockDim.x) {
      f32x4 p[ADAMW_U], m[ADAMW_U], v[ADAMW_U], g[ADAMW_U];
#pragma unroll
      for (int u = 0; u < ADAMW_U; ++u) {
        const long k = i + u * (long)blockDim.x;
        p[u] = P[k];
        m[u] = Mv[k];
        v[u] = Vv[k];
        g[u] = G[k];
      }
#pragma unroll
      for (int u = 0; u < ADAMW_U; ++u)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          float pj = p[u][j], mj = m[u][j], vj = v[u][j];
          adamw_elem(pj, g[u][j] * gs, mj, vj, decay, beta1, beta2, step_size, bc2s, eps);
          p[u][j] = pj;
          m[u][j] = mj;
          v[u][j] = vj;
        }
#pragma unroll
      for (int u = 0; u < ADAMW_U; ++u) {
        const long k = i + u * (long)blockDim.x;
        P[k] = p[u];
        Mv[k] = m[u];
        Vv[k] = v[u];
      }
    }
    for (; i < nv; i += blockDim.x) {
      f32x4 p = P[i], m = Mv[i], v = Vv[i];
      const f32x4 g = G[i];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float pj = p[j], mj = m[j], vj = v[j];
        adamw_elem(pj, g[j] * gs, mj, vj, decay, beta1, beta2, step_size, bc2s, eps);
        p[j] = pj;
        m[j] = mj;
        v[j] = vj;
      }
      P[i] = p;
      Mv[i] = m;
      Vv[i] = v;
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
  bool bad = false;  // a non-finite element (torch's per-element inf/NaN check)
  long i0 = 0;
  if (aligned16(d.g)) {
    const long nv = d.n / 4;
    for (long i = threadIdx.x; i < nv; i += blockDim.x) {
      const f32x4 g = ((const f32x4*)d.g)[i];
      bad |= !(isfinite(g[0]) && isfinite(g[1]) && isfinite(g[2]) && isfinite(g[3]));
      acc += g[0] * g[0] + g[1] * g[1] + g[2] * g[2] + g[3] * g[3];
    }
    i0 = nv * 4;
  }
  for (long i = i0 + threadIdx.x; i < d.n; i += blockDim.x) {
    bad |= !isfinite(d.g[i]);
    acc += d.g[i] * d.g[i];
  }
  acc = block_sum<256>(acc, red);
  bad = __syncthreads_or(bad);
  // the sum of squares passes through unchanged (an inf gradient gives +inf, a NaN one NaN,
  // as torch's norm); a chunk holding an inf/NaN element sets the partial's sign bit (a sum of
  // squares is otherwise >= 0, so the bit is free) — finite gradients whose squares overflow
  // give +inf without it, and norm_finalize raises found_inf only for the flagged ones
  if (threadIdx.x == 0) part[blockIdx.x] = bad ? copysignf(acc, -1.f) : acc;
}

// norm = sqrt(sum of partials); scale = clip coefficient (torch.nn.utils.clip_grad_norm_:
// min(1, max_norm / (norm + 1e-6))).  AMP form (loss_scale != NULL, torch.amp.GradScaler):
// the gradients hold loss_scale * g; found_inf = 1 when some gradient is inf/NaN; with
// unscale_first the clip sees the unscaled norm (scaler.unscale_ before the clip), otherwise
// the scaled one (the reference's order, TP:1056-1060: clip, then scaler.step unscales);
// scale additionally carries 1/loss_scale, so AdamW's grad_scale does the unscale.
__global__ __launch_bounds__(256) void norm_finalize_kernel(const float* __restrict__ part, int n,
                                                            float max_norm, float* norm,
                                                            float* scale,
                                                            const float* __restrict__ loss_scale,
                                                            int unscale_first, float* found_inf) {
  __shared__ float red[4];
  float acc = 0.f;
  bool bad = false;
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const float v = part[i];
    bad |= signbit(v);
    acc += fabsf(v);
  }
  acc = block_sum<256>(acc, red);
  bad = __syncthreads_or(bad);
  if (threadIdx.x == 0) {
    float nrm = sqrtf(acc);
    const float inv = loss_scale ? 1.f / loss_scale[0] : 1.f;
    if (loss_scale && unscale_first) nrm *= inv;
    norm[0] = nrm;
    // torch.nn.utils.clip_grad_norm_: clamp(max_norm / (norm + 1e-6), max=1) — 0 for an inf
    // norm, NaN for a NaN one (clamp keeps a NaN; fminf would return 1)
    float s = 1.f;
    if (max_norm > 0.f) {
      const float c = max_norm / (nrm + 1e-6f);
      s = isnan(c) ? c : fminf(1.f, c);
    }
    if (scale) scale[0] = s * inv;
    // found_inf: some gradient element is inf/NaN (its chunk's partial carries the sign
    // flag), as torch._amp_foreach_non_finite_check_and_unscale_; an overflow of the sum of
    // squares of finite gradients is not an overflow of the gradients
    if (found_inf) found_inf[0] = bad ? 1.f : 0.f;
  }
}

// torch._amp_update_scale_: overflow -> scale *= backoff, tracker = 0; otherwise tracker += 1
// and every `interval` clean steps scale *= growth (kept only while finite).
__global__ void amp_update_scale_kernel(float* scale, int* tracker, const float* found_inf,
                                        float growth, float backoff, int interval) {
  if (found_inf[0] != 0.f) {
    scale[0] *= backoff;
    tracker[0] = 0;
  } else {
    const int t = tracker[0] + 1;
    if (t == interval) {
      const float g = scale[0] * growth;
      if (isfinite(g)) scale[0] = g;
      tracker[0] = 0;
    } else {
      tracker[0] = t;
    }
  }
}

// out[i] = x[i] * s[0] (fp32; the loss scaling multiply and its backward)
__global__ void mul_dev_scalar_kernel(const float* __restrict__ x, long n,
                                      const float* __restrict__ s, float* __restrict__ out) {
  const float v = s[0];
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n;
       i += (long)gridDim.x * blockDim.x)
    out[i] = x[i] * v;
}

// Per-step refresh of the table's gradient column from kernel arguments (no host->device
// copy): row r of tensor t = row_tensor[r] in [t0, t0 + n) gets g = grads[t - t0] + off.
constexpr int kPatchPtrs = 256;
struct PatchArgs { const float* g[kPatchPtrs]; };

__global__ __launch_bounds__(256) void patch_grads_kernel(mmdx_adamw_tensor* __restrict__ tab,
                                                          const int* __restrict__ row_tensor,
                                                          int nchunks, int t0, int n,
                                                          PatchArgs a) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= nchunks) return;
  const int t = row_tensor[r] - t0;
  if (t < 0 || t >= n) return;
  tab[r].g = a.g[t] + tab[r].off;
}

}  // namespace mmdx

using namespace mmdx;

extern "C" int mmdx_adamw_multi_amp(int nchunks, const mmdx_adamw_tensor* table, float beta1,
                                    float beta2, float eps, float* step_dev,
                                    const float* grad_scale, const float* found_inf,
                                    void* stream) {
  MMDX_CHECK_ARG(nchunks > 0 && table && step_dev, "adamw: bad args");
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(step_incr_kernel, dim3(1), dim3(1), 0, st, step_dev, found_inf);
  hipLaunchKernelGGL(adamw_kernel, dim3(nchunks), dim3(256), 0, st, table, beta1, beta2, eps,
                     (const float*)step_dev, grad_scale, found_inf);
  MMDX_LAUNCH_CHECK();
  return 0;
}

extern "C" int mmdx_adamw_multi(int nchunks, const mmdx_adamw_tensor* table, float beta1,
                                float beta2, float eps, float* step_dev,
                                const float* grad_scale, void* stream) {
  return mmdx_adamw_multi_amp(nchunks, table, beta1, beta2, eps, step_dev, grad_scale, nullptr,
                              stream);
}

extern "C" int mmdx_amp_update_scale(float* scale, int* growth_tracker, const float* found_inf,
                                     float growth_factor, float backoff_factor,
                                     int growth_interval, void* stream) {
  MMDX_CHECK_ARG(scale && growth_tracker && found_inf && growth_interval > 0,
                 "amp_update_scale: bad args");
  hipLaunchKernelGGL(amp_update_scale_kernel, dim3(1), dim3(1), 0, (hipStream_t)stream, scale,
                     growth_tracker, found_inf, growth_factor, backoff_factor, growth_interval);
  MMDX_LAUNCH_CHECK();
  return 0;
}

extern "C" int mmdx_mul_dev_scalar(const float* x, long n, const float* s, float* out,
                                   void* stream) {
  MMDX_CHECK_ARG(x && s && out && n >= 0, "mul_dev_scalar: bad args");
  if (n == 0) return 0;
  const int blocks = (int)std::min<long>((n + 255) / 256, 4096);
  hipLaunchKernelGGL(mul_dev_scalar_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, x,
                     n, s, out);
  MMDX_LAUNCH_CHECK();
  return 0;
}

extern "C" size_t mmdx_grad_norm_workspace_size(int nchunks) {
  return (size_t)std::max(nchunks, 1) * sizeof(float);
}

extern "C" int mmdx_grad_norm_amp(int nchunks, const mmdx_adamw_tensor* table, float max_norm,
                                  const float* loss_scale, int unscale_first, float* norm,
                                  float* scale, float* found_inf, void* ws, size_t ws_bytes,
                                  void* stream) {
  MMDX_CHECK_ARG(nchunks > 0 && table && norm, "grad_norm: bad args");
  MMDX_CHECK_ARG(ws && ws_bytes >= mmdx_grad_norm_workspace_size(nchunks),
                 "grad_norm: workspace");
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(sumsq_kernel, dim3(nchunks), dim3(256), 0, st, table, (float*)ws);
  hipLaunchKernelGGL(norm_finalize_kernel, dim3(1), dim3(256), 0, st, (const float*)ws, nchunks,
                     max_norm, norm, scale, loss_scale, unscale_first, found_inf);
  MMDX_LAUNCH_CHECK();
  return 0;
}

extern "C" int mmdx_grad_norm(int nchunks, const mmdx_adamw_tensor* table, float max_norm,
                              float* norm, float* scale, void* ws, size_t ws_bytes,
                              void* stream) {
  return mmdx_grad_norm_amp(nchunks, table, max_norm, nullptr, 0, norm, scale, nullptr, ws,
                            ws_bytes, stream);
}

extern "C" int mmdx_scale_grads(int nchunks, const mmdx_adamw_tensor* table, const float* scale,
                                void* stream) {
  MMDX_CHECK_ARG(nchunks > 0 && table && scale, "scale_grads: bad args");
  hipLaunchKernelGGL(scale_grads_kernel, dim3(nchunks), dim3(256), 0, (hipStream_t)stream, table,
                     scale);
  MMDX_LAUNCH_CHECK();
  return 0;
}

extern "C" int mmdx_adamw_patch_grads(int nchunks, mmdx_adamw_tensor* table,
                                      const int* row_tensor, int n_tensors,
                                      const float* const* grads, void* stream) {
  MMDX_CHECK_ARG(nchunks > 0 && table && row_tensor && grads && n_tensors > 0,
                 "adamw_patch_grads: bad args");
  hipStream_t st = (hipStream_t)stream;
  for (int t0 = 0; t0 < n_tensors; t0 += kPatchPtrs) {
    PatchArgs a{};
    const int n = std::min(kPatchPtrs, n_tensors - t0);
    for (int j = 0; j < n; ++j) a.g[j] = grads[t0 + j];
    hipLaunchKernelGGL(patch_grads_kernel, dim3((nchunks + 255) / 256), dim3(256), 0, st, table,
                       row_tensor, nchunks, t0, n, a);
  }
  MMDX_LAUNCH_CHECK();
  return 0;
}
