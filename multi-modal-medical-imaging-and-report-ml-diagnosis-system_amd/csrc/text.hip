// Text-tower memory-bound kernels: BERT embeddings + LayerNorm, masked mean pooling,
// fused embedding-gather + masked mean (C2 tower), plain row gather/scatter (BiLSTM tower).
#include <algorithm>

#include "common.h"
#include "../../include/mmdx.h"

namespace mmdx {

constexpr int EMB_MAXE = 16;  // elements per lane: D <= 1024

// One wave per token: s = word[id] + pos[l] + type[tt]; y = LN(s).  (BertEmbeddings)
template <typename T>
__global__ __launch_bounds__(256) void embed_ln_kernel(
    const int64_t* __restrict__ ids, const int64_t* __restrict__ tt, int B, int L, int D,
    const float* __restrict__ word, const float* __restrict__ pos,
    const float* __restrict__ type, const float* __restrict__ gamma,
    const float* __restrict__ beta, float eps, T* __restrict__ y, T* __restrict__ xsum,
    float* smean, float* srstd) {
  const int lane = threadIdx.x & 63;
  const long row = blockIdx.x * 4L + (threadIdx.x >> 6);
  if (row >= (long)B * L) return;
  const int l = (int)(row % L);
  const long id = ids[row];
  const long t = tt ? tt[row] : 0;
  float v[EMB_MAXE];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < EMB_MAXE; ++i) {
    const int d = lane + i * 64;
    v[i] = 0.f;
    if (d < D) {
      v[i] = word[id * D + d] + pos[(long)l * D + d] + type[t * D + d];
      s += v[i];
      if (xsum) xsum[row * D + d] = from_f<T>(v[i]);
    }
  }
  const float mean = wave_sum(s) / D;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < EMB_MAXE; ++i)
    if (lane + i * 64 < D) q += (v[i] - mean) * (v[i] - mean);
  const float rstd = rsqrtf(wave_sum(q) / D + eps);
  if (lane == 0) { smean[row] = mean; srstd[row] = rstd; }
#pragma unroll
  for (int i = 0; i < EMB_MAXE; ++i) {
    const int d = lane + i * 64;
    if (d < D) y[row * D + d] = from_f<T>((v[i] - mean) * rstd * gamma[d] + beta[d]);
  }
}

// word-table grads: scatter-add (fp32 atomics; repeated ids collide)
template <typename T>
__global__ void embed_word_bwd_kernel(const int64_t* __restrict__ ids, long rows, int D,
                                      const T* __restrict__ ds, float* __restrict__ dword,
                                      int pad_id) {
  const long total = rows * D;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total;
       i += (long)gridDim.x * blockDim.x) {
    const long r = i / D;
    const int d = (int)(i - r * D);
    const long id = ids[r];
    if (id == pad_id) continue;  // nn.Embedding(padding_idx): no gradient for the pad row
    atomicAdd(&dword[id * D + d], to_f(ds[i]));
  }
}
// position grads: dpos[l,d] = sum_b ds[b,l,d] (deterministic)
template <typename T>
__global__ void embed_pos_bwd_kernel(const T* __restrict__ ds, int B, int L, int D,
                                     float* __restrict__ dpos) {
  const long total = (long)L * D;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total;
       i += (long)gridDim.x * blockDim.x) {
    float acc = 0.f;
    for (int b = 0; b < B; ++b) acc += to_f(ds[(long)b * L * D + i]);
    dpos[i] += acc;
  }
}
// token-type grads: dtype[t,d] += sum over rows with tt==t (deterministic).  A block owns 8
// column vectors (128 B of a row) x 32 row lanes striding all rows, then an LDS tree over the
// lanes.  (The first version ran one thread per column over every row: 3 blocks, 2.4 ms per
// C5 step.)
template <typename T>
__global__ __launch_bounds__(256) void embed_type_bwd_kernel(const int64_t* __restrict__ tt,
                                                             long rows, int D,
                                                             const T* __restrict__ ds,
                                                             float* __restrict__ dtab) {
  typedef typename Vec16<T>::type V;
  constexpr int VEC = Vec16<T>::N;
  __shared__ float red[32][8 * VEC][2];
  const int cv = threadIdx.x & 7, lane = threadIdx.x >> 3;
  const int j = blockIdx.x * 8 + cv;
  const bool ok = j < D / VEC;
  float a0[VEC], a1[VEC];
#pragma unroll
  for (int e = 0; e < VEC; ++e) a0[e] = a1[e] = 0.f;
  if (ok) {
#pragma unroll 4
    for (long r = lane; r < rows; r += 32) {
      const V v = ((const V*)(ds + r * D))[j];
      const bool one = tt && tt[r] == 1;
#pragma unroll
      for (int e = 0; e < VEC; ++e) {
        const float g = to_f(v[e]);
        a0[e] += one ? 0.f : g;
        a1[e] += one ? g : 0.f;
      }
    }
  }
#pragma unroll
  for (int e = 0; e < VEC; ++e) {
    red[lane][cv * VEC + e][0] = a0[e];
    red[lane][cv * VEC + e][1] = a1[e];
  }
  __syncthreads();
  if (threadIdx.x >= 8 * VEC * 2) return;
  const int c = threadIdx.x >> 1, t = threadIdx.x & 1;  // one (column, type) per thread
  if (blockIdx.x * 8 * VEC + c >= D) return;
  float s = 0.f;
  for (int l = 0; l < 32; ++l) s += red[l][c][t];
  dtab[(long)t * D + blockIdx.x * 8 * VEC + c] += s;
}
// D not a multiple of the vector width: one column per thread
template <typename T>
__global__ void embed_type_bwd_scalar_kernel(const int64_t* __restrict__ tt, long rows, int D,
                                             const T* __restrict__ ds, float* __restrict__ dtab) {
  const int d = blockIdx.x * blockDim.x + threadIdx.x;
  if (d >= D) return;
  float a0 = 0.f, a1 = 0.f;
  for (long r = 0; r < rows; ++r) {
    const float g = to_f(ds[r * D + d]);
    if (tt && tt[r] == 1) a1 += g; else a0 += g;
  }
  dtab[d] += a0;
  dtab[D + d] += a1;
}

// masked mean (TextEncoderTransformer.mean_pool TP:452-459)
template <typename T>
__global__ void masked_mean_fwd_kernel(const T* __restrict__ h, const int64_t* __restrict__ m,
                                       int B, int L, int D, T* __restrict__ out) {
  const long total = (long)B * D;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total;
       i += (long)gridDim.x * blockDim.x) {
    const int b = (int)(i / D), d = (int)(i % D);
    float acc = 0.f, cnt = 0.f;
    for (int l = 0; l < L; ++l) {
      const float w = (float)m[(long)b * L + l];
      acc += to_f(h[((long)b * L + l) * D + d]) * w;
      cnt += w;
    }
    out[i] = from_f<T>(acc / fmaxf(cnt, 1e-6f));
  }
}
template <typename T>
__global__ void masked_mean_bwd_kernel(const T* __restrict__ dout, const int64_t* __restrict__ m,
                                       int B, int L, int D, T* __restrict__ dh) {
  // one block per sample: token count once, then every (l, d) of the sample
  __shared__ float s_inv;
  const int b = blockIdx.x;
  if (threadIdx.x < 64) {
    float cnt = 0.f;
    for (int l = threadIdx.x; l < L; l += 64) cnt += (float)m[(long)b * L + l];
    cnt = wave_sum(cnt);
    if (threadIdx.x == 0) s_inv = 1.f / fmaxf(cnt, 1e-6f);
  }
  __syncthreads();
  const float inv = s_inv;
  for (int l = 0; l < L; ++l) {
    const float w = (float)m[(long)b * L + l] * inv;
    T* row = dh + ((long)b * L + l) * D;
    for (int d = threadIdx.x; d < D; d += blockDim.x)
      row[d] = from_f<T>(to_f(dout[(long)b * D + d]) * w);
  }
}

// fused gather + masked mean: one block per sample, threads over D
template <typename T>
__global__ void embed_mean_fwd_kernel(const int64_t* __restrict__ ids,
                                      const int64_t* __restrict__ m, int B, int L, int D,
                                      const float* __restrict__ tab, T* __restrict__ out) {
  const int b = blockIdx.x;
  float cnt = 0.f;
  for (int l = 0; l < L; ++l) cnt += (float)m[(long)b * L + l];
  const float inv = 1.f / fmaxf(cnt, 1e-6f);
  for (int d = threadIdx.x; d < D; d += blockDim.x) {
    float acc = 0.f;
    for (int l = 0; l < L; ++l) {
      const float w = (float)m[(long)b * L + l];
      if (w != 0.f) acc += tab[ids[(long)b * L + l] * D + d] * w;
    }
    out[(long)b * D + d] = from_f<T>(acc * inv);
  }
}
template <typename T>
__global__ void embed_mean_bwd_kernel(const int64_t* __restrict__ ids,
                                      const int64_t* __restrict__ m, int B, int L, int D,
                                      const T* __restrict__ dout, float* __restrict__ dtab) {
  const int b = blockIdx.x;
  float cnt = 0.f;
  for (int l = 0; l < L; ++l) cnt += (float)m[(long)b * L + l];
  const float inv = 1.f / fmaxf(cnt, 1e-6f);
  for (int l = 0; l < L; ++l) {
    const float w = (float)m[(long)b * L + l] * inv;
    if (w == 0.f) continue;
    const long row = ids[(long)b * L + l];
    for (int d = threadIdx.x; d < D; d += blockDim.x)
      atomicAdd(&dtab[row * D + d], to_f(dout[(long)b * D + d]) * w);
  }
}

template <typename T>
__global__ void gather_kernel(const int64_t* __restrict__ ids, long n, int D,
                              const float* __restrict__ tab, T* __restrict__ out) {
  const long total = n * D;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total;
       i += (long)gridDim.x * blockDim.x) {
    const long r = i / D;
    out[i] = from_f<T>(tab[ids[r] * D + (i - r * D)]);
  }
}
template <typename T>
__global__ void scatter_kernel(const int64_t* __restrict__ ids, long n, int D,
                               const T* __restrict__ dout, float* __restrict__ dtab) {
  const long total = n * D;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total;
       i += (long)gridDim.x * blockDim.x) {
    const long r = i / D;
    atomicAdd(&dtab[ids[r] * D + (i - r * D)], to_f(dout[i]));
  }
}

}  // namespace mmdx

using namespace mmdx;

#define DISPATCH_T(dtype, ...) MMDX_DISPATCH(dtype, __VA_ARGS__)

extern "C" int mmdx_embed_ln_fwd(int dtype, const int64_t* ids, const int64_t* tt, int B, int L,
                                 int D, const float* word, const float* pos, const float* type,
                                 const float* gamma, const float* beta, float eps, void* y,
                                 void* xsum, float* smean, float* srstd, void* stream) {
  MMDX_CHECK_ARG(D <= 64 * EMB_MAXE && smean && srstd, "embed_ln: D=%d unsupported", D);
  const long rows = (long)B * L;
  DISPATCH_T(dtype, hipLaunchKernelGGL(embed_ln_kernel<T>, dim3((rows + 3) / 4), dim3(256), 0,
                                       (hipStream_t)stream, ids, tt, B, L, D, word, pos, type,
                                       gamma, beta, eps, (T*)y, (T*)xsum, smean, srstd));
  MMDX_LAUNCH_CHECK();
  return 0;
}

extern "C" int mmdx_embed_bwd(int dtype, const int64_t* ids, const int64_t* tt, int B, int L,
                              int D, const void* dsum, float* dword, float* dpos,
                              float* dtype_tab, int pad_id, void* stream) {
  const long rows = (long)B * L;
  hipStream_t st = (hipStream_t)stream;
  DISPATCH_T(dtype, {
    if (dword)
      hipLaunchKernelGGL(embed_word_bwd_kernel<T>, dim3(grid_for(rows * D)), dim3(256), 0, st,
                         ids, rows, D, (const T*)dsum, dword, pad_id);
    if (dpos)
      hipLaunchKernelGGL(embed_pos_bwd_kernel<T>, dim3(grid_for((long)L * D)), dim3(256), 0, st,
                         (const T*)dsum, B, L, D, dpos);
    if (dtype_tab) {
      constexpr int VEC = Vec16<T>::N;
      if (D % VEC == 0 && ((uintptr_t)dsum & 15) == 0)
        hipLaunchKernelGGL(embed_type_bwd_kernel<T>, dim3((D / VEC + 7) / 8), dim3(256), 0, st,
                           tt, rows, D, (const T*)dsum, dtype_tab);
      else
        hipLaunchKernelGGL(embed_type_bwd_scalar_kernel<T>, dim3((D + 255) / 256), dim3(256), 0,
                           st, tt, rows, D, (const T*)dsum, dtype_tab);
    }
  });
  MMDX_LAUNCH_CHECK();
  return 0;
}

extern "C" int mmdx_masked_mean_fwd(int dtype, const void* h, const int64_t* mask, int B, int L,
                                    int D, void* out, void* stream) {
  DISPATCH_T(dtype, hipLaunchKernelGGL(masked_mean_fwd_kernel<T>, dim3(grid_for((long)B * D)),
                                       dim3(256), 0, (hipStream_t)stream, (const T*)h, mask, B,
                                       L, D, (T*)out));
  MMDX_LAUNCH_CHECK();
  return 0;
}

extern "C" int mmdx_masked_mean_bwd(int dtype, const void* dout, const int64_t* mask, int B,
                                    int L, int D, void* dh, void* stream) {
  DISPATCH_T(dtype, hipLaunchKernelGGL(masked_mean_bwd_kernel<T>, dim3(B), dim3(256), 0,
                                       (hipStream_t)stream, (const T*)dout, mask, B, L, D,
                                       (T*)dh));
  MMDX_LAUNCH_CHECK();
  return 0;
}

extern "C" int mmdx_embed_mean_fwd(int dtype, const int64_t* ids, const int64_t* mask, int B,
                                   int L, int D, const float* table, void* out, void* stream) {
  DISPATCH_T(dtype, hipLaunchKernelGGL(embed_mean_fwd_kernel<T>, dim3(B), dim3(256), 0,
                                       (hipStream_t)stream, ids, mask, B, L, D, table, (T*)out));
  MMDX_LAUNCH_CHECK();
  return 0;
}

extern "C" int mmdx_embed_mean_bwd(int dtype, const int64_t* ids, const int64_t* mask, int B,
                                   int L, int D, const void* dout, float* dtable, void* stream) {
  DISPATCH_T(dtype, hipLaunchKernelGGL(embed_mean_bwd_kernel<T>, dim3(B), dim3(256), 0,
                                       (hipStream_t)stream, ids, mask, B, L, D, (const T*)dout,
                                       dtable));
  MMDX_LAUNCH_CHECK();
  return 0;
}

extern "C" int mmdx_embed_gather(int dtype, const int64_t* ids, long n, int D,
                                 const float* table, void* out, void* stream) {
  DISPATCH_T(dtype, hipLaunchKernelGGL(gather_kernel<T>, dim3(grid_for(n * D)), dim3(256), 0,
                                       (hipStream_t)stream, ids, n, D, table, (T*)out));
  MMDX_LAUNCH_CHECK();
  return 0;
}

extern "C" int mmdx_embed_scatter(int dtype, const int64_t* ids, long n, int D,
                                  const void* dout, float* dtable, void* stream) {
  DISPATCH_T(dtype, hipLaunchKernelGGL(scatter_kernel<T>, dim3(grid_for(n * D)), dim3(256), 0,
                                       (hipStream_t)stream, ids, n, D, (const T*)dout, dtable));
  MMDX_LAUNCH_CHECK();
  return 0;
}
