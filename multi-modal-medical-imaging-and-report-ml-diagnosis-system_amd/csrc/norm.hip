// BatchNorm2d (+residual)(+ReLU) and LayerNorm, forward and backward, NHWC / row-major.
//
// BN statistics are reduced deterministically: every block writes a per-channel
// (mean, M2) partial over its row slab, and a finalize kernel merges the slabs in a
// fixed order with Chan's parallel-variance update (no float atomics, bitwise
// reproducible, no E[x^2]-E[x]^2 cancellation across the 10^5..10^6 rows of a layer).
// All elementwise passes move 16 B per lane (8 bf16 / 4 fp32).
#include <algorithm>
#include <type_traits>
#include <cstdlib>

#include "common.h"
#include "pool.h"
#include "../../include/mmdx.h"

namespace mmdx {

constexpr int BN_NT = 256;

struct BnLayout {
  int ct;        // channel-vector threads per block
  int rt;        // row threads per block
  int cgroups;   // blockIdx.y extent
  int rblocks;   // blockIdx.x extent
  long rows_per_block;
};

static BnLayout bn_layout(long rows, int C, int vec) {
  BnLayout L;
  const int cv = C / vec;
  L.ct = std::min(cv, 64);
  L.rt = BN_NT / L.ct;
  L.cgroups = (cv + L.ct - 1) / L.ct;
  long target = std::max(1L, 2048L / L.cgroups);  // ~8 blocks per CU for latency hiding
  long rpb = (rows + target - 1) / target;
  rpb = std::max<long>(rpb, L.rt);
  L.rows_per_block = (rpb + L.rt - 1) / L.rt * L.rt;
  L.rblocks = (int)((rows + L.rows_per_block - 1) / L.rows_per_block);
  return L;
}

__device__ __forceinline__ void chan_merge(float& n, float& mean, float& m2, float nb, float mb,
                                           float m2b) {
  const float nn = n + nb;
  if (nb == 0.f) return;
  if (n == 0.f) { n = nb; mean = mb; m2 = m2b; return; }
  const float d = mb - mean;
  const float f = nb / nn;
  mean += d * f;
  m2 += m2b + d * d * n * f;
  n = nn;
}

// partial[c][b] = (mean, M2) of rows [b*rpb, (b+1)*rpb) (channel-major: the finalize reads
// one channel's slabs contiguously)
template <typename T>
__global__ __launch_bounds__(BN_NT) void bn_stats_kernel(const T* __restrict__ x, long rows,
                                                         int C, int ct, long rpb,
                                                         float2* __restrict__ part) {
  typedef typename Vec16<T>::type V;
  constexpr int VEC = Vec16<T>::N;
  __shared__ float s_n[BN_NT], s_mean[BN_NT * VEC], s_m2[BN_NT * VEC];
  const int tx = threadIdx.x % ct, ty = threadIdx.x / ct, rt = BN_NT / ct;
  const int c0 = (blockIdx.y * ct + tx) * VEC;
  const long r0 = blockIdx.x * rpb, r1 = min(rows, r0 + rpb);
  float sum[VEC], sq[VEC];
#pragma unroll
  for (int j = 0; j < VEC; ++j) sum[j] = sq[j] = 0.f;
  int cnt = 0;
  if (c0 < C) {
    for (long r = r0 + ty; r < r1; r += rt) {
      const V v = *(const V*)(x + r * C + c0);
#pragma unroll
      for (int j = 0; j < VEC; ++j) {
        const float f = to_f(v[j]);
        sum[j] += f;
        sq[j] += f * f;
      }
      ++cnt;
    }
  }
  const int me = ty * ct + tx;
  s_n[me] = (float)cnt;
#pragma unroll
  for (int j = 0; j < VEC; ++j) {
    const float m = cnt ? sum[j] / cnt : 0.f;
    s_mean[me * VEC + j] = m;
    s_m2[me * VEC + j] = cnt ? fmaxf(sq[j] - sum[j] * m, 0.f) : 0.f;
  }
  __syncthreads();
  if (ty == 0 && c0 < C) {
#pragma unroll
    for (int j = 0; j < VEC; ++j) {
      float n = 0.f, mean = 0.f, m2 = 0.f;
      for (int y = 0; y < rt; ++y) {
        const int o = y * ct + tx;
        chan_merge(n, mean, m2, s_n[o], s_mean[o * VEC + j], s_m2[o * VEC + j]);
      }
      part[(long)(c0 + j) * gridDim.x + blockIdx.x] = make_float2(mean, m2);
    }
  }
}

// Merge slab partials; update running stats; emit scale/shift for the apply pass.
// One wave per channel, two passes over the slabs (all loads independent, so they pipeline):
// mean = sum(n_b mean_b) / N, then M2 = sum(M2_b + n_b (mean_b - mean)^2) — the exact
// two-level decomposition of the variance, reduced in a fixed lane/shuffle order
// (deterministic).  Conv-epilogue statistics give one slab per 128 output rows.
constexpr int FIN_W = 4;  // channels per 256-thread block when one wave serves a channel

// sum over this channel's slabs of f(b): TPC threads, 4 independent accumulators each
// (4 slab loads in flight), fixed-order wave / block reduction (deterministic)
template <int TPC, class F>
__device__ __forceinline__ float slab_sum(int nblk, int sub, float* red, F f) {
  float a4[4] = {0.f, 0.f, 0.f, 0.f};
  for (int b0 = sub; b0 < nblk; b0 += 4 * TPC) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int b = b0 + TPC * j;
      if (b < nblk) a4[j] += f(b);
    }
  }
  const float v = (a4[0] + a4[1]) + (a4[2] + a4[3]);
  if constexpr (TPC == 64) return wave_sum(v);
  else return block_sum<256>(v, red);
}

// slab_sum over slabs already held in registers (vals[j] = slab sub + TPC*j): the same
// accumulator assignment and order as slab_sum, so the result is bit-identical, but the
// channel's slabs are read from memory once for both passes of the finalize.
template <int TPC, int PER, class F>
__device__ __forceinline__ float slab_sum_regs(const float2* vals, int nblk, int sub, float* red,
                                               F f) {
  float a4[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const int b = sub + TPC * j;
    if (b < nblk) a4[j & 3] += f(b, vals[j]);
  }
  const float v = (a4[0] + a4[1]) + (a4[2] + a4[3]);
  if constexpr (TPC == 64) return wave_sum(v);
  else return block_sum<256>(v, red);
}

// slabs per thread held in registers by the finalize kernels (more: two passes over memory)
constexpr int FIN_PER = 16;

struct BnFinArgs {
  const float2* part;
  int nblk;
  long rows, rpb;
  int C;
  const float* gamma;
  const float* beta;
  float* running_mean;
  float* running_var;
  float momentum, eps;
  float* save_mean;
  float* save_rstd;
  float* scale;
  float* shift;
};

// TPC = threads per channel: 64 (one wave; few slabs) or 256 (whole block; thousands of
// slabs, e.g. the 3136 per-128-row slabs of a layer1 conv at batch 128).  `bid` is the
// finalize block index.
template <int TPC>
__device__ __forceinline__ void bn_finalize_body(const BnFinArgs& a, int bid, float* red) {
  const int sub = threadIdx.x % TPC;
  const int c = bid * (256 / TPC) + threadIdx.x / TPC;
  if (c >= a.C) return;  // uniform per wave (TPC = 64) or per block (TPC = 256)
  const int nblk = a.nblk;
  const long rows = a.rows, rpb = a.rpb;
  const long last = rows - (long)(nblk - 1) * rpb;  // rows of the final (short) slab
  const float2* pc = a.part + (long)c * nblk;        // this channel's slabs, contiguous
  float mean, m2;
  if (nblk <= TPC * FIN_PER) {  // one read of the slabs (all loads in flight together)
    float2 v[FIN_PER];
#pragma unroll
    for (int j = 0; j < FIN_PER; ++j) {
      const int b = sub + TPC * j;
      v[j] = b < nblk ? pc[b] : make_float2(0.f, 0.f);
    }
    mean = slab_sum_regs<TPC, FIN_PER>(v, nblk, sub, red, [&](int b, float2 p) {
      return (b == nblk - 1 ? (float)last : (float)rpb) * p.x;
    }) / (float)rows;
    m2 = slab_sum_regs<TPC, FIN_PER>(v, nblk, sub, red, [&](int b, float2 p) {
      const float d = p.x - mean;
      return p.y + (b == nblk - 1 ? (float)last : (float)rpb) * d * d;
    });
  } else {
    mean = slab_sum<TPC>(nblk, sub, red, [&](int b) {
      return (b == nblk - 1 ? (float)last : (float)rpb) * pc[b].x;
    }) / (float)rows;
    m2 = slab_sum<TPC>(nblk, sub, red, [&](int b) {
      const float2 p = pc[b];
      const float d = p.x - mean;
      return p.y + (b == nblk - 1 ? (float)last : (float)rpb) * d * d;
    });
  }
  if (sub != 0) return;
  const float var = m2 / (float)rows;
  const float rstd = rsqrtf(var + a.eps);
  a.save_mean[c] = mean;
  a.save_rstd[c] = rstd;
  if (a.running_mean) {
    const float unb = rows > 1 ? m2 / (float)(rows - 1) : var;
    a.running_mean[c] = (1.f - a.momentum) * a.running_mean[c] + a.momentum * mean;
    a.running_var[c] = (1.f - a.momentum) * a.running_var[c] + a.momentum * unb;
  }
  const float g = a.gamma ? a.gamma[c] : 1.f;
  a.scale[c] = g * rstd;
  a.shift[c] = (a.beta ? a.beta[c] : 0.f) - mean * g * rstd;
}

template <int TPC>
__global__ __launch_bounds__(256) void bn_finalize_kernel(BnFinArgs a) {
  __shared__ float red[4];
  bn_finalize_body<TPC>(a, blockIdx.x, red);
}

__global__ void bn_eval_coef_kernel(int C, const float* __restrict__ gamma,
                                    const float* __restrict__ beta, const float* rm,
                                    const float* rv, float eps, float* save_mean,
                                    float* save_rstd, float* scale, float* shift) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const float rstd = rsqrtf(rv[c] + eps);
  const float g = gamma ? gamma[c] : 1.f;
  save_mean[c] = rm[c];
  save_rstd[c] = rstd;
  scale[c] = g * rstd;
  shift[c] = (beta ? beta[c] : 0.f) - rm[c] * g * rstd;
}

// Row-tiled channel-vector layout for the elementwise BN passes: a 256-thread block covers
// `tpr` 16-B channel vectors of `rpi` rows; each thread keeps its channels' coefficients in
// registers for every row it visits (no per-element index math or coefficient reloads).
struct RowTile { int cv, tpr, rpi; };
__host__ __device__ inline RowTile row_tile(int C, int vec) {
  RowTile t;
  t.cv = C / vec;
  t.tpr = t.cv < 256 ? t.cv : 256;
  t.rpi = 256 / t.tpr;
  return t;
}

// VEC consecutive per-channel floats (16-B aligned: C % VEC == 0) with vector loads
template <int VEC>
__device__ __forceinline__ void load_coef(const float* p, float* out) {
#pragma unroll
  for (int e = 0; e < VEC; e += 4) {
    const f32x4 v = *(const f32x4*)(p + e);
    out[e] = v[0]; out[e + 1] = v[1]; out[e + 2] = v[2]; out[e + 3] = v[3];
  }
}

// The forward's per-channel scale/shift, recomputed with the same expression order as
// bn_finalize_kernel / bn_eval_coef_kernel so the recomputed pre-activation is bit-equal.
__device__ __forceinline__ void bn_coef(const float* gamma, const float* beta, float mean,
                                        float rstd, int c, float& scale, float& shift) {
  const float g = gamma ? gamma[c] : 1.f;
  scale = g * rstd;
  shift = (beta ? beta[c] : 0.f) - mean * g * rstd;
}

// y = act(x*scale[c] + shift[c] (+ res)); mask (optional): one byte per channel vector of a
// row, bit e = (stored y[e] > 0) — the ReLU mask the backward of a residual unit reads
// instead of y itself (1 bit per element instead of 16)
template <typename T>
__device__ __forceinline__ void bn_apply_vec(const typename Vec16<T>::type& v,
                                             const typename Vec16<T>::type& rr, bool has_res,
                                             const float* sc, const float* sh, int relu, long i,
                                             T* __restrict__ y, uint8_t* __restrict__ mask) {
  typedef typename Vec16<T>::type V;
  constexpr int VEC = Vec16<T>::N;
  V o;
#pragma unroll
  for (int e = 0; e < VEC; ++e) {
    float f = to_f(v[e]) * sc[e] + sh[e];
    if (has_res) f += to_f(rr[e]);
    if (relu) f = fmaxf(f, 0.f);
    o[e] = from_f<T>(f);
  }
  ((V*)y)[i] = o;
  if (mask) {
    unsigned b = 0;
#pragma unroll
    for (int e = 0; e < VEC; ++e) b |= (to_f(o[e]) > 0.f ? 1u : 0u) << e;
    mask[i] = (uint8_t)b;
  }
}

template <typename T>
__global__ __launch_bounds__(256) void bn_apply_kernel(const T* __restrict__ x,
                                                       const T* __restrict__ res, long rows,
                                                       int C, const float* __restrict__ scale,
                                                       const float* __restrict__ shift, int relu,
                                                       T* __restrict__ y,
                                                       uint8_t* __restrict__ mask) {
  typedef typename Vec16<T>::type V;
  constexpr int VEC = Vec16<T>::N;
  const RowTile rt = row_tile(C, VEC);
  const int j0 = threadIdx.x % rt.tpr, ro = threadIdx.x / rt.tpr;
  for (int j = j0; j < rt.cv; j += rt.tpr) {
    float sc[VEC], sh[VEC];
    load_coef<VEC>(scale + j * VEC, sc);
    load_coef<VEC>(shift + j * VEC, sh);
    for (long r = (long)blockIdx.x * rt.rpi + ro; r < rows; r += (long)gridDim.x * rt.rpi) {
      const long i = r * rt.cv + j;
      // nontemporal loads: the conv output and the residual are read once here (their next
      // readers come in the backward, long after): C4 +0.9 % (profiles/r06_nt_store_ab.txt)
      const V v = __builtin_nontemporal_load((const V*)x + i);
      V rr{};
      if (res) rr = __builtin_nontemporal_load((const V*)res + i);
      bn_apply_vec<T>(v, rr, res != nullptr, sc, sh, relu, i, y, mask);
    }
  }
}

// backward reduce: partial[c][b] = (sum g, sum g*xhat), g = dy * relu'(y); dy row r comes
// from the gradient source G (DenseGrad: the [rows][C] tensor; Pool3s2Grad: gathered from the
// stem pool's output gradient and argmax, pool.h); MODE as bn_bwd_apply_kernel's
template <typename T, class G, int MODE>
__global__ __launch_bounds__(BN_NT) void bn_bwd_reduce_kernel(
    const T* __restrict__ x, const T* __restrict__ y, const G dy, long rows, int C,
    int ct, long rpb, const float* __restrict__ mean, const float* __restrict__ rstd,
    const float* __restrict__ gamma, const float* __restrict__ bbeta, float2* __restrict__ part,
    const uint8_t* __restrict__ mask_k) {
  constexpr int relu = MODE != 0;
  const uint8_t* mask = MODE == 1 ? mask_k : nullptr;
  typedef typename Vec16<T>::type V;
  constexpr int VEC = Vec16<T>::N;
  __shared__ float s_a[BN_NT * VEC], s_b[BN_NT * VEC];
  const int tx = threadIdx.x % ct, ty = threadIdx.x / ct, rt = BN_NT / ct;
  const int c0 = (blockIdx.y * ct + tx) * VEC;
  const long r0 = blockIdx.x * rpb, r1 = min(rows, r0 + rpb);
  float sg[VEC], sgx[VEC], mu[VEC], rs[VEC], sc[VEC], sh[VEC];
  // ReLU mask source: the forward's bit mask, else y (the unit's output), else recomputed
  // from x (no residual)
  constexpr bool mask_x = MODE == 3;
#pragma unroll
  for (int j = 0; j < VEC; ++j) sg[j] = sgx[j] = mu[j] = rs[j] = sc[j] = sh[j] = 0.f;
  if (c0 < C) {
    load_coef<VEC>(mean + c0, mu);
    load_coef<VEC>(rstd + c0, rs);
    if constexpr (mask_x) {
      float ga[VEC], be[VEC];
      if (gamma) load_coef<VEC>(gamma + c0, ga);
      if (bbeta) load_coef<VEC>(bbeta + c0, be);
#pragma unroll
      for (int j = 0; j < VEC; ++j) {  // same expression order as bn_coef / the forward
        const float g = gamma ? ga[j] : 1.f;
        sc[j] = g * rs[j];
        sh[j] = (bbeta ? be[j] : 0.f) - mu[j] * g * rs[j];
      }
    }
  }
  if (c0 < C) {
    for (long r = r0 + ty; r < r1; r += rt) {
      const V vx = *(const V*)(x + r * C + c0);
      const V vd = dy.row(r, c0);
      V vy{};
      unsigned mb = 0;
      if (MODE == 1) mb = mask[r * (C / VEC) + c0 / VEC];
      else if (MODE == 2) vy = *(const V*)(y + r * C + c0);
#pragma unroll
      for (int j = 0; j < VEC; ++j) {
        float g = to_f(vd[j]);
        const float a = mask_x ? to_f(vx[j]) * sc[j] + sh[j] : to_f(vy[j]);
        const bool pos = MODE == 1 ? ((mb >> j) & 1u) != 0 : a > 0.f;
        if (relu && !pos) g = 0.f;
        sg[j] += g;
        sgx[j] += g * (to_f(vx[j]) - mu[j]) * rs[j];
      }
    }
  }
  const int me = ty * ct + tx;
#pragma unroll
  for (int j = 0; j < VEC; ++j) {
    s_a[me * VEC + j] = sg[j];
    s_b[me * VEC + j] = sgx[j];
  }
  __syncthreads();
  if (ty == 0 && c0 < C) {
#pragma unroll
    for (int j = 0; j < VEC; ++j) {
      float a = 0.f, b = 0.f;
      for (int yy = 0; yy < rt; ++yy) {
        a += s_a[(yy * ct + tx) * VEC + j];
        b += s_b[(yy * ct + tx) * VEC + j];
      }
      part[(long)(c0 + j) * gridDim.x + blockIdx.x] = make_float2(a, b);
    }
  }
}

// coef: a[c] = gamma*rstd, b[c] = -gamma*rstd*sum_g/n, k[c] = -gamma*rstd*sum_gx/n
// Per channel: sum the (sum g, sum g*xhat) slab partials (slab_sum), then the apply-pass
// coefficients.
struct BnBwdFinArgs {
  const float2* part;
  int nblk;
  long rows;
  int C, train;
  const float* gamma;
  const float* bbeta;
  const float* mean;
  const float* rstd;
  float* dgamma;
  float* dbeta;
  float beta_acc;
  float* coef;
};

template <int TPC>
__device__ __forceinline__ void bn_bwd_finalize_body(const BnBwdFinArgs& a, int bid,
                                                     float* red) {
  const int sub = threadIdx.x % TPC;
  const int c = bid * (256 / TPC) + threadIdx.x / TPC;
  const int C = a.C, nblk = a.nblk;
  if (c >= C) return;
  const float2* pc = a.part + (long)c * nblk;  // this channel's slabs, contiguous
  float sg, sgx;
  if (nblk <= TPC * FIN_PER) {  // one read of the slabs for both sums
    float2 v[FIN_PER];
#pragma unroll
    for (int j = 0; j < FIN_PER; ++j) {
      const int b = sub + TPC * j;
      v[j] = b < nblk ? pc[b] : make_float2(0.f, 0.f);
    }
    sg = slab_sum_regs<TPC, FIN_PER>(v, nblk, sub, red, [](int, float2 p) { return p.x; });
    sgx = slab_sum_regs<TPC, FIN_PER>(v, nblk, sub, red, [](int, float2 p) { return p.y; });
  } else {
    sg = slab_sum<TPC>(nblk, sub, red, [&](int b) { return pc[b].x; });
    sgx = slab_sum<TPC>(nblk, sub, red, [&](int b) { return pc[b].y; });
  }
  if (sub != 0) return;
  const float beta_acc = a.beta_acc;
  if (a.dgamma) a.dgamma[c] = beta_acc != 0.f ? beta_acc * a.dgamma[c] + sgx : sgx;
  if (a.dbeta) a.dbeta[c] = beta_acc != 0.f ? beta_acc * a.dbeta[c] + sg : sg;
  // dx = a*g + cb + ck*x  (== a*g + b + k*xhat);  scale/shift: the forward's pre-activation
  const float rs = a.rstd[c], mu = a.mean[c];
  const float ga = (a.gamma ? a.gamma[c] : 1.f) * rs;
  const float b = a.train ? -ga * sg / (float)a.rows : 0.f;
  const float k = (a.train ? -ga * sgx / (float)a.rows : 0.f) * rs;
  a.coef[c] = ga;
  a.coef[C + c] = b - k * mu;
  a.coef[2 * C + c] = k;
  float sc, sh;
  bn_coef(a.gamma, a.bbeta, mu, rs, c, sc, sh);
  a.coef[3 * C + c] = sc;
  a.coef[4 * C + c] = sh;
}

template <int TPC>
__global__ __launch_bounds__(256) void bn_bwd_finalize_kernel(BnBwdFinArgs a) {
  __shared__ float red[4];
  bn_bwd_finalize_body<TPC>(a, blockIdx.x, red);
}

// dx = a*g + b + k*xhat  ==  a*g + (b - k*mean*rstd) + (k*rstd)*x,  g = dy*relu'(y)
// One channel vector of one row: its loads (BnBwdIn) and its arithmetic (bn_bwd_vec), split so
// the fused finalize + apply kernel can issue the loads before its coefficients exist.
template <typename T>
struct BnBwdIn {
  typename Vec16<T>::type vx, vd, vy;
  unsigned mb;
};

template <typename T, class G>
__device__ __forceinline__ BnBwdIn<T> bn_bwd_load(const T* __restrict__ x,
                                                  const T* __restrict__ y, const G& dy, long r,
                                                  int j, long i, int relu, bool mask_x,
                                                  const uint8_t* __restrict__ mask) {
  typedef typename Vec16<T>::type V;
  constexpr int VEC = Vec16<T>::N;
  BnBwdIn<T> in;
  in.vx = __builtin_nontemporal_load((const V*)x + i);  // (read once: see bn_apply_kernel)
  in.vd = dy.row(r, j * VEC);
  in.vy = V{};
  in.mb = 0;
  if (relu && mask) in.mb = mask[i];
  else if (relu && !mask_x) in.vy = ((const V*)y)[i];
  return in;
}

template <typename T>
__device__ __forceinline__ void bn_bwd_vec(const BnBwdIn<T>& in, const float* ca,
                                           const float* cb, const float* ck, const float* sc,
                                           const float* sh, int relu, bool mask_x, bool has_mask,
                                           long i, T* __restrict__ dx, T* __restrict__ dres) {
  typedef typename Vec16<T>::type V;
  constexpr int VEC = Vec16<T>::N;
  V o, og;
#pragma unroll
  for (int e = 0; e < VEC; ++e) {
    float g = to_f(in.vd[e]);
    const float a = mask_x ? to_f(in.vx[e]) * sc[e] + sh[e] : to_f(in.vy[e]);
    const bool pos = has_mask ? ((in.mb >> e) & 1u) != 0 : a > 0.f;
    if (relu && !pos) g = 0.f;
    // explicit: the compiler may contract a*g + b + k*x either way round, per call site
    o[e] = from_f<T>(fmaf(ck[e], to_f(in.vx[e]), fmaf(ca[e], g, cb[e])));
    og[e] = from_f<T>(g);
  }
  ((V*)dx)[i] = o;
  if (dres) ((V*)dres)[i] = og;
}

// MODE (host-chosen): 0 no ReLU, 1 ReLU mask saved by the forward, 2 ReLU from y, 3 ReLU
// recomputed from x (the only mode that needs scale/shift: keeping them out of the others'
// registers lifts the bf16 kernel from 5 to 6+ waves per SIMD)
template <typename T, class G, int MODE>
__device__ __forceinline__ void bn_bwd_apply_body(
    const T* __restrict__ x, const T* __restrict__ y, const G& dy, long rows, int C,
    const float* __restrict__ coef, T* __restrict__ dx, T* __restrict__ dres,
    const uint8_t* __restrict__ mask) {
  constexpr int relu = MODE != 0;
  constexpr bool mask_x = MODE == 3;
  constexpr int VEC = Vec16<T>::N;
  const uint8_t* mk = MODE == 1 ? mask : nullptr;
  const RowTile rt = row_tile(C, VEC);
  const int j0 = threadIdx.x % rt.tpr, ro = threadIdx.x / rt.tpr;
  for (int j = j0; j < rt.cv; j += rt.tpr) {
    // the forward's scale (coef[3C..]) is bit-equal to a = gamma * rstd (coef[0..C)), both
    // formed as (gamma ? gamma[c] : 1) * rstd: MODE 3 reads only the shift besides a
    float ca[VEC], cb[VEC], ck[VEC], sh[VEC] = {};
    load_coef<VEC>(coef + j * VEC, ca);
    load_coef<VEC>(coef + C + j * VEC, cb);
    load_coef<VEC>(coef + 2 * C + j * VEC, ck);
    if constexpr (mask_x) load_coef<VEC>(coef + 4 * C + j * VEC, sh);
    for (long r = (long)blockIdx.x * rt.rpi + ro; r < rows; r += (long)gridDim.x * rt.rpi) {
      const long i = r * rt.cv + j;
      const BnBwdIn<T> in = bn_bwd_load<T, G>(x, y, dy, r, j, i, relu, mask_x, mk);
      bn_bwd_vec<T>(in, ca, cb, ck, ca, sh, relu, mask_x, MODE == 1, i, dx, dres);
    }
  }
}

template <typename T, class G, int MODE>
__global__ __launch_bounds__(256) void bn_bwd_apply_kernel(
    const T* __restrict__ x, const T* __restrict__ y, const G dy, long rows, int C,
    const float* __restrict__ coef, T* __restrict__ dx, T* __restrict__ dres,
    const uint8_t* __restrict__ mask) {
  bn_bwd_apply_body<T, G, MODE>(x, y, dy, rows, C, coef, dx, dres, mask);
}

// the dense-gradient instances with a 7-waves-per-SIMD register target (MODE 3: 76 -> 72
// VGPRs, no scratch; the gathered-gradient instances would spill under it)
template <typename T, int MODE>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(7))) void
bn_bwd_apply_dense_kernel(const T* __restrict__ x, const T* __restrict__ y, const DenseGrad<T> dy,
                          long rows, int C, const float* __restrict__ coef, T* __restrict__ dx,
                          T* __restrict__ dres, const uint8_t* __restrict__ mask) {
  bn_bwd_apply_body<T, DenseGrad<T>, MODE>(x, y, dy, rows, C, coef, dx, dres, mask);
}

// slab count above which a whole block (not one wave) reduces a channel's partials
// (C4 step: 128 and 512 tie, 2048 -1.6 %)
static int fin_wide() { return 512; }

// >= 4 row iterations per block so the per-channel coefficient loads are amortised
static int grid_rows(long rows, int C, int vec) {
  // row iterations per block and grid cap, measured in the C4 step: 2 and 4 iterations tie,
  // 8 is 0.5 % slower; cap 8192 beat 4096 in 4 of 4 paired runs (+0.3 %), 2048 -1 %
  const long per = 4L;
  const long cap = 8192L;
  const RowTile rt = row_tile(C, vec);
  const long iters = (rows + rt.rpi - 1) / rt.rpi;
  return (int)std::max<long>(1, std::min<long>((iters + per - 1) / per, cap));
}

template <typename T>
static int bn_fwd_t(int train, const void* x, long rows, int C, const float* stat_part,
                    int stat_blocks, long stat_rows, const float* gamma, const float* beta,
                    float* rm, float* rv, float momentum, float eps, float* smean, float* srstd,
                    const void* res, int relu, void* y, void* ws, size_t ws_bytes,
                    hipStream_t st, uint8_t* mask = nullptr) {
  constexpr int VEC = Vec16<T>::N;
  MMDX_CHECK_ARG(C % VEC == 0, "bn: C=%d must be a multiple of %d", C, VEC);
  const BnLayout L = bn_layout(rows, C, VEC);
  const bool ext = train && stat_part;
  const size_t part_bytes = ext ? 0 : (size_t)L.rblocks * C * sizeof(float2);
  const size_t need = part_bytes + 2 * (size_t)C * sizeof(float);
  MMDX_CHECK_ARG(ws && ws_bytes >= need, "bn fwd: workspace %zu < %zu", ws_bytes, need);
  float2* part = (float2*)ws;
  float* scale = (float*)((char*)ws + part_bytes);
  float* shift = scale + C;
  if (train) {
    int nblk = L.rblocks;
    long rpb = L.rows_per_block;
    if (ext) {
      part = (float2*)stat_part;
      nblk = stat_blocks;
      rpb = stat_rows;
    } else {
      hipLaunchKernelGGL(bn_stats_kernel<T>, dim3(L.rblocks, L.cgroups), dim3(BN_NT), 0, st,
                         (const T*)x, rows, C, L.ct, L.rows_per_block, part);
    }
    const BnFinArgs fa{(const float2*)part, nblk, rows, rpb, C, gamma, beta, rm, rv,
                       momentum, eps, smean, srstd, scale, shift};
    const bool wide = nblk > fin_wide();
    const int nfin = wide ? C : (C + FIN_W - 1) / FIN_W;
    if (wide)
      hipLaunchKernelGGL(bn_finalize_kernel<256>, dim3(nfin), dim3(256), 0, st, fa);
    else
      hipLaunchKernelGGL(bn_finalize_kernel<64>, dim3(nfin), dim3(256), 0, st, fa);
  } else {
    MMDX_CHECK_ARG(rm && rv, "bn eval: running stats required");
    hipLaunchKernelGGL(bn_eval_coef_kernel, dim3((C + 255) / 256), dim3(256), 0, st, C, gamma,
                       beta, (const float*)rm, (const float*)rv, eps, smean, srstd, scale,
                       shift);
  }
  if (y)  // (y == NULL: statistics only, the consumer applies the normalisation itself)
    hipLaunchKernelGGL(bn_apply_kernel<T>, dim3(grid_rows(rows, C, VEC)), dim3(256), 0, st,
                       (const T*)x, (const T*)res, rows, C, (const float*)scale,
                       (const float*)shift, relu, (T*)y, relu ? mask : nullptr);
  MMDX_LAUNCH_CHECK();
  return 0;
}

template <typename T, class G>
static int bn_bwd_t(int train, const void* x, const void* y, const G& dy, long rows, int C,
                    const float* gamma, const float* bbeta, const float* smean,
                    const float* srstd, int relu, const float* stat_part, int stat_blocks,
                    void* dx, void* dres, float* dgamma, float* dbeta, float beta_acc, void* ws,
                    size_t ws_bytes, hipStream_t st, const uint8_t* mask = nullptr) {
  constexpr int VEC = Vec16<T>::N;
  MMDX_CHECK_ARG(C % VEC == 0, "bn bwd: C=%d must be a multiple of %d", C, VEC);
  const BnLayout L = bn_layout(rows, C, VEC);
  const size_t need = (size_t)L.rblocks * C * sizeof(float2) + 5 * (size_t)C * sizeof(float);
  MMDX_CHECK_ARG(ws && ws_bytes >= need, "bn bwd: workspace %zu < %zu", ws_bytes, need);
  float2* part = (float2*)ws;
  float* coef = (float*)((char*)ws + (size_t)L.rblocks * C * sizeof(float2));
  int nblk = L.rblocks;
  // ReLU mask source (the MODE of the reduce and apply kernels): none, the forward's bit mask,
  // y (the unit's output), or recomputed from x (no residual)
  const int mode = !relu ? 0 : mask ? 1 : y ? 2 : 3;
  if (stat_part) {  // (sum g, sum g*xhat) partials already made by the dgrad epilogue
    MMDX_CHECK_ARG(stat_blocks > 0 && relu, "bn bwd: precomputed partials need a ReLU unit");
    part = (float2*)stat_part;
    nblk = stat_blocks;
  } else {
    const dim3 g(L.rblocks, L.cgroups);
#define MMDX_BN_BWD_REDUCE(M)                                                                \
  hipLaunchKernelGGL((bn_bwd_reduce_kernel<T, G, M>), g, dim3(BN_NT), 0, st, (const T*)x,   \
                     (const T*)y, dy, rows, C, L.ct, L.rows_per_block, smean, srstd, gamma,  \
                     bbeta, part, mask)
    switch (mode) {
      case 0: MMDX_BN_BWD_REDUCE(0); break;
      case 1: MMDX_BN_BWD_REDUCE(1); break;
      case 2: MMDX_BN_BWD_REDUCE(2); break;
      default: MMDX_BN_BWD_REDUCE(3); break;
    }
#undef MMDX_BN_BWD_REDUCE
  }
  const BnBwdFinArgs fa{(const float2*)part, nblk, rows, C, train, gamma, bbeta, smean, srstd,
                        dgamma, dbeta, beta_acc, coef};
  const bool wide = nblk > fin_wide();
  const int nfin = wide ? C : (C + FIN_W - 1) / FIN_W;
  if (wide)
    hipLaunchKernelGGL(bn_bwd_finalize_kernel<256>, dim3(nfin), dim3(256), 0, st, fa);
  else
    hipLaunchKernelGGL(bn_bwd_finalize_kernel<64>, dim3(nfin), dim3(256), 0, st, fa);
  const dim3 g(grid_rows(rows, C, VEC));
#define MMDX_BN_BWD_APPLY(M)                                                                 \
  if constexpr (std::is_same<G, DenseGrad<T>>::value)                                        \
    hipLaunchKernelGGL((bn_bwd_apply_dense_kernel<T, M>), g, dim3(256), 0, st, (const T*)x,  \
                       (const T*)y, dy, rows, C, (const float*)coef, (T*)dx, (T*)dres, mask); \
  else                                                                                       \
    hipLaunchKernelGGL((bn_bwd_apply_kernel<T, G, M>), g, dim3(256), 0, st, (const T*)x,    \
                       (const T*)y, dy, rows, C, (const float*)coef, (T*)dx, (T*)dres, mask)
  switch (mode) {
    case 0: MMDX_BN_BWD_APPLY(0); break;
    case 1: MMDX_BN_BWD_APPLY(1); break;
    case 2: MMDX_BN_BWD_APPLY(2); break;
    default: MMDX_BN_BWD_APPLY(3); break;
  }
#undef MMDX_BN_BWD_APPLY
  MMDX_LAUNCH_CHECK();
  return 0;
}

// ------------------------------------------------------------------------ LayerNorm
// One wave per row; D <= 64 * LN_MAXV * VEC handled from registers (two-pass stats).
constexpr int LN_MAXV = 4;

// Dropout on the x input (DROP; BertSelfOutput / BertOutput: LayerNorm(dropout(dense) + res)):
// element e = row * D + c of x is kept when hash(base + e) >= p, base = seed * phi +
// (counter << 32) as mmdx_dropout_fwd draws it, and the kept value is rounded to T after the
// 1 / (1 - p) scale as that kernel stores it — so the normalised rows are bit-identical to
// mmdx_dropout_fwd followed by mmdx_layernorm_fwd, without the dropped tensor or its mask.
__device__ __forceinline__ uint32_t ln_drop_hash(uint64_t x) {
  x ^= x >> 33; x *= 0xff51afd7ed558ccdULL;
  x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ULL;
  x ^= x >> 33;
  return (uint32_t)x;
}
__device__ __forceinline__ bool ln_keep(uint64_t base, long e, float p) {
  return (ln_drop_hash(base + (uint64_t)e) >> 8) * (1.f / 16777216.f) >= p;
}

template <typename T, bool DROP = false>
__global__ __launch_bounds__(256) void ln_fwd_kernel(const T* __restrict__ x,
                                                     const T* __restrict__ res, long rows, int D,
                                                     const float* __restrict__ gamma,
                                                     const float* __restrict__ beta, float eps,
                                                     T* __restrict__ y, T* __restrict__ xsum,
                                                     float* smean, float* srstd, float p = 0.f,
                                                     uint64_t seed = 0,
                                                     const uint64_t* __restrict__ ctr = nullptr,
                                                     uint64_t* __restrict__ rng_out = nullptr) {
  typedef typename Vec16<T>::type V;
  constexpr int VEC = Vec16<T>::N;
  const int lane = threadIdx.x & 63;
  const long row = blockIdx.x * 4L + (threadIdx.x >> 6);
  uint64_t dbase = 0;
  float dscale = 1.f;
  if constexpr (DROP) {
    dbase = seed * 0x9E3779B97F4A7C15ULL + (ctr ? ctr[0] << 32 : 0ull);
    dscale = 1.f / (1.f - p);
    if (rng_out && blockIdx.x == 0 && threadIdx.x == 0) rng_out[0] = dbase;
  }
  if (row >= rows) return;
  const int nv = D / VEC;
  float v[LN_MAXV][VEC];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < LN_MAXV; ++i) {
    const int vi = lane + i * 64;
    if (vi < nv) {
      const V a = *(const V*)(x + row * D + vi * VEC);
      V b{};
      if (res) b = *(const V*)(res + row * D + vi * VEC);
#pragma unroll
      for (int j = 0; j < VEC; ++j) {
        float av = to_f(a[j]);
        if constexpr (DROP)
          av = to_f(from_f<T>(ln_keep(dbase, row * D + vi * VEC + j, p) ? av * dscale : 0.f));
        v[i][j] = av + (res ? to_f(b[j]) : 0.f);
        s += v[i][j];
      }
      if (xsum) {
        V o;
#pragma unroll
        for (int j = 0; j < VEC; ++j) o[j] = from_f<T>(v[i][j]);
        *(V*)(xsum + row * D + vi * VEC) = o;
      }
    }
  }
  const float mean = wave_sum(s) / D;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < LN_MAXV; ++i)
    if (lane + i * 64 < nv)
#pragma unroll
      for (int j = 0; j < VEC; ++j) {
        const float d = v[i][j] - mean;
        q += d * d;
      }
  const float rstd = rsqrtf(wave_sum(q) / D + eps);
  if (lane == 0) {
    if (smean) smean[row] = mean;
    if (srstd) srstd[row] = rstd;
  }
#pragma unroll
  for (int i = 0; i < LN_MAXV; ++i) {
    const int vi = lane + i * 64;
    if (vi < nv) {
      V o;
#pragma unroll
      for (int j = 0; j < VEC; ++j) {
        const int c = vi * VEC + j;
        o[j] = from_f<T>((v[i][j] - mean) * rstd * gamma[c] + beta[c]);
      }
      *(V*)(y + row * D + vi * VEC) = o;
    }
  }
}

// rows per block = 4 waves x rpw rows; each wave loads its next row while reducing the
// current one (isolated bwd at 12608 x 768 fp16 was 25.9 us, 2.3 TB/s, with 8 rows per wave
// and no prefetch).  The workspace is sized for the smallest rpw (the most partials).
constexpr int LN_RPW_MIN = 4;
constexpr int LN_BWD_ROWS = 4 * LN_RPW_MIN;   // rows per block at LN_RPW_MIN
static int ln_bwd_rpw() { return knobs().ln_bwd_rpw; }   // MMDX_LN_BWD_RPW = 4 | 8 (8)

// dx per row; per-block partial dgamma/dbeta -> part[blk][2][D]
// MV: 16-B vectors per lane (ceil(D / VEC / 64)), a template argument so the register arrays
// are sized for D (MV everywhere held 194 VGPRs at D = 768: two waves per SIMD)
// DROP: dx_drop = dropout's backward of the stored dx (the same keep bits from rng[0], the
// base the forward left): mmdx_dropout_bwd's result, bit for bit, without the mask tensor.
template <typename T, int MV, bool DROP = false>
__global__ __launch_bounds__(256) void ln_bwd_kernel(const T* __restrict__ xs,
                                                     const T* __restrict__ dy, long rows, int D,
                                                     const float* __restrict__ gamma,
                                                     const float* __restrict__ smean,
                                                     const float* __restrict__ srstd,
                                                     T* __restrict__ dx,
                                                     float* __restrict__ part, int rpw,
                                                     float p = 0.f,
                                                     const uint64_t* __restrict__ rng = nullptr,
                                                     T* __restrict__ dx_drop = nullptr,
                                                     const T* __restrict__ addin = nullptr) {
  typedef typename Vec16<T>::type V;
  constexpr int VEC = Vec16<T>::N;
  extern __shared__ __attribute__((aligned(16))) float red[];  // [4][2][D]
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int nv = D / VEC;
  float pg[MV][VEC], pb[MV][VEC];
#pragma unroll
  for (int i = 0; i < MV; ++i)
#pragma unroll
    for (int j = 0; j < VEC; ++j) pg[i][j] = pb[i][j] = 0.f;
  const long row0 = (blockIdx.x * 4L + w) * rpw;
  V an[MV], dn[MV];
  float mean_n = 0.f, rstd_n = 0.f;
  auto fetch = [&](long row) {
#pragma unroll
    for (int i = 0; i < MV; ++i) {
      const int vi = lane + i * 64;
      if (vi < nv) {
        an[i] = *(const V*)(xs + row * D + vi * VEC);
        dn[i] = *(const V*)(dy + row * D + vi * VEC);
      }
    }
    mean_n = smean[row];
    rstd_n = srstd[row];
  };
  if (row0 < rows) fetch(row0);
  for (int rr = 0; rr < rpw; ++rr) {
    const long row = row0 + rr;
    if (row >= rows) break;
    const float mean = mean_n, rstd = rstd_n;
    V av[MV], dv[MV];
#pragma unroll
    for (int i = 0; i < MV; ++i) {
      av[i] = an[i];
      dv[i] = dn[i];
    }
    if (rr + 1 < rpw && row + 1 < rows) fetch(row + 1);
    // the residual branch's gradient is loaded here, not at the store: a load issued after
    // the row's wave sums left its whole latency exposed on every row (C5 -1.5 %)
    V ai[MV];
    if (addin) {
#pragma unroll
      for (int i = 0; i < MV; ++i) {
        const int vi = lane + i * 64;
        if (vi < nv) ai[i] = *(const V*)(addin + row * D + vi * VEC);
      }
    }
    float xh[MV][VEC], g[MV][VEC];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < MV; ++i) {
      const int vi = lane + i * 64;
      if (vi < nv) {
        const V a = av[i];
        const V d = dv[i];
#pragma unroll
        for (int j = 0; j < VEC; ++j) {
          const int c = vi * VEC + j;
          xh[i][j] = (to_f(a[j]) - mean) * rstd;
          const float dd = to_f(d[j]);
          g[i][j] = dd * gamma[c];
          s1 += g[i][j];
          s2 += g[i][j] * xh[i][j];
          pg[i][j] += dd * xh[i][j];
          pb[i][j] += dd;
        }
      }
    }
    s1 = wave_sum(s1) / D;
    s2 = wave_sum(s2) / D;
#pragma unroll
    for (int i = 0; i < MV; ++i) {
      const int vi = lane + i * 64;
      if (vi < nv) {
        V o;
        if (addin) {   // dx + a residual branch's gradient, one rounding (ViT: da = dO + LN'(.))
#pragma unroll
          for (int j = 0; j < VEC; ++j)
            o[j] = from_f<T>(rstd * (g[i][j] - s1 - xh[i][j] * s2) + to_f(ai[i][j]));
        } else {
#pragma unroll
          for (int j = 0; j < VEC; ++j) o[j] = from_f<T>(rstd * (g[i][j] - s1 - xh[i][j] * s2));
        }
        *(V*)(dx + row * D + vi * VEC) = o;
        if constexpr (DROP) {
          const uint64_t dbase = rng[0];
          const float dscale = 1.f / (1.f - p);
          V od;
#pragma unroll
          for (int j = 0; j < VEC; ++j)
            od[j] = from_f<T>(ln_keep(dbase, row * D + vi * VEC + j, p) ? to_f(o[j]) * dscale
                                                                         : 0.f);
          *(V*)(dx_drop + row * D + vi * VEC) = od;
        }
      }
    }
  }
#pragma unroll
  for (int i = 0; i < MV; ++i) {
    const int vi = lane + i * 64;
    if (vi < nv)
#pragma unroll
      for (int j = 0; j < VEC; ++j) {
        red[(w * 2 + 0) * D + vi * VEC + j] = pg[i][j];
        red[(w * 2 + 1) * D + vi * VEC + j] = pb[i][j];
      }
  }
  __syncthreads();
  for (int c = threadIdx.x; c < D; c += 256) {
    float a = 0.f, b = 0.f;
#pragma unroll
    for (int ww = 0; ww < 4; ++ww) {
      a += red[(ww * 2 + 0) * D + c];
      b += red[(ww * 2 + 1) * D + c];
    }
    part[((long)blockIdx.x * 2 + 0) * D + c] = a;
    part[((long)blockIdx.x * 2 + 1) * D + c] = b;
  }
}

// dgamma / dbeta from the per-block partials [nblk][2][D]: 32 columns x 32 lanes per block,
// the lanes stride the blocks with 8 loads in flight each (the first version had one thread
// per column over all nblk partials — 3 blocks at D = 768: 82 us per call, 4.5 ms per C5
// step; 8 lanes with 4 loads in flight still left ~12 us at 394 partials)
constexpr int LN_FIN_LANES = 32;
__global__ __launch_bounds__(1024) void ln_bwd_finalize_kernel(const float* __restrict__ part,
                                                               int nblk, int D, float* dgamma,
                                                               float* dbeta, float beta_acc) {
  __shared__ float red[LN_FIN_LANES][33];
  const int cc = threadIdx.x & 31, lane = threadIdx.x >> 5;
  const int c = blockIdx.x * 32 + cc, which = blockIdx.y;  // 0: dgamma, 1: dbeta
  float acc = 0.f;
  if (c < D) {
#pragma unroll 8
    for (int k = lane; k < nblk; k += LN_FIN_LANES) acc += part[((long)k * 2 + which) * D + c];
  }
  red[lane][cc] = acc;
  __syncthreads();
  if (lane != 0 || c >= D) return;
  float s = 0.f;
#pragma unroll
  for (int l = 0; l < LN_FIN_LANES; ++l) s += red[l][cc];
  float* out = which ? dbeta : dgamma;
  if (out) out[c] = beta_acc != 0.f ? beta_acc * out[c] + s : s;
}

}  // namespace mmdx

using namespace mmdx;

extern "C" size_t mmdx_bn_workspace_size(long rows, int C) {
  const BnLayout L = bn_layout(rows, C, 4);  // fp32 layout has the most row blocks
  const BnLayout L8 = bn_layout(rows, C, 8);
  const int nb = std::max(L.rblocks, L8.rblocks);
  return (size_t)nb * C * sizeof(float2) + 5 * (size_t)C * sizeof(float);
}

extern "C" int mmdx_bn_fwd_ex(int dtype, int train, const void* x, long rows, int C,
                              const float* stat_part, int stat_blocks, long stat_rows,
                              const float* gamma, const float* beta, float* running_mean,
                              float* running_var, float momentum, float eps, float* save_mean,
                              float* save_rstd, const void* residual, int relu, void* y,
                              uint8_t* relu_mask, void* ws, size_t ws_bytes, void* stream) {
  MMDX_CHECK_ARG(dtype != F16, "mmdx_bn_fwd: fp16 is the C5 path only");
  MMDX_CHECK_ARG(rows > 0 && C > 0 && save_mean && save_rstd, "bn fwd: bad args");
  MMDX_CHECK_ARG(!stat_part || (stat_blocks > 0 && stat_rows > 0 &&
                                (long)stat_blocks * stat_rows >= rows),
                 "bn fwd: bad precomputed statistics layout");
  MMDX_CHECK_ARG(!relu_mask || (relu && y), "bn fwd: a ReLU mask needs relu and y");
  hipStream_t st = (hipStream_t)stream;
  if (dtype == BF16)
    return bn_fwd_t<bf16>(train, x, rows, C, stat_part, stat_blocks, stat_rows, gamma, beta,
                          running_mean, running_var, momentum, eps, save_mean, save_rstd,
                          residual, relu, y, ws, ws_bytes, st, relu_mask);
  return bn_fwd_t<float>(train, x, rows, C, stat_part, stat_blocks, stat_rows, gamma, beta,
                         running_mean, running_var, momentum, eps, save_mean, save_rstd,
                         residual, relu, y, ws, ws_bytes, st, relu_mask);
}

// The finalize alone (slabs from a conv epilogue -> mean / rstd / running stats / scale /
// shift) and the apply alone: the two halves of mmdx_bn_fwd_ex's train forward, as separate
// entry points (plan op MMDX_OP_BN_APPLY).
extern "C" int mmdx_bn_finalize(const float* stat_part, int stat_blocks, long stat_rows,
                                long rows, int C, const float* gamma, const float* beta,
                                float* running_mean, float* running_var, float momentum,
                                float eps, float* save_mean, float* save_rstd, float* scale,
                                float* shift, void* stream) {
  MMDX_CHECK_ARG(stat_part && stat_blocks > 0 && stat_rows > 0 && rows > 0 && C > 0 &&
                     (long)stat_blocks * stat_rows >= rows && save_mean && save_rstd && scale &&
                     shift,
                 "bn finalize: bad args");
  hipStream_t st = (hipStream_t)stream;
  const BnFinArgs fa{(const float2*)stat_part, stat_blocks, rows, stat_rows, C, gamma, beta,
                     running_mean, running_var, momentum, eps, save_mean, save_rstd, scale,
                     shift};
  if (stat_blocks > fin_wide())
    hipLaunchKernelGGL(bn_finalize_kernel<256>, dim3(C), dim3(256), 0, st, fa);
  else
    hipLaunchKernelGGL(bn_finalize_kernel<64>, dim3((C + FIN_W - 1) / FIN_W), dim3(256), 0, st,
                       fa);
  MMDX_LAUNCH_CHECK();
  return 0;
}

extern "C" int mmdx_bn_apply(int dtype, const void* x, const void* residual, long rows, int C,
                             const float* scale, const float* shift, int relu, void* y,
                             uint8_t* relu_mask, void* stream) {
  MMDX_CHECK_ARG(dtype != F16, "mmdx_bn_apply: fp16 is the C5 path only");
  MMDX_CHECK_ARG(x && y && scale && shift && rows > 0 && C > 0, "bn apply: bad args");
  MMDX_CHECK_ARG(!relu_mask || relu, "bn apply: a ReLU mask needs relu");
  hipStream_t st = (hipStream_t)stream;
  if (dtype == BF16) {
    MMDX_CHECK_ARG(C % 8 == 0, "bn apply: C=%d must be a multiple of 8", C);
    hipLaunchKernelGGL(bn_apply_kernel<bf16>, dim3(grid_rows(rows, C, 8)), dim3(256), 0, st,
                       (const bf16*)x, (const bf16*)residual, rows, C, scale, shift, relu,
                       (bf16*)y, relu ? relu_mask : nullptr);
  } else {
    MMDX_CHECK_ARG(C % 4 == 0, "bn apply: C=%d must be a multiple of 4", C);
    hipLaunchKernelGGL(bn_apply_kernel<float>, dim3(grid_rows(rows, C, 4)), dim3(256), 0, st,
                       (const float*)x, (const float*)residual, rows, C, scale, shift, relu,
                       (float*)y, relu ? relu_mask : nullptr);
  }
  MMDX_LAUNCH_CHECK();
  return 0;
}

extern "C" int mmdx_bn_fwd(int dtype, int train, const void* x, long rows, int C,
                           const float* stat_part, int stat_blocks, long stat_rows,
                           const float* gamma, const float* beta, float* running_mean,
                           float* running_var, float momentum, float eps, float* save_mean,
                           float* save_rstd, const void* residual, int relu, void* y,
                           void* ws, size_t ws_bytes, void* stream) {
  return mmdx_bn_fwd_ex(dtype, train, x, rows, C, stat_part, stat_blocks, stat_rows, gamma,
                        beta, running_mean, running_var, momentum, eps, save_mean, save_rstd,
                        residual, relu, y, nullptr, ws, ws_bytes, stream);
}

extern "C" int mmdx_bn_bwd_ex(int dtype, int train, const void* x, const void* y,
                              const void* dy, long rows, int C, const float* gamma,
                              const float* bn_beta, const float* save_mean,
                              const float* save_rstd, int relu, const float* stat_part,
                              int stat_blocks, void* dx, void* d_residual, float* dgamma,
                              float* dbeta, float beta_acc, const uint8_t* relu_mask, void* ws,
                              size_t ws_bytes, void* stream) {
  MMDX_CHECK_ARG(dtype != F16, "mmdx_bn_bwd: fp16 is the C5 path only");
  MMDX_CHECK_ARG(rows > 0 && C > 0, "bn bwd: bad args");
  MMDX_CHECK_ARG(!(relu && !y && !relu_mask && d_residual),
                 "bn bwd: a residual unit needs its output y or its ReLU mask");
  hipStream_t st = (hipStream_t)stream;
  const uint8_t* mk = relu ? relu_mask : nullptr;
  if (dtype == BF16)
    return bn_bwd_t<bf16>(train, x, y, DenseGrad<bf16>{(const bf16*)dy, C}, rows, C, gamma,
                          bn_beta, save_mean, save_rstd, relu, stat_part, stat_blocks, dx,
                          d_residual, dgamma, dbeta, beta_acc, ws, ws_bytes, st, mk);
  return bn_bwd_t<float>(train, x, y, DenseGrad<float>{(const float*)dy, C}, rows, C, gamma,
                         bn_beta, save_mean, save_rstd, relu, stat_part, stat_blocks, dx,
                         d_residual, dgamma, dbeta, beta_acc, ws, ws_bytes, st, mk);
}

extern "C" int mmdx_bn_bwd_masked_dy(int dtype, int train, const void* x, const void* dy,
                                     const uint8_t* dy_mask, long rows, int C,
                                     const float* gamma, const float* bn_beta,
                                     const float* save_mean, const float* save_rstd, void* dx,
                                     float* dgamma, float* dbeta, float beta_acc, void* ws,
                                     size_t ws_bytes, void* stream) {
  MMDX_CHECK_ARG(dtype != F16, "mmdx_bn_bwd_masked_dy: fp16 is the C5 path only");
  MMDX_CHECK_ARG(rows > 0 && C > 0 && dy && dy_mask, "bn bwd masked dy: bad args");
  hipStream_t st = (hipStream_t)stream;
  if (dtype == BF16)
    return bn_bwd_t<bf16>(train, x, nullptr, MaskedGrad<bf16>{(const bf16*)dy, dy_mask, C}, rows,
                          C, gamma, bn_beta, save_mean, save_rstd, 0, nullptr, 0, dx, nullptr,
                          dgamma, dbeta, beta_acc, ws, ws_bytes, st);
  return bn_bwd_t<float>(train, x, nullptr, MaskedGrad<float>{(const float*)dy, dy_mask, C},
                         rows, C, gamma, bn_beta, save_mean, save_rstd, 0, nullptr, 0, dx,
                         nullptr, dgamma, dbeta, beta_acc, ws, ws_bytes, st);
}

extern "C" int mmdx_bn_bwd(int dtype, int train, const void* x, const void* y, const void* dy,
                           long rows, int C, const float* gamma, const float* bn_beta,
                           const float* save_mean, const float* save_rstd, int relu,
                           const float* stat_part, int stat_blocks, void* dx,
                           void* d_residual, float* dgamma, float* dbeta, float beta_acc,
                           void* ws, size_t ws_bytes, void* stream) {
  return mmdx_bn_bwd_ex(dtype, train, x, y, dy, rows, C, gamma, bn_beta, save_mean, save_rstd,
                        relu, stat_part, stat_blocks, dx, d_residual, dgamma, dbeta, beta_acc,
                        nullptr, ws, ws_bytes, stream);
}

extern "C" int mmdx_bn_bwd_pool(int dtype, int train, const void* x, const uint8_t* argmax,
                                const void* dy_pooled, int N, int H, int W, int C, int k, int s,
                                int p, int P, int Q, const float* gamma, const float* bn_beta,
                                const float* save_mean, const float* save_rstd, int relu,
                                void* dx, float* dgamma, float* dbeta, float beta_acc, void* ws,
                                size_t ws_bytes, void* stream) {
  MMDX_CHECK_ARG(dtype != F16, "mmdx_bn_bwd_pool: fp16 is the C5 path only");
  MMDX_CHECK_ARG(N > 0 && H > 0 && W > 0 && C > 0 && argmax && dy_pooled,
                 "bn bwd pool: bad args");
  MMDX_CHECK_ARG(k == 3 && s == 2 && p <= 1, "bn bwd pool: only the 3x3 / stride-2 stem pool");
  MMDX_CHECK_ARG(P == (H + 2 * p - k) / s + 1 && Q == (W + 2 * p - k) / s + 1,
                 "bn bwd pool: inconsistent pool output size");
  const long rows = (long)N * H * W;
  MMDX_CHECK_ARG(rows < (1L << 31), "bn bwd pool: more than 2^31 rows");
  hipStream_t st = (hipStream_t)stream;
  if (dtype == BF16)
    return bn_bwd_t<bf16>(train, x, nullptr,
                          Pool3s2Grad<bf16>{argmax, (const bf16*)dy_pooled, H, W, C, p, P, Q},
                          rows, C, gamma, bn_beta, save_mean, save_rstd, relu, nullptr, 0, dx,
                          nullptr, dgamma, dbeta, beta_acc, ws, ws_bytes, st);
  return bn_bwd_t<float>(train, x, nullptr,
                         Pool3s2Grad<float>{argmax, (const float*)dy_pooled, H, W, C, p, P, Q},
                         rows, C, gamma, bn_beta, save_mean, save_rstd, relu, nullptr, 0, dx,
                         nullptr, dgamma, dbeta, beta_acc, ws, ws_bytes, st);
}

extern "C" int mmdx_layernorm_fwd(int dtype, const void* x, const void* residual, long rows,
                                  int D, const float* gamma, const float* beta, float eps,
                                  void* y, void* sum_out, float* save_mean, float* save_rstd,
                                  void* stream) {
  const int VEC = dtype == F32 ? 4 : 8;
  MMDX_CHECK_ARG(rows > 0 && D % VEC == 0 && D <= 64 * LN_MAXV * VEC && gamma && beta,
                 "layernorm: D=%d unsupported", D);
  hipStream_t st = (hipStream_t)stream;
  const int blocks = (int)((rows + 3) / 4);
  MMDX_DISPATCH(dtype, hipLaunchKernelGGL(ln_fwd_kernel<T>, dim3(blocks), dim3(256), 0, st,
                                          (const T*)x, (const T*)residual, rows, D, gamma, beta,
                                          eps, (T*)y, (T*)sum_out, save_mean, save_rstd));
  MMDX_LAUNCH_CHECK();
  return 0;
}

__global__ void ln_counter_incr_kernel(uint64_t* c) { c[0] += 1; }

extern "C" int mmdx_layernorm_fwd_dropout(int dtype, const void* x, const void* residual,
                                          long rows, int D, const float* gamma,
                                          const float* beta, float eps, float p, uint64_t seed,
                                          uint64_t* counter, void* y, void* sum_out,
                                          float* save_mean, float* save_rstd, uint64_t* rng,
                                          void* stream) {
  const int VEC = dtype == F32 ? 4 : 8;
  MMDX_CHECK_ARG(rows > 0 && D % VEC == 0 && D <= 64 * LN_MAXV * VEC && gamma && beta,
                 "layernorm: D=%d unsupported", D);
  MMDX_CHECK_ARG(p >= 0.f && p < 1.f && rng, "layernorm dropout: p=%g / rng", (double)p);
  hipStream_t st = (hipStream_t)stream;
  const int blocks = (int)((rows + 3) / 4);
  MMDX_DISPATCH(dtype, hipLaunchKernelGGL((ln_fwd_kernel<T, true>), dim3(blocks), dim3(256), 0,
                                          st, (const T*)x, (const T*)residual, rows, D, gamma,
                                          beta, eps, (T*)y, (T*)sum_out, save_mean, save_rstd, p,
                                          seed, (const uint64_t*)counter, rng));
  if (counter)
    hipLaunchKernelGGL(ln_counter_incr_kernel, dim3(1), dim3(1), 0, st, counter);
  MMDX_LAUNCH_CHECK();
  return 0;
}

extern "C" size_t mmdx_layernorm_workspace_size(long rows, int D) {
  const long nblk = (rows + LN_BWD_ROWS - 1) / LN_BWD_ROWS;
  return (size_t)nblk * 2 * D * sizeof(float);
}

static int layernorm_bwd_t(int dtype, const void* xsum, const void* dy, long rows, int D,
                           const float* gamma, const float* save_mean, const float* save_rstd,
                           void* dx, float* dgamma, float* dbeta, float beta_acc, void* ws,
                           size_t ws_bytes, float p, const uint64_t* rng, void* dx_drop,
                           void* stream, const void* addin = nullptr) {
  const int VEC = dtype == F32 ? 4 : 8;
  MMDX_CHECK_ARG(rows > 0 && D % VEC == 0 && D <= 64 * LN_MAXV * VEC, "layernorm bwd: D=%d", D);
  const int rpw = ln_bwd_rpw();
  const long nblk = (rows + 4 * rpw - 1) / (4 * rpw);
  MMDX_CHECK_ARG(ws && ws_bytes >= mmdx_layernorm_workspace_size(rows, D),
                 "layernorm bwd: workspace too small");
  hipStream_t st = (hipStream_t)stream;
  const size_t shm = 8 * (size_t)D * sizeof(float);
  const int mv = (D / VEC + 63) / 64;
  const bool drop = dx_drop != nullptr;
  MMDX_DISPATCH(dtype, {
    auto launch = [&](auto kern) {
      hipLaunchKernelGGL(kern, dim3(nblk), dim3(256), shm, st, (const T*)xsum, (const T*)dy,
                         rows, D, gamma, save_mean, save_rstd, (T*)dx, (float*)ws, rpw, p, rng,
                         (T*)dx_drop, (const T*)addin);
    };
    if (drop) {
      if (mv == 1) launch(ln_bwd_kernel<T, 1, true>);
      else if (mv == 2) launch(ln_bwd_kernel<T, 2, true>);
      else if (mv == 3) launch(ln_bwd_kernel<T, 3, true>);
      else launch(ln_bwd_kernel<T, 4, true>);
    } else {
      if (mv == 1) launch(ln_bwd_kernel<T, 1>);
      else if (mv == 2) launch(ln_bwd_kernel<T, 2>);
      else if (mv == 3) launch(ln_bwd_kernel<T, 3>);
      else launch(ln_bwd_kernel<T, 4>);
    }
  });
  hipLaunchKernelGGL(ln_bwd_finalize_kernel, dim3((D + 31) / 32, 2), dim3(32 * LN_FIN_LANES), 0,
                     st,
                     (const float*)ws, (int)nblk, D, dgamma, dbeta, beta_acc);
  MMDX_LAUNCH_CHECK();
  return 0;
}

extern "C" int mmdx_layernorm_bwd(int dtype, const void* xsum, const void* dy, long rows, int D,
                                  const float* gamma, const float* save_mean,
                                  const float* save_rstd, void* dx, float* dgamma, float* dbeta,
                                  float beta_acc, void* ws, size_t ws_bytes, void* stream) {
  return layernorm_bwd_t(dtype, xsum, dy, rows, D, gamma, save_mean, save_rstd, dx, dgamma,
                         dbeta, beta_acc, ws, ws_bytes, 0.f, nullptr, nullptr, stream);
}

extern "C" int mmdx_layernorm_bwd_residual(int dtype, const void* xsum, const void* dy,
                                           long rows, int D, const float* gamma,
                                           const float* save_mean, const float* save_rstd,
                                           const void* residual_grad, void* dx, float* dgamma,
                                           float* dbeta, float beta_acc, void* ws,
                                           size_t ws_bytes, void* stream) {
  MMDX_CHECK_ARG(residual_grad && residual_grad != dx,
                 "layernorm bwd residual: residual_grad missing or aliasing dx");
  return layernorm_bwd_t(dtype, xsum, dy, rows, D, gamma, save_mean, save_rstd, dx, dgamma,
                         dbeta, beta_acc, ws, ws_bytes, 0.f, nullptr, nullptr, stream,
                         residual_grad);
}

extern "C" int mmdx_layernorm_bwd_dropout(int dtype, const void* xsum, const void* dy, long rows,
                                          int D, const float* gamma, const float* save_mean,
                                          const float* save_rstd, float p, const uint64_t* rng,
                                          void* dx, void* dx_drop, float* dgamma, float* dbeta,
                                          float beta_acc, void* ws, size_t ws_bytes,
                                          void* stream) {
  MMDX_CHECK_ARG(p >= 0.f && p < 1.f && rng && dx_drop, "layernorm bwd dropout: bad args");
  return layernorm_bwd_t(dtype, xsum, dy, rows, D, gamma, save_mean, save_rstd, dx, dgamma,
                         dbeta, beta_acc, ws, ws_bytes, p, rng, dx_drop, stream);
}
