// T5-small report head: the kernels the decoder needs beyond the
// GEMM / attention / dropout / embedding ones it shares with the towers.
//
// The reference conditions T5's DECODER on K = 4 synthetic encoder tokens
// (cond_proj(z_fuse), training_pipeline.py:553-558, 574-578) and trains it teacher-forced
// with CrossEntropyLoss(ignore_index=-100) (TP:983-991, 1049-1053), beam-generates at
// predict (IP:190-196).  Arithmetic of transformers' T5 (modeling_t5.py):
//   * T5LayerNorm = RMSNorm: y = w * x * rsqrt(mean(x^2) + eps), no mean, no bias;
//   * self-attention without 1/sqrt(d) scaling, plus a learned relative-position bias
//     table[bucket(k - q)][h] (causal buckets, layer 0 owns it, all layers share it);
//   * cross-attention over the 4 condition tokens (no bias, no mask);
//   * lm_head tied to the embedding, on the final hidden state scaled by d_model^-0.5.
// Row-wise kernels use one wave per row and 16-B vectors; the cross-attention over K <= 16
// keys is a per-(row, head) CUDA-core kernel (its FLOPs are negligible next to the GEMMs).
#include <algorithm>
#include <climits>

#include "common.h"
#include "../../include/mmdx.h"

namespace mmdx {

constexpr int RMS_MAXV = 4;   // D <= 64 lanes * 4 vectors * VEC
constexpr int RMS_BWD_ROWS = 32;

template <typename T>
__global__ __launch_bounds__(256) void rms_fwd_kernel(const T* __restrict__ x, long rows, int D,
                                                      const float* __restrict__ w, float eps,
                                                      T* __restrict__ y, float* srstd) {
  typedef typename Vec16<T>::type V;
  constexpr int VEC = Vec16<T>::N;
  const int lane = threadIdx.x & 63;
  const long row = blockIdx.x * 4L + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int nv = D / VEC;
  float v[RMS_MAXV][VEC];
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < RMS_MAXV; ++i) {
    const int vi = lane + i * 64;
    if (vi < nv) {
      const V a = *(const V*)(x + row * D + vi * VEC);
#pragma unroll
      for (int j = 0; j < VEC; ++j) {
        v[i][j] = to_f(a[j]);
        q += v[i][j] * v[i][j];
      }
    }
  }
  const float rstd = rsqrtf(wave_sum(q) / D + eps);
  if (lane == 0 && srstd) srstd[row] = rstd;
#pragma unroll
  for (int i = 0; i < RMS_MAXV; ++i) {
    const int vi = lane + i * 64;
    if (vi < nv) {
      V o;
#pragma unroll
      for (int j = 0; j < VEC; ++j) o[j] = from_f<T>(w[vi * VEC + j] * (v[i][j] * rstd));
      *(V*)(y + row * D + vi * VEC) = o;
    }
  }
}

// dx = rstd * (w*dy - x * rstd^2 * mean(w*dy*x)) (+ beta * dx); per-block partial dw.
template <typename T>
__global__ __launch_bounds__(256) void rms_bwd_kernel(const T* __restrict__ x,
                                                      const T* __restrict__ dy, long rows, int D,
                                                      const float* __restrict__ w,
                                                      const float* __restrict__ srstd,
                                                      float beta, T* __restrict__ dx,
                                                      float* __restrict__ part) {
  typedef typename Vec16<T>::type V;
  constexpr int VEC = Vec16<T>::N;
  extern __shared__ __attribute__((aligned(16))) float red[];  // [4][D]
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int nv = D / VEC;
  float pw[RMS_MAXV][VEC];
#pragma unroll
  for (int i = 0; i < RMS_MAXV; ++i)
#pragma unroll
    for (int j = 0; j < VEC; ++j) pw[i][j] = 0.f;
  for (int rr = 0; rr < RMS_BWD_ROWS / 4; ++rr) {
    const long row = blockIdx.x * (long)RMS_BWD_ROWS + wv * (RMS_BWD_ROWS / 4) + rr;
    if (row >= rows) break;
    const float rstd = srstd[row];
    float xv[RMS_MAXV][VEC], g[RMS_MAXV][VEC];
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < RMS_MAXV; ++i) {
      const int vi = lane + i * 64;
      if (vi < nv) {
        const V a = *(const V*)(x + row * D + vi * VEC);
        const V d = *(const V*)(dy + row * D + vi * VEC);
#pragma unroll
        for (int j = 0; j < VEC; ++j) {
          xv[i][j] = to_f(a[j]);
          const float dd = to_f(d[j]);
          g[i][j] = dd * w[vi * VEC + j];
          s += g[i][j] * xv[i][j];
          pw[i][j] += dd * xv[i][j] * rstd;
        }
      }
    }
    const float c = wave_sum(s) / D * rstd * rstd;
#pragma unroll
    for (int i = 0; i < RMS_MAXV; ++i) {
      const int vi = lane + i * 64;
      if (vi < nv) {
        V prev{};
        if (beta != 0.f) prev = *(const V*)(dx + row * D + vi * VEC);
        V o;
#pragma unroll
        for (int j = 0; j < VEC; ++j) {
          float r = rstd * (g[i][j] - xv[i][j] * c);
          if (beta != 0.f) r += beta * to_f(prev[j]);
          o[j] = from_f<T>(r);
        }
        *(V*)(dx + row * D + vi * VEC) = o;
      }
    }
  }
#pragma unroll
  for (int i = 0; i < RMS_MAXV; ++i) {
    const int vi = lane + i * 64;
    if (vi < nv)
#pragma unroll
      for (int j = 0; j < VEC; ++j) red[wv * D + vi * VEC + j] = pw[i][j];
  }
  __syncthreads();
  for (int c = threadIdx.x; c < D; c += 256)
    part[(long)blockIdx.x * D + c] = (red[c] + red[D + c]) + (red[2 * D + c] + red[3 * D + c]);
}

__global__ void rms_bwd_finalize_kernel(const float* __restrict__ part, int nblk, int D,
                                        float* dw, float beta_acc) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= D) return;
  float a = 0.f;
  for (int k = 0; k < nblk; ++k) a += part[(long)k * D + c];
  dw[c] = beta_acc != 0.f ? beta_acc * dw[c] + a : a;
}

// transformers T5Attention._relative_position_bucket, bidirectional = False (decoder):
// n = max(q - k, 0); n < nb/2 exact, else nb/2 + log(n/(nb/2)) / log(maxd/(nb/2)) * (nb/2)
__device__ __forceinline__ int t5_bucket_causal(int n, int nb, int maxd) {
  const int exact = nb / 2;
  if (n < exact) return n;
  const int v = exact + (int)(logf((float)n / exact) / logf((float)maxd / exact) *
                              (float)(nb - exact));
  return min(v, nb - 1);
}

// bias[h][q][k] = table[bucket(q - k)][h]  (fp32, shared by the batch and all layers)
__global__ void t5_pos_bias_kernel(const float* __restrict__ table, int H, int L, int nb,
                                   int maxd, float* __restrict__ bias) {
  GRID_STRIDE(i, (long)H * L * L) {
    const int k = (int)(i % L);
    const long t = i / L;
    const int q = (int)(t % L), h = (int)(t / L);
    bias[i] = table[t5_bucket_causal(max(q - k, 0), nb, maxd) * H + h];
  }
}

// dtable[b][h] (+)= sum over batch and the (q, k <= q) cells whose relative position falls in
// bucket b of dS[n][h][q][k] (the bias gradient is the score gradient; masked cells k > q
// have dS = 0).  One block per (h, bucket), fixed-order block reduction (deterministic).
template <typename T>
__global__ __launch_bounds__(256) void t5_pos_bias_bwd_kernel(
    const T* __restrict__ ds, int B, int H, int L, int LP, int nb, int maxd,
    float* __restrict__ dtable, float beta) {
  __shared__ float red[4];
  const int h = blockIdx.x, bk = blockIdx.y;
  // relative positions n in [lo, hi) map to bucket bk (monotone bucket function)
  int lo = -1, hi = -1;
  for (int n = 0; n < L; ++n) {
    const int b = t5_bucket_causal(n, nb, maxd);
    if (b == bk) {
      if (lo < 0) lo = n;
      hi = n + 1;
    }
  }
  float acc = 0.f;
  if (lo >= 0) {
    // cells with q - k = n, n in [lo, hi): for each n, q = n .. L-1
    const long per_b = 0;
    (void)per_b;
    for (int n = lo; n < hi; ++n) {
      const int cnt = L - n;
      for (long e = threadIdx.x; e < (long)B * cnt; e += blockDim.x) {
        const int b = (int)(e / cnt), q = n + (int)(e % cnt);
        acc += to_f(ds[(((long)b * H + h) * L + q) * LP + (q - n)]);
      }
    }
  }
  acc = block_sum<256>(acc, red);
  if (threadIdx.x == 0) {
    float* o = dtable + bk * H + h;
    *o = beta != 0.f ? beta * *o + acc : acc;
  }
}

// Cross-attention over LK <= 16 condition tokens, head dim 64, no bias / mask:
// S = scale * Q K^T, P = softmax(S), O = dropout(P) V.  One thread per (n, q, h) row.
// q: [B][Lq] rows of ld_q elements (head h at +h*64); kv: [B][Lk][2][H][64] (k | v);
// probs [B][H][Lq][Lk] fp32 with the dropout keep bit in the sign (as mmdx_attention_fwd).
constexpr int XA_MAXK = 16;
__device__ __forceinline__ uint32_t xa_hash64(uint64_t x) {
  x ^= x >> 33; x *= 0xff51afd7ed558ccdULL;
  x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ULL;
  x ^= x >> 33;
  return (uint32_t)x;
}

template <typename T>
__global__ __launch_bounds__(256) void xattn_fwd_kernel(
    const T* __restrict__ q, long ldq, const T* __restrict__ kv, int B, int Lq, int Lk, int H,
    float scale, float p_drop, uint64_t seed, const uint64_t* __restrict__ ctr,
    T* __restrict__ out, float* __restrict__ probs) {
  const long i = blockIdx.x * (long)blockDim.x + threadIdx.x;
  if (i >= (long)B * Lq * H) return;
  const int h = (int)(i % H);
  const long t = i / H;
  const int qi = (int)(t % Lq), b = (int)(t / Lq);
  const T* qr = q + ((long)b * Lq + qi) * ldq + h * 64;
  float qv[64];
#pragma unroll
  for (int d = 0; d < 64; ++d) qv[d] = to_f(qr[d]);
  float s[XA_MAXK];
  float mx = -INFINITY;
  for (int j = 0; j < Lk; ++j) {
    const T* kr = kv + (((long)b * Lk + j) * 2 * H + h) * 64;
    float a = 0.f;
#pragma unroll
    for (int d = 0; d < 64; ++d) a += qv[d] * to_f(kr[d]);
    s[j] = a * scale;
    mx = fmaxf(mx, s[j]);
  }
  float sum = 0.f;
  for (int j = 0; j < Lk; ++j) {
    s[j] = __expf(s[j] - mx);
    sum += s[j];
  }
  const float inv = 1.f / sum;
  const bool drop = p_drop > 0.f;
  const float keep_scale = drop ? 1.f / (1.f - p_drop) : 1.f;
  const uint64_t rbase = drop ? seed * 0x9E3779B97F4A7C15ULL + (ctr ? ctr[0] << 32 : 0ull) : 0ull;
  float o[64];
#pragma unroll
  for (int d = 0; d < 64; ++d) o[d] = 0.f;
  float* pr = probs ? probs + (((long)b * H + h) * Lq + qi) * Lk : nullptr;
  for (int j = 0; j < Lk; ++j) {
    const float p = s[j] * inv;
    bool keep = true;
    if (drop) {
      const uint64_t idx = (((uint64_t)b * H + h) * Lq + qi) * (uint64_t)Lk + j;
      keep = (xa_hash64(rbase + idx) >> 8) * (1.f / 16777216.f) >= p_drop;
    }
    if (pr) pr[j] = keep ? p : -p;
    const float pe = keep ? p * keep_scale : 0.f;
    const T* vr = kv + (((long)b * Lk + j) * 2 * H + H + h) * 64;
#pragma unroll
    for (int d = 0; d < 64; ++d) o[d] += pe * to_f(vr[d]);
  }
  T* orow = out + (((long)b * Lq + qi) * H + h) * 64;
#pragma unroll
  for (int d = 0; d < 64; ++d) orow[d] = from_f<T>(o[d]);
}

// Backward part 1, per (n, q, h): dP'_j = dO . v_j, dP_j = keep * dP'_j / (1 - p),
// dS_j = P_j (dP_j - sum_i P_i dP_i); dq = scale * sum_j dS_j k_j; dS and P' saved for part 2.
template <typename T>
__global__ __launch_bounds__(256) void xattn_bwd_q_kernel(
    const T* __restrict__ kv, const float* __restrict__ probs, const T* __restrict__ dout,
    int B, int Lq, int Lk, int H, float scale, float keep_scale, T* __restrict__ dq, long lddq,
    float* __restrict__ ds_out, float* __restrict__ pe_out) {
  const long i = blockIdx.x * (long)blockDim.x + threadIdx.x;
  if (i >= (long)B * Lq * H) return;
  const int h = (int)(i % H);
  const long t = i / H;
  const int qi = (int)(t % Lq), b = (int)(t / Lq);
  const T* dor = dout + (((long)b * Lq + qi) * H + h) * 64;
  float dov[64];
#pragma unroll
  for (int d = 0; d < 64; ++d) dov[d] = to_f(dor[d]);
  const long prow = (((long)b * H + h) * Lq + qi) * Lk;
  float p[XA_MAXK], dp[XA_MAXK];
  float dot = 0.f;
  for (int j = 0; j < Lk; ++j) {
    const float v = probs[prow + j];
    const bool keep = !__builtin_signbitf(v);
    p[j] = fabsf(v);
    const T* vr = kv + (((long)b * Lk + j) * 2 * H + H + h) * 64;
    float a = 0.f;
#pragma unroll
    for (int d = 0; d < 64; ++d) a += dov[d] * to_f(vr[d]);
    dp[j] = keep ? a * keep_scale : 0.f;
    pe_out[prow + j] = keep ? p[j] * keep_scale : 0.f;
    dot += p[j] * dp[j];
  }
  float g[64];
#pragma unroll
  for (int d = 0; d < 64; ++d) g[d] = 0.f;
  for (int j = 0; j < Lk; ++j) {
    const float dsj = p[j] * (dp[j] - dot);
    ds_out[prow + j] = dsj;
    const T* kr = kv + (((long)b * Lk + j) * 2 * H + h) * 64;
#pragma unroll
    for (int d = 0; d < 64; ++d) g[d] += dsj * to_f(kr[d]);
  }
  T* dqr = dq + ((long)b * Lq + qi) * lddq + h * 64;
#pragma unroll
  for (int d = 0; d < 64; ++d) dqr[d] = from_f<T>(g[d] * scale);
}

// Backward part 2, per (n, j, h, d): dk = scale * sum_q dS_qj q[q][d], dv = sum_q P'_qj dO[q][d]
template <typename T>
__global__ __launch_bounds__(256) void xattn_bwd_kv_kernel(
    const T* __restrict__ q, long ldq, const T* __restrict__ dout, const float* __restrict__ ds,
    const float* __restrict__ pe, int B, int Lq, int Lk, int H, float scale,
    T* __restrict__ dkv) {
  const long i = blockIdx.x * (long)blockDim.x + threadIdx.x;
  if (i >= (long)B * Lk * H * 64) return;
  const int d = (int)(i & 63);
  const long t = i >> 6;
  const int h = (int)(t % H);
  const long t2 = t / H;
  const int j = (int)(t2 % Lk), b = (int)(t2 / Lk);
  float ak = 0.f, av = 0.f;
  const long pb = ((long)b * H + h) * Lq;
  for (int qi = 0; qi < Lq; ++qi) {
    const long pj = (pb + qi) * Lk + j;
    ak += ds[pj] * to_f(q[((long)b * Lq + qi) * ldq + h * 64 + d]);
    av += pe[pj] * to_f(dout[(((long)b * Lq + qi) * H + h) * 64 + d]);
  }
  T* row = dkv + (((long)b * Lk + j) * 2 * H + h) * 64 + d;
  row[0] = from_f<T>(ak * scale);
  row[(long)H * 64] = from_f<T>(av);
}

// CrossEntropyLoss(ignore_index=-100, mean over the non-ignored rows) over fp32 logits.
// Forward per row: lse = log sum exp; row_loss = lse - logit[target]; then one block sums
// (fixed order) and divides by the count.  Backward: dlogits = (softmax - onehot) * g / count.
__global__ __launch_bounds__(256) void ce_row_kernel(const float* __restrict__ logits,
                                                     const int64_t* __restrict__ tgt, long V,
                                                     float* __restrict__ lse,
                                                     float* __restrict__ row_loss) {
  __shared__ float red[4];
  const long r = blockIdx.x;
  const float* x = logits + r * V;
  float mx = -INFINITY;
  for (long v = threadIdx.x; v < V; v += 256) mx = fmaxf(mx, x[v]);
  mx = wave_max(mx);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = mx;
  __syncthreads();
  mx = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  __syncthreads();
  float s = 0.f;
  for (long v = threadIdx.x; v < V; v += 256) s += __expf(x[v] - mx);
  s = block_sum<256>(s, red);
  if (threadIdx.x == 0) {
    const float l = mx + logf(s);
    lse[r] = l;
    const int64_t t = tgt ? tgt[r] : -100;
    row_loss[r] = (t >= 0 && t < V) ? l - x[t] : 0.f;
    row_loss[r + gridDim.x] = (t >= 0 && t < V) ? 1.f : 0.f;  // valid flag
  }
}

__global__ __launch_bounds__(256) void ce_reduce_kernel(const float* __restrict__ row_loss,
                                                        long R, float* loss, float* count) {
  __shared__ float red[4];
  float s = 0.f, c = 0.f;
  for (long r = threadIdx.x; r < R; r += 256) {
    s += row_loss[r];
    c += row_loss[r + R];
  }
  s = block_sum<256>(s, red);
  c = block_sum<256>(c, red);
  if (threadIdx.x == 0) {
    *count = c;
    *loss = c > 0.f ? s / c : NAN;  // torch: mean over zero elements is nan
  }
}

template <typename T>
__global__ __launch_bounds__(256) void ce_bwd_kernel(const float* __restrict__ logits,
                                                     const int64_t* __restrict__ tgt, long V,
                                                     const float* __restrict__ lse,
                                                     const float* __restrict__ gscale,
                                                     const float* __restrict__ count,
                                                     T* __restrict__ dlogits) {
  const long r = blockIdx.x;
  const int64_t t = tgt[r];
  const bool valid = t >= 0 && t < V;
  const float g = valid && *count > 0.f ? (gscale ? *gscale : 1.f) / *count : 0.f;
  const float l = lse[r];
  const float* x = logits + r * V;
  T* o = dlogits + r * V;
  for (long v = threadIdx.x; v < V; v += 256) {
    const float p = valid ? __expf(x[v] - l) : 0.f;
    o[v] = from_f<T>(g * (p - (v == t ? 1.f : 0.f)));
  }
}

__global__ __launch_bounds__(256) void log_softmax_kernel(const float* __restrict__ logits,
                                                          long V, float* __restrict__ out) {
  __shared__ float red[4];
  const long r = blockIdx.x;
  const float* x = logits + r * V;
  float mx = -INFINITY;
  for (long v = threadIdx.x; v < V; v += 256) mx = fmaxf(mx, x[v]);
  mx = wave_max(mx);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = mx;
  __syncthreads();
  mx = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  __syncthreads();
  float s = 0.f;
  for (long v = threadIdx.x; v < V; v += 256) s += __expf(x[v] - mx);
  s = block_sum<256>(s, red);
  const float l = mx + logf(s);
  for (long v = threadIdx.x; v < V; v += 256) out[r * V + v] = x[v] - l;
}

template <typename T>
__global__ void relu_bwd_kernel(const T* __restrict__ y, const T* __restrict__ dy, long n,
                                T* __restrict__ dx) {
  GRID_STRIDE(i, n) dx[i] = to_f(y[i]) > 0.f ? dy[i] : from_f<T>(0.f);
}

// One incremental beam-search step of the decoder's causal self-attention with a KV cache
// (generate, IP:190-196 / TP:613-618; transformers appends each step's K/V to a cache instead
// of re-running the prefix).  Block (r, h), one wave: the query of position `pos` of row r
// attends keys 0..pos of head h.  Beam search reorders rows without moving the cache: key j
// of row r lives in cache row slots[r * Lmax + j]; this step's own K/V (qkv) are used
// directly for j == pos and appended to the cache at (row r, pos) at the end (nothing reads
// position pos of the cache in this launch).  Scores are unscaled (T5) plus the relative-
// position bias[h][pos][j]; lanes own keys for the scores (<= DEC_MAXL / 64 per lane), then
// dims for P.V.  fp32 math.
constexpr int DEC_MAXL = 512;

template <typename T>
__global__ __launch_bounds__(64) void t5_decode_attn_kernel(
    const T* __restrict__ qkv, int H, int pos, int Lmax, T* __restrict__ kc,
    T* __restrict__ vc, const int* __restrict__ slots, const float* __restrict__ bias,
    T* __restrict__ out) {
  constexpr int NI = DEC_MAXL / 64;
  const int r = blockIdx.x, h = blockIdx.y, lane = threadIdx.x;
  const long D = (long)H * 64;
  const T* qrow = qkv + (long)r * 3 * D + h * 64;
  const T* knew = qrow + D;
  const T* vnew = qrow + 2 * D;
  float q[64];
#pragma unroll
  for (int d = 0; d < 64; ++d) q[d] = to_f(qrow[d]);
  const float* brow = bias + ((long)h * Lmax + pos) * Lmax;
  const int* srow = slots + (long)r * Lmax;
  float sc[NI];
  float mx = -INFINITY;
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    const int j = lane + 64 * i;
    sc[i] = -INFINITY;
    if (j <= pos) {
      const T* kr = j == pos ? knew : kc + ((long)srow[j] * Lmax + j) * D + h * 64;
      float acc = 0.f;
#pragma unroll
      for (int d = 0; d < 64; ++d) acc += q[d] * to_f(kr[d]);
      sc[i] = acc + brow[j];
      mx = fmaxf(mx, sc[i]);
    }
  }
  mx = wave_max(mx);
  float sum = 0.f;
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    sc[i] = lane + 64 * i <= pos ? __expf(sc[i] - mx) : 0.f;
    sum += sc[i];
  }
  sum = wave_sum(sum);
  const float inv = 1.f / sum;
  float o = 0.f;
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    const int jn = min(64, pos + 1 - 64 * i);
    for (int jj = 0; jj < jn; ++jj) {
      const int j = 64 * i + jj;
      const float pj = __shfl(sc[i], jj, 64);
      const T* vr = j == pos ? vnew : vc + ((long)srow[j] * Lmax + j) * D + h * 64;
      o += pj * to_f(vr[lane]);
    }
  }
  out[(long)r * D + h * 64 + lane] = from_f<T>(o * inv);
  kc[((long)r * Lmax + pos) * D + h * 64 + lane] = knew[lane];
  vc[((long)r * Lmax + pos) * D + h * 64 + lane] = vnew[lane];
}

// Beam-search candidate selection (transformers' _beam_search: topk over the nb*V running
// scores of a batch row): per batch row b (one block), the k largest of
// lp[b*nb + i][v] + run_sc[b*nb + i] over (i, v), ordered by value descending then by flat
// index i*V + v ascending (numpy's stable argsort order).  Before the scan the block writes
// -inf into its rows of lp at the banned (row, token) pairs (no_repeat_ngram_size) and, when
// eos >= 0, at the EOS column (min_new_tokens) — the logits processors of the step.
// Each thread keeps a sorted top-KMAX of its strided slice in registers; k rounds of a block
// arg-max over the threads' heads then pop the winners.
constexpr int TOPK_MAX = 16;

__device__ __forceinline__ bool beats(float va, long ia, float vb, long ib) {
  return va > vb || (va == vb && ia < ib);
}

__global__ __launch_bounds__(256) void beam_topk_kernel(float* __restrict__ lp, int nb, long V,
                                                        const float* __restrict__ run_sc,
                                                        const int* __restrict__ ban, int nban,
                                                        int eos, int k, float* __restrict__ oval,
                                                        long* __restrict__ oidx) {
  __shared__ float sv[256];
  __shared__ long si[256];
  __shared__ int swin;
  const int b = blockIdx.x, tid = threadIdx.x;
  const long r0 = (long)b * nb;
  for (int i = tid; i < nban; i += 256) {
    const long r = ban[2 * i], t = ban[2 * i + 1];
    if (r >= r0 && r < r0 + nb && t >= 0 && t < V) lp[r * V + t] = -INFINITY;
  }
  if (eos >= 0 && eos < V)
    for (int i = tid; i < nb; i += 256) lp[(r0 + i) * V + eos] = -INFINITY;
  __syncthreads();
  float tv[TOPK_MAX];
  long ti[TOPK_MAX];
#pragma unroll
  for (int j = 0; j < TOPK_MAX; ++j) { tv[j] = -INFINITY; ti[j] = LONG_MAX; }
  const long n = (long)nb * V;
  for (long e = tid; e < n; e += 256) {
    const long i = e / V;
    const float v = lp[r0 * V + e] + run_sc[r0 + i];
    if (!beats(v, e, tv[TOPK_MAX - 1], ti[TOPK_MAX - 1])) continue;
    // insertion into the sorted register list (compile-time indices only)
    float cv = v;
    long ci = e;
#pragma unroll
    for (int j = 0; j < TOPK_MAX; ++j) {
      if (beats(cv, ci, tv[j], ti[j])) {
        const float xv = tv[j];
        const long xi = ti[j];
        tv[j] = cv; ti[j] = ci;
        cv = xv; ci = xi;
      }
    }
  }
  for (int q = 0; q < k; ++q) {
    sv[tid] = tv[0];
    si[tid] = ti[0];
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
      if (tid < w && beats(sv[tid + w], si[tid + w], sv[tid], si[tid])) {
        sv[tid] = sv[tid + w];
        si[tid] = si[tid + w];
      }
      __syncthreads();
    }
    if (tid == 0) {
      oval[(long)b * k + q] = sv[0];
      oidx[(long)b * k + q] = si[0];
    }
    if (ti[0] == si[0]) {  // the winner pops its head (indices are unique)
#pragma unroll
      for (int j = 0; j < TOPK_MAX - 1; ++j) { tv[j] = tv[j + 1]; ti[j] = ti[j + 1]; }
      tv[TOPK_MAX - 1] = -INFINITY;
      ti[TOPK_MAX - 1] = LONG_MAX;
    }
    __syncthreads();
  }
}

}  // namespace mmdx

using namespace mmdx;

#define T5_DISPATCH(dtype, ...) MMDX_DISPATCH(dtype, __VA_ARGS__)

extern "C" int mmdx_beam_topk(float* log_probs, int B, int nb, long V, const float* run_scores,
                              const int* ban_pairs, int n_ban, int eos_ban, int k,
                              float* out_val, long* out_idx, void* stream) {
  MMDX_CHECK_ARG(log_probs && run_scores && out_val && out_idx && B > 0 && nb > 0 && V > 0 &&
                     k > 0 && k <= TOPK_MAX && k <= (long)nb * V && (n_ban == 0 || ban_pairs),
                 "beam topk: bad args (k=%d <= %d)", k, TOPK_MAX);
  hipLaunchKernelGGL(beam_topk_kernel, dim3(B), dim3(256), 0, (hipStream_t)stream, log_probs, nb,
                     V, run_scores, ban_pairs, n_ban, eos_ban, k, out_val, out_idx);
  MMDX_LAUNCH_CHECK();
  return 0;
}

extern "C" int mmdx_t5_decode_attn(int dtype, const void* qkv, int R, int H, int pos, int Lmax,
                                   void* k_cache, void* v_cache, const int* slots,
                                   const float* bias, void* out, void* stream) {
  MMDX_CHECK_ARG(qkv && k_cache && v_cache && slots && bias && out && R > 0 && H > 0 &&
                     Lmax > 0 && Lmax <= DEC_MAXL && pos >= 0 && pos < Lmax,
                 "t5 decode attention: bad args (pos=%d, Lmax=%d <= %d)", pos, Lmax, DEC_MAXL);
  T5_DISPATCH(dtype, hipLaunchKernelGGL(t5_decode_attn_kernel<T>, dim3(R, H), dim3(64), 0,
                                        (hipStream_t)stream, (const T*)qkv, H, pos, Lmax,
                                        (T*)k_cache, (T*)v_cache, slots, bias, (T*)out));
  MMDX_LAUNCH_CHECK();
  return 0;
}

extern "C" int mmdx_rmsnorm_fwd(int dtype, const void* x, long rows, int D, const float* w,
                                float eps, void* y, float* save_rstd, void* stream) {
  const int VEC = dtype == F32 ? 4 : 8;
  MMDX_CHECK_ARG(rows > 0 && D % VEC == 0 && D <= 64 * RMS_MAXV * VEC && w,
                 "rmsnorm: D=%d unsupported", D);
  T5_DISPATCH(dtype, hipLaunchKernelGGL(rms_fwd_kernel<T>, dim3((rows + 3) / 4), dim3(256), 0,
                                        (hipStream_t)stream, (const T*)x, rows, D, w, eps,
                                        (T*)y, save_rstd));
  MMDX_LAUNCH_CHECK();
  return 0;
}

extern "C" size_t mmdx_rmsnorm_workspace_size(long rows, int D) {
  return (size_t)((rows + RMS_BWD_ROWS - 1) / RMS_BWD_ROWS) * D * sizeof(float);
}

extern "C" int mmdx_rmsnorm_bwd(int dtype, const void* x, const void* dy, long rows, int D,
                                const float* w, const float* save_rstd, void* dx, float beta,
                                float* dw, float dw_beta, void* ws, size_t ws_bytes,
                                void* stream) {
  const int VEC = dtype == F32 ? 4 : 8;
  MMDX_CHECK_ARG(rows > 0 && D % VEC == 0 && D <= 64 * RMS_MAXV * VEC, "rmsnorm bwd: D=%d", D);
  MMDX_CHECK_ARG(ws && ws_bytes >= mmdx_rmsnorm_workspace_size(rows, D),
                 "rmsnorm bwd: workspace too small");
  hipStream_t st = (hipStream_t)stream;
  const long nblk = (rows + RMS_BWD_ROWS - 1) / RMS_BWD_ROWS;
  const size_t shm = 4 * (size_t)D * sizeof(float);
  T5_DISPATCH(dtype, hipLaunchKernelGGL(rms_bwd_kernel<T>, dim3(nblk), dim3(256), shm, st,
                                        (const T*)x, (const T*)dy, rows, D, w, save_rstd, beta,
                                        (T*)dx, (float*)ws));
  if (dw)
    hipLaunchKernelGGL(rms_bwd_finalize_kernel, dim3((D + 255) / 256), dim3(256), 0, st,
                       (const float*)ws, (int)nblk, D, dw, dw_beta);
  MMDX_LAUNCH_CHECK();
  return 0;
}

extern "C" int mmdx_t5_position_bias(const float* table, int H, int L, int num_buckets,
                                     int max_distance, float* bias, void* stream) {
  MMDX_CHECK_ARG(table && bias && H > 0 && L > 0 && num_buckets >= 2 && max_distance > 0,
                 "t5 position bias: bad args");
  const long n = (long)H * L * L;
  hipLaunchKernelGGL(t5_pos_bias_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream,
                     table, H, L, num_buckets, max_distance, bias);
  MMDX_LAUNCH_CHECK();
  return 0;
}

extern "C" int mmdx_t5_position_bias_bwd(int dtype, const void* dscores, int B, int H, int L,
                                         int ld, int num_buckets, int max_distance,
                                         float* dtable, float beta, void* stream) {
  MMDX_CHECK_ARG(dscores && dtable && B > 0 && H > 0 && L > 0 && ld >= L,
                 "t5 position bias bwd: bad args");
  T5_DISPATCH(dtype, hipLaunchKernelGGL(t5_pos_bias_bwd_kernel<T>, dim3(H, num_buckets),
                                        dim3(256), 0, (hipStream_t)stream, (const T*)dscores, B,
                                        H, L, ld, num_buckets, max_distance, dtable, beta));
  MMDX_LAUNCH_CHECK();
  return 0;
}

__global__ void xattn_counter_incr_kernel(uint64_t* c) { c[0] += 1; }

extern "C" int mmdx_xattn_fwd(int dtype, const void* q, long ldq, const void* kv, int B, int Lq,
                              int Lk, int H, float scale, float p_drop, uint64_t seed,
                              uint64_t* counter, void* out, float* probs, void* stream) {
  MMDX_CHECK_ARG(B > 0 && Lq > 0 && Lk > 0 && Lk <= XA_MAXK && H > 0 && ldq >= 64L * H,
                 "cross attention: Lk=%d (<= %d)", Lk, XA_MAXK);
  MMDX_CHECK_ARG(p_drop >= 0.f && p_drop < 1.f && (p_drop == 0.f || probs),
                 "cross attention: bad dropout");
  hipStream_t st = (hipStream_t)stream;
  const long n = (long)B * Lq * H;
  T5_DISPATCH(dtype, hipLaunchKernelGGL(xattn_fwd_kernel<T>, dim3((n + 255) / 256), dim3(256),
                                        0, st, (const T*)q, ldq, (const T*)kv, B, Lq, Lk, H,
                                        scale, p_drop, seed, (const uint64_t*)counter, (T*)out,
                                        probs));
  if (p_drop > 0.f && counter)
    hipLaunchKernelGGL(xattn_counter_incr_kernel, dim3(1), dim3(1), 0, st, counter);
  MMDX_LAUNCH_CHECK();
  return 0;
}

extern "C" size_t mmdx_xattn_workspace_size(int B, int Lq, int Lk, int H) {
  return 2 * (size_t)B * H * Lq * Lk * sizeof(float);
}

extern "C" int mmdx_xattn_bwd(int dtype, const void* q, long ldq, const void* kv,
                              const float* probs, const void* dout, int B, int Lq, int Lk, int H,
                              float scale, float p_drop, void* dq, long lddq, void* dkv,
                              void* ws, size_t ws_bytes, void* stream) {
  MMDX_CHECK_ARG(B > 0 && Lq > 0 && Lk > 0 && Lk <= XA_MAXK && probs && p_drop >= 0.f &&
                     p_drop < 1.f,
                 "cross attention bwd: bad args");
  MMDX_CHECK_ARG(ws && ws_bytes >= mmdx_xattn_workspace_size(B, Lq, Lk, H),
                 "cross attention bwd: workspace too small");
  hipStream_t st = (hipStream_t)stream;
  float* ds = (float*)ws;
  float* pe = ds + (size_t)B * H * Lq * Lk;
  const float keep_scale = 1.f / (1.f - p_drop);
  const long n = (long)B * Lq * H;
  const long nkv = (long)B * Lk * H * 64;
  T5_DISPATCH(dtype, {
    hipLaunchKernelGGL(xattn_bwd_q_kernel<T>, dim3((n + 255) / 256), dim3(256), 0, st,
                       (const T*)kv, probs, (const T*)dout, B, Lq, Lk, H, scale, keep_scale,
                       (T*)dq, lddq, ds, pe);
    hipLaunchKernelGGL(xattn_bwd_kv_kernel<T>, dim3((nkv + 255) / 256), dim3(256), 0, st,
                       (const T*)q, ldq, (const T*)dout, ds, pe, B, Lq, Lk, H, scale, (T*)dkv);
  });
  MMDX_LAUNCH_CHECK();
  return 0;
}

extern "C" size_t mmdx_cross_entropy_workspace_size(long rows) {
  return (size_t)rows * 3 * sizeof(float) + 256;
}

extern "C" int mmdx_cross_entropy_fwd(const float* logits, const int64_t* targets, long rows,
                                      long V, float* loss, float* count, void* ws,
                                      size_t ws_bytes, void* stream) {
  MMDX_CHECK_ARG(logits && targets && rows > 0 && V > 0 && loss && count,
                 "cross entropy: bad args");
  MMDX_CHECK_ARG(ws && ws_bytes >= mmdx_cross_entropy_workspace_size(rows),
                 "cross entropy: workspace too small");
  hipStream_t st = (hipStream_t)stream;
  float* lse = (float*)ws;
  float* row = lse + rows;
  hipLaunchKernelGGL(ce_row_kernel, dim3(rows), dim3(256), 0, st, logits, targets, V, lse, row);
  hipLaunchKernelGGL(ce_reduce_kernel, dim3(1), dim3(256), 0, st, (const float*)row, rows, loss,
                     count);
  MMDX_LAUNCH_CHECK();
  return 0;
}

extern "C" int mmdx_cross_entropy_bwd(int dtype, const float* logits, const int64_t* targets,
                                      long rows, long V, const float* dloss, const float* count,
                                      const void* ws, void* dlogits, void* stream) {
  MMDX_CHECK_ARG(logits && targets && rows > 0 && V > 0 && count && ws && dlogits,
                 "cross entropy bwd: bad args");
  T5_DISPATCH(dtype, hipLaunchKernelGGL(ce_bwd_kernel<T>, dim3(rows), dim3(256), 0,
                                        (hipStream_t)stream, logits, targets, V,
                                        (const float*)ws, dloss, count, (T*)dlogits));
  MMDX_LAUNCH_CHECK();
  return 0;
}

extern "C" int mmdx_log_softmax(const float* logits, long rows, long V, float* out,
                                void* stream) {
  MMDX_CHECK_ARG(logits && out && rows > 0 && V > 0, "log_softmax: bad args");
  hipLaunchKernelGGL(log_softmax_kernel, dim3(rows), dim3(256), 0, (hipStream_t)stream, logits,
                     V, out);
  MMDX_LAUNCH_CHECK();
  return 0;
}

extern "C" int mmdx_relu_bwd(int dtype, const void* y, const void* dy, long n, void* dx,
                             void* stream) {
  MMDX_CHECK_ARG(y && dy && dx && n > 0, "relu bwd: bad args");
  T5_DISPATCH(dtype, hipLaunchKernelGGL(relu_bwd_kernel<T>, dim3(grid_for(n)), dim3(256), 0,
                                        (hipStream_t)stream, (const T*)y, (const T*)dy, n,
                                        (T*)dx));
  MMDX_LAUNCH_CHECK();
  return 0;
}
