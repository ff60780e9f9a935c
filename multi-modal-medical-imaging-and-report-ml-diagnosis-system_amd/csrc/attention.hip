// Multi-head self-attention core for BERT-base / ViT-B (head dim 64, L <= 256).
//
// Forward: one workgroup per (query block, head, batch); K and V of the head live in LDS.
// bf16 / f16 (the training dtypes) use swapped products (attn_fwd16_kernel, 8 waves = 128
// queries): S^T = K Q^T leaves each query on one lane column, the row softmax is a per-lane
// sum plus two shuffles, and P^T feeds O^T = V^T P^T straight from registers (V^T through
// transposed LDS reads).  fp32: S = Q K^T, 16-lane softmax, P -> LDS, O = P V.
// Probabilities are saved (fp32) for the backward.
// Backward: kernel A per query block: dP = dO V^T, dS = P o (dP - rowsum(P o dP)),
// dQ = scale dS K; kernel B per key block: dV = P^T dO, dK = scale dS^T Q (fp32: streaming
// query chunks through LDS; 16-bit: swapped as the forward, the head's Q and dO staged whole,
// P' and dS read straight into registers).  Blocks of one head share an XCD (attn_block).
// Additive key mask as BertSelfAttention (large negative on pads).
// Attention-probability dropout (BertSelfAttention's dropout on attention_probs, train
// mode): P' = P * keep / (1 - p) feeds O = P' V; keep comes from a counter-based hash of
// (seed, device launch counter, b, h, q, key).  The saved probabilities carry the keep bit
// in their sign (P >= 0: a dropped element is saved as -P), so the backward needs no RNG
// and no mask tensor: dV = P'^T dO, dP = keep * (dO V^T) / (1 - p),
// dS = P o (dP - rowsum(P o dP)).
#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include "igemm.h"
#include "../../include/mmdx.h"
#include <mutex>
#include <set>
#include <utility>

// hipFuncSetAttribute(MaxDynamicSharedMemorySize -> the full 160 KB of LDS) once per kernel
// and device, so no attribute call is issued again on the launch path: a launch sequence
// captured into a hipGraph then holds nothing but kernel nodes (the first call of each kernel
// runs eagerly, e.g. torch.cuda.make_graphed_callables' warm-up iterations).
static void mmdx_lds_max_once(const void* kern) {
  static std::mutex mu;
  static std::set<std::pair<int, const void*>> done;
  int dev = 0;
  (void)hipGetDevice(&dev);
  std::lock_guard<std::mutex> g(mu);
  if (done.insert({dev, kern}).second)
    (void)hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
}


namespace mmdx {

constexpr int HD = 64;           // head dim
constexpr int MAXKT = 16;        // max 16-key tiles (L <= 256)
constexpr float MASK_NEG = -1e30f;

template <typename T> struct AttnCfg;
template <> struct AttnCfg<bf16> { static constexpr int NW = 4; };   // 64 query rows / block
template <> struct AttnCfg<float> { static constexpr int NW = 2; };  // 32 query rows / block
template <> struct AttnCfg<f16> { static constexpr int NW = 4; };

__device__ __forceinline__ float rowgroup_max(float v) {
#pragma unroll
  for (int o = 1; o < 16; o <<= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ float rowgroup_sum(float v) {
#pragma unroll
  for (int o = 1; o < 16; o <<= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Global -> LDS staging of rows x 64-element head slices (16-B vectors, zero beyond
// rows_valid).  Every thread issues all U loads of a round before its first LDS store, so a
// round costs one memory latency; the former load-store-per-vector loop serialised 7-16 of
// them per block and made the attention kernels latency bound (isolated ViT fwd 128 us).
template <typename T, bool TR>
__device__ __forceinline__ void put_row_vec(T* dst, int ld, int r, int c,
                                            const typename Vec16<T>::type& v) {
  if (TR) {  // dst[c][r] = src[r][c]
#pragma unroll
    for (int j = 0; j < Vec16<T>::N; ++j) dst[(c + j) * ld + r] = v[j];
  } else {
    *(typename Vec16<T>::type*)(dst + r * ld + c) = v;
  }
}
// Two tiles of identical row geometry (K and V, or V and K, of one head): U vectors of each
// in flight per thread per round.  TA / TB: whether tile a / b is stored transposed.
template <typename T, int U, bool TA, bool TB>
__device__ __forceinline__ void stage_pair(T* da, int lda, const T* sa, T* db, int ldb,
                                           const T* sb, long src_ld, int rows, int rows_valid,
                                           int nthreads) {
  typedef typename Vec16<T>::type V;
  constexpr int VEC = Vec16<T>::N, VPR = HD / VEC;
  const int total = rows * VPR;
  for (int i0 = threadIdx.x; i0 < total; i0 += U * nthreads) {
    V va[U], vb[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = i0 + u * nthreads, r = i / VPR, c = (i - r * VPR) * VEC;
      va[u] = V{};
      vb[u] = V{};
      if (i < total && r < rows_valid) {
        va[u] = *(const V*)(sa + r * src_ld + c);
        vb[u] = *(const V*)(sb + r * src_ld + c);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = i0 + u * nthreads, r = i / VPR, c = (i - r * VPR) * VEC;
      if (i < total) {
        put_row_vec<T, TA>(da, lda, r, c, va[u]);
        put_row_vec<T, TB>(db, ldb, r, c, vb[u]);
      }
    }
  }
}
template <typename T, int U, bool TR>
__device__ __forceinline__ void stage_rows(T* dst, int ld, const T* src, long src_ld, int rows,
                                           int rows_valid, int nthreads) {
  typedef typename Vec16<T>::type V;
  constexpr int VEC = Vec16<T>::N, VPR = HD / VEC;
  const int total = rows * VPR;
  for (int i0 = threadIdx.x; i0 < total; i0 += U * nthreads) {
    V v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = i0 + u * nthreads, r = i / VPR, c = (i - r * VPR) * VEC;
      v[u] = V{};
      if (i < total && r < rows_valid) v[u] = *(const V*)(src + r * src_ld + c);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = i0 + u * nthreads, r = i / VPR, c = (i - r * VPR) * VEC;
      if (i < total) put_row_vec<T, TR>(dst, ld, r, c, v[u]);
    }
  }
}

// XCD-aware block order for a 1-D grid of nb blocks per (batch, head): the 8 XCDs take linear
// block ids round-robin and each has its own L2, so the nb blocks of one head, which all read
// that head's K and V (or Q, dO, P), get ids congruent mod 8 and share one XCD's L2 instead
// of fetching the head once per XCD.
__device__ __forceinline__ void attn_block(int nb, int H, int& blk, int& h, int& b) {
  const int n = blockIdx.x, bh = gridDim.x / nb;
  int hl;
  if ((bh & 7) == 0) {
    const int k = n >> 3;
    blk = k % nb;
    hl = (k / nb) * 8 + (n & 7);
  } else {
    blk = n % nb;
    hl = n / nb;
  }
  h = hl % H;
  b = hl / H;
}

__device__ __forceinline__ uint32_t attn_hash64(uint64_t x) {
  x ^= x >> 33; x *= 0xff51afd7ed558ccdULL;
  x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ULL;
  x ^= x >> 33;
  return (uint32_t)x;
}

// (launch bounds: the LDS footprint allows two blocks per CU; the default 1024-thread budget
// of 128 VGPRs spilled the staged K / V vectors)
template <typename T>
__global__ __launch_bounds__(AttnCfg<T>::NW * 64, 2) void attn_fwd_kernel(
    const T* __restrict__ qkv, const int64_t* __restrict__ mask, const float* __restrict__ bias,
    int causal, int L, int H, float scale, float p_drop, uint64_t seed,
    const uint64_t* __restrict__ ctr, T* __restrict__ out, float* __restrict__ probs) {
  typedef MfmaOp<T> Op;
  constexpr int NW = AttnCfg<T>::NW, QB = NW * 16, PAD = Vec16<T>::N;
  constexpr int LDQ = HD + PAD;
  const int LP = (L + 31) & ~31;  // multiple of the bf16 MFMA K (32)
  const int LDV = LP + PAD;
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  const int KP = max(LP * LDQ, QB * LDV);
  T* Ks = (T*)smem_raw;                 // [LP][LDQ]; P [QB][LDV] reuses it after S = QK^T
  T* Ps = Ks;
  T* Vt = Ks + KP;                      // [HD][LDV]
  T* Qs = Vt + HD * LDV;                // [QB][LDQ]
  const int q0 = blockIdx.x * QB, h = blockIdx.y, b = blockIdx.z;
  const int nth = NW * 64;
  const long row_ld = 3L * H * HD;
  const T* base = qkv + (long)b * L * row_ld + h * HD;
  stage_pair<T, 4, false, true>(Ks, LDQ, base + (long)H * HD, Vt, LDV, base + 2L * H * HD,
                                row_ld, LP, L, nth);
  stage_rows<T, 4, false>(Qs, LDQ, base + (long)q0 * row_ld, row_ld, QB, min(QB, L - q0), nth);
  __syncthreads();
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int nkt = LP / 16;
  f32x4 s[MAXKT];
  const T* a_s = Qs + (wid * 16 + (lane & 15)) * LDQ + (lane >> 4) * Op::FRAG;
#pragma unroll
  for (int j = 0; j < MAXKT; ++j) {
    s[j] = f32x4{0.f, 0.f, 0.f, 0.f};
    if (j < nkt) {
      const T* b_s = Ks + (j * 16 + (lane & 15)) * LDQ + (lane >> 4) * Op::FRAG;
#pragma unroll
      for (int k = 0; k < HD; k += Op::KS) s[j] = Op::mma(Op::ld(a_s + k), Op::ld(b_s + k), s[j]);
    }
  }
  // scale + mask + row softmax (rows (lane>>4)*4+r of this wave's 16)
  float mx[4] = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
#pragma unroll
  for (int j = 0; j < MAXKT; ++j) {
    if (j >= nkt) continue;
    const int key = j * 16 + (lane & 15);
    const float madd = key < L ? (mask && mask[(long)b * L + key] == 0 ? MASK_NEG : 0.f) : -INFINITY;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int q = q0 + wid * 16 + (lane >> 4) * 4 + r;
      float v = s[j][r] * scale + madd;
      // additive score bias [H][L][L] (T5 relative position bias) and causal mask
      if (bias && key < L && q < L) v += bias[((long)h * L + q) * L + key];
      if (causal && key > q && key < L) v = MASK_NEG;
      s[j][r] = v;
      mx[r] = fmaxf(mx[r], s[j][r]);
    }
  }
  float sum[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) { mx[r] = rowgroup_max(mx[r]); sum[r] = 0.f; }
#pragma unroll
  for (int j = 0; j < MAXKT; ++j) {
    if (j >= nkt) continue;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      s[j][r] = __expf(s[j][r] - mx[r]);
      sum[r] += s[j][r];
    }
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) sum[r] = 1.f / rowgroup_sum(sum[r]);
  __syncthreads();  // every wave is done reading K: P may overwrite it
  float* prow = probs ? probs + (((long)b * H + h) * L) * L : nullptr;
  const bool drop = p_drop > 0.f;
  const float keep_scale = drop ? 1.f / (1.f - p_drop) : 1.f;
  const uint64_t rbase = drop ? seed * 0x9E3779B97F4A7C15ULL + (ctr ? ctr[0] << 32 : 0ull) +
                                    (((uint64_t)b * H + h) * L) * (uint64_t)L
                              : 0ull;
#pragma unroll
  for (int j = 0; j < MAXKT; ++j) {
    if (j >= nkt) continue;
    const int key = j * 16 + (lane & 15);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int rl = wid * 16 + (lane >> 4) * 4 + r;
      const float p = s[j][r] * sum[r];
      const int q = q0 + rl;
      bool keep = true;
      if (drop) {
        const float u = (attn_hash64(rbase + (uint64_t)q * L + key) >> 8) * (1.f / 16777216.f);
        keep = u >= p_drop;
      }
      Ps[rl * LDV + key] = from_f<T>(keep ? p * keep_scale : 0.f);
      if (prow && q < L && key < L) prow[(long)q * L + key] = keep ? p : -p;
    }
  }
  __syncthreads();
  // O[16][64] = P[16][LP] V[LP][64]
  f32x4 o[HD / 16];
#pragma unroll
  for (int j = 0; j < HD / 16; ++j) o[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const T* p_s = Ps + (wid * 16 + (lane & 15)) * LDV + (lane >> 4) * Op::FRAG;
  for (int k = 0; k < LP; k += Op::KS) {
    const typename Op::frag_t af = Op::ld(p_s + k);
#pragma unroll
    for (int j = 0; j < HD / 16; ++j) {
      const T* v_s = Vt + (j * 16 + (lane & 15)) * LDV + (lane >> 4) * Op::FRAG;
      o[j] = Op::mma(af, Op::ld(v_s + k), o[j]);
    }
  }
#pragma unroll
  for (int j = 0; j < HD / 16; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int q = q0 + wid * 16 + (lane >> 4) * 4 + r;
      if (q < L) out[(((long)b * L + q) * H + h) * HD + j * 16 + (lane & 15)] = from_f<T>(o[j][r]);
    }
}

// Backward A: per query block -> dS (T, global scratch [B,H,L,LP]) and dQ.
template <typename T>
// (launch bounds: without them the compiler budgets registers for 1024-thread blocks, 128
// VGPRs, and spilled 17 of the dP row tiles to scratch; the LDS footprint allows two blocks
// per CU = two waves per SIMD anyway)
__global__ __launch_bounds__(AttnCfg<T>::NW * 64, 2) void attn_bwd_q_kernel(
    const T* __restrict__ qkv, const float* __restrict__ probs,
                                  const T* __restrict__ dout, int L, int H, float scale,
                                  float keep_scale, T* __restrict__ dS_g,
                                  T* __restrict__ dqkv) {
  typedef MfmaOp<T> Op;
  constexpr int NW = AttnCfg<T>::NW, QB = NW * 16, PAD = Vec16<T>::N;
  constexpr int LDQ = HD + PAD;
  const int LP = (L + 31) & ~31;  // multiple of the bf16 MFMA K (32)
  const int LDV = LP + PAD;
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  const int KP = max(LP * LDQ, QB * LDV);
  T* Vs = (T*)smem_raw;                 // [LP][LDQ] V rows (K-major for dP); dS reuses it
  T* dSs = Vs;                          // [QB][LDV]
  T* Kt = Vs + KP;                      // [HD][LDV]   K^T (for dQ)
  T* dOs = Kt + HD * LDV;               // [QB][LDQ]
  const int q0 = blockIdx.x * QB, h = blockIdx.y, b = blockIdx.z;
  const int nth = NW * 64;
  const long row_ld = 3L * H * HD;
  const T* base = qkv + (long)b * L * row_ld + h * HD;
  stage_pair<T, 8, false, true>(Vs, LDQ, base + 2L * H * HD, Kt, LDV, base + (long)H * HD,
                                row_ld, LP, L, nth);
  stage_rows<T, 4, false>(dOs, LDQ, dout + ((long)b * L + q0) * H * HD + h * HD, (long)H * HD,
                          QB, min(QB, L - q0), nth);
  __syncthreads();
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int nkt = LP / 16;
  f32x4 s[MAXKT];
  const T* a_s = dOs + (wid * 16 + (lane & 15)) * LDQ + (lane >> 4) * Op::FRAG;
#pragma unroll
  for (int j = 0; j < MAXKT; ++j) {
    s[j] = f32x4{0.f, 0.f, 0.f, 0.f};
    if (j < nkt) {
      const T* b_s = Vs + (j * 16 + (lane & 15)) * LDQ + (lane >> 4) * Op::FRAG;
#pragma unroll
      for (int k = 0; k < HD; k += Op::KS) s[j] = Op::mma(Op::ld(a_s + k), Op::ld(b_s + k), s[j]);
    }
  }
  const float* prow = probs + (((long)b * H + h) * L) * L;
  float pv[MAXKT][4];
  float dot[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int j = 0; j < MAXKT; ++j) {
    if (j >= nkt) continue;
    const int key = j * 16 + (lane & 15);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int q = q0 + wid * 16 + (lane >> 4) * 4 + r;
      const float v = (q < L && key < L) ? prow[(long)q * L + key] : 0.f;
      // dP = keep * dP' / (1 - p); dropped elements are saved with the sign bit set
      s[j][r] = __builtin_signbitf(v) ? 0.f : s[j][r] * keep_scale;
      pv[j][r] = fabsf(v);
      dot[r] += pv[j][r] * s[j][r];
    }
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) dot[r] = rowgroup_sum(dot[r]);
  __syncthreads();  // every wave is done reading V: dS may overwrite it
  T* dsg = dS_g + (((long)b * H + h) * L) * LP;
#pragma unroll
  for (int j = 0; j < MAXKT; ++j) {
    if (j >= nkt) continue;
    const int key = j * 16 + (lane & 15);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int rl = wid * 16 + (lane >> 4) * 4 + r;
      const float ds = pv[j][r] * (s[j][r] - dot[r]);
      const T dst = from_f<T>(ds);
      dSs[rl * LDV + key] = dst;
      const int q = q0 + rl;
      if (q < L) dsg[(long)q * LP + key] = dst;
    }
  }
  __syncthreads();
  f32x4 o[HD / 16];
#pragma unroll
  for (int j = 0; j < HD / 16; ++j) o[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const T* p_s = dSs + (wid * 16 + (lane & 15)) * LDV + (lane >> 4) * Op::FRAG;
  for (int k = 0; k < LP; k += Op::KS) {
    const typename Op::frag_t af = Op::ld(p_s + k);
#pragma unroll
    for (int j = 0; j < HD / 16; ++j) {
      const T* k_s = Kt + (j * 16 + (lane & 15)) * LDV + (lane >> 4) * Op::FRAG;
      o[j] = Op::mma(af, Op::ld(k_s + k), o[j]);
    }
  }
#pragma unroll
  for (int j = 0; j < HD / 16; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int q = q0 + wid * 16 + (lane >> 4) * 4 + r;
      if (q < L)
        dqkv[((long)b * L + q) * 3 * H * HD + h * HD + j * 16 + (lane & 15)] =
            from_f<T>(o[j][r] * scale);
    }
}

// Backward B: per key block (16*NW keys): dV = P^T dO, dK = scale * dS^T Q, streaming
// 32-query chunks through LDS.
constexpr int QC = 32;
template <typename T>
__global__ __launch_bounds__(AttnCfg<T>::NW * 64, 2) void attn_bwd_kv_kernel(const T* __restrict__ qkv, const float* __restrict__ probs,
                                   const T* __restrict__ dout, const T* __restrict__ dS_g, int L,
                                   int H, float scale, float keep_scale, T* __restrict__ dqkv) {
  typedef MfmaOp<T> Op;
  constexpr int NW = AttnCfg<T>::NW, KB = NW * 16, PAD = Vec16<T>::N;
  constexpr int LDC = QC + PAD;
  __shared__ __attribute__((aligned(16))) T Pt[KB * LDC];    // [key][q]
  __shared__ __attribute__((aligned(16))) T dSt[KB * LDC];   // [key][q]
  __shared__ __attribute__((aligned(16))) T dOt[HD * LDC];   // [d][q]
  __shared__ __attribute__((aligned(16))) T Qt[HD * LDC];    // [d][q]
  int kb, h, b;
  attn_block((L + KB - 1) / KB, H, kb, h, b);
  const int k0 = kb * KB;
  const int LP = (L + 31) & ~31;  // multiple of the bf16 MFMA K (32)
  const long row_ld = 3L * H * HD;
  const T* qbase = qkv + (long)b * L * row_ld + h * HD;
  const float* pb = probs + (((long)b * H + h) * L) * L;
  const T* dsb = dS_g + (((long)b * H + h) * L) * LP;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  f32x4 dv[HD / 16], dk[HD / 16];
#pragma unroll
  for (int j = 0; j < HD / 16; ++j) dv[j] = dk[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // Chunk staging: thread (kk, qg) owns key k0+kk and the 8 queries qg*8.. of a chunk, so
  // the P / dS reads are key-contiguous across lanes (coalesced rows of [q][key]) and land in
  // LDS as one [key][q] vector store each; the dO / Q slices of the chunk are NV vectors per
  // thread.  The next chunk's loads are issued into registers before this chunk's MFMAs.
  typedef typename Vec16<T>::type V;
  constexpr int VEC = Vec16<T>::N, VPR = HD / VEC, NTH = NW * 64;
  constexpr int QG = 8, NV = QC * VPR / NTH;
  static_assert(KB * QC == NTH * QG && NV * NTH == QC * VPR, "chunk staging shape");
  const int kk = threadIdx.x % KB, qg = threadIdx.x / KB;
  float pr[QG];
  T dsr[QG];
  V dov[NV], qv[NV];
  auto fetch = [&](int qc) {
    const int key = k0 + kk;
#pragma unroll
    for (int u = 0; u < QG; ++u) {
      const int q = qc + qg * QG + u;
      const bool ok = key < L && q < L;
      pr[u] = ok ? pb[(long)q * L + key] : 0.f;
      dsr[u] = ok ? dsb[(long)q * LP + key] : from_f<T>(0.f);
    }
#pragma unroll
    for (int n = 0; n < NV; ++n) {
      const int i = threadIdx.x + n * NTH, r = i / VPR, c = (i - r * VPR) * VEC;
      const int q = qc + r;
      dov[n] = V{};
      qv[n] = V{};
      if (q < L) {
        dov[n] = *(const V*)(dout + ((long)b * L + q) * H * HD + h * HD + c);
        qv[n] = *(const V*)(qbase + (long)q * row_ld + c);
      }
    }
  };
  fetch(0);
  for (int qc = 0; qc < L; qc += QC) {
#pragma unroll
    for (int w = 0; w < QG / VEC; ++w) {
      V pv, sv;
#pragma unroll
      for (int j = 0; j < VEC; ++j) {
        const float v = pr[w * VEC + j];
        pv[j] = from_f<T>(__builtin_signbitf(v) ? 0.f : v * keep_scale);  // P'
        sv[j] = dsr[w * VEC + j];
      }
      *(V*)(Pt + kk * LDC + qg * QG + w * VEC) = pv;
      *(V*)(dSt + kk * LDC + qg * QG + w * VEC) = sv;
    }
#pragma unroll
    for (int n = 0; n < NV; ++n) {
      const int i = threadIdx.x + n * NTH, r = i / VPR, c = (i - r * VPR) * VEC;
      put_row_vec<T, true>(dOt, LDC, r, c, dov[n]);
      put_row_vec<T, true>(Qt, LDC, r, c, qv[n]);
    }
    __syncthreads();
    if (qc + QC < L) fetch(qc + QC);
    const T* ap = Pt + (wid * 16 + (lane & 15)) * LDC + (lane >> 4) * Op::FRAG;
    const T* as = dSt + (wid * 16 + (lane & 15)) * LDC + (lane >> 4) * Op::FRAG;
#pragma unroll
    for (int k = 0; k < QC; k += Op::KS) {
      const typename Op::frag_t fp = Op::ld(ap + k), fs = Op::ld(as + k);
#pragma unroll
      for (int j = 0; j < HD / 16; ++j) {
        const int off = (j * 16 + (lane & 15)) * LDC + (lane >> 4) * Op::FRAG + k;
        dv[j] = Op::mma(fp, Op::ld(dOt + off), dv[j]);
        dk[j] = Op::mma(fs, Op::ld(Qt + off), dk[j]);
      }
    }
    __syncthreads();
  }
#pragma unroll
  for (int j = 0; j < HD / 16; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int key = k0 + wid * 16 + (lane >> 4) * 4 + r;
      if (key < L) {
        T* row = dqkv + ((long)b * L + key) * 3 * H * HD + h * HD + j * 16 + (lane & 15);
        row[(long)H * HD] = from_f<T>(dk[j][r] * scale);
        row[2L * H * HD] = from_f<T>(dv[j][r]);
      }
    }
}

// ---------------------------------------------------------------------------------------
// 16-bit (bf16 / f16) kernels with swapped products.  S^T = K Q^T (and dP^T = V dO^T) puts
// one query on each lane's column: lane (ql = lane & 15, g = lane >> 4) of wave w holds,
// for every 16-key tile j, the four keys j*16 + g*4 + r (r = 0..3) of query q0 + w*16 + ql.
// Consequences:
//  * the row softmax (and the dP row dot) is a per-lane sum plus two cross-group shuffles;
//  * a lane's 4 consecutive keys are one 16-B probability store / load;
//  * the 8 keys of tiles (2t, 2t+1) at offsets g*4 .. g*4+3 are, in that order, the k
//    elements of the MFMA B operand P^T (dS^T) of the next product O^T = V^T P^T
//    (dQ^T = K^T dS^T): no LDS round trip for P / dS.  The A operand V^T (K^T) takes the
//    same permuted key order from a row-major LDS image with two ds_read_b64_tr_b16;
//  * Q and dO, the B operands of the first product, come straight from HBM into registers.
// ---------------------------------------------------------------------------------------
constexpr int LDR = HD + 8;    // 144-B rows: ds_read_b128 operand rows
constexpr int LDT = HD + 16;   // 160-B rows: 8 consecutive rows of a 32-B column block fall
                               // on distinct banks -> conflict-free transposed reads
constexpr int LDP = 20;        // fp32 [16][16] probability tile transpose, padded: conflict-free
                               // 16-B writes and 4-B column reads
typedef short s16x4v __attribute__((__vector_size__(4 * sizeof(short))));
typedef __attribute__((address_space(3))) s16x4v lds_s16x4v;

// Rows row0 .. row0+3 of 16 columns col0.. of a row-major [rows][LDT] 16-bit LDS tile,
// delivered column-major: lane i of each 16-lane group gets column col0 + i, row e in
// element e.  Every lane of the wave must execute it (EXEC all ones).
template <typename T>
__device__ __forceinline__ s16x4v tr_read4(const T* tile, int row0, int col0) {
  const int l = threadIdx.x & 15;
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (lds_s16x4v*)(tile + (row0 + (l >> 2)) * LDT + col0 + 4 * (l & 3)));
}
template <typename T>
__device__ __forceinline__ typename MfmaOp<T>::frag_t join_frag(s16x4v lo, s16x4v hi) {
  union { s16x4v h[2]; typename MfmaOp<T>::frag_t f; } u;
  u.h[0] = lo;
  u.h[1] = hi;
  return u.f;
}
// 4 consecutive 16-bit elements as one 8-B store
template <typename T>
__device__ __forceinline__ void store4(T* dst, float a, float b, float c, float d) {
  union { T e[4]; uint2 u; } pk;
  pk.e[0] = from_f<T>(a); pk.e[1] = from_f<T>(b); pk.e[2] = from_f<T>(c); pk.e[3] = from_f<T>(d);
  *(uint2*)dst = pk.u;
}

template <typename T, int NW>
__global__ __launch_bounds__(NW * 64, NW >= 8 ? 1 : 8 / NW) void attn_fwd16_kernel(
    const T* __restrict__ qkv, const int64_t* __restrict__ mask, const float* __restrict__ bias,
    int causal, int L, int H, float scale, float p_drop, uint64_t seed,
    const uint64_t* __restrict__ ctr, T* __restrict__ out, float* __restrict__ probs,
    float* __restrict__ lse, uint64_t* __restrict__ rng_out) {
  typedef MfmaOp<T> Op;
  typedef typename Op::frag_t F;
  static_assert(Op::FRAG == 8 && Op::KS == 32, "16-bit MFMA 16x16x32 operands");
  constexpr int QB = NW * 16;
  const int LP = (L + 31) & ~31;
  const int nkt = LP / 16;
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  T* Ks = (T*)smem_raw;               // [LP][LDR]  A operand rows of S^T
  T* Vs = Ks + LP * LDR;              // [LP][LDT]  transposed reads for V^T
  float* madd = (float*)(Vs + LP * LDT);   // [LP] additive key mask
  int qb, h, b;
  attn_block((L + QB - 1) / QB, H, qb, h, b);
  const int q0 = qb * QB;
  const long row_ld = 3L * H * HD;
  const T* base = qkv + (long)b * L * row_ld + h * HD;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, ql = lane & 15, g = lane >> 4;
  const int q = q0 + wid * 16 + ql;
  const bool idle = q0 + wid * 16 >= L;   // a wave of padding queries: stage, then leave
  F qf[2];
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    qf[k] = F{};
    if (q < L) qf[k] = *(const F*)(base + (long)q * row_ld + k * 32 + g * 8);
  }
  stage_pair<T, 4, false, false>(Ks, LDR, base + (long)H * HD, Vs, LDT, base + 2L * H * HD,
                                 row_ld, LP, L, NW * 64);
  for (int k = threadIdx.x; k < LP; k += NW * 64)
    madd[k] = k < L ? (mask && mask[(long)b * L + k] == 0 ? MASK_NEG : 0.f) : -INFINITY;
  __syncthreads();   // the only barrier: idle waves may leave after it
  if (idle) return;
  // s[j][r] = S[q][j*16 + g*4 + r]
  f32x4 s[MAXKT];
  float mx = -INFINITY;
#pragma unroll
  for (int j = 0; j < MAXKT; ++j) {
    s[j] = f32x4{0.f, 0.f, 0.f, 0.f};
    if (j >= nkt) continue;
    const T* a = Ks + (j * 16 + ql) * LDR + g * 8;
#pragma unroll
    for (int k = 0; k < 2; ++k) s[j] = Op::mma(Op::ld(a + k * 32), qf[k], s[j]);
    const f32x4 ma = *(const f32x4*)(madd + j * 16 + g * 4);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int key = j * 16 + g * 4 + r;
      float v = s[j][r] * scale + ma[r];
      // additive score bias [H][L][L] (T5 relative position bias) and causal mask
      if (bias && key < L && q < L) v += bias[((long)h * L + q) * L + key];
      if (causal && key > q && key < L) v = MASK_NEG;
      s[j][r] = v;
      mx = fmaxf(mx, v);
    }
  }
  mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
  mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
  float sum = 0.f;
#pragma unroll
  for (int j = 0; j < MAXKT; ++j) {
    if (j >= nkt) continue;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      s[j][r] = __expf(s[j][r] - mx);
      sum += s[j][r];
    }
  }
  sum += __shfl_xor(sum, 16, 64);
  sum += __shfl_xor(sum, 32, 64);
  const float inv = 1.f / sum;
  // flash-style save (mmdx_attention_fwd_lse): the row log-sum-exp instead of P
  if (lse && g == 0 && q < L) lse[((long)b * H + h) * L + q] = mx + __logf(sum);
  float* pbase = probs ? probs + (((long)b * H + h) * L) * L : nullptr;
  const bool vec_p = (L & 3) == 0;
  // L % 4 != 0: the lane's 4 keys are not a 16-B aligned run of a row; the wave transposes
  // each 16 x 16 tile through its LDS scratch so a store covers 64 contiguous bytes of 4 rows
  float* pscr = madd + LP + wid * 16 * LDP;
  const bool drop = p_drop > 0.f;
  const float keep_scale = drop ? 1.f / (1.f - p_drop) : 1.f;
  const uint64_t rb0 = seed * 0x9E3779B97F4A7C15ULL + (ctr ? ctr[0] << 32 : 0ull);
  if (rng_out && blockIdx.x == 0 && threadIdx.x == 0) rng_out[0] = rb0;  // for the backward
  const uint64_t rbase = drop ? rb0 + (((uint64_t)b * H + h) * L) * (uint64_t)L : 0ull;
  F pf[MAXKT / 2];
#pragma unroll
  for (int j = 0; j < MAXKT; ++j) {
    if (j >= nkt) continue;
    f32x4 pv;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int key = j * 16 + g * 4 + r;
      const float p = s[j][r] * inv;
      bool keep = true;
      if (drop) {
        const float u = (attn_hash64(rbase + (uint64_t)q * L + key) >> 8) * (1.f / 16777216.f);
        keep = u >= p_drop;
      }
      pf[j >> 1][(j & 1) * 4 + r] = from_f<T>(keep ? p * keep_scale : 0.f);
      pv[r] = keep ? p : -p;
    }
    if (pbase) {
      const int k0 = j * 16 + g * 4;
      if (vec_p) {
        if (q < L && k0 < L) *(f32x4*)(pbase + (long)q * L + k0) = pv;
      } else {
        *(f32x4*)(pscr + ql * LDP + g * 4) = pv;   // [q][key] of the tile
        const int key = j * 16 + ql;
#pragma unroll
        for (int r = 0; r < 4; ++r) {   // in-order LDS within the wave: no barrier
          const int qr = q0 + wid * 16 + g * 4 + r;
          const float v = pscr[(g * 4 + r) * LDP + ql];
          if (qr < L && key < L) pbase[(long)qr * L + key] = v;
        }
      }
    }
  }
  // O^T[d][q] = sum_key V^T[d][key] P'^T[key][q]
  f32x4 o[HD / 16];
#pragma unroll
  for (int dt = 0; dt < HD / 16; ++dt) o[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int t = 0; t < MAXKT / 2; ++t) {
    if (2 * t >= nkt) continue;
#pragma unroll
    for (int dt = 0; dt < HD / 16; ++dt) {
      const F vf = join_frag<T>(tr_read4(Vs, 2 * t * 16 + g * 4, dt * 16),
                                tr_read4(Vs, (2 * t + 1) * 16 + g * 4, dt * 16));
      o[dt] = Op::mma(vf, pf[t], o[dt]);
    }
  }
  if (q < L) {
    T* orow = out + ((long)b * L + q) * H * HD + h * HD;
#pragma unroll
    for (int dt = 0; dt < HD / 16; ++dt)
      store4<T>(orow + dt * 16 + g * 4, o[dt][0], o[dt][1], o[dt][2], o[dt][3]);
  }
}

// Backward A (16-bit): dP^T = V dO^T, dS = P o (dP - rowsum(P o dP)) -> dS_g [B,H,L,LP],
// dQ^T = scale K^T dS^T.  Two passes over the key tiles: the first only accumulates the row
// dot, the second recomputes each dP tile pair (28 extra MFMAs per wave), forms dS and feeds
// it straight into the dQ product, so no dP / dS tile array stays live (<= 128 VGPRs: two
// 8-wave blocks per CU).
template <typename T, int NW>
__global__ __launch_bounds__(NW * 64, 8 / NW) void attn_bwd_q16_kernel(
    const T* __restrict__ qkv, const float* __restrict__ probs, const T* __restrict__ dout,
    int L, int H, float scale, float keep_scale, T* __restrict__ dS_g, T* __restrict__ dqkv) {
  typedef MfmaOp<T> Op;
  typedef typename Op::frag_t F;
  constexpr int QB = NW * 16;
  const int LP = (L + 31) & ~31;
  const int nkt = LP / 16;
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  T* Vs = (T*)smem_raw;               // [LP][LDR]  A operand rows of dP^T
  T* Ks = Vs + LP * LDR;              // [LP][LDT]  transposed reads for K^T
  int qb, h, b;
  attn_block((L + QB - 1) / QB, H, qb, h, b);
  const int q0 = qb * QB;
  const long row_ld = 3L * H * HD;
  const T* base = qkv + (long)b * L * row_ld + h * HD;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, ql = lane & 15, g = lane >> 4;
  const int q = q0 + wid * 16 + ql;
  const bool idle = q0 + wid * 16 >= L;   // a wave of padding queries: stage, then leave
  F of[2];
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    of[k] = F{};
    if (q < L) of[k] = *(const F*)(dout + ((long)b * L + q) * H * HD + h * HD + k * 32 + g * 8);
  }
  stage_pair<T, 4, false, false>(Vs, LDR, base + 2L * H * HD, Ks, LDT, base + (long)H * HD,
                                 row_ld, LP, L, NW * 64);
  __syncthreads();   // the only barrier: idle waves may leave after it
  if (idle) return;
  // saved probabilities P[q][j*16 + g*4 + r] -> pv[j][r]: one 16-B load per tile when
  // L % 4 == 0; otherwise 4 loads of 64 contiguous bytes of 4 rows each, transposed through
  // the wave's LDS scratch (in-order LDS within the wave: no barrier)
  const float* pbase = probs + (((long)b * H + h) * L) * L;
  f32x4 pv[MAXKT];
  if ((L & 3) == 0) {
#pragma unroll
    for (int j = 0; j < MAXKT; ++j) {
      pv[j] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (j < nkt && q < L && j * 16 + g * 4 < L)
        pv[j] = *(const f32x4*)(pbase + (long)q * L + j * 16 + g * 4);
    }
  } else {
    float* pscr = (float*)(Ks + LP * LDT) + LP + wid * 16 * LDP;
#pragma unroll
    for (int j = 0; j < MAXKT; ++j) {
      pv[j] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (j >= nkt) continue;
      const int key = j * 16 + ql;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int qr = q0 + wid * 16 + g * 4 + r;
        if (qr < L && key < L) pv[j][r] = pbase[(long)qr * L + key];
      }
    }
#pragma unroll
    for (int j = 0; j < MAXKT; ++j) {
      if (j >= nkt) continue;
#pragma unroll
      for (int r = 0; r < 4; ++r) pscr[(g * 4 + r) * LDP + ql] = pv[j][r];
      pv[j] = *(const f32x4*)(pscr + ql * LDP + g * 4);
    }
  }
  // dP'[q][j*16 + g*4 + r] -> dP = keep * dP' / (1 - p); dropped elements are saved with the
  // sign bit set
  auto dp_tile = [&](int j) {
    f32x4 t = f32x4{0.f, 0.f, 0.f, 0.f};
    const T* a = Vs + (j * 16 + ql) * LDR + g * 8;
#pragma unroll
    for (int k = 0; k < 2; ++k) t = Op::mma(Op::ld(a + k * 32), of[k], t);
#pragma unroll
    for (int r = 0; r < 4; ++r) t[r] = __builtin_signbitf(pv[j][r]) ? 0.f : t[r] * keep_scale;
    return t;
  };
  float dot = 0.f;
#pragma unroll
  for (int j = 0; j < MAXKT; ++j) {
    if (j >= nkt) continue;
    const f32x4 t = dp_tile(j);
#pragma unroll
    for (int r = 0; r < 4; ++r) dot += fabsf(pv[j][r]) * t[r];
  }
  dot += __shfl_xor(dot, 16, 64);
  dot += __shfl_xor(dot, 32, 64);
  T* dsrow = dS_g + ((((long)b * H + h) * L) + q) * LP;
  // dQ^T[d][q] = sum_key K^T[d][key] dS^T[key][q]
  f32x4 o[HD / 16];
#pragma unroll
  for (int dt = 0; dt < HD / 16; ++dt) o[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int t = 0; t < MAXKT / 2; ++t) {
    if (2 * t >= nkt) continue;
    F df;
#pragma unroll
    for (int h2 = 0; h2 < 2; ++h2) {
      const int j = 2 * t + h2;
      const f32x4 tp = dp_tile(j);
      float ds[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const T dst = from_f<T>(fabsf(pv[j][r]) * (tp[r] - dot));
        df[h2 * 4 + r] = dst;
        ds[r] = (float)dst;
      }
      if (q < L) store4<T>(dsrow + j * 16 + g * 4, ds[0], ds[1], ds[2], ds[3]);
    }
#pragma unroll
    for (int dt = 0; dt < HD / 16; ++dt) {
      const F kf = join_frag<T>(tr_read4(Ks, 2 * t * 16 + g * 4, dt * 16),
                                tr_read4(Ks, (2 * t + 1) * 16 + g * 4, dt * 16));
      o[dt] = Op::mma(kf, df, o[dt]);
    }
  }
  if (q < L) {
    T* drow = dqkv + ((long)b * L + q) * 3 * H * HD + h * HD;
#pragma unroll
    for (int dt = 0; dt < HD / 16; ++dt)
      store4<T>(drow + dt * 16 + g * 4, o[dt][0] * scale, o[dt][1] * scale, o[dt][2] * scale,
                o[dt][3] * scale);
  }
}

// Backward B (16-bit), swapped products, per key block of 16*NW keys, one key
// per lane column: dV^T[d][key] = sum_q dO^T[d][q] P'[q][key] and
// dK^T[d][key] = scale * sum_q Q^T[d][q] dS[q][key].  The head's Q and dO rows are staged
// whole in LDS (one barrier) and read as the A operands through transposed reads; the
// B operands P' and dS come straight from HBM into registers, 8 queries per lane per step
// (each load instruction covers 64 contiguous bytes of 4 rows).
template <typename T, int NW>
__global__ __launch_bounds__(NW * 64, 8 / NW) void attn_bwd_kv16_kernel(
    const T* __restrict__ qkv, const float* __restrict__ probs, const T* __restrict__ dout,
    const T* __restrict__ dS_g, int L, int H, float scale, float keep_scale,
    T* __restrict__ dqkv) {
  typedef MfmaOp<T> Op;
  typedef typename Op::frag_t F;
  constexpr int KB = NW * 16;
  const int LP = (L + 31) & ~31;
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  T* Qs = (T*)smem_raw;               // [LP][LDT]
  T* Os = Qs + LP * LDT;              // [LP][LDT]  dO
  int kb, h, b;
  attn_block((L + KB - 1) / KB, H, kb, h, b);
  const int k0 = kb * KB;
  const long row_ld = 3L * H * HD;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, kl = lane & 15, g = lane >> 4;
  const int key = k0 + wid * 16 + kl;
  const bool idle = k0 + wid * 16 >= L;   // a wave of padding keys: stage, then leave
  stage_rows<T, 4, false>(Qs, LDT, qkv + (long)b * L * row_ld + h * HD, row_ld, LP, L, NW * 64);
  stage_rows<T, 4, false>(Os, LDT, dout + (long)b * L * H * HD + h * HD, (long)H * HD, LP, L,
                          NW * 64);
  __syncthreads();   // the only barrier
  if (idle) return;
  const float* pb = probs + (((long)b * H + h) * L) * L;
  const T* dsb = dS_g + (((long)b * H + h) * L) * LP;
  const bool kok = key < L;
  f32x4 dv[HD / 16], dk[HD / 16];
#pragma unroll
  for (int dt = 0; dt < HD / 16; ++dt) dv[dt] = dk[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int qs = 0; qs < LP; qs += 32) {
    F pf, sf;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int q = qs + g * 8 + e;
      const bool ok = kok && q < L;
      const float v = ok ? pb[(long)q * L + key] : 0.f;
      pf[e] = from_f<T>(__builtin_signbitf(v) ? 0.f : v * keep_scale);  // P'
      sf[e] = ok ? dsb[(long)q * LP + key] : from_f<T>(0.f);
    }
#pragma unroll
    for (int dt = 0; dt < HD / 16; ++dt) {
      const F of = join_frag<T>(tr_read4(Os, qs + g * 8, dt * 16),
                                tr_read4(Os, qs + g * 8 + 4, dt * 16));
      dv[dt] = Op::mma(of, pf, dv[dt]);
      const F qf = join_frag<T>(tr_read4(Qs, qs + g * 8, dt * 16),
                                tr_read4(Qs, qs + g * 8 + 4, dt * 16));
      dk[dt] = Op::mma(qf, sf, dk[dt]);
    }
  }
  if (kok) {
    T* row = dqkv + ((long)b * L + key) * 3 * H * HD + h * HD;
#pragma unroll
    for (int dt = 0; dt < HD / 16; ++dt) {
      store4<T>(row + (long)H * HD + dt * 16 + g * 4, dk[dt][0] * scale, dk[dt][1] * scale,
                dk[dt][2] * scale, dk[dt][3] * scale);
      store4<T>(row + 2L * H * HD + dt * 16 + g * 4, dv[dt][0], dv[dt][1], dv[dt][2],
                dv[dt][3]);
    }
  }
}

// ---------------------------------------------------------------------------------------
// Flash-style backward (16-bit; mmdx_attention_bwd_lse): nothing of size L^2 is saved or
// exchanged.  P is recomputed from Q, K and the forward's row log-sum-exp, the dropout keep
// bits from the counter hash (the forward left the stream's base in rng[0]), and the row term
// rowsum(P o dP) of the softmax gradient is D = dO . O (with dropout: sum_k P'_k dP'_k, the
// same number), so each kernel makes one pass:
//   A (per query block, swapped products as attn_bwd_q16_kernel): D, then per key-tile pair
//     S^T = K Q^T and dP'^T = V dO^T, dS = P o (keep * dP' / (1-p) - D), dQ^T += K^T dS^T;
//     D is left in the workspace for B.
//   B (per key block, one key per lane column): per 32-query chunk S = Q K^T and
//     dP' = dO V^T as two 16-query tiles (queries g*4+r and 16+g*4+r of the lane: the MFMA
//     k order of the next products, matched by the permuted transposed reads of Q / dO),
//     P' and dS formed in registers, dV^T += dO^T P', dK^T += Q^T dS.
// K (A) and Q, dO (B) are staged once per block as [LP][LDT] images: plain 16-B reads give
// the S / dP operands, ds_read_b64_tr_b16 the transposed ones.
// ---------------------------------------------------------------------------------------
template <typename T, int NW>
__global__ __launch_bounds__(NW * 64, 8 / NW) void attn_bwd_q16_lse_kernel(
    const T* __restrict__ qkv, const T* __restrict__ outp, const float* __restrict__ lse,
    const uint64_t* __restrict__ rng, const T* __restrict__ dout, const int64_t* __restrict__ mask,
    int L, int H, float scale, float p_drop, float* __restrict__ Dg, T* __restrict__ dqkv) {
  typedef MfmaOp<T> Op;
  typedef typename Op::frag_t F;
  constexpr int QB = NW * 16;
  const int LP = (L + 31) & ~31;
  const int nkt = LP / 16;
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  T* Vs = (T*)smem_raw;               // [LP][LDR]  A operand rows of dP^T
  T* Ks = Vs + LP * LDR;              // [LP][LDT]  A operand rows of S^T / transposed K^T
  float* madd = (float*)(Ks + LP * LDT);   // [LP]
  int qb, h, b;
  attn_block((L + QB - 1) / QB, H, qb, h, b);
  const int q0 = qb * QB;
  const long row_ld = 3L * H * HD;
  const T* base = qkv + (long)b * L * row_ld + h * HD;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, ql = lane & 15, g = lane >> 4;
  const int q = q0 + wid * 16 + ql;
  const bool idle = q0 + wid * 16 >= L;
  F qf[2], of[2];
  float dot = 0.f;
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    qf[k] = of[k] = F{};
    if (q < L) {
      qf[k] = *(const F*)(base + (long)q * row_ld + k * 32 + g * 8);
      const long orow = ((long)b * L + q) * H * HD + h * HD + k * 32 + g * 8;
      of[k] = *(const F*)(dout + orow);
      const F ov = *(const F*)(outp + orow);
#pragma unroll
      for (int e = 0; e < 8; ++e) dot += (float)of[k][e] * (float)ov[e];
    }
  }
  dot += __shfl_xor(dot, 16, 64);
  dot += __shfl_xor(dot, 32, 64);
  stage_pair<T, 4, false, false>(Vs, LDR, base + 2L * H * HD, Ks, LDT, base + (long)H * HD,
                                 row_ld, LP, L, NW * 64);
  for (int k = threadIdx.x; k < LP; k += NW * 64)
    madd[k] = k < L ? (mask && mask[(long)b * L + k] == 0 ? MASK_NEG : 0.f) : -INFINITY;
  __syncthreads();   // the only barrier
  if (idle) return;
  if (g == 0 && q < L) Dg[((long)b * H + h) * L + q] = dot;
  const float lq = q < L ? lse[((long)b * H + h) * L + q] : 0.f;
  const bool drop = p_drop > 0.f;
  const float keep_scale = drop ? 1.f / (1.f - p_drop) : 1.f;
  const uint64_t rbase = drop ? rng[0] + (((uint64_t)b * H + h) * L) * (uint64_t)L : 0ull;
  f32x4 o[HD / 16];
#pragma unroll
  for (int dt = 0; dt < HD / 16; ++dt) o[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int t = 0; t < MAXKT / 2; ++t) {
    if (2 * t >= nkt) continue;
    F df;
#pragma unroll
    for (int h2 = 0; h2 < 2; ++h2) {
      const int j = 2 * t + h2;
      f32x4 st = f32x4{0.f, 0.f, 0.f, 0.f}, tp = st;
      const T* ak = Ks + (j * 16 + ql) * LDT + g * 8;
      const T* av = Vs + (j * 16 + ql) * LDR + g * 8;
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        st = Op::mma(Op::ld(ak + k * 32), qf[k], st);
        tp = Op::mma(Op::ld(av + k * 32), of[k], tp);
      }
      const f32x4 ma = *(const f32x4*)(madd + j * 16 + g * 4);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int key = j * 16 + g * 4 + r;
        const float p = __expf(st[r] * scale + ma[r] - lq);
        bool keep = true;
        if (drop) {
          const float u = (attn_hash64(rbase + (uint64_t)q * L + key) >> 8) * (1.f / 16777216.f);
          keep = u >= p_drop;
        }
        const float dp = keep ? tp[r] * keep_scale : 0.f;
        df[h2 * 4 + r] = from_f<T>(p * (dp - dot));
      }
    }
#pragma unroll
    for (int dt = 0; dt < HD / 16; ++dt) {
      const F kf = join_frag<T>(tr_read4(Ks, 2 * t * 16 + g * 4, dt * 16),
                                tr_read4(Ks, (2 * t + 1) * 16 + g * 4, dt * 16));
      o[dt] = Op::mma(kf, df, o[dt]);
    }
  }
  if (q < L) {
    T* drow = dqkv + ((long)b * L + q) * 3 * H * HD + h * HD;
#pragma unroll
    for (int dt = 0; dt < HD / 16; ++dt)
      store4<T>(drow + dt * 16 + g * 4, o[dt][0] * scale, o[dt][1] * scale, o[dt][2] * scale,
                o[dt][3] * scale);
  }
}

template <typename T, int NW>
__global__ __launch_bounds__(NW * 64, 8 / NW) void attn_bwd_kv16_lse_kernel(
    const T* __restrict__ qkv, const float* __restrict__ lse, const uint64_t* __restrict__ rng,
    const T* __restrict__ dout, const int64_t* __restrict__ mask, const float* __restrict__ Dg,
    int L, int H, float scale, float p_drop, T* __restrict__ dqkv) {
  typedef MfmaOp<T> Op;
  typedef typename Op::frag_t F;
  constexpr int KB = NW * 16;
  const int LP = (L + 31) & ~31;
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  T* Qs = (T*)smem_raw;               // [LP][LDT]
  T* Os = Qs + LP * LDT;              // [LP][LDT]  dO
  float* ls = (float*)(Os + LP * LDT);   // [LP] lse (0 beyond L)
  float* ds_ = ls + LP;                  // [LP] D
  int kb, h, b;
  attn_block((L + KB - 1) / KB, H, kb, h, b);
  const int k0 = kb * KB;
  const long row_ld = 3L * H * HD;
  const T* base = qkv + (long)b * L * row_ld + h * HD;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, kl = lane & 15, g = lane >> 4;
  const int key = k0 + wid * 16 + kl;
  const bool idle = k0 + wid * 16 >= L;
  const bool kok = key < L;
  F kf[2], vf[2];
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    kf[k] = vf[k] = F{};
    if (kok) {
      kf[k] = *(const F*)(base + (long)key * row_ld + (long)H * HD + k * 32 + g * 8);
      vf[k] = *(const F*)(base + (long)key * row_ld + 2L * H * HD + k * 32 + g * 8);
    }
  }
  stage_rows<T, 4, false>(Qs, LDT, base, row_ld, LP, L, NW * 64);
  stage_rows<T, 4, false>(Os, LDT, dout + (long)b * L * H * HD + h * HD, (long)H * HD, LP, L,
                          NW * 64);
  const long hq = ((long)b * H + h) * L;
  for (int i = threadIdx.x; i < LP; i += NW * 64) {
    ls[i] = i < L ? lse[hq + i] : 0.f;
    ds_[i] = i < L ? Dg[hq + i] : 0.f;
  }
  __syncthreads();   // the only barrier
  if (idle) return;
  const float mk = kok ? (mask && mask[(long)b * L + key] == 0 ? MASK_NEG : 0.f) : -INFINITY;
  const bool drop = p_drop > 0.f;
  const float keep_scale = drop ? 1.f / (1.f - p_drop) : 1.f;
  const uint64_t rbase = drop ? rng[0] + (uint64_t)hq * (uint64_t)L : 0ull;
  f32x4 dv[HD / 16], dk[HD / 16];
#pragma unroll
  for (int dt = 0; dt < HD / 16; ++dt) dv[dt] = dk[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int qs = 0; qs < LP; qs += 32) {
    F pf, sf;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      f32x4 st = f32x4{0.f, 0.f, 0.f, 0.f}, tp = st;
      const T* aq = Qs + (qs + 16 * u + kl) * LDT + g * 8;
      const T* ao = Os + (qs + 16 * u + kl) * LDT + g * 8;
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        st = Op::mma(Op::ld(aq + k * 32), kf[k], st);   // S[q][key]
        tp = Op::mma(Op::ld(ao + k * 32), vf[k], tp);   // dP'[q][key]
      }
      const int qr0 = qs + 16 * u + g * 4;
      const f32x4 lq = *(const f32x4*)(ls + qr0);
      const f32x4 dq = *(const f32x4*)(ds_ + qr0);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int qq = qr0 + r;
        const float p = __expf(st[r] * scale + mk - lq[r]);
        bool keep = true;
        if (drop) {
          const float uu =
              (attn_hash64(rbase + (uint64_t)qq * L + key) >> 8) * (1.f / 16777216.f);
          keep = uu >= p_drop;
        }
        const float dp = keep ? tp[r] * keep_scale : 0.f;
        pf[u * 4 + r] = from_f<T>(keep ? p * keep_scale : 0.f);
        sf[u * 4 + r] = from_f<T>(p * (dp - dq[r]));
      }
    }
#pragma unroll
    for (int dt = 0; dt < HD / 16; ++dt) {
      const F of = join_frag<T>(tr_read4(Os, qs + g * 4, dt * 16),
                                tr_read4(Os, qs + 16 + g * 4, dt * 16));
      dv[dt] = Op::mma(of, pf, dv[dt]);
      const F qf = join_frag<T>(tr_read4(Qs, qs + g * 4, dt * 16),
                                tr_read4(Qs, qs + 16 + g * 4, dt * 16));
      dk[dt] = Op::mma(qf, sf, dk[dt]);
    }
  }
  if (kok) {
    T* row = dqkv + ((long)b * L + key) * 3 * H * HD + h * HD;
#pragma unroll
    for (int dt = 0; dt < HD / 16; ++dt) {
      store4<T>(row + (long)H * HD + dt * 16 + g * 4, dk[dt][0] * scale, dk[dt][1] * scale,
                dk[dt][2] * scale, dk[dt][3] * scale);
      store4<T>(row + 2L * H * HD + dt * 16 + g * 4, dv[dt][0], dv[dt][1], dv[dt][2],
                dv[dt][3]);
    }
  }
}

static size_t smem16(int L, int nw) {
  const size_t LP = (L + 31) & ~31;
  return LP * (LDR + LDT) * 2 + (LP + (size_t)nw * 16 * LDP) * sizeof(float);
}

// queries per forward block: 128 (8 waves) halves the K/V staging per query and doubles the
// resident waves per CU (the LDS, not the registers, bounds residency); MMDX_ATTN_FWD_NW=4
// selects 64
static int fwd16_nw() { return knobs().attn_fwd_nw == 4 ? 4 : 8; }
// the flash-style forward's block: 8 waves (128 queries); MMDX_ATTN_FWD_NW = 4 | 16 selects
// 64 / 256 (16 waves = one block per ViT head, K and V staged once instead of twice: C5
// 2631 / 2640 vs 2653 / 2664 samples/s with 8, paired, tools/lab_attnnw.sh)
static int fwd16_lse_nw(int L) {
  (void)L;
  const int v = knobs().attn_fwd_nw;
  return v == 4 || v == 16 ? v : 8;
}
static int bwd16_nw() {   // the same for the dQ kernel; MMDX_ATTN_BWD_NW=4 selects 64
  return knobs().attn_bwd_nw == 4 ? 4 : 8;
}

template <typename T>
static size_t fwd_smem(int L) {
  constexpr int NW = AttnCfg<T>::NW, QB = NW * 16, PAD = Vec16<T>::N;
  const int LP = (L + 31) & ~31;  // multiple of the bf16 MFMA K (32)
  const size_t kp = std::max((size_t)LP * (HD + PAD), (size_t)QB * (LP + PAD));
  return sizeof(T) * (kp + (size_t)HD * (LP + PAD) + (size_t)QB * (HD + PAD));
}

}  // namespace mmdx

using namespace mmdx;

__global__ void attn_counter_incr_kernel(uint64_t* c) { c[0] += 1; }

extern "C" int mmdx_attention_fwd_ex(int dtype, const void* qkv, const int64_t* mask,
                                     const float* bias, int causal, int B, int L, int H,
                                     float scale, float p_drop, uint64_t seed,
                                     uint64_t* counter, void* out, float* probs, void* stream) {
  MMDX_CHECK_ARG(B > 0 && H > 0 && L > 0 && L <= 16 * MAXKT, "attention: L=%d > 256", L);
  MMDX_CHECK_ARG(p_drop >= 0.f && p_drop < 1.f, "attention: dropout p=%g out of range",
                 (double)p_drop);
  MMDX_CHECK_ARG(p_drop == 0.f || probs,
                 "attention: dropout needs the saved probabilities (training)");
  hipStream_t st = (hipStream_t)stream;
  MMDX_DISPATCH(dtype, {
    if constexpr (std::is_same<T, float>::value) {
      constexpr int QB = AttnCfg<T>::NW * 16;
      const size_t sm = fwd_smem<T>(L);
      MMDX_CHECK_ARG(sm <= 160 * 1024, "attention: L=%d needs %zu B LDS", L, sm);
      mmdx_lds_max_once((const void*)attn_fwd_kernel<T>);
      hipLaunchKernelGGL(attn_fwd_kernel<T>, dim3((L + QB - 1) / QB, H, B),
                         dim3(AttnCfg<T>::NW * 64), sm, st, (const T*)qkv, mask, bias, causal,
                         L, H, scale, p_drop, seed, (const uint64_t*)counter, (T*)out, probs);
    } else {
      auto launch = [&](auto kern, int nw) {
        const size_t sm = smem16(L, nw);
        mmdx_lds_max_once((const void*)kern);
        const int qb = nw * 16;
        hipLaunchKernelGGL(kern, dim3((L + qb - 1) / qb * H * B), dim3(nw * 64), sm, st,
                           (const T*)qkv, mask, bias, causal, L, H, scale, p_drop, seed,
                           (const uint64_t*)counter, (T*)out, probs, (float*)nullptr,
                           (uint64_t*)nullptr);
      };
      if (fwd16_nw() == 8) launch(attn_fwd16_kernel<T, 8>, 8);
      else launch(attn_fwd16_kernel<T, 4>, 4);
    }
  });
  if (p_drop > 0.f && counter)
    hipLaunchKernelGGL(attn_counter_incr_kernel, dim3(1), dim3(1), 0, st, counter);
  MMDX_LAUNCH_CHECK();
  return 0;
}

extern "C" int mmdx_attention_fwd(int dtype, const void* qkv, const int64_t* mask, int B, int L,
                                  int H, float scale, float p_drop, uint64_t seed,
                                  uint64_t* counter, void* out, float* probs, void* stream) {
  return mmdx_attention_fwd_ex(dtype, qkv, mask, nullptr, 0, B, L, H, scale, p_drop, seed,
                               counter, out, probs, stream);
}

extern "C" size_t mmdx_attention_workspace_size(int dtype, int B, int L, int H) {
  const int LP = (L + 31) & ~31;  // multiple of the bf16 MFMA K (32)
  return (size_t)B * H * L * LP * (dtype == F32 ? 4 : 2);
}

extern "C" int mmdx_attention_bwd(int dtype, const void* qkv, const float* probs,
                                  const void* dout, const int64_t* mask, int B, int L, int H,
                                  float scale, float p_drop, void* dqkv, void* ws,
                                  size_t ws_bytes, void* stream) {
  (void)mask;  // encoded in probs (masked keys have p = 0)
  MMDX_CHECK_ARG(L <= 16 * MAXKT && probs && p_drop >= 0.f && p_drop < 1.f,
                 "attention bwd: bad args");
  const float keep_scale = 1.f / (1.f - p_drop);
  MMDX_CHECK_ARG(ws && ws_bytes >= mmdx_attention_workspace_size(dtype, B, L, H),
                 "attention bwd: workspace too small");
  hipStream_t st = (hipStream_t)stream;
  MMDX_DISPATCH(dtype, {
    constexpr int QB = AttnCfg<T>::NW * 16;
    if constexpr (std::is_same<T, float>::value) {
      const size_t sm = fwd_smem<T>(L);
      MMDX_CHECK_ARG(sm <= 160 * 1024, "attention bwd: L=%d needs %zu B LDS", L, sm);
      mmdx_lds_max_once((const void*)attn_bwd_q_kernel<T>);
      hipLaunchKernelGGL(attn_bwd_q_kernel<T>, dim3((L + QB - 1) / QB, H, B),
                         dim3(AttnCfg<T>::NW * 64), sm, st, (const T*)qkv, probs,
                         (const T*)dout, L, H, scale, keep_scale, (T*)ws, (T*)dqkv);
    } else {
      auto launch = [&](auto kern, int nw) {
        const size_t sm = smem16(L, nw);
        mmdx_lds_max_once((const void*)kern);
        const int qb = nw * 16;
        hipLaunchKernelGGL(kern, dim3((L + qb - 1) / qb * H * B), dim3(nw * 64), sm, st,
                           (const T*)qkv, probs, (const T*)dout, L, H, scale, keep_scale,
                           (T*)ws, (T*)dqkv);
      };
      if (bwd16_nw() == 8) launch(attn_bwd_q16_kernel<T, 8>, 8);
      else launch(attn_bwd_q16_kernel<T, 4>, 4);
    }
    if constexpr (std::is_same<T, float>::value) {
      hipLaunchKernelGGL(attn_bwd_kv_kernel<T>, dim3((L + QB - 1) / QB * H * B),
                         dim3(AttnCfg<T>::NW * 64), 0, st, (const T*)qkv, probs,
                         (const T*)dout, (const T*)ws, L, H, scale, keep_scale, (T*)dqkv);
    } else {
      const size_t sm = (size_t)((L + 31) & ~31) * LDT * 2 * sizeof(T);
      auto kv16 = attn_bwd_kv16_kernel<T, 8>;
      mmdx_lds_max_once((const void*)kv16);
      hipLaunchKernelGGL(kv16, dim3((L + 127) / 128 * H * B), dim3(512),
                         sm, st, (const T*)qkv, probs, (const T*)dout, (const T*)ws, L, H,
                         scale, keep_scale, (T*)dqkv);
    }
  });
  MMDX_LAUNCH_CHECK();
  return 0;
}

extern "C" int mmdx_attention_fwd_lse(int dtype, const void* qkv, const int64_t* mask, int B,
                                      int L, int H, float scale, float p_drop, uint64_t seed,
                                      uint64_t* counter, void* out, float* lse, uint64_t* rng,
                                      void* stream) {
  MMDX_CHECK_ARG(dtype != F32, "attention (lse): 16-bit compute dtypes only");
  MMDX_CHECK_ARG(B > 0 && H > 0 && L > 0 && L <= 16 * MAXKT, "attention: L=%d > 256", L);
  MMDX_CHECK_ARG(p_drop >= 0.f && p_drop < 1.f && lse && rng,
                 "attention (lse): bad dropout p=%g or missing lse / rng", (double)p_drop);
  hipStream_t st = (hipStream_t)stream;
  MMDX_DISPATCH(dtype, {
    if constexpr (!std::is_same<T, float>::value) {
      auto launch = [&](auto kern, int nw) {
        // (no probability tiles to transpose: the K / V images and the key mask only)
        const size_t LP = (L + 31) & ~31;
        const size_t sm = LP * (LDR + LDT) * sizeof(T) + LP * sizeof(float);
        mmdx_lds_max_once((const void*)kern);
        const int qb = nw * 16;
        hipLaunchKernelGGL(kern, dim3((L + qb - 1) / qb * H * B), dim3(nw * 64), sm, st,
                           (const T*)qkv, mask, (const float*)nullptr, 0, L, H, scale, p_drop,
                           seed, (const uint64_t*)counter, (T*)out, (float*)nullptr, lse, rng);
      };
      const int nw = fwd16_lse_nw(L);
      if (nw == 16) launch(attn_fwd16_kernel<T, 16>, 16);
      else if (nw == 8) launch(attn_fwd16_kernel<T, 8>, 8);
      else launch(attn_fwd16_kernel<T, 4>, 4);
    }
  });
  if (p_drop > 0.f && counter)
    hipLaunchKernelGGL(attn_counter_incr_kernel, dim3(1), dim3(1), 0, st, counter);
  MMDX_LAUNCH_CHECK();
  return 0;
}

extern "C" size_t mmdx_attention_lse_workspace_size(int dtype, int B, int L, int H) {
  (void)dtype;
  return (size_t)B * H * L * sizeof(float);   // D = rowsum(dO o O)
}

extern "C" int mmdx_attention_bwd_lse(int dtype, const void* qkv, const void* out,
                                      const float* lse, const uint64_t* rng, const void* dout,
                                      const int64_t* mask, int B, int L, int H, float scale,
                                      float p_drop, void* dqkv, void* ws, size_t ws_bytes,
                                      void* stream) {
  MMDX_CHECK_ARG(dtype != F32, "attention bwd (lse): 16-bit compute dtypes only");
  MMDX_CHECK_ARG(B > 0 && H > 0 && L > 0 && L <= 16 * MAXKT && lse && rng && out &&
                     p_drop >= 0.f && p_drop < 1.f,
                 "attention bwd (lse): bad args");
  MMDX_CHECK_ARG(ws && ws_bytes >= mmdx_attention_lse_workspace_size(dtype, B, L, H),
                 "attention bwd (lse): workspace too small");
  hipStream_t st = (hipStream_t)stream;
  const int LP = (L + 31) & ~31;
  MMDX_DISPATCH(dtype, {
    if constexpr (!std::is_same<T, float>::value) {
      const size_t sma = (size_t)LP * (LDR + LDT) * sizeof(T) + (size_t)LP * sizeof(float);
      auto qk = attn_bwd_q16_lse_kernel<T, 8>;
      mmdx_lds_max_once((const void*)qk);
      hipLaunchKernelGGL(qk, dim3((L + 127) / 128 * H * B), dim3(512), sma, st, (const T*)qkv,
                         (const T*)out, lse, rng, (const T*)dout, mask, L, H, scale, p_drop,
                         (float*)ws, (T*)dqkv);
      const size_t smb = (size_t)LP * LDT * 2 * sizeof(T) + (size_t)LP * 2 * sizeof(float);
      auto kv = attn_bwd_kv16_lse_kernel<T, 8>;
      mmdx_lds_max_once((const void*)kv);
      hipLaunchKernelGGL(kv, dim3((L + 127) / 128 * H * B), dim3(512), smb, st, (const T*)qkv,
                         lse, rng, (const T*)dout, mask, (const float*)ws, L, H, scale, p_drop,
                         (T*)dqkv);
    }
  });
  MMDX_LAUNCH_CHECK();
  return 0;
}
