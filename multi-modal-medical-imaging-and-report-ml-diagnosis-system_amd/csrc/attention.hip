// Multi-head self-attention core for BERT-base / ViT-B (head dim 64, L <= 256).
//
// Forward: one workgroup per (query block, head, batch); K, V^T of the head and the Q block
// live in LDS; S = Q K^T on MFMA, row softmax in registers (16-lane shuffles on the 16x16
// C layout), P -> LDS, O = P V on MFMA.  Probabilities are saved (fp32) for the backward.
// Backward: kernel A per query block: dP = dO V^T, dS = P o (dP - rowsum(P o dP)),
// dQ = scale dS K; kernel B per key block, streaming query chunks: dV = P^T dO,
// dK = scale dS^T Q.  Additive key mask as BertSelfAttention (large negative on pads).
// Attention-probability dropout (BertSelfAttention's dropout on attention_probs, train
// mode): P' = P * keep / (1 - p) feeds O = P' V; keep comes from a counter-based hash of
// (seed, device launch counter, b, h, q, key).  The saved probabilities carry the keep bit
// in their sign (P >= 0: a dropped element is saved as -P), so the backward needs no RNG
// and no mask tensor: dV = P'^T dO, dP = keep * (dO V^T) / (1 - p),
// dS = P o (dP - rowsum(P o dP)).
#include <algorithm>

#include "igemm.h"
#include "../../include/mmdx.h"

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

template <typename T>
__device__ __forceinline__ void load_rows(T* dst, int ld, const T* src, long src_ld, int rows,
                                          int rows_valid, int nthreads) {
  // rows x 64 elements (16-B vectors), zero beyond rows_valid
  typedef typename Vec16<T>::type V;
  constexpr int VEC = Vec16<T>::N;
  constexpr int VPR = HD / VEC;
  for (int i = threadIdx.x; i < rows * VPR; i += nthreads) {
    const int r = i / VPR, c = (i - r * VPR) * VEC;
    V v{};
    if (r < rows_valid) v = *(const V*)(src + r * src_ld + c);
    *(V*)(dst + r * ld + c) = v;
  }
}
template <typename T>
__device__ __forceinline__ void load_rows_T(T* dst, int ld, const T* src, long src_ld, int rows,
                                            int rows_valid, int nthreads) {
  // dst[c][r] = src[r][c] for rows x 64
  typedef typename Vec16<T>::type V;
  constexpr int VEC = Vec16<T>::N;
  constexpr int VPR = HD / VEC;
  for (int i = threadIdx.x; i < rows * VPR; i += nthreads) {
    const int r = i / VPR, c = (i - r * VPR) * VEC;
    V v{};
    if (r < rows_valid) v = *(const V*)(src + r * src_ld + c);
#pragma unroll
    for (int j = 0; j < VEC; ++j) dst[(c + j) * ld + r] = v[j];
  }
}

__device__ __forceinline__ uint32_t attn_hash64(uint64_t x) {
  x ^= x >> 33; x *= 0xff51afd7ed558ccdULL;
  x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ULL;
  x ^= x >> 33;
  return (uint32_t)x;
}

template <typename T>
__global__ void attn_fwd_kernel(const T* __restrict__ qkv, const int64_t* __restrict__ mask,
                                const float* __restrict__ bias, int causal, int L, int H,
                                float scale, float p_drop, uint64_t seed,
                                const uint64_t* __restrict__ ctr, T* __restrict__ out,
                                float* __restrict__ probs) {
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
  load_rows<T>(Qs, LDQ, base + (long)q0 * row_ld, row_ld, QB, min(QB, L - q0), nth);
  load_rows<T>(Ks, LDQ, base + (long)H * HD, row_ld, LP, L, nth);
  load_rows_T<T>(Vt, LDV, base + 2L * H * HD, row_ld, LP, L, nth);
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
  load_rows<T>(dOs, LDQ, dout + ((long)b * L + q0) * H * HD + h * HD, (long)H * HD, QB,
               min(QB, L - q0), nth);
  load_rows<T>(Vs, LDQ, base + 2L * H * HD, row_ld, LP, L, nth);
  load_rows_T<T>(Kt, LDV, base + (long)H * HD, row_ld, LP, L, nth);
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
__global__ void attn_bwd_kv_kernel(const T* __restrict__ qkv, const float* __restrict__ probs,
                                   const T* __restrict__ dout, const T* __restrict__ dS_g, int L,
                                   int H, float scale, float keep_scale, T* __restrict__ dqkv) {
  typedef MfmaOp<T> Op;
  constexpr int NW = AttnCfg<T>::NW, KB = NW * 16, PAD = Vec16<T>::N;
  constexpr int LDC = QC + PAD;
  __shared__ __attribute__((aligned(16))) T Pt[KB * LDC];    // [key][q]
  __shared__ __attribute__((aligned(16))) T dSt[KB * LDC];   // [key][q]
  __shared__ __attribute__((aligned(16))) T dOt[HD * LDC];   // [d][q]
  __shared__ __attribute__((aligned(16))) T Qt[HD * LDC];    // [d][q]
  const int k0 = blockIdx.x * KB, h = blockIdx.y, b = blockIdx.z;
  const int nth = NW * 64;
  const int LP = (L + 31) & ~31;  // multiple of the bf16 MFMA K (32)
  const long row_ld = 3L * H * HD;
  const T* qbase = qkv + (long)b * L * row_ld + h * HD;
  const float* pb = probs + (((long)b * H + h) * L) * L;
  const T* dsb = dS_g + (((long)b * H + h) * L) * LP;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  f32x4 dv[HD / 16], dk[HD / 16];
#pragma unroll
  for (int j = 0; j < HD / 16; ++j) dv[j] = dk[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int qc = 0; qc < L; qc += QC) {
    for (int i = threadIdx.x; i < KB * QC; i += nth) {
      const int kk = i / QC, qq = i - kk * QC;
      const int key = k0 + kk, q = qc + qq;
      const bool ok = key < L && q < L;
      const float v = ok ? pb[(long)q * L + key] : 0.f;
      Pt[kk * LDC + qq] = from_f<T>(__builtin_signbitf(v) ? 0.f : v * keep_scale);  // P'
      dSt[kk * LDC + qq] = ok ? dsb[(long)q * LP + key] : from_f<T>(0.f);
    }
    load_rows_T<T>(dOt, LDC, dout + ((long)b * L + qc) * H * HD + h * HD, (long)H * HD, QC,
                   min(QC, L - qc), nth);
    load_rows_T<T>(Qt, LDC, qbase + (long)qc * row_ld, row_ld, QC, min(QC, L - qc), nth);
    __syncthreads();
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
    constexpr int QB = AttnCfg<T>::NW * 16;
    const size_t sm = fwd_smem<T>(L);
    MMDX_CHECK_ARG(sm <= 160 * 1024, "attention: L=%d needs %zu B LDS", L, sm);
    (void)hipFuncSetAttribute((const void*)attn_fwd_kernel<T>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)sm);
    hipLaunchKernelGGL(attn_fwd_kernel<T>, dim3((L + QB - 1) / QB, H, B),
                       dim3(AttnCfg<T>::NW * 64), sm, st, (const T*)qkv, mask, bias, causal, L,
                       H, scale, p_drop, seed, (const uint64_t*)counter, (T*)out, probs);
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
#define ATTN_BWD(T)                                                                            \
  {                                                                                            \
    constexpr int QB = AttnCfg<T>::NW * 16;                                                    \
    const size_t sm = fwd_smem<T>(L);                                                          \
    MMDX_CHECK_ARG(sm <= 160 * 1024, "attention bwd: L=%d needs %zu B LDS", L, sm);           \
    (void)hipFuncSetAttribute((const void*)attn_bwd_q_kernel<T>,                                     \
                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)sm);                  \
    hipLaunchKernelGGL(attn_bwd_q_kernel<T>, dim3((L + QB - 1) / QB, H, B),                    \
                       dim3(AttnCfg<T>::NW * 64), sm, st, (const T*)qkv, probs,                \
                       (const T*)dout, L, H, scale, keep_scale, (T*)ws, (T*)dqkv);             \
    hipLaunchKernelGGL(attn_bwd_kv_kernel<T>, dim3((L + QB - 1) / QB, H, B),                   \
                       dim3(AttnCfg<T>::NW * 64), 0, st, (const T*)qkv, probs, (const T*)dout, \
                       (const T*)ws, L, H, scale, keep_scale, (T*)dqkv);                       \
  }
  if (dtype == BF16) ATTN_BWD(bf16) else if (dtype == F16) ATTN_BWD(f16) else ATTN_BWD(float)
#undef ATTN_BWD
  MMDX_LAUNCH_CHECK();
  return 0;
}
