// Implicit-GEMM core for gfx950: C[M,N] = sum_k A(m,k) * B(n,k).
//
// One templated MFMA main loop serves every contraction on the hot path:
//   * Linear fwd / dX / dW           (dense operands, either majorness)
//   * conv fwd  (A = im2col gather of the NHWC input, on the fly)
//   * conv dgrad (A = strided gather of dY, B = packed [Cin][R][S][Cout] weights)
//   * conv wgrad (A = dY^T, B = im2col gather, split-K over N*P*Q pixels)
//
// Tiling: 256 threads = 4 waves laid out WM x WN over a BM x BN block tile; each wave
// owns (BM/WM) x (BN/WN) built from 16x16 MFMA tiles (bf16: v_mfma_f32_16x16x32_bf16,
// f32: v_mfma_f32_16x16x4_f32 = exact f32 fmaf chain, used for the parity path).
// Operands are staged global -> registers -> LDS (two buffers, one barrier per K tile);
// the LDS image is always [row][k] (k contiguous, rows padded by 16 B so the 16 lanes of
// a ds_read_b128 group hit 16 distinct 16-B slots).  Operands whose K is not the
// contiguous global dimension ("R-major") are transposed on the LDS write.
#pragma once
#include "common.h"

namespace mmdx {

constexpr int NT = 256;  // threads per GEMM block

template <typename T> struct MfmaOp;
template <> struct MfmaOp<bf16> {
  static constexpr int KS = 32;    // k per MFMA
  static constexpr int FRAG = 8;   // operand elements per lane
  typedef bf16x8 frag_t;
  __device__ __forceinline__ static f32x4 mma(frag_t a, frag_t b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
  }
  __device__ __forceinline__ static frag_t ld(const bf16* p) { return *(const bf16x8*)p; }
};
template <> struct MfmaOp<float> {
  static constexpr int KS = 4;
  static constexpr int FRAG = 1;
  typedef float frag_t;
  __device__ __forceinline__ static f32x4 mma(frag_t a, frag_t b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
  }
  __device__ __forceinline__ static frag_t ld(const float* p) { return *p; }
};

template <typename T> struct KTile;               // K depth of one LDS stage
template <> struct KTile<bf16> { static constexpr int BK = 64; };
template <> struct KTile<float> { static constexpr int BK = 32; };

template <typename T, int BK>
struct LdsGeom {
  static constexpr int VEC = Vec16<T>::N;
  static constexpr int LDK = BK + VEC;  // +16 B row pad
};

// --------------------------------------------------------------------------------------
// Operand sources. Each maps (row, k) -> element pointer or nullptr (= zero).
// K-major sources return a pointer to VEC consecutive k's; R-major ones to VEC
// consecutive rows.  `klim` is the exclusive K bound of the current split.
// --------------------------------------------------------------------------------------

// Dense, K contiguous: element (r, k) at base[r*ld + k].  `vec` = ld and base allow
// 16-B vector loads; otherwise (and for a vector crossing klim) elements load one by one.
template <typename T>
struct DenseK {
  const T* base; long ld; int R; bool vec;
  typedef const T* RowState;
  typedef typename Vec16<T>::type V;
  __device__ RowState row(int r) const { return r < R ? base + (long)r * ld : nullptr; }
  __device__ V load(RowState rs, int k, int klim) const {
    constexpr int VEC = Vec16<T>::N;
    V v{};
    if (!rs || k >= klim) return v;
    if (vec && k + VEC <= klim) return *(const V*)(rs + k);
#pragma unroll
    for (int j = 0; j < VEC; ++j)
      if (k + j < klim) v[j] = rs[k + j];
    return v;
  }
};

// Dense, rows contiguous: element (r, k) at base[k*ld + r].
template <typename T>
struct DenseR {
  const T* base; long ld; int R; bool vec;
  typedef int RowState;
  typedef typename Vec16<T>::type V;
  __device__ RowState row(int r) const { return r < R ? r : -1; }
  __device__ V load(RowState rs, int k, int klim) const {
    constexpr int VEC = Vec16<T>::N;
    V v{};
    if (rs < 0 || k >= klim) return v;
    const T* p = base + (long)k * ld + rs;
    if (vec && rs + VEC <= R) return *(const V*)p;
#pragma unroll
    for (int j = 0; j < VEC; ++j)
      if (rs + j < R) v[j] = p[j];
    return v;
  }
};

struct ConvGeom {
  int N, H, W, C;      // input NHWC
  int K;               // output channels
  int R, S;            // filter h, w
  int sh, sw, ph, pw;  // stride, pad
  int P, Q;            // output h, w
};

// conv fwd A operand: rows = output pixels (n,p,q), k = (r, s, c) with c contiguous.
template <typename T>
struct Im2colK {
  const T* x; ConvGeom g; int M;
  struct RowState { const T* img; int ih0, iw0; };
  __device__ RowState row(int m) const {
    RowState rs;
    if (m >= M) { rs.img = nullptr; rs.ih0 = rs.iw0 = 0; return rs; }
    const int pq = g.P * g.Q;
    const int n = m / pq, rem = m - n * pq;
    const int p = rem / g.Q, q = rem - p * g.Q;
    rs.img = x + (long)n * g.H * g.W * g.C;
    rs.ih0 = p * g.sh - g.ph;
    rs.iw0 = q * g.sw - g.pw;
    return rs;
  }
  typedef typename Vec16<T>::type V;
  __device__ V load(const RowState& rs, int k, int klim) const {
    const T* p = at(rs, k, klim);
    return p ? *(const V*)p : V{};
  }
  __device__ const T* at(const RowState& rs, int k, int klim) const {
    if (!rs.img || k >= klim) return nullptr;
    const int tap = k / g.C, c = k - tap * g.C;
    const int r = tap / g.S, s = tap - r * g.S;
    const int ih = rs.ih0 + r, iw = rs.iw0 + s;
    if ((unsigned)ih >= (unsigned)g.H || (unsigned)iw >= (unsigned)g.W) return nullptr;
    return rs.img + ((long)ih * g.W + iw) * g.C + c;
  }
};

// conv dgrad A operand: rows = input pixels (n,h,w), k = (r, s, kout) with kout contiguous.
// dX[n,h,w,c] = sum_{r,s,k} dY[n,(h+ph-r)/sh,(w+pw-s)/sw,k] * W[k,r,s,c]  (divisible taps only)
template <typename T>
struct DgradK {
  const T* dy; ConvGeom g; int M;
  struct RowState { const T* img; int h, w; };
  __device__ RowState row(int m) const {
    RowState rs;
    if (m >= M) { rs.img = nullptr; rs.h = rs.w = 0; return rs; }
    const int hw = g.H * g.W;
    const int n = m / hw, rem = m - n * hw;
    rs.h = rem / g.W + g.ph;
    rs.w = rem - (rem / g.W) * g.W + g.pw;
    rs.img = dy + (long)n * g.P * g.Q * g.K;
    return rs;
  }
  typedef typename Vec16<T>::type V;
  __device__ V load(const RowState& rs, int k, int klim) const {
    const T* p = at(rs, k, klim);
    return p ? *(const V*)p : V{};
  }
  __device__ const T* at(const RowState& rs, int k, int klim) const {
    if (!rs.img || k >= klim) return nullptr;
    const int tap = k / g.K, ko = k - tap * g.K;
    const int r = tap / g.S, s = tap - r * g.S;
    const int th = rs.h - r, tw = rs.w - s;
    if (th < 0 || tw < 0) return nullptr;
    const int p = th / g.sh, q = tw / g.sw;
    if (p * g.sh != th || q * g.sw != tw || p >= g.P || q >= g.Q) return nullptr;
    return rs.img + ((long)p * g.Q + q) * g.K + ko;
  }
};

// conv wgrad B operand: rows = (r, s, c) with c contiguous, k = output pixel (n,p,q).
template <typename T>
struct Im2colR {
  const T* x; ConvGeom g; int Rows;
  struct RowState { int r, s, c; };
  __device__ RowState row(int row) const {
    RowState rs;
    if (row >= Rows) { rs.r = -1; rs.s = rs.c = 0; return rs; }
    const int tap = row / g.C;
    rs.c = row - tap * g.C;
    rs.r = tap / g.S;
    rs.s = tap - rs.r * g.S;
    return rs;
  }
  typedef typename Vec16<T>::type V;
  __device__ V load(const RowState& rs, int k, int klim) const {
    const T* p = at(rs, k, klim);
    return p ? *(const V*)p : V{};
  }
  __device__ const T* at(const RowState& rs, int k, int klim) const {
    if (rs.r < 0 || k >= klim) return nullptr;
    const int pq = g.P * g.Q;
    const int n = k / pq, rem = k - n * pq;
    const int p = rem / g.Q, q = rem - p * g.Q;
    const int ih = p * g.sh - g.ph + rs.r, iw = q * g.sw - g.pw + rs.s;
    if ((unsigned)ih >= (unsigned)g.H || (unsigned)iw >= (unsigned)g.W) return nullptr;
    return x + (((long)n * g.H + ih) * g.W + iw) * g.C + rs.c;
  }
};

// --------------------------------------------------------------------------------------
// Tile loaders (global -> registers -> LDS).
// --------------------------------------------------------------------------------------
template <typename T, int ROWS, int BK, class Src>
struct KMajorLoader {
  typedef typename Vec16<T>::type V;
  static constexpr int VEC = Vec16<T>::N;
  static constexpr int KV = BK / VEC;    // vectors per row
  static constexpr int RPP = NT / KV;    // rows per pass
  static constexpr int CH = ROWS / RPP;  // vectors per thread
  static_assert(ROWS % RPP == 0, "tile rows");
  typename Src::RowState rs[CH];
  int kv, r0;
  __device__ void init(const Src& s, int row0) {
    kv = threadIdx.x % KV;
    r0 = threadIdx.x / KV;
#pragma unroll
    for (int i = 0; i < CH; ++i) rs[i] = s.row(row0 + r0 + i * RPP);
  }
  __device__ void fetch(const Src& s, int k0, int klim, V* regs) const {
    const int k = k0 + kv * VEC;
#pragma unroll
    for (int i = 0; i < CH; ++i) regs[i] = s.load(rs[i], k, klim);
  }
  __device__ void store(T* lds, const V* regs) const {
    constexpr int LDK = LdsGeom<T, BK>::LDK;
#pragma unroll
    for (int i = 0; i < CH; ++i) *(V*)(lds + (r0 + i * RPP) * LDK + kv * VEC) = regs[i];
  }
};

template <typename T, int ROWS, int BK, class Src>
struct RMajorLoader {
  typedef typename Vec16<T>::type V;
  static constexpr int VEC = Vec16<T>::N;
  static constexpr int RV = ROWS / VEC;  // vectors per k
  static constexpr int KPP = NT / RV;    // k per pass
  static constexpr int CH = BK / KPP;
  static_assert(NT % RV == 0 && BK % KPP == 0, "tile shape");
  typename Src::RowState rs;
  int rv, kk0;
  __device__ void init(const Src& s, int row0) {
    rv = threadIdx.x % RV;
    kk0 = threadIdx.x / RV;
    rs = s.row(row0 + rv * VEC);
  }
  __device__ void fetch(const Src& s, int k0, int klim, V* regs) const {
#pragma unroll
    for (int i = 0; i < CH; ++i) regs[i] = s.load(rs, k0 + kk0 + i * KPP, klim);
  }
  __device__ void store(T* lds, const V* regs) const {
    constexpr int LDK = LdsGeom<T, BK>::LDK;
#pragma unroll
    for (int i = 0; i < CH; ++i)
#pragma unroll
      for (int j = 0; j < VEC; ++j) lds[(rv * VEC + j) * LDK + kk0 + i * KPP] = regs[i][j];
  }
};

// --------------------------------------------------------------------------------------
// Epilogues. `apply(m, n, v)` is called per output element with the fp32 accumulator.
// --------------------------------------------------------------------------------------
template <typename OutT>
struct EpiStore {
  OutT* C; long ldc; int M, N;
  const float* bias;  // [N] or null
  const float* addend;  // [M][ldc] fp32 or null, added before the activation
  int act;            // Act
  float alpha, beta;  // C = act(alpha*acc + bias) + beta*C
  OutT* preact;       // optional copy of alpha*acc+bias (for GELU backward), ld = ldc
  __device__ __forceinline__ void apply(int m, int n, float v) const {
    if (m >= M || n >= N) return;
    v = alpha * v;
    if (bias) v += bias[n];
    const long off = (long)m * ldc + n;
    if (addend) v += addend[off];
    if (preact) preact[off] = from_f<OutT>(v);
    if (act == ACT_RELU) v = fmaxf(v, 0.f);
    else if (act == ACT_GELU) v = gelu_erf(v);
    if (beta != 0.f) v += beta * to_f(C[off]);
    C[off] = from_f<OutT>(v);
  }
};

// Raw fp32 partial for split-K: ws[z][M][N].
struct EpiPartial {
  float* ws; int M, N;
  __device__ __forceinline__ void apply(int m, int n, float v) const {
    if (m >= M || n >= N) return;
    ws[((long)blockIdx.z * M + m) * N + n] = v;
  }
};

// Bijective XCD-aware remap: blocks that share an A panel land on one XCD's L2.
__device__ __forceinline__ int xcd_swizzle(int orig, int nwg) {
  const int q = nwg / 8, r = nwg % 8, xcd = orig % 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / 8;
}

template <typename T, int BM, int BN, int WM, int WN, class LA, class LB, class Epi>
__global__ __launch_bounds__(NT, 2) void igemm_kernel(typename LA::SrcT sa, typename LB::SrcT sb,
                                                      Epi epi, int M, int N, int K, int kper) {
  constexpr int BK = KTile<T>::BK;
  constexpr int LDK = LdsGeom<T, BK>::LDK;
  constexpr int WTM = BM / WM, WTN = BN / WN;
  constexpr int RM = WTM / 16, RN = WTN / 16;
  typedef MfmaOp<T> Op;
  __shared__ __attribute__((aligned(16))) T lds[2 * (BM + BN) * LDK];
  T* const As = lds;                  // [2][BM][LDK]
  T* const Bs = lds + 2 * BM * LDK;   // [2][BN][LDK]

  const int tiles_n = (N + BN - 1) / BN;
  const int tiles_m = (M + BM - 1) / BM;
  const int tile = xcd_swizzle(blockIdx.x, tiles_m * tiles_n);
  const int tm = tile / tiles_n, tn = tile - tm * tiles_n;
  const int kbeg = blockIdx.z * kper;
  const int kend = min(K, kbeg + kper);
  const int nt = kend > kbeg ? (kend - kbeg + BK - 1) / BK : 0;

  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int wm = wid / WN, wn = wid % WN;

  LA la; la.init(sa, tm * BM);
  LB lb; lb.init(sb, tn * BN);
  typename LA::V ra[LA::CH];
  typename LB::V rb[LB::CH];

  f32x4 acc[RM][RN];
#pragma unroll
  for (int i = 0; i < RM; ++i)
#pragma unroll
    for (int j = 0; j < RN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  if (nt > 0) {
    la.fetch(sa, kbeg, kend, ra);
    lb.fetch(sb, kbeg, kend, rb);
    la.store(As, ra);
    lb.store(Bs, rb);
    __syncthreads();
  }
  const int frow = lane & 15, fk = (lane >> 4) * Op::FRAG;
  for (int t = 0; t < nt; ++t) {
    const int cur = t & 1;
    const bool more = t + 1 < nt;
    if (more) {
      la.fetch(sa, kbeg + (t + 1) * BK, kend, ra);
      lb.fetch(sb, kbeg + (t + 1) * BK, kend, rb);
    }
    const T* a_s = As + cur * BM * LDK + (wm * WTM + frow) * LDK + fk;
    const T* b_s = Bs + cur * BN * LDK + (wn * WTN + frow) * LDK + fk;
#pragma unroll
    for (int ks = 0; ks < BK; ks += Op::KS) {
      typename Op::frag_t af[RM], bfr[RN];
#pragma unroll
      for (int i = 0; i < RM; ++i) af[i] = Op::ld(a_s + i * 16 * LDK + ks);
#pragma unroll
      for (int j = 0; j < RN; ++j) bfr[j] = Op::ld(b_s + j * 16 * LDK + ks);
#pragma unroll
      for (int i = 0; i < RM; ++i)
#pragma unroll
        for (int j = 0; j < RN; ++j) acc[i][j] = Op::mma(af[i], bfr[j], acc[i][j]);
    }
    if (more) {
      la.store(As + (cur ^ 1) * BM * LDK, ra);
      lb.store(Bs + (cur ^ 1) * BN * LDK, rb);
    }
    __syncthreads();
  }

  // C/D map of 16x16 MFMA: col = lane&15, row = (lane>>4)*4 + reg.
  const int m0 = tm * BM + wm * WTM + (lane >> 4) * 4;
  const int n0 = tn * BN + wn * WTN + (lane & 15);
#pragma unroll
  for (int i = 0; i < RM; ++i)
#pragma unroll
    for (int j = 0; j < RN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) epi.apply(m0 + i * 16 + r, n0 + j * 16, acc[i][j][r]);
}

// Loader bundles (give the kernel template one type per operand).
template <typename T, int ROWS, class Src>
struct KLoad : KMajorLoader<T, ROWS, KTile<T>::BK, Src> { typedef Src SrcT; };
template <typename T, int ROWS, class Src>
struct RLoad : RMajorLoader<T, ROWS, KTile<T>::BK, Src> { typedef Src SrcT; };

}  // namespace mmdx
