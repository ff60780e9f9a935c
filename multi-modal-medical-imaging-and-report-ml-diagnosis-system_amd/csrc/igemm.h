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
// Operands are staged global -> registers -> LDS (two buffers, one barrier per K tile).
//   * K-major operands (k contiguous in global): LDS image [row][k], rows padded 16 B so
//     a ds_read_b128 lane group touches 16 distinct 16-B slots.
//   * R-major operands (rows contiguous in global; wgrad/Linear-dW): LDS image [k][row]
//     written with 16-B stores as loaded; bf16 fragments come back k-contiguous through
//     ds_read_b64_tr_b16 (hardware transpose), fp32 fragments through ds_read_b32.
// The k decomposition of a gather (filter tap, channel block) is computed ONCE per K tile
// in scalar registers when the channel count is a multiple of the K tile (every ResNet
// layer but the 3-channel stem), so the per-vector address math is an add + bounds check.
// The epilogue stages the fp32 accumulators through LDS and stores 4 outputs per lane.
#pragma once
#include <type_traits>
#include <utility>

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
template <> struct MfmaOp<f16> {
  static constexpr int KS = 32;
  static constexpr int FRAG = 8;
  typedef f16x8 frag_t;
  __device__ __forceinline__ static f32x4 mma(frag_t a, frag_t b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
  }
  __device__ __forceinline__ static frag_t ld(const f16* p) { return *(const f16x8*)p; }
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
template <> struct KTile<f16> { static constexpr int BK = 64; };
template <> struct KTile<float> { static constexpr int BK = 32; };

// Generic per-K-tile context: just the tile origin and the split's k bound.
struct KCtx { int k0, klim; };

// a / b for 0 <= a < 2^22, b >= 1 (uniform): float reciprocal estimate + one correction
// step (the estimate is within 1 of the quotient) — ~8 VALU instead of the ~30 of an integer
// division; the LDS-DMA prologue decodes every row it loads with it.
__device__ __forceinline__ int fdivu(int a, int b) {
  int q = (int)((float)a * __builtin_amdgcn_rcpf((float)b));
  const int r = a - q * b;
  q += (r >= b) - (r < 0);
  return q;
}

// Bit mask of the valid filter taps (bit r*S + s) for r in [rlo, rhi) x s in [slo, shi),
// bounds clamped to [0, R) x [0, S) (R*S <= 32): two bit ranges and R shifted copies instead of
// an R*S loop of bounds tests.
__device__ __forceinline__ unsigned tap_mask(int rlo, int rhi, int slo, int shi, int R, int S) {
  rlo = max(rlo, 0); rhi = min(rhi, R);
  slo = max(slo, 0); shi = min(shi, S);
  if (rhi <= rlo || shi <= slo) return 0u;
  const unsigned sb = (unsigned)((1ull << shi) - (1ull << slo));
  const unsigned rb = (unsigned)((1ull << rhi) - (1ull << rlo));
  unsigned m = 0u;
  for (int r = 0; r < R; ++r) m |= ((rb >> r) & 1u) ? sb << (r * S) : 0u;
  return m;
}

// --------------------------------------------------------------------------------------
// Operand sources.  `row(r)` -> per-row state (computed once per block), `ktile(k0,klim)`
// -> per-K-tile state (scalar, once per tile), `load(rs, kt, off)` -> one 16-B vector:
// K-major sources: VEC consecutive k at k0+off of row rs; R-major: VEC consecutive rows
// starting at rs, at k = k0+off.  Out-of-range elements read as zero.
// --------------------------------------------------------------------------------------

// Dense, K contiguous: element (r, k) at base[r*ld + k].  `vec` = ld and base allow 16-B
// vector loads; otherwise (and for a vector crossing klim) elements load one by one.
template <typename T>
struct DenseK {
  const T* base; long ld; int R; bool vec;
  typedef const T* RowState;
  typedef KCtx KT;
  typedef typename Vec16<T>::type V;
  __device__ RowState row(int r) const { return r < R ? base + (long)r * ld : nullptr; }
  __device__ KT ktile(int k0, int klim) const { return KT{k0, klim}; }
  __device__ V load(RowState rs, const KT& kt, int off) const {
    constexpr int VEC = Vec16<T>::N;
    const int k = kt.k0 + off;
    V v{};
    if (!rs || k >= kt.klim) return v;
    if (vec && k + VEC <= kt.klim) return *(const V*)(rs + k);
#pragma unroll
    for (int j = 0; j < VEC; ++j)
      if (k + j < kt.klim) v[j] = rs[k + j];
    return v;
  }
  // LDS-DMA path (vec, K tiles whole): address of the VEC elements at k0+off, or null = zeros
  __device__ const T* ptr(RowState rs, const KT& kt, int off) const {
    return rs && kt.k0 + off < kt.klim ? rs + kt.k0 + off : nullptr;
  }
  // buffer-DMA interface: byte offset of (row, k = 0) and tap-validity bits; per K tile the
  // uniform byte offset and tap index.  Offsets are relative to bbase().
  __device__ const void* bbase() const { return base; }
  __device__ unsigned bbytes() const { return (unsigned)((long)R * ld * sizeof(T)); }
  typedef unsigned Mask;
  static constexpr bool LANE_TAP = false;
  __device__ void lane_decode(int, int&, int&, int&) const {}
  __device__ bool lane_ok(unsigned, int, int) const { return false; }
  __device__ int brow(int r, unsigned& mask) const {
    mask = r < R ? ~0u : 0u;
    return r < R ? (int)((long)r * ld * sizeof(T)) : 0;
  }
  __device__ void btile(int k0, int& toff, int& tap) const { toff = k0 * (int)sizeof(T); tap = 0; }
  // K-tile iterator (DmaK): k = (u * T2 + v) * Cblk + c0; here one block spanning all of K
  __device__ void tdims(int& cblk, int& t2) const { cblk = 1 << 30; t2 = 1; }
  __device__ void tmap(int, int, int c0, int& toff, int& tap) const {
    toff = c0 * (int)sizeof(T); tap = 0;
  }
};

// The pointwise (1x1 / stride 1 / unpadded) conv's activation operands: plain dense
// matrices, given their own names so a kernel trace tells the conv family's dispatches
// (PointFwdK: x in the forward, PointDgradK: dY in the dgrad) from the Linear layers' DenseK.
template <typename T> struct PointFwdK : DenseK<T> {};
template <typename T> struct PointDgradK : DenseK<T> {};

// Dense, rows contiguous: element (r, k) at base[k*ld + r].
template <typename T>
struct DenseR {
  const T* base; long ld; int R; bool vec; int vrows;  // vrows: k extent (buffer size)
  typedef int RowState;
  typedef KCtx KT;
  typedef typename Vec16<T>::type V;
  // an out-of-range row is a large negative marker: its DMA offsets stay negative (= zeros)
  // without a per-DMA row test
  __device__ RowState row(int r) const { return r < R ? r : -(1 << 30); }
  __device__ KT ktile(int k0, int klim) const { return KT{k0, klim}; }
  __device__ V load(RowState rs, const KT& kt, int off) const {
    constexpr int VEC = Vec16<T>::N;
    const int k = kt.k0 + off;
    V v{};
    if (rs < 0 || k >= kt.klim) return v;
    const T* p = base + (long)k * ld + rs;
    if (vec && rs + VEC <= R) return *(const V*)p;
#pragma unroll
    for (int j = 0; j < VEC; ++j)
      if (rs + j < R) v[j] = p[j];
    return v;
  }
  // LDS-DMA path (vec, R % 8 == 0): the 8 rows from rs at k = k0 + kk, or null = zeros
  __device__ const T* ptr(RowState rs, const KT& kt, int kk) const {
    const int k = kt.k0 + kk;
    return rs >= 0 && k < kt.klim ? base + (long)k * ld + rs : nullptr;
  }
  __device__ const void* bbase() const { return base; }
  __device__ unsigned bbytes() const { return (unsigned)((long)vrows * ld * sizeof(T)); }
  // LDS-DMA lane state: element offset k*ld of this lane's k-line, stepped one 64-deep K tile
  // per issue (an add instead of a multiply per DMA; the operand is < 2 GiB)
  static constexpr bool STEP = true;
  static constexpr bool STEP_ANY = true;  // any K-tile depth (lane_step_by)
  struct Lane { int koff; };
  __device__ Lane lane_at(int k) const { return Lane{k * (int)ld}; }
  __device__ void lane_step(Lane& l) const { l.koff += (int)ld << 6; }
  __device__ void lane_step_by(Lane& l, int bk) const { l.koff += (int)ld * bk; }
  template <bool CHECK_K>
  __device__ int roff_at(RowState rs, const Lane& l, int k, int klim) const {
    const int o = (l.koff + rs) * (int)sizeof(T);  // < 0 for an out-of-range row
    return CHECK_K && k >= klim ? -1 : o;
  }
  // byte offset of the 8 rows from rs at k, or -1 (zeros)
  __device__ int roff(RowState rs, int k, int klim) const {
    return rs >= 0 && k < klim ? (int)(((long)k * ld + rs) * sizeof(T)) : -1;
  }
  // DmaRq: every row of every ROWS-row tile is in range (quarters share one validity test)
  __device__ bool rows_one_tap(int rows) const { return R % rows == 0; }
};

// x^T of a pointwise conv in its weight gradient (named apart from DenseR, see PointFwdK)
template <typename T> struct PointWgradR : DenseR<T> {};

// exactly the plain-matrix sources (the conv operands derived from them are not)
template <class S> struct IsDenseSrc { static constexpr bool value = false; };
template <typename T> struct IsDenseSrc<DenseK<T>> { static constexpr bool value = true; };
template <typename T> struct IsDenseSrc<DenseR<T>> { static constexpr bool value = true; };

struct ConvGeom {
  int N, H, W, C;      // input NHWC
  int K;               // output channels
  int R, S;            // filter h, w
  int sh, sw, ph, pw;  // stride, pad
  int P, Q;            // output h, w
};

// conv fwd A operand: rows = output pixels (n,p,q), k = (r, s, c) with c contiguous.
// FAST: C % BK == 0, so one K tile = one filter tap and a contiguous channel block.
template <typename T, bool FAST>
struct Im2colK {
  const T* x; ConvGeom g; int M; int cshift = 0; float inv_s = 0.f;  // !FAST DMA: log2(C), 1/S
  struct RowState { const T* base; int ih0, iw0; };  // base = &x[n, ih0, iw0, 0]
  struct KT { int r, s, k0, klim; long off; };
  typedef typename Vec16<T>::type V;
  __device__ RowState row(int m) const {
    RowState rs;
    if (m >= M) { rs.base = nullptr; rs.ih0 = rs.iw0 = 0; return rs; }
    const int pq = g.P * g.Q;
    const int n = m / pq, rem = m - n * pq;
    const int p = rem / g.Q, q = rem - p * g.Q;
    rs.ih0 = p * g.sh - g.ph;
    rs.iw0 = q * g.sw - g.pw;
    rs.base = x + (((long)n * g.H + rs.ih0) * g.W + rs.iw0) * g.C;
    return rs;
  }
  __device__ KT ktile(int k0, int klim) const {
    KT kt;
    kt.k0 = k0; kt.klim = klim;
    kt.r = kt.s = 0; kt.off = 0;
    if (FAST) {
      const int tap = k0 / g.C;
      const int c0 = k0 - tap * g.C;
      kt.r = tap / g.S;
      kt.s = tap - kt.r * g.S;
      kt.off = ((long)kt.r * g.W + kt.s) * g.C + c0;
    }
    return kt;
  }
  __device__ V load(const RowState& rs, const KT& kt, int off) const {
    if (!rs.base) return V{};
    int r, s;
    long o;
    if (FAST) {
      r = kt.r; s = kt.s;
      o = kt.off + off;
    } else {
      const int k = kt.k0 + off;
      if (k >= kt.klim) return V{};
      const int tap = k / g.C, c = k - tap * g.C;
      r = tap / g.S;
      s = tap - r * g.S;
      o = ((long)r * g.W + s) * g.C + c;
    }
    const int ih = rs.ih0 + r, iw = rs.iw0 + s;
    if ((unsigned)ih >= (unsigned)g.H || (unsigned)iw >= (unsigned)g.W) return V{};
    return *(const V*)(rs.base + o);
  }
  __device__ const T* ptr(const RowState& rs, const KT& kt, int off) const {  // FAST only
    const int ih = rs.ih0 + kt.r, iw = rs.iw0 + kt.s;
    if (!rs.base || (unsigned)ih >= (unsigned)g.H || (unsigned)iw >= (unsigned)g.W)
      return nullptr;
    return rs.base + kt.off + off;
  }
  __device__ const void* bbase() const { return x; }
  __device__ unsigned bbytes() const { return (unsigned)((long)g.N * g.H * g.W * g.C * sizeof(T)); }
  // FAST: 32-bit tap mask (R*S <= 32), one tap per K tile.  !FAST (power-of-two C >= 8,
  // e.g. the 3-channel stem padded to 8): every lane's 8-channel chunk is its own tap,
  // decoded per lane; the row keeps its packed (ih0, iw0) instead of a mask.
  typedef typename std::conditional<FAST, unsigned, int>::type Mask;
  static constexpr bool LANE_TAP = !FAST;
  __device__ int brow(int m, Mask& mask) const {
    const int pq = g.P * g.Q;
    const int n = fdivu(m, pq), rem = m - n * pq;
    const int p = fdivu(rem, g.Q), q = rem - p * g.Q;
    const int ih0 = p * g.sh - g.ph, iw0 = q * g.sw - g.pw;
    if constexpr (FAST) {
      mask = 0u;
      if (m >= M) return 0;
      mask = tap_mask(-ih0, g.H - ih0, -iw0, g.W - iw0, g.R, g.S);
    } else {
      mask = m < M ? (int)(((unsigned)ih0 << 16) | ((unsigned)iw0 & 0xffffu)) : (int)0x80008000;
      if (m >= M) return 0;
    }
    return (int)((((long)n * g.H + ih0) * g.W + iw0) * g.C * (long)sizeof(T));
  }
  // per-lane tap of element k: byte offset from the row base, and the (r, s) it needs
  __device__ void lane_decode(int k, int& toff, int& r, int& s) const {
    const int tap = k >> cshift, c = k & (g.C - 1);
    r = (int)((float)tap * inv_s + 1e-3f);  // tap < 64: exact
    s = tap - r * g.S;
    toff = ((r * g.W + s) * g.C + c) * (int)sizeof(T);
  }
  __device__ bool lane_ok(Mask mk, int r, int s) const {
    const int ih = (mk >> 16) + r, iw = (int)(short)(mk & 0xffff) + s;
    return (unsigned)ih < (unsigned)g.H && (unsigned)iw < (unsigned)g.W;
  }
  __device__ void btile(int k0, int& toff, int& tap) const {
    tap = k0 / g.C;
    const int c0 = k0 - tap * g.C, r = tap / g.S, s = tap - r * g.S;
    toff = ((r * g.W + s) * g.C + c0) * (int)sizeof(T);
  }
  // K-tile iterator: (u, v) = filter tap (r, s), c0 = channel block
  __device__ void tdims(int& cblk, int& t2) const { cblk = g.C; t2 = g.S; }
  __device__ void tmap(int r, int s, int c0, int& toff, int& tap) const {
    toff = ((r * g.W + s) * g.C + c0) * (int)sizeof(T);
    tap = r * g.S + s;
  }
};

// conv dgrad A operand: rows = input pixels (n,h,w), k = (r, s, kout) with kout contiguous.
// dX[n,h,w,c] = sum_{r,s,k} dY[n,(h+ph-r)/sh,(w+pw-s)/sw,k] * W[k,r,s,c]  (divisible taps only)
template <typename T, bool FAST>
struct DgradK {
  const T* dy; ConvGeom g; int M;
  struct RowState { const T* img; int h, w; };
  struct KT { int r, s, k0, klim, kb; };
  typedef typename Vec16<T>::type V;
  __device__ RowState row(int m) const {
    RowState rs;
    if (m >= M) { rs.img = nullptr; rs.h = rs.w = 0; return rs; }
    const int hw = g.H * g.W;
    const int n = m / hw, rem = m - n * hw;
    const int hh = rem / g.W;
    rs.h = hh + g.ph;
    rs.w = rem - hh * g.W + g.pw;
    rs.img = dy + (long)n * g.P * g.Q * g.K;
    return rs;
  }
  __device__ KT ktile(int k0, int klim) const {
    KT kt;
    kt.k0 = k0; kt.klim = klim;
    kt.r = kt.s = kt.kb = 0;
    if (FAST) {
      const int tap = k0 / g.K;
      kt.kb = k0 - tap * g.K;
      kt.r = tap / g.S;
      kt.s = tap - kt.r * g.S;
    }
    return kt;
  }
  __device__ V load(const RowState& rs, const KT& kt, int off) const {
    if (!rs.img) return V{};
    int r, s, ko;
    if (FAST) {
      r = kt.r; s = kt.s; ko = kt.kb + off;
    } else {
      const int k = kt.k0 + off;
      if (k >= kt.klim) return V{};
      const int tap = k / g.K;
      ko = k - tap * g.K;
      r = tap / g.S;
      s = tap - r * g.S;
    }
    const int th = rs.h - r, tw = rs.w - s;
    if (th < 0 || tw < 0) return V{};
    int p, q;
    if (g.sh == 1 && g.sw == 1) {
      p = th; q = tw;
    } else {
      p = th / g.sh; q = tw / g.sw;
      if (p * g.sh != th || q * g.sw != tw) return V{};
    }
    if (p >= g.P || q >= g.Q) return V{};
    return *(const V*)(rs.img + ((long)p * g.Q + q) * g.K + ko);
  }
  __device__ const T* ptr(const RowState& rs, const KT& kt, int off) const {  // FAST only
    if (!rs.img) return nullptr;
    const int th = rs.h - kt.r, tw = rs.w - kt.s;
    if (th < 0 || tw < 0) return nullptr;
    int p = th, q = tw;
    if (g.sh != 1 || g.sw != 1) {
      p = th / g.sh; q = tw / g.sw;
      if (p * g.sh != th || q * g.sw != tw) return nullptr;
    }
    if (p >= g.P || q >= g.Q) return nullptr;
    return rs.img + ((long)p * g.Q + q) * g.K + kt.kb + off;
  }
  __device__ const void* bbase() const { return dy; }
  __device__ unsigned bbytes() const { return (unsigned)((long)g.N * g.P * g.Q * g.K * sizeof(T)); }
  typedef unsigned Mask;
  static constexpr bool LANE_TAP = false;
  __device__ void lane_decode(int, int&, int&, int&) const {}
  __device__ bool lane_ok(unsigned, int, int) const { return false; }
  __device__ int brow(int m, unsigned& mask) const {  // FAST, stride 1, R*S <= 32
    mask = 0u;
    if (m >= M) return 0;
    const int hw = g.H * g.W;
    const int n = fdivu(m, hw), rem = m - n * hw;
    const int h = fdivu(rem, g.W), w = rem - h * g.W;
    // valid taps: 0 <= h + ph - r < P, 0 <= w + pw - s < Q
    mask = tap_mask(h + g.ph - g.P + 1, h + g.ph + 1, w + g.pw - g.Q + 1, w + g.pw + 1, g.R, g.S);
    return (int)((((long)n * g.P + h + g.ph) * g.Q + w + g.pw) * g.K * (long)sizeof(T));
  }
  __device__ void btile(int k0, int& toff, int& tap) const {
    tap = k0 / g.K;
    const int kb = k0 - tap * g.K, r = tap / g.S, s = tap - r * g.S;
    toff = (kb - (r * g.Q + s) * g.K) * (int)sizeof(T);
  }
  __device__ void tdims(int& cblk, int& t2) const { cblk = g.K; t2 = g.S; }
  __device__ void tmap(int r, int s, int kb, int& toff, int& tap) const {
    toff = (kb - (r * g.Q + s) * g.K) * (int)sizeof(T);
    tap = r * g.S + s;
  }
};

// Strided-conv dgrad, one output phase (a, b) = (h mod sh, w mod sw) at a time: only the
// taps r = r0 + sh*u (s = s0 + sw*v) reach those pixels, so the GEMM runs over
// M = N*Hp*Wp phase pixels and K = ntaps*Kout instead of all H*W pixels and all R*S taps
// (a stride-2 3x3 conv does 1/4 of the MACs of the dense dgrad; a stride-2 1x1 only the
// (0,0) phase).  Requires Kout % BK == 0 (each K tile = one tap, contiguous channel block).
struct PhaseGeom {
  int Hp, Wp;      // phase grid
  int r0, s0;      // first tap of the phase
  int ntr, nts;    // taps in r / s
  int dr0, ds0;    // (a + ph - r0) / sh, (b + pw - s0) / sw
};

// Merged-phase launches (gridDim.z = phases, conv_dgrad_phases): the A / B sources and the
// epilogue carry every phase's geometry and each block selects its own (select(blockIdx.z))
// before anything else, so the sh*sw phase GEMMs of a strided dgrad fill the chip as one grid
// instead of sh*sw launches of a quarter of it each.
constexpr int MAX_PHASES = 4;

template <typename T>
struct DgradPhaseK {
  const T* dy; ConvGeom g; PhaseGeom ph; int M;
  PhaseGeom phs[MAX_PHASES]; int Ms[MAX_PHASES];
  // phase p's geometry from the (unwritten) kernel argument `k` (igemm_dma_kernel): p is
  // block-uniform (blockIdx.z), so these are scalar loads from the kernarg segment
  __device__ void select_from(const DgradPhaseK& k, int p) {
    ph = k.phs[p];
    M = k.Ms[p];
  }
  struct RowState { const T* img; int i, j; };
  struct KT { int dr, ds, kb, k0, klim; };
  typedef typename Vec16<T>::type V;
  __device__ RowState row(int m) const {
    RowState rs;
    if (m >= M) { rs.img = nullptr; rs.i = rs.j = 0; return rs; }
    const int hw = ph.Hp * ph.Wp;
    const int n = m / hw, rem = m - n * hw;
    rs.i = rem / ph.Wp;
    rs.j = rem - rs.i * ph.Wp;
    rs.img = dy + (long)n * g.P * g.Q * g.K;
    return rs;
  }
  __device__ KT ktile(int k0, int klim) const {
    KT kt;
    const int t = k0 / g.K;
    kt.kb = k0 - t * g.K;
    const int u = t / ph.nts, v = t - u * ph.nts;
    kt.dr = ph.dr0 - u;  // tap r0 + sh*u moves the source row up by u
    kt.ds = ph.ds0 - v;
    kt.k0 = k0; kt.klim = klim;
    return kt;
  }
  __device__ V load(const RowState& rs, const KT& kt, int off) const {
    if (!rs.img || kt.k0 + off >= kt.klim) return V{};
    const int p = rs.i + kt.dr, q = rs.j + kt.ds;
    if ((unsigned)p >= (unsigned)g.P || (unsigned)q >= (unsigned)g.Q) return V{};
    return *(const V*)(rs.img + ((long)p * g.Q + q) * g.K + kt.kb + off);
  }
  __device__ const T* ptr(const RowState& rs, const KT& kt, int off) const {
    if (!rs.img || kt.k0 + off >= kt.klim) return nullptr;
    const int p = rs.i + kt.dr, q = rs.j + kt.ds;
    if ((unsigned)p >= (unsigned)g.P || (unsigned)q >= (unsigned)g.Q) return nullptr;
    return rs.img + ((long)p * g.Q + q) * g.K + kt.kb + off;
  }
  __device__ const void* bbase() const { return dy; }
  __device__ unsigned bbytes() const { return (unsigned)((long)g.N * g.P * g.Q * g.K * sizeof(T)); }
  typedef unsigned Mask;
  static constexpr bool LANE_TAP = false;
  __device__ void lane_decode(int, int&, int&, int&) const {}
  __device__ bool lane_ok(unsigned, int, int) const { return false; }
  __device__ int brow(int m, unsigned& mask) const {  // ntr * nts <= 32
    mask = 0u;
    if (m >= M) return 0;
    const int hw = ph.Hp * ph.Wp;
    const int n = fdivu(m, hw), rem = m - n * hw;
    const int i = fdivu(rem, ph.Wp), j = rem - i * ph.Wp;
    // valid taps: 0 <= i + dr0 - u < P, 0 <= j + ds0 - v < Q
    mask = tap_mask(i + ph.dr0 - g.P + 1, i + ph.dr0 + 1, j + ph.ds0 - g.Q + 1, j + ph.ds0 + 1,
                    ph.ntr, ph.nts);
    return (int)((((long)n * g.P + i) * g.Q + j) * g.K * (long)sizeof(T));
  }
  __device__ void btile(int k0, int& toff, int& tap) const {
    tap = k0 / g.K;
    const int kb = k0 - tap * g.K, u = tap / ph.nts, v = tap - u * ph.nts;
    toff = (((ph.dr0 - u) * g.Q + (ph.ds0 - v)) * g.K + kb) * (int)sizeof(T);
  }
  __device__ void tdims(int& cblk, int& t2) const { cblk = g.K; t2 = ph.nts; }
  __device__ void tmap(int u, int v, int kb, int& toff, int& tap) const {
    toff = (((ph.dr0 - u) * g.Q + (ph.ds0 - v)) * g.K + kb) * (int)sizeof(T);
    tap = u * ph.nts + v;
  }
};

// B operand of the phase dgrad: packed CRSK weights, k = (phase tap t, kout).
template <typename T>
struct PhaseTapK {
  const T* w; long ld; int C, K, S, sh, sw; PhaseGeom ph;  // w[c][r][s][k], ld = R*S*K
  PhaseGeom phs[MAX_PHASES];
  __device__ void select_from(const PhaseTapK& k, int p) { ph = k.phs[p]; }  // (DgradPhaseK)
  typedef const T* RowState;
  struct KT { long kg; int k0, klim; };
  typedef typename Vec16<T>::type V;
  __device__ RowState row(int c) const { return c < C ? w + (long)c * ld : nullptr; }
  __device__ KT ktile(int k0, int klim) const {
    KT kt;
    const int t = k0 / K, kb = k0 - t * K;
    const int u = t / ph.nts, v = t - u * ph.nts;
    kt.kg = ((long)(ph.r0 + sh * u) * S + (ph.s0 + sw * v)) * K + kb;
    kt.k0 = k0; kt.klim = klim;
    return kt;
  }
  __device__ V load(RowState rs, const KT& kt, int off) const {
    if (!rs || kt.k0 + off >= kt.klim) return V{};
    return *(const V*)(rs + kt.kg + off);
  }
  __device__ const T* ptr(RowState rs, const KT& kt, int off) const {
    return rs && kt.k0 + off < kt.klim ? rs + kt.kg + off : nullptr;
  }
  __device__ const void* bbase() const { return w; }
  __device__ unsigned bbytes() const { return (unsigned)((long)C * ld * sizeof(T)); }
  typedef unsigned Mask;
  static constexpr bool LANE_TAP = false;
  __device__ void lane_decode(int, int&, int&, int&) const {}
  __device__ bool lane_ok(unsigned, int, int) const { return false; }
  __device__ int brow(int c, unsigned& mask) const {
    mask = c < C ? ~0u : 0u;
    return c < C ? (int)((long)c * ld * sizeof(T)) : 0;
  }
  __device__ void btile(int k0, int& toff, int& tap) const {
    const int t = k0 / K, kb = k0 - t * K;
    const int u = t / ph.nts, v = t - u * ph.nts;
    toff = (((ph.r0 + sh * u) * S + (ph.s0 + sw * v)) * K + kb) * (int)sizeof(T);
    tap = 0;
  }
  __device__ void tdims(int& cblk, int& t2) const { cblk = K; t2 = ph.nts; }
  __device__ void tmap(int u, int v, int kb, int& toff, int& tap) const {
    toff = (((ph.r0 + sh * u) * S + (ph.s0 + sw * v)) * K + kb) * (int)sizeof(T);
    tap = 0;
  }
};

// conv wgrad B operand: rows = (r, s, c) with c contiguous, k = output pixel (n,p,q).
template <typename T>
struct Im2colR {
  const T* x; ConvGeom g; int Rows; float inv_pq, inv_q;  // 1/(P*Q), 1/Q for roff()
  int dn, dp, dq;  // one 64-pixel K tile = dn*P*Q + dp*Q + dq pixels (lane stepping)
  // lane stepping in input coordinates (set by the host, im2colr_steps): one K tile moves a
  // lane's window origin (ih0, iw0) by (dp*sh, dq*sw) and its element offset by doff; a q
  // (p) wrap moves it by (sh, -Q*sw) (-P*sh) and the offset by wq (wp)
  int dih, diw, doff, qlim, qspan, wq, plim, pspan, wp;
  struct RowState { int r, s, c, toff; };  // toff = element offset of tap (r, s), channel c
  typedef KCtx KT;
  typedef typename Vec16<T>::type V;
  __device__ RowState row(int row) const {
    RowState rs;
    if (row >= Rows) { rs.r = -1; rs.s = rs.c = rs.toff = 0; return rs; }
    const int tap = row / g.C;
    rs.c = row - tap * g.C;
    rs.r = tap / g.S;
    rs.s = tap - rs.r * g.S;
    rs.toff = (rs.r * g.W + rs.s) * g.C + rs.c;
    return rs;
  }
  __device__ KT ktile(int k0, int klim) const { return KT{k0, klim}; }
  __device__ V load(const RowState& rs, const KT& kt, int off) const {
    const int k = kt.k0 + off;
    if (rs.r < 0 || k >= kt.klim) return V{};
    const int pq = g.P * g.Q;
    const int n = k / pq, rem = k - n * pq;
    const int p = rem / g.Q, q = rem - p * g.Q;
    const int ih = p * g.sh - g.ph + rs.r, iw = q * g.sw - g.pw + rs.s;
    if ((unsigned)ih >= (unsigned)g.H || (unsigned)iw >= (unsigned)g.W) return V{};
    return *(const V*)(x + (((long)n * g.H + ih) * g.W + iw) * g.C + rs.c);
  }
  __device__ const T* ptr(const RowState& rs, const KT& kt, int kk) const {
    const int k = kt.k0 + kk;
    if (rs.r < 0 || k >= kt.klim) return nullptr;
    const int pq = g.P * g.Q;
    const int n = k / pq, rem = k - n * pq;
    const int p = rem / g.Q, q = rem - p * g.Q;
    const int ih = p * g.sh - g.ph + rs.r, iw = q * g.sw - g.pw + rs.s;
    if ((unsigned)ih >= (unsigned)g.H || (unsigned)iw >= (unsigned)g.W) return nullptr;
    return x + (((long)n * g.H + ih) * g.W + iw) * g.C + rs.c;
  }
  __device__ const void* bbase() const { return x; }
  __device__ unsigned bbytes() const { return (unsigned)((long)g.N * g.H * g.W * g.C * sizeof(T)); }
  // LDS-DMA lane state: the window origin (ih0, iw0) of this lane's pixel and the element
  // offset of (n, ih0, iw0, 0), advanced one K tile per issue with adds and two wrap selects
  // (no multiplies in the K loop; the tensor is < 2 GiB, so 32-bit offsets)
  static constexpr bool STEP = true;
  struct Lane { int ih0, iw0, off; };
  __device__ Lane lane_at(int k) const {
    const int pq = g.P * g.Q;
    int n = (int)((float)k * inv_pq);
    int rem = k - n * pq;
    if (rem < 0) { --n; rem += pq; } else if (rem >= pq) { ++n; rem -= pq; }
    int p = (int)((float)rem * inv_q);
    int q = rem - p * g.Q;
    if (q < 0) { --p; q += g.Q; } else if (q >= g.Q) { ++p; q -= g.Q; }
    Lane l;
    l.ih0 = p * g.sh - g.ph;
    l.iw0 = q * g.sw - g.pw;
    l.off = ((n * g.H + l.ih0) * g.W + l.iw0) * g.C;
    return l;
  }
  __device__ void lane_step(Lane& l) const {
    l.iw0 += diw; l.ih0 += dih; l.off += doff;
    const bool wq_ = l.iw0 >= qlim;
    l.iw0 -= wq_ ? qspan : 0;
    l.ih0 += wq_ ? g.sh : 0;
    l.off += wq_ ? wq : 0;
    const bool wp_ = l.ih0 >= plim;
    l.ih0 -= wp_ ? pspan : 0;
    l.off += wp_ ? wp : 0;
  }
  template <bool CHECK_K>
  __device__ int roff_at(const RowState& rs, const Lane& l, int k, int klim) const {
    // an out-of-range row has r = -1: ih = ih0 - 1 may still be valid, so it is tested
    const int ih = l.ih0 + rs.r, iw = l.iw0 + rs.s;
    const bool ok = rs.r >= 0 && (!CHECK_K || k < klim) && (unsigned)ih < (unsigned)g.H &&
                    (unsigned)iw < (unsigned)g.W;
    return ok ? (l.off + rs.toff) * (int)sizeof(T) : -1;
  }
  // DmaRq: a ROWS-row tile lies in one filter tap (C % ROWS == 0, so tiles start on a tap and
  // every row is in range): its quarters share the pixel's bounds test
  __device__ bool rows_one_tap(int rows) const { return g.C % rows == 0; }
  // pixel k -> (n, p, q) by float reciprocals (k < 2^23: one correction step is exact)
  __device__ int roff(const RowState& rs, int k, int klim) const {
    if (rs.r < 0 || k >= klim) return -1;
    const int pq = g.P * g.Q;
    int n = (int)((float)k * inv_pq);
    int rem = k - n * pq;
    if (rem < 0) { --n; rem += pq; } else if (rem >= pq) { ++n; rem -= pq; }
    int p = (int)((float)rem * inv_q);
    int q = rem - p * g.Q;
    if (q < 0) { --p; q += g.Q; } else if (q >= g.Q) { ++p; q -= g.Q; }
    const int ih = p * g.sh - g.ph + rs.r, iw = q * g.sw - g.pw + rs.s;
    if ((unsigned)ih >= (unsigned)g.H || (unsigned)iw >= (unsigned)g.W) return -1;
    return (int)(((((long)n * g.H + ih) * g.W + iw) * g.C + rs.c) * (long)sizeof(T));
  }
};

// Host: the wgrad im2col^T operand with its per-K-tile lane-stepping constants (64 pixels).
template <typename T>
inline Im2colR<T> make_im2colr(const T* x, const ConvGeom& g, int rows) {
  Im2colR<T> s{};
  s.x = x; s.g = g; s.Rows = rows;
  const int pq = g.P * g.Q;
  s.inv_pq = 1.f / (float)pq;
  s.inv_q = 1.f / (float)g.Q;
  s.dn = 64 / pq;
  s.dp = (64 % pq) / g.Q;
  s.dq = (64 % pq) % g.Q;
  const int HWC = g.H * g.W * g.C, WC = g.W * g.C;
  s.dih = s.dp * g.sh;
  s.diw = s.dq * g.sw;
  s.doff = s.dn * HWC + s.dih * WC + s.diw * g.C;
  s.qlim = g.Q * g.sw - g.pw;
  s.qspan = g.Q * g.sw;
  s.wq = -s.qspan * g.C + g.sh * WC;
  s.plim = g.P * g.sh - g.ph;
  s.pspan = g.P * g.sh;
  s.wp = -s.pspan * WC + HWC;
  return s;
}

// --------------------------------------------------------------------------------------
// Tile loaders (global -> registers -> LDS) and MFMA fragment reads from their LDS image.
// --------------------------------------------------------------------------------------
template <typename T, int ROWS, int BK, class Src>
struct KMajorLoader {
  typedef typename Vec16<T>::type V;
  typedef Src SrcT;
  static constexpr int VEC = Vec16<T>::N;
  static constexpr int LDK = BK + VEC;   // +16 B row pad
  static constexpr int LDS_ELEMS = ROWS * LDK;
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
    const typename Src::KT kt = s.ktile(k0, klim);
#pragma unroll
    for (int i = 0; i < CH; ++i) regs[i] = s.load(rs[i], kt, kv * VEC);
  }
  __device__ void store(T* lds, const V* regs) const {
#pragma unroll
    for (int i = 0; i < CH; ++i) *(V*)(lds + (r0 + i * RPP) * LDK + kv * VEC) = regs[i];
  }
  // fragment of the 16-row MFMA tile starting at row `r16`, k-step `ks`
  __device__ static typename MfmaOp<T>::frag_t frag(const T* lds, int r16, int ks) {
    const int lane = threadIdx.x & 63;
    return MfmaOp<T>::ld(lds + (r16 + (lane & 15)) * LDK + ks + (lane >> 4) * MfmaOp<T>::FRAG);
  }
};

template <typename T, int ROWS, int BK, class Src>
struct RMajorLoader {
  typedef typename Vec16<T>::type V;
  typedef Src SrcT;
  static constexpr int VEC = Vec16<T>::N;
  static constexpr int RV = ROWS / VEC;  // vectors per k
  static constexpr int KPP = NT / RV;    // k per pass
  static constexpr int CH = BK / KPP;
  static_assert(NT % RV == 0 && BK % KPP == 0, "tile shape");
  // [k][row] image; each group of 8 consecutive k rows is skewed by 64 elements so the
  // 4-row blocks that the two 16-lane groups of a ds_read_b64_tr_b16 half-wave read
  // (k and k+8) land on different banks.
  static constexpr int LDR = ROWS + 16;
  static constexpr int LDS_ELEMS = BK * LDR + (BK / 8) * 64;
  __device__ static int kaddr(int k) { return k * LDR + (k >> 3) * 64; }
  typename Src::RowState rs;
  int rv, kk0;
  __device__ void init(const Src& s, int row0) {
    rv = threadIdx.x % RV;
    kk0 = threadIdx.x / RV;
    rs = s.row(row0 + rv * VEC);
  }
  __device__ void fetch(const Src& s, int k0, int klim, V* regs) const {
    const typename Src::KT kt = s.ktile(k0, klim);
#pragma unroll
    for (int i = 0; i < CH; ++i) regs[i] = s.load(rs, kt, kk0 + i * KPP);
  }
  __device__ void store(T* lds, const V* regs) const {
#pragma unroll
    for (int i = 0; i < CH; ++i) *(V*)(lds + kaddr(kk0 + i * KPP) + rv * VEC) = regs[i];
  }
  __device__ static typename MfmaOp<T>::frag_t frag(const T* lds, int r16, int ks) {
    const int lane = threadIdx.x & 63;
    if constexpr (sizeof(T) == 2) {
      // lane 4q+p of 16-lane group g addresses row k = ks+8g+q (+4), columns 4p..4p+3 and
      // receives column (lane&15) of the 4 rows: 8 consecutive k, as the MFMA wants.
      const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
      const int k = ks + 8 * g + q;
      typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
      const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
          (lds_s16x4*)(lds + kaddr(k) + r16 + 4 * p));
      const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
          (lds_s16x4*)(lds + kaddr(k + 4) + r16 + 4 * p));
      typedef __attribute__((ext_vector_type(8))) short s16x8;
      const s16x8 v = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
      return __builtin_bit_cast(typename MfmaOp<T>::frag_t, v);
    } else {
      return lds[kaddr(ks + (lane >> 4)) + r16 + (lane & 15)];
    }
  }
};

// --------------------------------------------------------------------------------------
// Epilogues. `apply4(m, n, v)` handles 4 consecutive columns n..n+3 of row m.
// --------------------------------------------------------------------------------------
// Statistics of a consumer BatchNorm's backward, fused into the epilogue of the dgrad that
// produces its input gradient dout (units without a residual: their ReLU mask is recomputed
// from the BN input y with the forward's scale/shift).  Per column n over the tile's rows:
// (sum g, sum g*xhat), g = dout * [y*scale + shift > 0], xhat = (y - mean) * rstd — the
// partials bn_bwd_reduce_kernel would compute, written [N][tiles] at tile0 + tm.  The dout
// values used are the stored (rounded) ones, as the separate reduce would read them.
struct BnStat {
  const void* y; const float *gamma, *beta, *mean, *rstd; float2* part; int relu, tiles, tile0;
  const void* out;  // residual unit: its output relu(bn(y) + res), the ReLU mask source
};

struct BnCoef8 { float mu[8], rs[8], sc[8], sh[8]; };

__device__ __forceinline__ void bn_coef8(const BnStat& b, int n, int N, BnCoef8& c) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const bool ok = n + j < N;
    const float mu = ok ? b.mean[n + j] : 0.f, rs = ok ? b.rstd[n + j] : 0.f;
    const float g = ok && b.gamma ? b.gamma[n + j] : 1.f;
    c.mu[j] = mu;
    c.rs[j] = rs;
    c.sc[j] = g * rs;  // same expression order as bn_coef / bn_bwd_reduce_kernel
    c.sh[j] = (ok && b.beta ? b.beta[n + j] : 0.f) - mu * g * rs;
  }
}

typedef __attribute__((ext_vector_type(8))) __bf16 bn_y8;

template <typename T>
__device__ __forceinline__ void bn_acc8(const bn_y8& yv, const bn_y8& ov, f32x4 lo, f32x4 hi,
                                        const BnStat& b, const BnCoef8& c, float* sg,
                                        float* sgx) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    float g = to_f(from_f<T>(j < 4 ? lo[j] : hi[j - 4]));
    const float y = to_f(yv[j]);
    const float a = b.out ? to_f(ov[j]) : y * c.sc[j] + c.sh[j];  // the forward's ReLU input
    if (b.relu && !(a > 0.f)) g = 0.f;
    sg[j] += g;
    sgx[j] += g * (y - c.mu[j]) * c.rs[j];
  }
}

// The fused-statistics epilogue stores the final values itself (alpha = 1): (lo, hi) +=
// beta * C[m][n..n+7] first, so the statistics see the accumulated gradient of a residual
// branch (beta = 1), then a plain store.  Epi::bn_off maps (m, n) to the element offset.
template <class Epi>
__device__ __forceinline__ void bst_accum8(const Epi& e, int m, int n, f32x4& lo, f32x4& hi) {
  if constexpr (Epi::BNSTAT) {
    if (e.beta == 0.f || m >= e.M) return;
    const long off = e.bn_off(m, n);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (n + j < e.N) lo[j] += e.beta * to_f(e.C[off + j]);
      if (n + 4 + j < e.N) hi[j] += e.beta * to_f(e.C[off + 4 + j]);
    }
  }
}

template <class Epi>
__device__ __forceinline__ void bst_store8(const Epi& e, int m, int n, f32x4 lo, f32x4 hi) {
  if constexpr (Epi::BNSTAT) {
    if (m >= e.M) return;
    const long off = e.bn_off(m, n);
    typedef typename std::remove_pointer<decltype(e.C)>::type OutT;
    if (n + 8 > e.N) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (n + j < e.N) e.C[off + j] = from_f<OutT>(lo[j]);
        if (n + 4 + j < e.N) e.C[off + 4 + j] = from_f<OutT>(hi[j]);
      }
      return;
    }
    typedef __attribute__((ext_vector_type(8))) OutT O8;
    O8 o;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      o[j] = from_f<OutT>(lo[j]);
      o[j + 4] = from_f<OutT>(hi[j]);
    }
    __builtin_nontemporal_store(o, (O8*)(e.C + off));  // (streaming: see apply8_fast)
  }
}

// Merge the per-thread column sums of the vec8 epilogue loop (threads with equal
// threadIdx % C8 own the same 8 columns) and store the tile's partials.
// SLABS > 1 (256-row tiles): the partial slots stay per 128 rows (what the consumer's
// stat_blocks counts); the sums are additive, so the tile's sums go to its first slot and its
// other slots inside the GEMM's M rows get zeros.
template <int BN, int NW, int SLABS = 1>
__device__ __forceinline__ void bn_stat_store(const BnStat& b, float* sg, float* sgx, float* red,
                                              int tm, int tn, int N, int M = 0) {
  constexpr int C8 = BN / 8;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int x = C8; x < 64; x <<= 1)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      sg[j] += __shfl_xor(sg[j], x, 64);
      sgx[j] += __shfl_xor(sgx[j], x, 64);
    }
  if (lane < C8)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      red[(wid * BN + lane * 8 + j) * 2] = sg[j];
      red[(wid * BN + lane * 8 + j) * 2 + 1] = sgx[j];
    }
  __syncthreads();
  const int col = threadIdx.x;
  if (col < BN && tn * BN + col < N) {
    float a = 0.f, c = 0.f;
#pragma unroll
    for (int w = 0; w < NW; ++w) {
      a += red[(w * BN + col) * 2];
      c += red[(w * BN + col) * 2 + 1];
    }
    float2* dst = b.part + (long)(tn * BN + col) * b.tiles + b.tile0 + tm * SLABS;
    dst[0] = make_float2(a, c);
#pragma unroll
    for (int s = 1; s < SLABS; ++s)
      if ((tm * SLABS + s) * 128 < M) dst[s] = make_float2(0.f, 0.f);
  }
}

// VEC_EPI: the 16-B-per-8-columns epilogue also for bias / addend / pre-activation / ReLU /
// GELU (the dense GEMMs of gemm_dense.hip).  The conv instantiations keep the lean form
// (their epilogues never carry those): the extra branch cost the C4 step 2.3 % when it was
// compiled into every conv kernel (8955 vs 8750 samples/s, tools/lab_ab3c4.sh).
template <typename OutT, bool VEC_EPI = false>
struct EpiStore {
  OutT* C; long ldc; int M, N;
  const float* bias;    // [N] or null
  const float* addend;  // [M][ldc] fp32 or null, added before the activation
  int act;              // Act
  float alpha, beta;    // C = act(alpha*acc + bias + addend) + beta*C
  OutT* preact;         // optional copy of the pre-activation value, ld = ldc
  float2* stats;        // optional per-column (mean, M2) of each BM-row tile: [N][tiles_m]
  BnStat bs{};          // optional fused consumer-BN backward statistics (bs.part != null)
  // optional masked accumulation source (beta must be 0): C = acc + (bit ? acc_src : 0), bit
  // from a 1-bit ReLU mask ([M][N / VEC] bytes, bit e of byte n / VEC = column n) — the
  // gradient a residual unit's identity path adds, without materialising it
  const OutT* acc_src = nullptr;
  const uint8_t* acc_mask = nullptr;
  // optional residual [M][ldc] (OutT) added last, as beta*C with beta 1 would add a copy of
  // it (ViT's out = a + f W2^T + b2 without copying a into C first)
  const OutT* res = nullptr;
  static constexpr bool BNSTAT = true;
  static constexpr bool SPLIT = false;
  __device__ __forceinline__ long bn_off(int m, int n) const { return (long)m * ldc + n; }
  __device__ __forceinline__ float acc_at(int m, int n) const {
    constexpr int VM = 16 / (int)sizeof(OutT);
    const unsigned b = acc_mask[(long)m * (N / VM) + n / VM];
    return (b >> (n % VM)) & 1u ? to_f(acc_src[(long)m * ldc + n]) : 0.f;
  }
  // Per-column (mean, M2) over this tile's valid rows, from the fp32 accumulators staged in
  // LDS (cst [BM][LDC]) — the BatchNorm statistics of a conv output without re-reading it.
  // Two passes (mean, then squared deviations) over NT/BN row slices, merged with Chan.
  template <int BM, int BN, int LDC>
  __device__ __forceinline__ void tile_stats(const float* cst, float* red, int tm, int tn) const {
    if (!stats) return;
    constexpr int PARTS = NT / BN, RPP = BM / PARTS;
    const int col = threadIdx.x % BN, part = threadIdx.x / BN;
    const int rows_valid = min(BM, M - tm * BM);
    const int r0 = part * RPP, r1 = min(r0 + RPP, rows_valid);
    // one pass, shifted by the slice's first value (no cancellation within <= 64 rows)
    const float x0 = r1 > r0 ? cst[r0 * LDC + col] : 0.f;
    float s = 0.f, q = 0.f;
    for (int r = r0; r < r1; ++r) {
      const float d = cst[r * LDC + col] - x0;
      s += d;
      q += d * d;
    }
    const float cnt = (float)max(r1 - r0, 0);
    const float mean = cnt > 0.f ? x0 + s / cnt : 0.f;
    const float m2 = cnt > 0.f ? fmaxf(q - s * s / cnt, 0.f) : 0.f;
    red[threadIdx.x * 3 + 0] = cnt;
    red[threadIdx.x * 3 + 1] = mean;
    red[threadIdx.x * 3 + 2] = m2;
    __syncthreads();
    const int n = tn * BN + col;
    if (part == 0 && n < N) {
      float nn = 0.f, mu = 0.f, mm = 0.f;
#pragma unroll
      for (int q = 0; q < PARTS; ++q) {
        const int o = (q * BN + col) * 3;
        const float nb = red[o], mb = red[o + 1], m2b = red[o + 2];
        if (nb == 0.f) continue;
        if (nn == 0.f) { nn = nb; mu = mb; mm = m2b; continue; }
        const float tot = nn + nb, d = mb - mu, f = nb / tot;
        mu += d * f;
        mm += m2b + d * d * nn * f;
        nn = tot;
      }
      stats[(long)n * ((M + BM - 1) / BM) + tm] = make_float2(mu, mm);  // [N][tiles_m]
    }
  }
  __device__ __forceinline__ void apply(int m, int n, float v) const {
    if (m >= M || n >= N) return;
    v = alpha * v;
    const long off = (long)m * ldc + n;
    if (act == ACT_GELU_BWD) v *= gelu_erf_grad(to_f(preact[off]));  // preact is an input
    if (bias) v += bias[n];
    if (addend) v += addend[off];
    if (preact && act != ACT_GELU_BWD) preact[off] = from_f<OutT>(v);
    if (act == ACT_RELU) v = fmaxf(v, 0.f);
    else if (act == ACT_GELU) v = gelu_erf(v);
    if (beta != 0.f) v += beta * to_f(C[off]);
    if (res) v += to_f(res[off]);
    if (acc_src) v += acc_at(m, n);
    C[off] = from_f<OutT>(v);
  }
  // Block-uniform: every 8-column chunk can take one 16-B (bf16) / 2x16-B (fp32) store —
  // with a bias (8 consecutive fp32 per chunk), an addend row, a pre-activation copy and a
  // ReLU / GELU activation too (the forward Linear layers of the BERT / ViT stacks all carry
  // a bias; the per-element epilogue stored them 2 bytes at a time)
  __device__ __forceinline__ bool vec8_ok() const {
    if constexpr (!VEC_EPI)
      return !bias && !addend && !res && ldc % 8 == 0 && ((uintptr_t)C & 15) == 0 &&
             ((!preact && act == ACT_NONE) ||
              (act == ACT_GELU_BWD && !acc_src && ((uintptr_t)preact & 15) == 0));
    if (ldc % 8 != 0 || ((uintptr_t)C & 15) != 0) return false;
    if (bias && ((uintptr_t)bias & 15) != 0) return false;
    if (addend && ((uintptr_t)addend & 15) != 0) return false;
    if (preact && ((uintptr_t)preact & 15) != 0) return false;
    if (res && ((uintptr_t)res & 15) != 0) return false;
    // the vector GELU-backward branch computes alpha*acc*gelu'(pre) + beta*C only: a bias or
    // addend takes the per-element path (apply() adds them)
    if (act == ACT_GELU_BWD) return !acc_src && !res && !bias && !addend && preact;
    return !(acc_src && (bias || addend || preact || res || act != ACT_NONE));
  }
  // 8 consecutive columns n..n+7 of row m (vec8_ok() checked by the caller)
  __device__ __forceinline__ void apply8_fast(int m, int n, f32x4 lo, f32x4 hi) const {
    if (m >= M) return;
    if (n + 8 > N) {
      apply4(m, n, lo);
      if (n + 4 < N) apply4(m, n + 4, hi);
      return;
    }
    const long off = (long)m * ldc + n;
    typedef __attribute__((ext_vector_type(8))) OutT O8;
    O8 o;
    if (act == ACT_GELU_BWD) {  // C = alpha*acc * gelu'(pre) (+ beta*C)
      const O8 pr = *(const O8*)(preact + off);
      O8 c{};
      if (beta != 0.f) c = *(const O8*)(C + off);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float v = alpha * (j < 4 ? lo[j] : hi[j - 4]) * gelu_erf_grad(to_f(pr[j]));
        if (beta != 0.f) v += beta * to_f(c[j]);
        o[j] = from_f<OutT>(v);
      }
      *(O8*)(C + off) = o;
      return;
    }
    if (VEC_EPI && (bias || addend || preact || res || act != ACT_NONE)) {
      // the general form, in apply()'s order: alpha*acc + bias + addend -> preact copy ->
      // activation -> + beta*C
      float v[8];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        v[j] = alpha * lo[j];
        v[j + 4] = alpha * hi[j];
      }
      if (bias) {
        const f32x4 b0 = *(const f32x4*)(bias + n), b1 = *(const f32x4*)(bias + n + 4);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          v[j] += b0[j];
          v[j + 4] += b1[j];
        }
      }
      if (addend) {
        const f32x4 a0 = *(const f32x4*)(addend + off), a1 = *(const f32x4*)(addend + off + 4);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          v[j] += a0[j];
          v[j + 4] += a1[j];
        }
      }
      if (preact) {
        O8 pr;
#pragma unroll
        for (int j = 0; j < 8; ++j) pr[j] = from_f<OutT>(v[j]);
        *(O8*)(preact + off) = pr;
      }
      O8 c{}, rr{};
      if (beta != 0.f) c = *(const O8*)(C + off);
      if (res) rr = *(const O8*)(res + off);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float x = v[j];
        if (act == ACT_RELU) x = fmaxf(x, 0.f);
        else if (act == ACT_GELU) x = gelu_erf(x);
        if (beta != 0.f) x += beta * to_f(c[j]);
        if (res) x += to_f(rr[j]);
        o[j] = from_f<OutT>(x);
      }
    } else if (acc_src) {  // 8 columns = one mask byte (bf16) or two (fp32)
      // (accumulation sources are read for the last time here: nontemporal loads, C4 +0.3 %
      // over three paired runs, profiles/r06_nt_store_ab.txt)
      const O8 c = __builtin_nontemporal_load((const O8*)(acc_src + off));
      constexpr int VM = 16 / (int)sizeof(OutT);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const unsigned b = acc_mask[(long)m * (N / VM) + (n + j) / VM];
        const float a = (b >> ((n + j) % VM)) & 1u ? to_f(c[j]) : 0.f;
        o[j] = from_f<OutT>(alpha * (j < 4 ? lo[j] : hi[j - 4]) + a);
      }
    } else if (beta != 0.f) {
      const O8 c = __builtin_nontemporal_load((const O8*)(C + off));
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        o[j] = from_f<OutT>(alpha * lo[j] + beta * to_f(c[j]));
        o[j + 4] = from_f<OutT>(alpha * hi[j] + beta * to_f(c[j + 4]));
      }
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        o[j] = from_f<OutT>(alpha * lo[j]);
        o[j + 4] = from_f<OutT>(alpha * hi[j]);
      }
    }
    // nontemporal (streaming) 16-B stores: an output tile is written once and next read by
    // another launch, long after it would have left the L2; isolated C4 conv fwd / dgrad
    // families 2.31 / 2.17 -> 2.20 / 2.11 ms, C4 9318 / 9335 -> 9516 / 9515 samples/s paired
    // (profiles/r06_nt_store_ab.txt)
    __builtin_nontemporal_store(o, (O8*)(C + off));
  }
  // Per-column (mean, M2) of this BM-row tile straight from the MFMA accumulators: each lane
  // reduces its 4*RM rows of a column exactly (two passes in registers), the four lane groups
  // sharing a column merge by Chan's formula through xor-shuffles, and the WM waves of a
  // column merge in LDS (`red`, WM*BN*3 floats).  Same result layout as tile_stats.
  static constexpr bool REG_STATS = true;
  template <int BM, int BN, int WM, int WN, int RM, int RN>
  __device__ __forceinline__ void reg_stats(const f32x4 (&acc)[RM][RN], float* red, int tm,
                                            int tn, int wm, int wn, int lane) const {
    if (!stats) return;
    // a full tile (every block but the last row of tiles) takes the branch-free instance: all
    // counts are the same power of two, so the masks, the divisions and the count shuffles
    // fold to constants — the same float operations on the same values (bit-identical)
    if (M - tm * BM >= BM)
      reg_stats_t<BM, BN, WM, WN, RM, RN, true>(acc, red, tm, tn, wm, wn, lane);
    else
      reg_stats_t<BM, BN, WM, WN, RM, RN, false>(acc, red, tm, tn, wm, wn, lane);
  }
  template <int BM, int BN, int WM, int WN, int RM, int RN, bool FULL>
  __device__ __forceinline__ void reg_stats_t(const f32x4 (&acc)[RM][RN], float* red, int tm,
                                              int tn, int wm, int wn, int lane) const {
    constexpr int WTM = BM / WM, WTN = BN / WN;
    const int rows_valid = min(BM, M - tm * BM);
#pragma unroll
    for (int j = 0; j < RN; ++j) {
      float cnt = 0.f, s = 0.f;
#pragma unroll
      for (int i = 0; i < RM; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const bool ok = FULL || wm * WTM + i * 16 + (lane >> 4) * 4 + r < rows_valid;
          cnt += ok ? 1.f : 0.f;
          s += ok ? acc[i][j][r] : 0.f;
        }
      if constexpr (FULL) cnt = (float)(RM * 4);
      const float mean = cnt > 0.f ? s / cnt : 0.f;
      float m2 = 0.f;
#pragma unroll
      for (int i = 0; i < RM; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const bool ok = FULL || wm * WTM + i * 16 + (lane >> 4) * 4 + r < rows_valid;
          const float d = acc[i][j][r] - mean;
          m2 += ok ? d * d : 0.f;
        }
      float n_a = cnt, mu = mean, mm = m2;
#pragma unroll
      for (int x = 16; x <= 32; x <<= 1) {
        const float n_b = FULL ? n_a : __shfl_xor(n_a, x, 64);
        const float mu_b = __shfl_xor(mu, x, 64), mm_b = __shfl_xor(mm, x, 64);
        const float tot = n_a + n_b;
        const float d = mu_b - mu, f = FULL ? 0.5f : (tot > 0.f ? n_b / tot : 0.f);
        mu += d * f;
        mm += mm_b + d * d * n_a * f;
        n_a = tot;
      }
      if constexpr (WTM == 128 && BM > 128) {
        // a wave row spans exactly one 128-row slab (the layout every consumer expects):
        // it is stored as is, no merge across wave rows
        const int slab = tm * WM + wm, n = tn * BN + wn * WTN + j * 16 + lane;
        if (lane < 16 && n_a > 0.f && n < N)
          stats[(long)n * ((M + 127) / 128) + slab] = make_float2(mu, mm);
        continue;
      }
      if (lane < 16) {
        float* o = red + (wm * BN + wn * WTN + j * 16 + lane) * 3;
        o[0] = n_a; o[1] = mu; o[2] = mm;
      }
    }
    if constexpr (WTM == 128 && BM > 128) return;
    __syncthreads();
    // the wave rows of each statistics slab (128 rows; the whole tile when BM <= 128) merge
    constexpr int SLAB = BM > 128 ? 128 : BM, SLABS = BM / SLAB, WPS = WM / SLABS;
    static_assert(WM % SLABS == 0, "wave rows per statistics slab");
    const int col = threadIdx.x % BN, slab = threadIdx.x / BN;
    if (slab < SLABS && tn * BN + col < N) {
      float nn = 0.f, mu = 0.f, mm = 0.f;
#pragma unroll
      for (int qq = 0; qq < WPS; ++qq) {
        const float* o = red + ((slab * WPS + qq) * BN + col) * 3;
        const float nb = FULL ? (float)WTM : o[0], mb = o[1], m2b = o[2];
        if (nb == 0.f) continue;
        if (nn == 0.f) { nn = nb; mu = mb; mm = m2b; continue; }
        // full tiles: equal counts, f = nb / (qq + 1) nb exactly
        const float tot = nn + nb, d = mb - mu, f = FULL ? 1.f / (float)(qq + 1) : nb / tot;
        mu += d * f;
        mm += m2b + d * d * nn * f;
        nn = tot;
      }
      if (nn > 0.f || SLABS == 1)
        stats[(long)(tn * BN + col) * ((M + SLAB - 1) / SLAB) + tm * SLABS + slab] =
            make_float2(mu, mm);
    }
  }
  __device__ __forceinline__ void apply4(int m, int n, f32x4 v) const {
    if (m >= M) return;
    const long off = (long)m * ldc + n;
    const bool fast = n + 4 <= N && (off & 3) == 0 && !bias && !addend && !preact &&
                      act == ACT_NONE && !acc_src && !res;
    if (!fast) {
#pragma unroll
      for (int j = 0; j < 4; ++j) apply(m, n + j, v[j]);
      return;
    }
    typedef __attribute__((ext_vector_type(4))) OutT O4;
    O4 o;
    if (beta != 0.f) {
      const O4 c = *(const O4*)(C + off);
#pragma unroll
      for (int j = 0; j < 4; ++j) o[j] = from_f<OutT>(alpha * v[j] + beta * to_f(c[j]));
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) o[j] = from_f<OutT>(alpha * v[j]);
    }
    *(O4*)(C + off) = o;
  }
};

// Eval-mode BatchNorm folded into the producing conv (TP:206 / TP:1000 / IP:170: the
// backbone in eval mode normalises with running statistics, an affine map per channel):
// C = act(acc * scale[n] + shift[n] (+ res[m][n])), scale = gamma * rsqrt(var + eps),
// shift = beta - mean * scale, computed in the epilogue from the BN's own tensors (no fold
// kernel, no re-packed weights, fp32 math on the fp32 accumulators).  Replaces the conv
// store + bn_apply pass of the eval forward.
template <typename OutT>
struct EpiBnEval : EpiStore<OutT> {
  static constexpr bool BNSTAT = false;
  const float *gamma, *beta_bn, *rmean, *rvar;
  float eps;
  const OutT* res;  // residual [M][ldc] or null
  bool relu;
  __device__ __forceinline__ void coef(int n, float& sc, float& sh) const {
    sc = gamma[n] * rsqrtf(rvar[n] + eps);
    sh = beta_bn[n] - rmean[n] * sc;
  }
  __device__ __forceinline__ float fin(float v, int n, long off) const {
    float sc, sh;
    coef(n, sc, sh);
    v = v * sc + sh;
    if (res) v += to_f(res[off]);
    return relu ? fmaxf(v, 0.f) : v;
  }
  __device__ __forceinline__ bool vec8_ok() const {
    return this->ldc % 8 == 0 && ((uintptr_t)this->C & 15) == 0 && ((uintptr_t)res & 15) == 0;
  }
  __device__ __forceinline__ void apply4(int m, int n, f32x4 v) const {
    if (m >= this->M) return;
    const long off = (long)m * this->ldc + n;
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (n + j < this->N) this->C[off + j] = from_f<OutT>(fin(v[j], n + j, off + j));
  }
  __device__ __forceinline__ void apply8_fast(int m, int n, f32x4 lo, f32x4 hi) const {
    if (m >= this->M) return;
    if (n + 8 > this->N) {
      apply4(m, n, lo);
      if (n + 4 < this->N) apply4(m, n + 4, hi);
      return;
    }
    const long off = (long)m * this->ldc + n;
    typedef __attribute__((ext_vector_type(8))) OutT O8;
    O8 r{};
    if (res) r = *(const O8*)(res + off);
    O8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float sc, sh;
      coef(n + j, sc, sh);
      float v = (j < 4 ? lo[j] : hi[j - 4]) * sc + sh;
      if (res) v += to_f(r[j]);
      o[j] = from_f<OutT>(relu ? fmaxf(v, 0.f) : v);
    }
    *(O8*)(this->C + off) = o;
  }
};

// Raw fp32 partial for split-K: ws[z][M][N].
struct EpiPartial {
  float* ws; int M, N;
  int z = 0;   // this block's K split (set by the kernel from its (tile, split) decode)
  static constexpr bool SPLIT = true;
  __device__ __forceinline__ void apply(int m, int n, float v) const {
    if (m >= M || n >= N) return;
    ws[((long)z * M + m) * N + n] = v;
  }
  __device__ __forceinline__ void apply4(int m, int n, f32x4 v) const {
    if (m >= M) return;
    const long off = ((long)z * M + m) * N + n;
    if (n + 4 <= N && (off & 3) == 0) {
      *(f32x4*)(ws + off) = v;
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) apply(m, n + j, v[j]);
    }
  }
  template <int BM, int BN, int LDC>
  __device__ __forceinline__ void tile_stats(const float*, float*, int, int) const {}
  static constexpr bool REG_STATS = false;
  template <int BM, int BN, int WM, int WN, int RM, int RN>
  __device__ __forceinline__ void reg_stats(const f32x4 (&)[RM][RN], float*, int, int, int,
                                            int, int) const {}
  BnStat bs{};
  static constexpr bool BNSTAT = false;
  __device__ __forceinline__ long bn_off(int, int) const { return 0; }
  __device__ __forceinline__ bool vec8_ok() const { return N % 4 == 0; }
  __device__ __forceinline__ void apply8_fast(int m, int n, f32x4 lo, f32x4 hi) const {
    if (m >= M) return;
    const long off = ((long)z * M + m) * N + n;
    if (n + 4 <= N) *(f32x4*)(ws + off) = lo;
    if (n + 8 <= N) *(f32x4*)(ws + off + 4) = hi;
  }
};

// Phase-dgrad epilogue: GEMM row m = phase pixel (n, i, j) -> dX pixel (n, a+sh*i, b+sw*j);
// dX = acc + beta*dX (beta = 1 accumulates a residual branch's gradient).
template <typename OutT>
struct EpiPhase {
  OutT* C; int ldc, M, N; float beta;
  int Hp, Wp, H, W, a, b, sh, sw;
  BnStat bs{};
  static constexpr bool BNSTAT = true;
  static constexpr bool SPLIT = false;
  // merged-phase launch: phase p's rows, K depth, pixel grid, offset and statistics tiles
  static constexpr bool PHASED = true;
  int Ms[MAX_PHASES], Ks[MAX_PHASES], Hps[MAX_PHASES], Wps[MAX_PHASES], as[MAX_PHASES],
      bs_[MAX_PHASES], tile0s[MAX_PHASES];
  int Kp = 0;  // the selected phase's K depth
  __device__ void select_from(const EpiPhase& k, int p) {  // (see DgradPhaseK::select_from)
    M = k.Ms[p]; Kp = k.Ks[p]; Hp = k.Hps[p]; Wp = k.Wps[p]; a = k.as[p]; b = k.bs_[p];
    bs.tile0 = k.tile0s[p];
  }
  __device__ __forceinline__ long bn_off(int m, int n) const { return pix(m) * ldc + n; }
  __device__ __forceinline__ long pix(int m) const {
    const int hw = Hp * Wp;
    const int n = m / hw, rem = m - n * hw;
    const int i = rem / Wp, j = rem - i * Wp;
    return ((long)n * H + a + sh * i) * W + b + sw * j;
  }
  __device__ __forceinline__ void apply(int m, int n, float v) const {
    if (m >= M || n >= N) return;
    const long off = pix(m) * ldc + n;
    if (beta != 0.f) v += beta * to_f(C[off]);
    C[off] = from_f<OutT>(v);
  }
  __device__ __forceinline__ void apply4(int m, int n, f32x4 v) const {
    if (m >= M) return;
    if (n + 4 > N) {
#pragma unroll
      for (int j = 0; j < 4; ++j) apply(m, n + j, v[j]);
      return;
    }
    const long off = pix(m) * ldc + n;
    typedef __attribute__((ext_vector_type(4))) OutT O4;
    O4 o;
    if (beta != 0.f) {
      const O4 c = *(const O4*)(C + off);
#pragma unroll
      for (int j = 0; j < 4; ++j) o[j] = from_f<OutT>(v[j] + beta * to_f(c[j]));
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) o[j] = from_f<OutT>(v[j]);
    }
    *(O4*)(C + off) = o;
  }
  template <int BM, int BN, int LDC>
  __device__ __forceinline__ void tile_stats(const float*, float*, int, int) const {}
  static constexpr bool REG_STATS = false;
  template <int BM, int BN, int WM, int WN, int RM, int RN>
  __device__ __forceinline__ void reg_stats(const f32x4 (&)[RM][RN], float*, int, int, int,
                                            int, int) const {}
  __device__ __forceinline__ bool vec8_ok() const { return ldc % 8 == 0 && ((uintptr_t)C & 15) == 0; }
  __device__ __forceinline__ void apply8_fast(int m, int n, f32x4 lo, f32x4 hi) const {
    if (m >= M) return;
    if (n + 8 > N) {
      apply4(m, n, lo);
      if (n + 4 < N) apply4(m, n + 4, hi);
      return;
    }
    const long off = pix(m) * ldc + n;
    typedef __attribute__((ext_vector_type(8))) OutT O8;
    O8 o;
    if (beta != 0.f) {
      const O8 c = __builtin_nontemporal_load((const O8*)(C + off));
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        o[j] = from_f<OutT>(lo[j] + beta * to_f(c[j]));
        o[j + 4] = from_f<OutT>(hi[j] + beta * to_f(c[j + 4]));
      }
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        o[j] = from_f<OutT>(lo[j]);
        o[j + 4] = from_f<OutT>(hi[j]);
      }
    }
    *(O8*)(C + off) = o;
  }
};

// Bias gradient fused into a weight-gradient GEMM (A R-major = dY^T): the blocks of column
// tile 0 also multiply their A fragments by a ones operand (one extra MFMA per A fragment
// and 32-deep k step, waves of column group 0 only), which leaves the row sums of A — the
// column sums of dY over this K split — in a 16 x 16 accumulator per row tile; they are
// stored to bpart[z][M] and reduced over the splits by gemm_dense.hip.
struct EpiPartialBias : EpiPartial {
  float* bpart;   // [splits][M]
  static constexpr bool BIAS_SUM = true;
};
template <class E, class = void> struct HasBiasSum { static constexpr bool value = false; };
template <class E> struct HasBiasSum<E, decltype((void)E::BIAS_SUM)> {
  static constexpr bool value = E::BIAS_SUM;
};

template <class E, class = void> struct IsPhased { static constexpr bool value = false; };
template <class E> struct IsPhased<E, decltype((void)E::PHASED)> {
  static constexpr bool value = E::PHASED;
};

// Bijective XCD-aware remap: blocks that share an A panel land on one XCD's L2.
__device__ __forceinline__ int xcd_swizzle(int orig, int nwg) {
  const int q = nwg / 8, r = nwg % 8, xcd = orig % 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / 8;
}

// (tile, K split) of this block.  Split-K grids (the weight gradients): the whole
// (split, tile) space is ordered split-major and XCD-swizzled as one, so all the tiles of a K
// split run on one XCD — they read the same dY / im2col pixel range, which then comes from
// that XCD's L2 once instead of once per XCD.  Measured on the C4 weight gradients
// (tools/conv_bench.py, isolated): splits of 2-32 tiles 4-30 % faster (layer2 3x3 74 -> 55 us),
// 64-144 tiles neutral, the 36-tile layer3 3x3 14 % slower, so rounds 3-4 kept the per-slice
// swizzle above 32 tiles.  Round 5 measured the traffic (PMC): split-major everywhere cuts the
// 540-block layer3 3x3 weight gradient from 214 to 89 MB of HBM traffic per call and the conv
// family from 152.2 to 144.3 MB per launch, with the C4 step unchanged (8942 / 8955 vs
// 8950 / 8935 samples/s, paired) and the isolated wgrad total 2.40 vs 2.33 ms — the lower HBM
// load is what the concurrent dgrad / BN chain shares, so split-major is the default.
// Dense split-K GEMMs (both operands plain matrices: the nn.Linear weight gradients) always
// use the split-major order: a K split's tiles share its dY / X row range, and on one XCD they
// read it from that XCD's L2.  Measured at C5 (r05, PMC): the 288-block weight-gradient GEMMs
// 262.7 -> 163.1 MB of HBM traffic per call, 52.7 -> 43.7 GB per step for the GEMM family,
// 2850 / 2851 vs 2833 / 2834 samples/s paired; C4 neutral.
#ifndef MMDX_SPLIT_XCD_MAX_TILES
#define MMDX_SPLIT_XCD_MAX_TILES (1 << 30)
#endif
#ifndef MMDX_DENSE_SPLIT_XCD_MAX_TILES
#define MMDX_DENSE_SPLIT_XCD_MAX_TILES (1 << 30)
#endif
// (tm, tn) of a linear tile index.  Wide grids (more than G tile columns) walk bands of G tile
// rows column by column, so the tiles one XCD holds at once (its contiguous share of the
// swizzled order, ~64 at two blocks per CU) span ~G rows x 64/G columns: ~20 distinct A / B
// panels in its L2 instead of ~3 + every column panel of the row-major order.  Mapping only:
// every tile computes exactly what it did (MMDX_TILE_GROUP=1: row-major).  Measured at C5
// (r05, paired): G 4 2830 / 2835, G 8 2815 / 2822, row-major 2788 / 2801 samples/s; G 8 cut the
// GEMM family's HBM traffic 43.7 -> 37.7 GB per step (the 2376-block FFN dgrad 380 -> 300 MB
// per call); C4 within noise (its conv grids are at most 16 tiles wide).
#ifndef MMDX_TILE_GROUP
#define MMDX_TILE_GROUP 4
#endif
__device__ __forceinline__ void tile_coords(int tile, int tiles_m, int tiles_n, int& tm, int& tn) {
  constexpr int G = MMDX_TILE_GROUP;
  if (G <= 1 || tiles_n <= G || tiles_m <= 1) {
    tm = tile / tiles_n;
    tn = tile - tm * tiles_n;
    return;
  }
  const int band = tile / (G * tiles_n);
  const int r0 = band * G;
  const int gh = min(G, tiles_m - r0);
  const int i = tile - band * G * tiles_n;
  tm = r0 + i % gh;
  tn = i / gh;
}

template <bool DENSE = false>
__device__ __forceinline__ void block_tile(int nwg, int& tile, int& z) {
  constexpr int MAXT = DENSE ? MMDX_DENSE_SPLIT_XCD_MAX_TILES : MMDX_SPLIT_XCD_MAX_TILES;
  if (gridDim.z > 1 && nwg <= MAXT) {
    const int lg = xcd_swizzle((int)(blockIdx.z * gridDim.x + blockIdx.x), nwg * (int)gridDim.z);
    z = lg / nwg;
    tile = lg - z * nwg;
  } else {
    z = blockIdx.z;
    tile = xcd_swizzle(blockIdx.x, nwg);
  }
}

template <typename T, int BM, int BN, int WM, int WN, class LA, class LB, class Epi>
__global__ __launch_bounds__(NT, 2) void igemm_kernel(typename LA::SrcT sa, typename LB::SrcT sb,
                                                      Epi epi, int M, int N, int K, int kper) {
  constexpr int BK = KTile<T>::BK;
  constexpr int WTM = BM / WM, WTN = BN / WN;
  constexpr int RM = WTM / 16, RN = WTN / 16;
  constexpr int A_EL = LA::LDS_ELEMS, B_EL = LB::LDS_ELEMS;
  constexpr int OP_BYTES = 2 * (A_EL + B_EL) * (int)sizeof(T);
  constexpr int LDC = BN + 4;
  constexpr int EPI_BYTES = BM * LDC * 4 + NT * 3 * 4;  // staged tile + stats scratch
  constexpr int LDS_BYTES = OP_BYTES > EPI_BYTES ? OP_BYTES : EPI_BYTES;
  typedef MfmaOp<T> Op;
  __shared__ __attribute__((aligned(16))) char lds_raw[LDS_BYTES];
  T* const As = (T*)lds_raw;          // [2][A_EL]
  T* const Bs = As + 2 * A_EL;        // [2][B_EL]

  const int tiles_n = (N + BN - 1) / BN;
  const int tiles_m = (M + BM - 1) / BM;
  int tile, zsplit;
  block_tile(tiles_m * tiles_n, tile, zsplit);
  if constexpr (Epi::SPLIT) epi.z = zsplit;
  const int tm = tile / tiles_n, tn = tile - tm * tiles_n;
  const int kbeg = zsplit * kper;
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
  for (int t = 0; t < nt; ++t) {
    const int cur = t & 1;
    const bool more = t + 1 < nt;
    if (more) {
      la.fetch(sa, kbeg + (t + 1) * BK, kend, ra);
      lb.fetch(sb, kbeg + (t + 1) * BK, kend, rb);
    }
    const T* a_s = As + cur * A_EL;
    const T* b_s = Bs + cur * B_EL;
#pragma unroll
    for (int ks = 0; ks < BK; ks += Op::KS) {
      typename Op::frag_t af[RM], bfr[RN];
#pragma unroll
      for (int i = 0; i < RM; ++i) af[i] = LA::frag(a_s, wm * WTM + i * 16, ks);
#pragma unroll
      for (int j = 0; j < RN; ++j) bfr[j] = LB::frag(b_s, wn * WTN + j * 16, ks);
#pragma unroll
      for (int i = 0; i < RM; ++i)
#pragma unroll
        for (int j = 0; j < RN; ++j) acc[i][j] = Op::mma(af[i], bfr[j], acc[i][j]);
    }
    if (more) {
      la.store(As + (cur ^ 1) * A_EL, ra);
      lb.store(Bs + (cur ^ 1) * B_EL, rb);
    }
    __syncthreads();
  }

  // Epilogue: C/D map of 16x16 MFMA (col = lane&15, row = (lane>>4)*4 + reg) -> fp32 LDS
  // tile [BM][BN+4] -> 4 consecutive columns per lane per store.
  float* cst = (float*)lds_raw;
#pragma unroll
  for (int i = 0; i < RM; ++i)
#pragma unroll
    for (int j = 0; j < RN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        cst[(wm * WTM + i * 16 + (lane >> 4) * 4 + r) * LDC + wn * WTN + j * 16 + (lane & 15)] =
            acc[i][j][r];
  __syncthreads();
  epi.template tile_stats<BM, BN, LDC>(cst, cst + BM * LDC, tm, tn);
  constexpr int C4 = BN / 4;
  for (int c = threadIdx.x; c < BM * C4; c += NT) {
    const int row = c / C4, col = (c - row * C4) * 4;
    const f32x4 v = *(const f32x4*)(cst + row * LDC + col);
    epi.apply4(tm * BM + row, tn * BN + col, v);
  }
}

// --------------------------------------------------------------------------------------
// LDS-DMA variant (bf16, both operands k-major, whole 64-deep K tiles): global_load_lds
// moves each 16-B chunk straight into LDS, so no staging registers and no ds_write pass.
// LDS image per operand and stage: [ROWS][64] bf16, 128-B rows, logical chunk c of row r at
// slot c ^ (r & 7) — conflict-free for the ds_read_b128 fragment reads.  Wave instruction j
// of wave w fills rows (4j + w)*8 .. +7 (1 KiB, lane-linear); each lane fetches the chunk
// that belongs at its slot (zeros through a zero line for padding / out-of-range rows).
// Two stages, one raw barrier per K tile: wait for this wave's DMAs of tile t, barrier,
// issue tile t+1 into the other stage, compute tile t.
// --------------------------------------------------------------------------------------
// Every DMA goes through a raw buffer resource over the operand tensor: a lane whose chunk is
// padding / out of range gets voffset = DMA_OOB, and the range check makes the hardware write
// zeros into LDS (verified on gfx950: tools/lab/oob_lds.hip).  Per K tile a lane's cost is
// one tap-validity bit test, an add and a select.
constexpr unsigned DMA_OOB = 0x80000000u;  // operand tensors are < 2 GiB (host-checked)

__device__ __forceinline__ __amdgpu_buffer_rsrc_t dma_rsrc(const void* base, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, (int)bytes, 0x00020000);
}

__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t rsrc, char* lds, unsigned voff) {
  typedef __attribute__((address_space(3))) void lds_void;
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (lds_void*)lds, 16, voff, 0, 0, 0);
}

// BK = 64: rows of 128 B (8 chunks), slot = chunk ^ (row & 7), an instruction fills 8 rows.
// BK = 32: rows of 64 B (4 chunks), slot = chunk ^ ((row >> 1) & 3) (conflict-free for the
// ds_read_b128 lane groups of a 16-row x 4-chunk fragment read), an instruction fills 16 rows.
template <int ROWS, class Src, int BK_ = 64, int NWV = NT / 64>
struct DmaK {
  static constexpr int BK = BK_;
  static constexpr bool RMAJOR = false;
  static constexpr int NW = NWV;                     // waves of the block
  static constexpr int CPR = BK / 8;                 // 16-B chunks per row
  static constexpr int RPI = 64 / CPR;               // rows per DMA instruction (1 KiB)
  static constexpr int INSTR = ROWS / (RPI * NW);    // DMAs per wave per stage
  static constexpr int BYTES = ROWS * BK * 2;
  static_assert(BK == 64 || BK == 32, "K tile depth");
  static_assert(ROWS % (RPI * NW) == 0, "rows per wave");
  typedef Src SrcT;
  typedef typename Src::Mask Mask;
  __amdgpu_buffer_rsrc_t rsrc;
  int off[INSTR];       // byte offset of this lane's chunk at tap 0
  Mask mask[INSTR];     // valid taps of the row
  int coff;             // element offset of this lane's logical chunk within the K tile
  // uniform K-tile iterator: the K tiles are issued in order, so the tile's filter tap is
  // stepped (k = (tu * tT + tv) * tC + tc0) instead of divided out of k0 every tile
  int tc0, tv, tu, tC, tT;
  __device__ static int swz(int row) { return BK == 64 ? (row & 7) : ((row >> 1) & 3); }
  __device__ void init(const Src& s, int row0, int lane, int wid, int kbeg) {
    const int rr = lane / CPR, slot = lane % CPR;
    coff = (slot ^ swz(rr)) * 8;  // instructions start at a multiple of RPI rows
    if constexpr (!Src::LANE_TAP) {
      s.tdims(tC, tT);
      const int tap = kbeg / tC;
      tc0 = kbeg - tap * tC;
      tu = tap / tT;
      tv = tap - tu * tT;
    }
    rsrc = dma_rsrc(s.bbase(), s.bbytes());
#pragma unroll
    for (int j = 0; j < INSTR; ++j)  // LANE_TAP sources fold the chunk offset into toff
      off[j] = s.brow(row0 + (j * NW + wid) * RPI + rr, mask[j]) + (Src::LANE_TAP ? 0 : coff * 2);
  }
  // called once per K tile, in order (k0 = kbeg, kbeg + BK, ...)
  __device__ void issue(const Src& s, char* stage, int k0, int klim, int wid) {
    const bool kok = k0 + coff < klim;
    if constexpr (Src::LANE_TAP) {  // this lane's chunk has its own tap
      int toff, r, sx;
      s.lane_decode(k0 + coff, toff, r, sx);
#pragma unroll
      for (int j = 0; j < INSTR; ++j) {
        const bool ok = kok && s.lane_ok(mask[j], r, sx);
        dma16(rsrc, stage + (j * NW + wid) * 1024, ok ? (unsigned)(off[j] + toff) : DMA_OOB);
      }
      return;
    }
    int toff, tap;
    s.tmap(tu, tv, tc0, toff, tap);  // one tap for the whole K tile (uniform)
    tc0 += BK;                       // C % BK == 0 (FAST sources): a tap ends on a tile edge
    if (tc0 >= tC) {
      tc0 = 0;
      if (++tv == tT) { tv = 0; ++tu; }
    }
#pragma unroll
    for (int j = 0; j < INSTR; ++j) {
      const bool ok = kok && ((mask[j] >> tap) & 1u);
      dma16(rsrc, stage + (j * NW + wid) * 1024, ok ? (unsigned)(off[j] + toff) : DMA_OOB);
    }
  }
  __device__ static bf16x8 frag(const char* stage, int r16, int ks, int lane) {
    const int row = r16 + (lane & 15);
    const int c = (ks >> 3) + (lane >> 4);
    return *(const bf16x8*)(stage + row * (BK * 2) + ((c ^ swz(row)) << 4));
  }
};

// R-major operand (rows contiguous in global: dY^T / im2col^T of the wgrad GEMM): LDS image
// [64 k][ROWS] bf16, one ROWS*2-byte line per k; a DMA instruction fills 1 KiB = KPI whole
// k-lines.  Chunk slots are XOR-swizzled per k so the ds_read_b64_tr_b16 fragment reads (8
// k-lines x 32 B per 32-lane group) hit every bank once.
template <int ROWS, class Src, int BK_ = 64, int NWV = NT / 64>
struct DmaR {
  static constexpr int BK = BK_;
  static constexpr bool RMAJOR = true;
  template <class S, class = void> struct AnyStep { static constexpr bool value = false; };
  template <class S> struct AnyStep<S, decltype((void)S::STEP_ANY)> {
    static constexpr bool value = S::STEP_ANY;
  };
  static_assert(!Src::STEP || BK == 64 || AnyStep<Src>::value,
                "lane stepping advances one 64-deep K tile");
  static constexpr int NW = NWV;
  static constexpr int CPR = ROWS / 8;          // 16-B chunks per k-line
  static constexpr int KPI = 64 / CPR;          // k-lines per DMA instruction
  static constexpr int INSTR = BK / (KPI * NW); // DMAs per wave per stage
  static constexpr int BYTES = BK * ROWS * 2;
  // ROWS = 256: two LDS bank rows per k-line; the swizzle only permutes the low 4 chunk
  // bits, so a fragment read's 16 chunk slots stay distinct mod 16 as for 128
  static_assert(ROWS == 64 || ROWS == 128 || ROWS == 256, "R-major DMA tile rows");
  static_assert(BK == 64 || BK == 32, "K tile depth");
  typedef Src SrcT;
  __amdgpu_buffer_rsrc_t rsrc;
  typename Src::RowState rs[INSTR];
  typename Src::Lane ln[INSTR];  // per-lane pixel state of stepping sources (im2col^T)
  int kr[INSTR];
  __device__ static int sw(int k) {
    return ROWS >= 128 ? 2 * ((k & 3) | (((k >> 3) & 1) << 2))
                       : 2 * (((k >> 1) & 1) | (((k >> 3) & 1) << 1));
  }
  __device__ void init(const Src& s, int row0, int lane, int wid, int kbeg) {
    const int slot = lane % CPR;
    rsrc = dma_rsrc(s.bbase(), s.bbytes());
#pragma unroll
    for (int j = 0; j < INSTR; ++j) {
      kr[j] = (j * NW + wid) * KPI + lane / CPR;
      rs[j] = s.row(row0 + (slot ^ sw(kr[j])) * 8);
      if constexpr (Src::STEP) ln[j] = s.lane_at(kbeg + kr[j]);
    }
  }
  // called once per K tile, in order (k0 = kbeg, kbeg + 64, ...)
  __device__ void issue(const Src& s, char* stage, int k0, int klim, int wid) {
    if (k0 + BK <= klim)  // uniform: every k-line of the tile is inside the split
      issue_t<false>(s, stage, k0, klim, wid);
    else
      issue_t<true>(s, stage, k0, klim, wid);
  }
  template <bool CHECK_K>
  __device__ void issue_t(const Src& s, char* stage, int k0, int klim, int wid) {
#pragma unroll
    for (int j = 0; j < INSTR; ++j) {
      const int o = s.template roff_at<CHECK_K>(rs[j], ln[j], k0 + kr[j], klim);
      dma16(rsrc, stage + (j * NW + wid) * 1024, o >= 0 ? (unsigned)o : DMA_OOB);
      if constexpr (Src::STEP) {
        if constexpr (BK == 64) s.lane_step(ln[j]);
        else s.lane_step_by(ln[j], BK);
      }
    }
  }
  // lane 4q+p of 16-lane group g reads k-line ks+8g+q (and +4), columns r16+4p..+3, and gets
  // column (lane & 15) of those 4 lines: 8 consecutive k, as the MFMA operand wants
  __device__ static bf16x8 frag(const char* stage, int r16, int ks, int lane) {
    const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
    const int k = ks + 8 * g + q;
    const int col = r16 + 4 * p;
    const int o = (((col >> 3) ^ sw(k)) << 4) + ((col >> 2) & 1) * 8;
    typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
    const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (lds_s16x4*)(stage + k * (ROWS * 2) + o));
    const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (lds_s16x4*)(stage + (k + 4) * (ROWS * 2) + o));
    return __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
  }
};

// R-major operand in a row-QUARTERED LDS image (BK = 64): the tile's ROWS rows are kept as
// QN = ROWS / 32 sub-images [64 k][32 rows] (64-B k-lines, 4 KiB each).  Wave w's instruction
// j fills k-lines 16w .. 16w+15 of quarter j (1 KiB, lane-linear: lane L -> k-line 16w + L/4,
// 16-B slot L % 4), so a lane serves ONE k-line (one pixel of the im2col^T operand) in all
// of its QN instructions: one pixel state per lane, stepped once per K tile, instead of DmaR's
// QN independent k-lines per lane (the im2col^T stepping and bounds tests were ~60 of the ~110
// VALU per K tile of the 3x3 weight-gradient loop, ~5 VALU per MFMA: PMC r05).
// When the tile's rows lie in one filter tap (C % ROWS == 0) the quarters share the pixel's
// validity and their offsets differ by 32 rows: one bounds test per lane per K tile.
// Slot swizzle: physical slot = logical ^ 2*((k >> 3) & 1), so the two 16-lane groups of a
// ds_read_b64_tr_b16 half-wave (k-lines k..k+3 and k+8..k+11, 32 B each) cover all 64 banks.
template <int ROWS, class Src>
struct DmaRq {
  static constexpr int BK = 64;
  static constexpr bool RMAJOR = true;
  static constexpr int NW = NT / 64;
  static constexpr int QN = ROWS / 32;           // quarters (32-row sub-images)
  static constexpr int INSTR = QN;               // DMAs per wave per stage (one per quarter)
  static constexpr int BYTES = BK * ROWS * 2;
  static_assert(ROWS == 64 || ROWS == 128, "quartered R-major tile rows");
  static_assert(NW == 4, "16 k-lines per wave");
  static_assert(Src::STEP, "lane-stepping source");
  typedef Src SrcT;
  __amdgpu_buffer_rsrc_t rsrc;
  typename Src::RowState rs[QN];
  typename Src::Lane ln;
  int kk;        // this lane's k-line within the K tile
  bool same;     // every quarter in the pixel's one tap: one bounds test (block-uniform)
  __device__ static int swq(int k) { return ((k >> 3) & 1) << 1; }
  __device__ void init(const Src& s, int row0, int lane, int wid, int kbeg) {
    rsrc = dma_rsrc(s.bbase(), s.bbytes());
    kk = wid * 16 + (lane >> 2);
    const int lc = (lane & 3) ^ swq(kk);          // logical 16-B chunk this lane fetches
#pragma unroll
    for (int j = 0; j < QN; ++j) rs[j] = s.row(row0 + 32 * j + lc * 8);
    ln = s.lane_at(kbeg + kk);
    same = s.rows_one_tap(ROWS);
  }
  __device__ void issue(const Src& s, char* stage, int k0, int klim, int wid) {
    if (k0 + BK <= klim)
      issue_t<false>(s, stage, k0, klim, wid);
    else
      issue_t<true>(s, stage, k0, klim, wid);
  }
  template <bool CHECK_K>
  __device__ void issue_t(const Src& s, char* stage, int k0, int klim, int wid) {
    char* dst = stage + wid * 1024;
    if (same) {
      const int o = s.template roff_at<CHECK_K>(rs[0], ln, k0 + kk, klim);
#pragma unroll
      for (int j = 0; j < QN; ++j)
        dma16(rsrc, dst + j * 4096, o >= 0 ? (unsigned)(o + j * 32 * (int)sizeof(bf16)) : DMA_OOB);
    } else {
#pragma unroll
      for (int j = 0; j < QN; ++j) {
        const int o = s.template roff_at<CHECK_K>(rs[j], ln, k0 + kk, klim);
        dma16(rsrc, dst + j * 4096, o >= 0 ? (unsigned)o : DMA_OOB);
      }
    }
    s.lane_step(ln);
  }
  // as DmaR::frag: lane 4q+p of 16-lane group g reads k-line ks+8g+q (and +4), columns
  // r16+4p..+3 (8 B inside one 16-B slot of quarter r16/32)
  __device__ static bf16x8 frag(const char* stage, int r16, int ks, int lane) {
    const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
    const int k = ks + 8 * g + q;
    const int col = r16 + 4 * p;
    const int cq = col & 31;
    const char* base = stage + (col >> 5) * 4096 + ((col >> 2) & 1) * 8;
    typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
    const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (lds_s16x4*)(base + k * 64 + (((cq >> 3) ^ swq(k)) << 4)));
    const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (lds_s16x4*)(base + (k + 4) * 64 + (((cq >> 3) ^ swq(k + 4)) << 4)));
    return __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
  }
};

// Stores a staged fp32 tile cst [BM][LDC] (CW columns) at output (m0, n0): 8 consecutive
// columns per lane -> one 16-B store where the epilogue allows it, else 4-column pieces.
template <int BM, int CW, int LDC, int NTH, class Epi>
__device__ __forceinline__ void epilogue_pass(const Epi& epi, const float* cst, int m0, int n0) {
  if (epi.vec8_ok()) {
    constexpr int C8 = CW / 8;
    static_assert(NTH % C8 == 0, "vec8 epilogue geometry");
    const int col = (threadIdx.x % C8) * 8;
#pragma unroll 2
    for (int c = threadIdx.x; c < BM * C8; c += NTH) {
      const int row = c / C8;
      const f32x4 lo = *(const f32x4*)(cst + row * LDC + col);
      const f32x4 hi = *(const f32x4*)(cst + row * LDC + col + 4);
      epi.apply8_fast(m0 + row, n0 + col, lo, hi);
    }
  } else {
    constexpr int C4 = CW / 4;
    for (int c = threadIdx.x; c < BM * C4; c += NTH) {
      const int row = c / C4, col = (c - row * C4) * 4;
      const f32x4 v = *(const f32x4*)(cst + row * LDC + col);
      epi.apply4(m0 + row, n0 + col, v);
    }
  }
}

// NS operand stages (2..5) of BK = OA::BK (64 or 32): NS - 1 K tiles are in flight while one
// is consumed (counted vmcnt).  NS = 3 at BK 64 where the grid leaves one block per CU anyway;
// BK 32 x NS 4-5 keeps two blocks per CU with twice the bytes in flight of BK 64 x NS 2.
// Epilogue: BatchNorm tile statistics straight from the accumulators (reg_stats), fp32
// staging through LDS, then 8 consecutive columns per lane -> one 16-B bf16 store.
// NTH = 512 (8 waves, one block per CU, 256 x 128 tiles, WM x WN = 4 x 2 waves of 64 x 64):
// half the operand bytes per MFMA of two 128 x 128 blocks and twice the K tiles in flight
// (NS = 3 stages of 48 KB) for the same LDS.
template <int BM, int BN, class OA, class OB, class Epi, int NS = 2, typename ET = bf16,
          int NTH = NT, int WM = 2, int WN = 2>
__global__ __launch_bounds__(NTH, 2) void igemm_dma_kernel(typename OA::SrcT sa_k,
                                                           typename OB::SrcT sb_k, Epi epi_k,
                                                           int M, int N, int K, int kper) {
  constexpr int BK = OA::BK;
  // working copies: the kernel arguments themselves are never written, so the merged-phase
  // selection below reads their per-phase arrays straight from the kernarg segment (a
  // by-value argument that is written is copied to scratch, and its phase arrays indexed
  // there: 208 B of scratch per lane in the phase dgrads before round 6)
  typename OA::SrcT sa = sa_k;
  typename OB::SrcT sb = sb_k;
  Epi epi = epi_k;
  static_assert(WM * WN * 64 == NTH && OA::NW * 64 == NTH && OB::NW * 64 == NTH, "waves");
  // fragments-first K loop (below): measured on the C4 conv shapes, 5-13 % faster for the
  // R-major (weight-gradient) operands and most 128-wide tiles, mixed on the 128x64 k-major
  // tiles (three blocks per CU there already cover the LDS latency)
  // (not at 128 x 64 per wave: the two K steps' fragments would not fit in 256 VGPRs)
  constexpr bool FRAG_FIRST = BN == 128 || (OA::RMAJOR && BN < 256);
  static_assert(OB::BK == BK, "operand K tile depths differ");
  constexpr int WTM = BM / WM, WTN = BN / WN;
  constexpr int RM = WTM / 16, RN = WTN / 16;
  constexpr int STAGE = OA::BYTES + OB::BYTES;
  constexpr int OP_BYTES = NS * STAGE;
  constexpr int RED = WM * 3 > (NTH / 64) * 2 ? WM * 3 : (NTH / 64) * 2;  // floats per column
  // the fp32 tile is staged through LDS in NCH column passes: two for 256 x 256 tiles, whose
  // full staging (266 KB) exceeds the CU's 160 KB
  constexpr int NCH = BM * (BN + 4) * 4 + RED * BN * 4 > 160 * 1024 ? 2 : 1;
  constexpr int CH = BN / NCH;  // staged columns per pass
  static_assert(NCH == 1 || (WN % NCH == 0 && (BN / WN) * (WN / NCH) == CH),
                "a staging pass holds whole wave columns");
  constexpr int LDC = CH + 4;
  constexpr int EPI_BYTES = BM * LDC * 4 + RED * BN * 4;  // staged tile + reduction scratch
  constexpr int LDS_BYTES = OP_BYTES > EPI_BYTES ? OP_BYTES : EPI_BYTES;
  // DMA instructions one wave issues per K tile (both operands)
  constexpr int PER_TILE = OA::INSTR + OB::INSTR;
  static_assert(NS >= 2 && NS <= 5 && PER_TILE * (NS - 2) <= 63, "stages");
  __shared__ __attribute__((aligned(1024))) char lds_raw[LDS_BYTES];  // the only LDS object

  int tile, zsplit;
  if constexpr (IsPhased<Epi>::value) {
    // merged strided-dgrad phases: blockIdx.z is this block's phase (not a K split)
    const int ph = blockIdx.z;
    sa.select_from(sa_k, ph);
    sb.select_from(sb_k, ph);
    epi.select_from(epi_k, ph);
    M = epi.M;
    K = kper = epi.Kp;
    const int nwg = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
    if ((int)blockIdx.x >= nwg) return;  // a phase with fewer tiles than the grid's x extent
    tile = xcd_swizzle(blockIdx.x, nwg);
    zsplit = 0;
  } else {
    block_tile<IsDenseSrc<typename OA::SrcT>::value && IsDenseSrc<typename OB::SrcT>::value>(
        ((M + BM - 1) / BM) * ((N + BN - 1) / BN), tile, zsplit);
  }
  const int tiles_n = (N + BN - 1) / BN;
  if constexpr (Epi::SPLIT) epi.z = zsplit;
  int tm, tn;
  tile_coords(tile, (M + BM - 1) / BM, tiles_n, tm, tn);
  const int kbeg = zsplit * kper;
  const int kend = min(K, kbeg + kper);
  const int nt = kend > kbeg ? (kend - kbeg + BK - 1) / BK : 0;
  // wave index as a scalar: the LDS-DMA destinations (M0) and fragment bases become SALU math
  const int lane = threadIdx.x & 63,
            wid = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const int wm = wid / WN, wn = wid % WN;

  OA oa;
  OB ob;
  oa.init(sa, tm * BM, lane, wid, kbeg);
  ob.init(sb, tn * BN, lane, wid, kbeg);

  f32x4 acc[RM][RN];
#pragma unroll
  for (int i = 0; i < RM; ++i)
#pragma unroll
    for (int j = 0; j < RN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // fused bias gradient (EpiPartialBias): row sums of A in the column-tile-0 blocks
  constexpr bool BSUM = HasBiasSum<Epi>::value;
  static_assert(!BSUM || FRAG_FIRST, "bias sums ride the fragments-first K loop");
  const bool bias_blk = BSUM && tn == 0 && wn == 0;   // wave-uniform
  f32x4 bsum[BSUM ? RM : 1];
#pragma unroll
  for (int i = 0; i < (BSUM ? RM : 1); ++i) bsum[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 ones8;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    if constexpr (std::is_same<ET, f16>::value)
      ones8[e] = __builtin_bit_cast(bf16, (f16)1.0f);
    else
      ones8[e] = (bf16)1.0f;
  }

#pragma unroll
  for (int t = 0; t < NS - 1; ++t) {
    if (t < nt) {
      char* st = lds_raw + t * STAGE;
      oa.issue(sa, st, kbeg + t * BK, kend, wid);
      ob.issue(sb, st + OA::BYTES, kbeg + t * BK, kend, wid);
    }
  }
  for (int t = 0; t < nt; ++t) {
    // wait for this wave's DMAs of tile t (tiles t+1 .. t+NS-2 may stay in flight)
    const int ahead = min(NS - 2, nt - 1 - t);
    if (NS >= 5 && ahead >= 3)
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(3 * PER_TILE) : "memory");
    else if (NS >= 4 && ahead == 2)
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * PER_TILE) : "memory");
    else if (NS >= 3 && ahead == 1)
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PER_TILE) : "memory");
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    const char* as = lds_raw + (t % NS) * STAGE;
    const char* bs = as + OA::BYTES;
    auto afrag = [&](int i, int ks) { return OA::frag(as, wm * WTM + i * 16, ks, lane); };
    if constexpr (FRAG_FIRST) {
      // every fragment of the tile is requested before the next tile's DMAs are issued, so
      // the LDS read latency runs under the DMA issue instead of in front of the MFMAs
      constexpr int KS = BK / 32;
      bf16x8 af[KS][RM], bfr[KS][RN];
#pragma unroll
      for (int s = 0; s < KS; ++s) {
#pragma unroll
        for (int i = 0; i < RM; ++i) af[s][i] = afrag(i, s * 32);
#pragma unroll
        for (int j = 0; j < RN; ++j) bfr[s][j] = OB::frag(bs, wn * WTN + j * 16, s * 32, lane);
      }
      if (t + NS - 1 < nt) {
        char* st = lds_raw + ((t + NS - 1) % NS) * STAGE;
        oa.issue(sa, st, kbeg + (t + NS - 1) * BK, kend, wid);
        ob.issue(sb, st + OA::BYTES, kbeg + (t + NS - 1) * BK, kend, wid);
      }
#pragma unroll
      for (int s = 0; s < KS; ++s)
#pragma unroll
        for (int i = 0; i < RM; ++i)
#pragma unroll
          for (int j = 0; j < RN; ++j) {
            if constexpr (std::is_same<ET, f16>::value)
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(
                  __builtin_bit_cast(f16x8, af[s][i]), __builtin_bit_cast(f16x8, bfr[s][j]),
                  acc[i][j], 0, 0, 0);
            else
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[s][i], bfr[s][j],
                                                                   acc[i][j], 0, 0, 0);
          }
      if constexpr (BSUM) {
        if (bias_blk) {
#pragma unroll
          for (int s = 0; s < KS; ++s)
#pragma unroll
            for (int i = 0; i < RM; ++i) {
              if constexpr (std::is_same<ET, f16>::value)
                bsum[i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(
                    __builtin_bit_cast(f16x8, af[s][i]), __builtin_bit_cast(f16x8, ones8),
                    bsum[i], 0, 0, 0);
              else
                bsum[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[s][i], ones8, bsum[i], 0,
                                                                   0, 0);
            }
        }
      }
      continue;
    }
    if (t + NS - 1 < nt) {  // its stage was consumed in iteration t-1 by every wave
      char* st = lds_raw + ((t + NS - 1) % NS) * STAGE;
      oa.issue(sa, st, kbeg + (t + NS - 1) * BK, kend, wid);
      ob.issue(sb, st + OA::BYTES, kbeg + (t + NS - 1) * BK, kend, wid);
    }
#pragma unroll
    for (int ks = 0; ks < BK; ks += 32) {
      bf16x8 af[RM], bfr[RN];
#pragma unroll
      for (int i = 0; i < RM; ++i) af[i] = afrag(i, ks);
#pragma unroll
      for (int j = 0; j < RN; ++j) bfr[j] = OB::frag(bs, wn * WTN + j * 16, ks, lane);
#pragma unroll
      for (int i = 0; i < RM; ++i)
#pragma unroll
        for (int j = 0; j < RN; ++j) {
          // the LDS-DMA path moves 16-bit elements; the MFMA reads them as ET
          if constexpr (std::is_same<ET, f16>::value)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(
                __builtin_bit_cast(f16x8, af[i]), __builtin_bit_cast(f16x8, bfr[j]), acc[i][j],
                0, 0, 0);
          else
            acc[i][j] =
                __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
        }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if constexpr (BSUM) {
    // every column of a bsum tile holds the row sums: lanes 0, 16, 32, 48 store rows
    // (lane >> 4) * 4 + r of each row tile
    if (bias_blk && (lane & 15) == 0) {
#pragma unroll
      for (int i = 0; i < RM; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = tm * BM + wm * WTM + i * 16 + (lane >> 4) * 4 + r;
          if (m < M) epi.bpart[(long)zsplit * M + m] = bsum[i][r];
        }
    }
  }

  float* cst = (float*)lds_raw;
  float* red = cst + BM * LDC;
  if constexpr (NCH == 1) {
    // fused consumer-BN backward statistics: the BN input y of this thread's output chunks
    // is loaded now, so its latency overlaps the accumulator staging below
    constexpr int C8 = BN / 8, ITERS = BM * C8 / NTH;
    static_assert(NTH % C8 == 0 && (BM * C8) % NTH == 0, "vec8 epilogue geometry");
    const bool bst = Epi::BNSTAT && epi.bs.part != nullptr && epi.vec8_ok();
    bn_y8 yv[ITERS], ov[ITERS];
    if (bst) {
      const int n = tn * BN + (threadIdx.x % C8) * 8;
#pragma unroll
      for (int it = 0; it < ITERS; ++it) {
        const int m = tm * BM + (threadIdx.x + it * NTH) / C8;
        const bool in = m < M && n < N;
        yv[it] = in ? *(const bn_y8*)((const bf16*)epi.bs.y + epi.bn_off(m, n)) : bn_y8{};
        ov[it] = in && epi.bs.out ? *(const bn_y8*)((const bf16*)epi.bs.out + epi.bn_off(m, n))
                                  : bn_y8{};
      }
    }
    if constexpr (Epi::REG_STATS)
      epi.template reg_stats<BM, BN, WM, WN, RM, RN>(acc, red, tm, tn, wm, wn, lane);
#pragma unroll
    for (int i = 0; i < RM; ++i)
#pragma unroll
      for (int j = 0; j < RN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          cst[(wm * WTM + i * 16 + (lane >> 4) * 4 + r) * LDC + wn * WTN + j * 16 +
              (lane & 15)] = acc[i][j][r];
    __syncthreads();
    if constexpr (!Epi::REG_STATS) epi.template tile_stats<BM, BN, LDC>(cst, red, tm, tn);
    if (bst) {  // vec8 stores + the statistics of every stored chunk (rows >= M excluded)
      const int col = (threadIdx.x % C8) * 8;
      BnCoef8 bc;
      float sg[8], sgx[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) sg[j] = sgx[j] = 0.f;
      bn_coef8(epi.bs, tn * BN + col, N, bc);
#pragma unroll
      for (int it = 0; it < ITERS; ++it) {
        const int row = (threadIdx.x + it * NTH) / C8;
        f32x4 lo = *(const f32x4*)(cst + row * LDC + col);
        f32x4 hi = *(const f32x4*)(cst + row * LDC + col + 4);
        const int m = tm * BM + row, n = tn * BN + col;
        bst_accum8(epi, m, n, lo, hi);
        bst_store8(epi, m, n, lo, hi);
        if (m < M && n < N) bn_acc8<bf16>(yv[it], ov[it], lo, hi, epi.bs, bc, sg, sgx);
      }
      bn_stat_store<BN, NTH / 64, (BM > 128 ? BM / 128 : 1)>(epi.bs, sg, sgx, red, tm, tn, N, M);
      return;
    }
  } else {
    // column passes (256 x 256 tiles): the waves whose columns fall in pass h stage them; the
    // epilogues used here take their statistics from the registers (REG_STATS) or keep none
    // (EpiPartial, EpiPhase), and the fused consumer-BN path is not instantiated
    if constexpr (Epi::REG_STATS)
      epi.template reg_stats<BM, BN, WM, WN, RM, RN>(acc, red, tm, tn, wm, wn, lane);
#pragma unroll
    for (int h = 0; h < NCH; ++h) {
      if (h > 0) __syncthreads();  // the previous pass's readers are done with cst
      if ((wn * WTN) / CH == h) {
#pragma unroll
        for (int i = 0; i < RM; ++i)
#pragma unroll
          for (int j = 0; j < RN; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r)
              cst[(wm * WTM + i * 16 + (lane >> 4) * 4 + r) * LDC + wn * WTN - h * CH +
                  j * 16 + (lane & 15)] = acc[i][j][r];
      }
      __syncthreads();
      epilogue_pass<BM, CH, LDC, NTH>(epi, cst, tm * BM, tn * BN + h * CH);
    }
    return;
  }
  epilogue_pass<BM, CH, LDC, NTH>(epi, cst, tm * BM, tn * BN);
}

// Loader bundles (give the kernel template one type per operand).
template <typename T, int ROWS, class Src>
struct KLoad : KMajorLoader<T, ROWS, KTile<T>::BK, Src> {};
template <typename T, int ROWS, class Src>
struct RLoad : RMajorLoader<T, ROWS, KTile<T>::BK, Src> {};

}  // namespace mmdx
