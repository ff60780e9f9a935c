// Bidirectional LSTM recurrence (build-defined C3/C4 text tower, nn.LSTM semantics).
//
// The recurrence couples time steps only within one batch row, so the grid is
// (direction x batch slices of 16 rows): every workgroup runs its rows through all L
// steps with no inter-workgroup synchronisation.  Per step the gate pre-activations
// G[16][4H] = xg[t] + h_{t-1} W_hh^T come from MFMA (h in LDS, W_hh streamed from L2),
// the cell update runs from an fp32 LDS image of G.  Input projections (x W_ih^T + b) for
// all steps are one large GEMM outside this kernel; so are dW_ih, dX and the bias grads.
#include <algorithm>
#include <atomic>

#include "igemm.h"
#include "../../include/mmdx.h"

namespace mmdx {

constexpr int LSTM_RB = 16;   // batch rows per workgroup
constexpr int LSTM_NW = 8;    // waves per workgroup

__device__ __forceinline__ float sigm(float x) { return 1.f / (1.f + __expf(-x)); }
// The bf16 recurrences' gate functions: v_exp + v_rcp (1 ulp each) instead of an IEEE divide
// and the libm tanh, whose VALU sequences made the cell update 3.7 of a 9.9 us step (probe,
// tools/lab/lstm_probe.py).  Absolute error <= ~1e-7, far below the bf16 rounding of h.
__device__ __forceinline__ float sigm_fast(float x) {
  return __builtin_amdgcn_rcpf(1.f + __expf(-x));
}
__device__ __forceinline__ float tanh_fast(float x) {
  return 1.f - 2.f * __builtin_amdgcn_rcpf(1.f + __expf(2.f * x));
}

// acc[j] += A[16 rows][K] (LDS, row base a_row = &A[lane&15][(lane>>4)*FRAG]) x B fragments
//           streamed from global (L2-resident weights): this lane's fragment of tile j at
//           k-step ks is at b + j*TS + ks*KSTR.  Row-major Bg^T (rows = output columns):
//           b = &Bg[col0 + lane&15][(lane>>4)*FRAG], TS = 16*ldb, KSTR = KS.  Fragment-packed
//           (lstm_pack_whh_kernel): TS = (K/KS)*64*FRAG, KSTR = 64*FRAG — one contiguous 1 KiB
//           per wave instruction.
// The weight stream is software-pipelined D k-steps deep (D*TILES fragments in flight).
// Short contractions are unrolled completely, so every fragment's wait is an exact vmcnt
// (a rolled loop with the refill under a branch compiled to vmcnt(0) at each iteration:
// one full L2 round trip per D k-steps instead of a full pipeline).
template <typename T, int TILES, int K, int D>
__device__ __forceinline__ void rowblock_mfma(const T* a_row, const T* b_row, long ts, int kstr,
                                              f32x4* acc) {
  typedef MfmaOp<T> Op;
  constexpr int NKS = K / Op::KS;
  static_assert(NKS % D == 0, "pipeline depth must divide the k-steps");
  typename Op::frag_t buf[D][TILES];
#pragma unroll
  for (int d = 0; d < D; ++d)
#pragma unroll
    for (int j = 0; j < TILES; ++j) buf[d][j] = Op::ld(b_row + (long)j * ts + d * kstr);
  auto kstep = [&](int ks, int d) {
    const typename Op::frag_t af = Op::ld(a_row + ks * Op::KS);
#pragma unroll
    for (int j = 0; j < TILES; ++j) acc[j] = Op::mma(af, buf[d][j], acc[j]);
    if (ks + D < NKS) {
#pragma unroll
      for (int j = 0; j < TILES; ++j)
        buf[d][j] = Op::ld(b_row + (long)j * ts + (ks + D) * kstr);
    }
    // keep the refill at this k-step: the scheduler otherwise sinks it next to its use and
    // the pipeline collapses to ~2 k-steps in flight
    __builtin_amdgcn_sched_barrier(0);
  };
  if constexpr (NKS <= 64) {
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) kstep(ks, ks % D);
  } else {
#pragma unroll 1
    for (int g = 0; g < NKS; g += D) {
#pragma unroll
      for (int d = 0; d < D; ++d) kstep(g + d, d);
    }
  }
}

template <typename T, int H> struct LstmDepth;
template <> struct LstmDepth<bf16, 256> { static constexpr int F = 2, B = 8; };
template <> struct LstmDepth<bf16, 128> { static constexpr int F = 4, B = 8; };
template <> struct LstmDepth<float, 256> { static constexpr int F = 8, B = 16; };
template <> struct LstmDepth<float, 128> { static constexpr int F = 8, B = 16; };

template <typename T, int H>
__global__ __launch_bounds__(LSTM_NW * 64) void lstm_fwd_kernel(
    const float* __restrict__ xg, const T* __restrict__ whh, int B, int L,
    T* __restrict__ hout, float* __restrict__ csave, float* __restrict__ gsave) {
  typedef MfmaOp<T> Op;
  constexpr int G4 = 4 * H;
  constexpr int LDH = H + Vec16<T>::N;
  constexpr int TILES = G4 / (LSTM_NW * 16);  // 16-col tiles per wave
  constexpr int CPT = LSTM_RB * H / (LSTM_NW * 64);
  __shared__ float sg[LSTM_RB * G4];
  __shared__ __attribute__((aligned(16))) T sh[LSTM_RB * LDH];
  const int dir = blockIdx.y;
  const int b0 = blockIdx.x * LSTM_RB;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const T* W = whh + (long)dir * G4 * H;
  for (int i = threadIdx.x; i < LSTM_RB * LDH; i += blockDim.x) sh[i] = from_f<T>(0.f);
  float creg[CPT];
#pragma unroll
  for (int i = 0; i < CPT; ++i) creg[i] = 0.f;
  __syncthreads();
  const int col0 = wid * TILES * 16;
  const T* a_row = sh + (lane & 15) * LDH + (lane >> 4) * Op::FRAG;
  const T* b_row = W + (long)(col0 + (lane & 15)) * H + (lane >> 4) * Op::FRAG;
  for (int s = 0; s < L; ++s) {
    const int t = dir == 0 ? s : L - 1 - s;
    f32x4 acc[TILES];
#pragma unroll
    for (int j = 0; j < TILES; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
    // the weight operand is re-streamed every step: an opaque zero offset keeps the compiler
    // from hoisting W_hh's fragments out of the step loop (they do not fit in VGPRs); an
    // offset, not the pointer, so the loads stay global (not flat) loads
    int zero = 0;
    asm volatile("" : "+s"(zero));
    rowblock_mfma<T, TILES, H, LstmDepth<T, H>::F>(a_row, b_row + zero, 16L * H, Op::KS, acc);
#pragma unroll
    for (int j = 0; j < TILES; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = (lane >> 4) * 4 + r, col = col0 + j * 16 + (lane & 15);
        const int b = b0 + row;
        float v = acc[j][r];
        // xg is unit-interleaved: gate g of unit u at column u * 4 + g
        if (b < B) v += xg[(((long)b * L + t) * 2 + dir) * G4 + (col % H) * 4 + col / H];
        sg[row * G4 + col] = v;
      }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < CPT; ++i) {
      const int e = threadIdx.x + i * LSTM_NW * 64;
      const int row = e / H, u = e - row * H;
      const int b = b0 + row;
      constexpr bool fast = sizeof(T) == 2;
      const float gi = fast ? sigm_fast(sg[row * G4 + u]) : sigm(sg[row * G4 + u]);
      const float gf = fast ? sigm_fast(sg[row * G4 + H + u]) : sigm(sg[row * G4 + H + u]);
      const float gg = fast ? tanh_fast(sg[row * G4 + 2 * H + u]) : tanhf(sg[row * G4 + 2 * H + u]);
      const float go = fast ? sigm_fast(sg[row * G4 + 3 * H + u]) : sigm(sg[row * G4 + 3 * H + u]);
      const float c = gf * creg[i] + gi * gg;
      creg[i] = c;
      const float h = go * (fast ? tanh_fast(c) : tanhf(c));
      sh[row * LDH + u] = from_f<T>(h);
      if (b < B) {
        hout[((long)b * L + t) * 2 * H + dir * H + u] = from_f<T>(h);
        const long sidx = (((long)dir * L + t) * B + b);
        csave[sidx * H + u] = c;
        // gates saved interleaved per unit ([2][L][B][H][4]): one 16-B store / load each
        *(f32x4*)(gsave + (sidx * H + u) * 4) = f32x4{gi, gf, gg, go};
      }
    }
    __syncthreads();
  }
}

// Recurrent backward.  dG (pre-activation gate grads) -> dxg [B][L][2][4H] (T) and the
// shifted hidden states hprev [2][B*L][H] (T) for the dW_hh GEMM.  whp: W_hh in the
// fragment-packed layout of lstm_pack_whh_kernel.
template <typename T, int H>
__global__ __launch_bounds__(LSTM_NW * 64) void lstm_bwd_kernel(
    const T* __restrict__ whp, const T* __restrict__ hout, const float* __restrict__ csave,
    const float* __restrict__ gsave, const T* __restrict__ dhout, int B, int L,
    T* __restrict__ dxg, T* __restrict__ hprev) {
  typedef MfmaOp<T> Op;
  constexpr int G4 = 4 * H;
  constexpr int LDG = G4 + Vec16<T>::N;
  constexpr int TILES = H / (LSTM_NW * 16);
  constexpr int CPT = LSTM_RB * H / (LSTM_NW * 64);
  __shared__ __attribute__((aligned(16))) T sdg[LSTM_RB * LDG];
  __shared__ float sdh[LSTM_RB * H];
  const int dir = blockIdx.y;
  const int b0 = blockIdx.x * LSTM_RB;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  constexpr int NKS = G4 / Op::KS;           // k-steps of the dh contraction
  float dcn[CPT];
#pragma unroll
  for (int i = 0; i < CPT; ++i) dcn[i] = 0.f;
  for (int i = threadIdx.x; i < LSTM_RB * H; i += blockDim.x) sdh[i] = 0.f;
  __syncthreads();
  const int col0 = wid * TILES * 16;
  const T* a_row = sdg + (lane & 15) * LDG + (lane >> 4) * Op::FRAG;
  constexpr long TS = (long)NKS * 64 * Op::FRAG;  // one 16-column tile, all k-steps
  const T* b_row = whp + ((long)dir * (H / 16) + col0 / 16) * TS + lane * Op::FRAG;
  for (int s = L - 1; s >= 0; --s) {
    const int t = dir == 0 ? s : L - 1 - s;
    const int tp = dir == 0 ? t - 1 : t + 1;  // previous step in forward order
    const bool has_prev = s > 0;
    // every global operand of this step's CPT elements is requested first (rows past B read
    // row B-1 and are discarded), then the cell math, then the stores: one memory round trip
    // per step instead of two per element
    float gv[CPT][4], cv[CPT], cpv[CPT], dhv[CPT];
    T hpv[CPT];
#pragma unroll
    for (int i = 0; i < CPT; ++i) {
      const int e = threadIdx.x + i * LSTM_NW * 64;
      const int row = e / H, u = e - row * H;
      const int b = min(b0 + row, B - 1);
      const long sidx = ((long)dir * L + t) * B + b;
      const f32x4 g4 = *(const f32x4*)(gsave + (sidx * H + u) * 4);
#pragma unroll
      for (int g = 0; g < 4; ++g) gv[i][g] = g4[g];
      cv[i] = csave[sidx * H + u];
      dhv[i] = to_f(dhout[((long)b * L + t) * 2 * H + dir * H + u]);
      if (has_prev) {
        cpv[i] = csave[(((long)dir * L + tp) * B + b) * H + u];
        hpv[i] = hout[((long)b * L + tp) * 2 * H + dir * H + u];
      } else {
        cpv[i] = 0.f;
        hpv[i] = from_f<T>(0.f);
      }
    }
#pragma unroll
    for (int i = 0; i < CPT; ++i) {
      const int e = threadIdx.x + i * LSTM_NW * 64;
      const int row = e / H, u = e - row * H;
      const int b = b0 + row;
      float dgi = 0.f, dgf = 0.f, dgg = 0.f, dgo = 0.f;
      if (b < B) {
        const float gi = gv[i][0], gf = gv[i][1], gg = gv[i][2], go = gv[i][3];
        const float c = cv[i];
        const float dh = dhv[i] + sdh[row * H + u];
        const float tc = sizeof(T) == 2 ? tanh_fast(c) : tanhf(c);
        const float dc = dh * go * (1.f - tc * tc) + dcn[i];
        const float d_o = dh * tc;
        dgi = dc * gg * gi * (1.f - gi);
        dgf = dc * cpv[i] * gf * (1.f - gf);
        dgg = dc * gi * (1.f - gg * gg);
        dgo = d_o * go * (1.f - go);
        dcn[i] = dc * gf;
        T* dp = dxg + (((long)b * L + t) * 2 + dir) * G4;
        dp[u] = from_f<T>(dgi);
        dp[H + u] = from_f<T>(dgf);
        dp[2 * H + u] = from_f<T>(dgg);
        dp[3 * H + u] = from_f<T>(dgo);
        hprev[((long)dir * B * L + (long)b * L + t) * H + u] = hpv[i];
      }
      sdg[row * LDG + u] = from_f<T>(dgi);
      sdg[row * LDG + H + u] = from_f<T>(dgf);
      sdg[row * LDG + 2 * H + u] = from_f<T>(dgg);
      sdg[row * LDG + 3 * H + u] = from_f<T>(dgo);
    }
    __syncthreads();
    // dh_next[16][H] = dG[16][4H] . W_hh  (B operand = W_hh^T rows, K-major)
    f32x4 acc[TILES];
#pragma unroll
    for (int j = 0; j < TILES; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
    int zero = 0;  // (see lstm_fwd_kernel: no hoisting of W_hh^T's fragments)
    asm volatile("" : "+s"(zero));
    rowblock_mfma<T, TILES, G4, LstmDepth<T, H>::B>(a_row, b_row + zero, TS, 64 * Op::FRAG,
                                                    acc);
    __syncthreads();
#pragma unroll
    for (int j = 0; j < TILES; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        sdh[((lane >> 4) * 4 + r) * H + col0 + j * 16 + (lane & 15)] = acc[j][r];
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------------------
// Cooperative forward (bf16, H = 256): per direction a group of COOP_NB workgroups, each
// owning COOP_UB hidden units (their i, f, g, o rows of W_hh = 128 x 256 bf16, held in
// REGISTERS for all L steps) and every batch row.  Per step a workgroup loads h_{t-1}
// (B x 256) into LDS, computes its 128 gate columns with MFMA, does the cell update in
// registers (each lane holds i, f, g, o of the same (row, unit) in the same accumulator
// slot) and publishes its h_t slice for the other workgroups of its direction.
// The h exchange is a write-through hand-off (cdna_hip_programming.md §6 Guideline 16, R1):
// the slice goes out as 16-B `sc1` stores, every wave drains them, then ONE agent atomic add
// signals; a consumer polls that counter and reads h with `sc1` loads (L1 bypassed), so no
// L2 writeback / L1 invalidate fence sits on the recurrence's critical path — the release
// fence alone cost 1.7-6.5 us per step with the image tower's dirty lines in the same L2.
// The step's xg operands are loaded before the wait, the c / gate / h saves for the
// backward are issued after the signal.  Outputs use the batch-partitioned kernel's layouts.
// ---------------------------------------------------------------------------------------
constexpr int COOP_NB = 8;                 // workgroups per direction
constexpr int COOP_H = 256;
constexpr int COOP_UB = COOP_H / COOP_NB;  // 32 units per workgroup
constexpr int COOP_LDH = COOP_H + 8;       // padded h row (bf16): conflict-free b128 reads
constexpr int COOP_SC1 = 16;               // buffer instruction aux: sc1 (write-through / L1 bypass)
constexpr long COOP_SPIN_MAX = 1L << 26;   // default bounded wait (~2 s): a lost peer ends the kernel
constexpr int COOP_DEBUG_DROP_PEER = 1;    // debug flag: workgroup 0 of direction 0 never signals
constexpr int COOP_DEBUG_TIMING = 2;       // debug flag: per-step phase timestamps (lab probe)
constexpr int COOP_TS_PHASES = 8;          // timestamps per (workgroup, step)

typedef unsigned coop_v4u __attribute__((ext_vector_type(4)));

// RT = 16-row tiles per wave (RT = 1: B <= 64; RT = 2: 128-row groups, grid z): 8 waves =
// 2 unit groups x 4 row groups.  The workgroup's W_hh slice (128 gate columns x 256, 64 KB)
// lives in LDS in fragment order (one contiguous 1 KiB per wave read): held in registers
// (128 VGPRs per lane) the B = 128 kernel needed 275 registers and spilled 19 to scratch
// inside the step loop, and a 256-row workgroup spilled 121.
constexpr int COOP_WLDS_BYTES = 2 * 4 * (COOP_H / 32) * 64 * 16;  // [ug][g][ks][lane] x 16 B

// Zeroes the cooperative recurrence's step counters ahead of its launch.  A kernel rather than
// hipMemsetAsync: the launch sequence captured into a hipGraph is then kernel nodes only,
// ordered on the stream like any other launch.
__global__ void lstm_coop_ctr_zero_kernel(unsigned* __restrict__ ctr, int n) {
  if ((int)threadIdx.x < n) ctr[threadIdx.x] = 0u;
}

template <int RT>
__global__ __launch_bounds__(512, 1) void lstm_fwd_coop_kernel(
    const float* __restrict__ xg, const bf16* __restrict__ whh, int B, int L,
    bf16* __restrict__ hout, float* __restrict__ csave, float* __restrict__ gsave,
    bf16* __restrict__ hx, unsigned* __restrict__ ctr, int* __restrict__ status, long spin_max,
    int debug, unsigned long long* __restrict__ tst) {
  constexpr int H = COOP_H, G4 = 4 * H, KS = H / 32;
  constexpr int NROWS = 64 * RT;
  static_assert(RT == 1 || RT == 2, "row tiles per wave");
  constexpr int WB = COOP_WLDS_BYTES / 2;  // bf16 elements of the W_hh image
  // [0, WB): the W_hh fragments; then h_{t-1} [NROWS][COOP_LDH] (MFMA A operand); then
  // this workgroup's h_t slice [NROWS][32]; then one int: the poller's verdict
  __shared__ __attribute__((aligned(16))) bf16 sh_all[WB + NROWS * COOP_LDH + NROWS * COOP_UB + 8];
  bf16* sh = sh_all + WB;
  bf16* sout = sh + NROWS * COOP_LDH;
  int* sgiveup = (int*)(sout + NROWS * COOP_UB);
  // the recurrence is the text tower's latency-critical chain and shares its CUs with the
  // image tower's conv blocks: its waves take issue priority over them
  __builtin_amdgcn_s_setprio(3);
  const int dir = blockIdx.y, blk = blockIdx.x;
  // blockIdx.z: this group's NROWS batch rows (B > 128 runs as independent 128-row groups of
  // COOP_NB workgroups: the recurrence of a row needs only its own row's hidden state)
  const int rb0 = blockIdx.z * NROWS;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int ug = wid & 1, rg = wid >> 1;
  const int u0 = blk * COOP_UB + ug * 16;   // this wave's 16 units
  const int ucol = u0 + (lane & 15);        // this lane's unit (accumulator column)
  // W fragments: gate g, unit u0 + (lane & 15), k = ks*32 + 8*(lane >> 4) .. +7
  const bf16* W = whh + (long)dir * G4 * H;
  // fragment (g, ks) of unit group ug at sh_all[(((ug * 4 + g) * KS + ks) * 64 + lane) * 8]:
  // gate g, unit blk * 32 + ug * 16 + (lane & 15), k = ks*32 + 8*(lane >> 4) .. +7; wave w
  // copies unit group (w & 1)'s fragments g * KS + ks = w >> 1, + 4, ...
  for (int f = wid >> 1; f < 4 * KS; f += 4) {
    const int g = f / KS, ks = f - g * KS;
    *(bf16x8*)(sh_all + ((((wid & 1) * 4 + g) * KS + ks) * 64 + lane) * 8) =
        *(const bf16x8*)(W + (long)(g * H + blk * COOP_UB + (wid & 1) * 16 + (lane & 15)) * H +
                         ks * 32 + 8 * (lane >> 4));
  }
  __syncthreads();
  const bf16* wl = sh_all + ((ug * 4) * KS * 64 + lane) * 8;  // this wave's fragment base
  float creg[RT][4];
#pragma unroll
  for (int i = 0; i < RT; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) creg[i][r] = 0.f;
  unsigned* myctr = ctr + dir * gridDim.z + blockIdx.z;
  bf16* hxd = hx + (long)dir * 2 * B * H;
  const __amdgpu_buffer_rsrc_t hrs =
      __builtin_amdgcn_make_buffer_rsrc((void*)hxd, (short)0, 2 * B * H * 2, 0x00020000);
  // lab probe (COOP_DEBUG_TIMING): thread 0 stamps the 100 MHz realtime clock at the phase
  // boundaries of every step, [group][dir][blk][step][phase]
  unsigned long long* tsw =
      tst ? tst + ((long)(blockIdx.z * 2 + dir) * COOP_NB + blk) * L * COOP_TS_PHASES : nullptr;
#define COOP_STAMP(k)                                                                       \
  do {                                                                                      \
    if (tsw && threadIdx.x == 0) tsw[s * COOP_TS_PHASES + (k)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
  // The input-projection operands of step s+1 and the backward's saves of step s-1 are issued
  // while step s's gates run: issued right after the publish (as before round 5) they sat in
  // front of the next wait's counter poll in thread 0's memory queue, so the last workgroup to
  // publish also saw the counter last (4.4 us behind its peers) and stayed last every step
  // (probe: tools/lab/lstm_probe.py).  Only the poll and the h loads touch memory between a
  // publish and the next step's gates.
#define COOP_LOAD_XV(XV, TT)                                                                 \
  do {                                                                                       \
    _Pragma("unroll") for (int i = 0; i < RT; ++i)                                            \
    _Pragma("unroll") for (int r = 0; r < 4; ++r) {                                           \
      const int b = rb0 + (rg + 4 * i) * 16 + (lane >> 4) * 4 + r;                           \
      const f32x4 x4 = *(const f32x4*)(xg + ((((long)min(b, B - 1) * L + (TT)) * 2 + dir) * H + ucol) * 4); \
      _Pragma("unroll") for (int g = 0; g < 4; ++g) XV[i][r][g] = x4[g];                      \
    }                                                                                        \
  } while (0)
  float xv[RT][4][4];
  COOP_LOAD_XV(xv, dir == 0 ? 0 : L - 1);
  float hv[RT][4], cv[RT][4], gv[RT][4][4];   // step s-1's outputs, saved during step s
  int tprev = 0;
  auto save = [&](int tt) {
#pragma unroll
    for (int i = 0; i < RT; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int b = rb0 + (rg + 4 * i) * 16 + (lane >> 4) * 4 + r;
        if (b >= B) continue;
        hout[((long)b * L + tt) * 2 * H + dir * H + ucol] = from_f<bf16>(hv[i][r]);
        const long sidx = ((long)dir * L + tt) * B + b;
        csave[sidx * H + ucol] = cv[i][r];
        *(f32x4*)(gsave + (sidx * H + ucol) * 4) =
            f32x4{gv[i][r][0], gv[i][r][1], gv[i][r][2], gv[i][r][3]};
      }
  };
  for (int s = 0; s < L; ++s) {
    const int t = dir == 0 ? s : L - 1 - s;
    COOP_STAMP(0);
    // wait until every workgroup of this direction has published h_{t-1}.  The wait is
    // bounded: a peer that never arrives (not co-resident, lost) makes the waiter set the
    // sticky status word and every workgroup leave, so the grid always drains; the host
    // reads the status word and raises (bilstm.py, mmdx_lstm_fwd's contract).
    if (s > 0) {
      if (threadIdx.x == 0) {
        const unsigned target = (unsigned)(COOP_NB * s);
        long spins = 0;
        int giveup = 0;
        while (__hip_atomic_load(myctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
          __builtin_amdgcn_s_sleep(1);
          ++spins;
          if (spins > spin_max) {
            __hip_atomic_store(status, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            giveup = 1;
            break;
          }
          // another workgroup already gave up: stop waiting for it
          if ((spins & 255) == 0 &&
              __hip_atomic_load(status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) {
            giveup = 1;
            break;
          }
        }
        *sgiveup = giveup;  // through LDS: no second memory round trip on the chain
      }
      __syncthreads();
      if (*sgiveup) return;
    }
    COOP_STAMP(1);
    // h_{t-1} -> LDS (zeros at the first step); sc1 loads: the producers' sc1 stores are
    // visible to them without an L1 invalidate
    // All of a thread's chunks are requested before any is written to LDS: one memory round
    // trip per batch of COOP_HB loads instead of one per chunk (a predicated load-then-store
    // loop compiles to a vmcnt(0) wait per chunk).  Rows >= B read out of the buffer's range
    // and come back as zeros.
    // Thread t moves rows (t >> 5) + 16 i, chunk t & 31: one base offset, the rest constants
    // (so nothing per chunk is kept live across steps).
    constexpr int HCH = NROWS * (H / 8) / 512;     // 16-B chunks per thread
    constexpr int HB = HCH < 8 ? HCH : 8;
    const int hrow = threadIdx.x >> 5;
    bf16* hdst = sh + hrow * COOP_LDH + (threadIdx.x & 31) * 8;
    if (s > 0) {
      const unsigned hsrc = (unsigned)(((s + 1) & 1) * B * H * 2 +  // the h_{t-1} buffer
                                       ((rb0 + hrow) * H + (threadIdx.x & 31) * 8) * 2);
#pragma unroll
      for (int i0 = 0; i0 < HCH; i0 += HB) {
        coop_v4u v[HB];
#pragma unroll
        for (int i = 0; i < HB; ++i)
          v[i] = __builtin_amdgcn_raw_buffer_load_b128(
              hrs, rb0 + hrow + 16 * (i0 + i) < B ? hsrc + (i0 + i) * 16 * H * 2 : DMA_OOB, 0,
              COOP_SC1);
#pragma unroll
        for (int i = 0; i < HB; ++i) *(coop_v4u*)(hdst + (i0 + i) * 16 * COOP_LDH) = v[i];
      }
    } else {
#pragma unroll
      for (int i = 0; i < HCH; ++i) *(coop_v4u*)(hdst + i * 16 * COOP_LDH) = coop_v4u{0u, 0u, 0u, 0u};
    }
    __syncthreads();
    COOP_STAMP(2);
    if (s > 0) save(tprev);
    float xn[RT][4][4];
    if (s + 1 < L) COOP_LOAD_XV(xn, dir == 0 ? s + 1 : L - 2 - s);
    COOP_STAMP(3);
    // every W fragment is read from LDS once per step, for all of the wave's row tiles
    constexpr int IB = RT;
#pragma unroll
    for (int i0 = 0; i0 < RT; i0 += IB) {
      f32x4 accs[IB][4];
#pragma unroll
      for (int ii = 0; ii < IB; ++ii)
#pragma unroll
        for (int g = 0; g < 4; ++g) accs[ii][g] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        bf16x8 w4[4];
#pragma unroll
        for (int g = 0; g < 4; ++g) w4[g] = *(const bf16x8*)(wl + (g * KS + ks) * 64 * 8);
#pragma unroll
        for (int ii = 0; ii < IB; ++ii) {
          const bf16x8 af = *(const bf16x8*)(sh + ((rg + 4 * (i0 + ii)) * 16 + (lane & 15)) *
                                                       COOP_LDH + 8 * (lane >> 4) + ks * 32);
#pragma unroll
          for (int g = 0; g < 4; ++g)
            accs[ii][g] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, w4[g], accs[ii][g], 0, 0, 0);
        }
      }
#pragma unroll
      for (int ii = 0; ii < IB; ++ii) {
        const int i = i0 + ii;
        const int rt16 = (rg + 4 * i) * 16;  // this row tile's first row
        const f32x4* acc = accs[ii];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float gi = sigm_fast(acc[0][r] + xv[i][r][0]);
          const float gf = sigm_fast(acc[1][r] + xv[i][r][1]);
          const float gg = tanh_fast(acc[2][r] + xv[i][r][2]);
          const float go = sigm_fast(acc[3][r] + xv[i][r][3]);
          const float c = gf * creg[i][r] + gi * gg;
          creg[i][r] = c;
          const bf16 h = from_f<bf16>(go * tanh_fast(c));
          hv[i][r] = (float)h;
          cv[i][r] = c;
          gv[i][r][0] = gi; gv[i][r][1] = gf; gv[i][r][2] = gg; gv[i][r][3] = go;
          const int row = rt16 + (lane >> 4) * 4 + r;
          sout[row * COOP_UB + ug * 16 + (lane & 15)] = h;
        }
      }
    }
    __syncthreads();
    COOP_STAMP(4);
    // publish h_t: 16-B sc1 stores of the [B][32] slice, drain, one agent atomic add (the
    // drain also covers the saves and operand loads issued above, long since complete)
    if (s + 1 < L) {
      const int par_out = (s & 1) * B * H * 2;
      const int nrow = min(NROWS, B - rb0);
      for (int e = threadIdx.x; e < nrow * (COOP_UB / 8); e += 512) {
        const int row = e / (COOP_UB / 8), c8 = e - row * (COOP_UB / 8);
        const coop_v4u v = *(const coop_v4u*)(sout + row * COOP_UB + c8 * 8);
        __builtin_amdgcn_raw_buffer_store_b128(
            v, hrs, par_out + ((rb0 + row) * H + blk * COOP_UB + c8 * 8) * 2, 0, COOP_SC1);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (threadIdx.x == 0 && !((debug & COOP_DEBUG_DROP_PEER) && blk == 0 && dir == 0))
        __hip_atomic_fetch_add(myctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    COOP_STAMP(5);
#pragma unroll
    for (int i = 0; i < RT; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int g = 0; g < 4; ++g) xv[i][r][g] = xn[i][r][g];
    tprev = t;
  }
  save(tprev);   // the last step's outputs
#undef COOP_LOAD_XV
#undef COOP_STAMP
}

// (The 4-wave register-W_hh variant of this forward, MMDX_LSTM_FWD_COOP4, was retired in
// round 6: 1.10 vs 0.81 ms per launch isolated, tools/lab/RETIRED.md.)

// W_hh [2][4H][H] -> the backward's B-operand fragments, [2][H/16][4H/KS][64 lanes][FRAG]:
// lane l of k-step ks of column tile c holds W_hh[ks*KS + (l>>4)*FRAG + e][16c + (l&15)],
// so every streaming load of the recurrence is one contiguous 1 KiB per wave.
template <typename T>
__global__ void lstm_pack_whh_kernel(const T* __restrict__ w, int H, T* __restrict__ wp) {
  typedef MfmaOp<T> Op;
  const int G4 = 4 * H, nks = G4 / Op::KS;
  const long total = 2L * G4 * H;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total;
       i += (long)gridDim.x * blockDim.x) {
    const int e = (int)(i % Op::FRAG);
    long r = i / Op::FRAG;
    const int l = (int)(r % 64);
    r /= 64;
    const int ks = (int)(r % nks);
    r /= nks;
    const int c = (int)(r % (H / 16)), d = (int)(r / (H / 16));
    const int u = 16 * c + (l & 15), j = ks * Op::KS + (l >> 4) * Op::FRAG + e;
    wp[i] = w[((long)d * G4 + j) * H + u];
  }
}

// ---------------------------------------------------------------------------------------
// Cooperative recurrent backward (bf16, H = 256).  The batch-partitioned lstm_bwd_kernel
// streams all of W_hh (512 KB) from L2 into every workgroup at every step (7.9 us per step,
// L2-bound).  Here a group of CB_NU workgroups shares each 16-row block of one direction: a
// workgroup owns CB_UB hidden units, holds its W_hh^T columns in REGISTERS for all L steps
// (wave w: one 16-unit tile, 32 k-step fragments = 128 VGPRs; one wave per SIMD) and per step
//   1. forms dG for (16 rows, its units, 4 gates) elementwise in the MFMA accumulator layout
//      (lane: rows 4*(lane>>4) + r, unit lane & 15) from dh_out + its own dh_next,
//   2. writes its dG slice into the step's A image in LDS and publishes it (16-B sc1 stores,
//      drained, one agent counter add: cdna_hip_programming.md §6 G16) next to the plain
//      dxg stores of the same chunks,
//   3. waits for its peers' slices (sc1 loads into the A image) and
//   4. runs dh_next[16][its units] = dG[16][4H] . W_hh[4H][its units] on MFMA.
// The arithmetic is the batch-partitioned kernel's: the same bf16 dG A operand, the same packed
// B fragments, the same k order, so the outputs are bit-identical (tests/test_text_gpu.py).
// The A image is 16 rows x 1024 bf16 with the 16-B chunk index XORed with the row (row < 16:
// conflict-free fragment reads without padding).  The exchange buffer is double-buffered by
// step parity; a slot is rewritten two steps later, after every peer has published the step
// in between (which it does only after reading this one).  Bounded wait like the forward's.
// ---------------------------------------------------------------------------------------
constexpr int CB_RB = 16;                   // batch rows per group
constexpr int CB_NU = 4;                    // workgroups per (row block, direction)
constexpr int CB_NT = 256;                  // threads: 4 waves, one 16-unit tile each
constexpr int CB_UB = COOP_H / CB_NU;       // units per workgroup (4 waves x 16)
constexpr int CB_G4 = 4 * COOP_H;
constexpr int CB_NKS = CB_G4 / 32;          // k-steps of the dh contraction
constexpr int CB_MAX_GROUPS = 32;           // row blocks per direction (B <= 512)

__device__ __forceinline__ int cb_swz(int row, int col) {  // bf16 element offset in the A image
  return row * CB_G4 + ((((col >> 3) ^ row) << 3) | (col & 7));
}

__global__ __launch_bounds__(CB_NT, 1) void lstm_bwd_coop_kernel(
    const bf16* __restrict__ whp, const bf16* __restrict__ hout, const float* __restrict__ csave,
    const float* __restrict__ gsave, const bf16* __restrict__ dhout, int B, int L,
    bf16* __restrict__ dxg, bf16* __restrict__ hprev, bf16* __restrict__ xbuf,
    unsigned* __restrict__ ctr, int* __restrict__ status, long spin_max,
    unsigned long long* __restrict__ tst, int debug) {
  constexpr int H = COOP_H;
  __shared__ __attribute__((aligned(16))) bf16 sA[CB_RB * CB_G4];
  __shared__ int sgiveup;
  const int j = blockIdx.x, dir = blockIdx.y, rb = blockIdx.z, nrb = gridDim.z;
  const int b0 = rb * CB_RB;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int unit = j * CB_UB + wid * 16 + (lane & 15);
  // this wave's B fragments (tile j*8 + wid of lstm_pack_whh_kernel's layout), all k-steps
  bf16x8 wf[CB_NKS];
  {
    const bf16* wp = whp + ((long)(dir * (H / 16) + j * (CB_UB / 16) + wid) * CB_NKS) * 512 +
                     lane * 8;
#pragma unroll
    for (int ks = 0; ks < CB_NKS; ++ks) wf[ks] = *(const bf16x8*)(wp + ks * 512);
  }
  unsigned* myctr = ctr + dir * nrb + rb;
  bf16* xb = xbuf + (long)(dir * nrb + rb) * 2 * CB_RB * CB_G4;
  const __amdgpu_buffer_rsrc_t xrs =
      __builtin_amdgcn_make_buffer_rsrc((void*)xb, (short)0, 2 * CB_RB * CB_G4 * 2, 0x00020000);
  // operands of one step for this lane's 4 (row, unit) elements
  f32x4 gq[4];
  float cq[4], cpq[4], dhq[4];
  bf16 hpq[4];
  auto load_ops = [&](int ss) {
    const int tt = dir == 0 ? ss : L - 1 - ss;
    const int tpp = dir == 0 ? tt - 1 : tt + 1;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int b = min(b0 + (lane >> 4) * 4 + r, B - 1);
      const long sidx = ((long)dir * L + tt) * B + b;
      gq[r] = *(const f32x4*)(gsave + (sidx * H + unit) * 4);
      cq[r] = csave[sidx * H + unit];
      dhq[r] = to_f(dhout[((long)b * L + tt) * 2 * H + dir * H + unit]);
      if (ss > 0) {
        cpq[r] = csave[(((long)dir * L + tpp) * B + b) * H + unit];
        hpq[r] = hout[((long)b * L + tpp) * 2 * H + dir * H + unit];
      } else {
        cpq[r] = 0.f;
        hpq[r] = from_f<bf16>(0.f);
      }
    }
  };
  float dcn[4] = {0.f, 0.f, 0.f, 0.f};
  f32x4 dhn = f32x4{0.f, 0.f, 0.f, 0.f};
  // lab probe (MMDX_LSTM_BWD_PROBE): [group][dir][wg][step][phase] realtime stamps
  unsigned long long* tsw =
      tst ? tst + ((long)(rb * 2 + dir) * CB_NU + j) * L * COOP_TS_PHASES : nullptr;
#define CB_STAMP(k)                                                                          \
  do {                                                                                       \
    if (tsw && threadIdx.x == 0) tsw[(L - 1 - s) * COOP_TS_PHASES + (k)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
  load_ops(L - 1);
  for (int s = L - 1; s >= 0; --s) {
    const int t = dir == 0 ? s : L - 1 - s;
    CB_STAMP(0);
    // 1. dG of this lane's elements -> the A image (rows >= B contribute zeros)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = (lane >> 4) * 4 + r, b = b0 + row;
      float dgi = 0.f, dgf = 0.f, dgg = 0.f, dgo = 0.f;
      if (b < B) {
        const float gi = gq[r][0], gf = gq[r][1], gg = gq[r][2], go = gq[r][3];
        const float c = cq[r];
        const float dh = dhq[r] + dhn[r];
        const float tc = tanh_fast(c);
        const float dc = dh * go * (1.f - tc * tc) + dcn[r];
        const float d_o = dh * tc;
        dgi = dc * gg * gi * (1.f - gi);
        dgf = dc * cpq[r] * gf * (1.f - gf);
        dgg = dc * gi * (1.f - gg * gg);
        dgo = d_o * go * (1.f - go);
        dcn[r] = dc * gf;
        hprev[((long)dir * B * L + (long)b * L + t) * H + unit] = hpq[r];
      }
      sA[cb_swz(row, unit)] = from_f<bf16>(dgi);
      sA[cb_swz(row, H + unit)] = from_f<bf16>(dgf);
      sA[cb_swz(row, 2 * H + unit)] = from_f<bf16>(dgg);
      sA[cb_swz(row, 3 * H + unit)] = from_f<bf16>(dgo);
    }
    __syncthreads();
    CB_STAMP(1);
    // 2. this workgroup's slice (16 rows x 4 gates x CB_UB units, 16-B chunks) -> dxg, and to
    //    the exchange slot of this step's parity for the peers
    const bool more = s > 0;
    constexpr int OWN = CB_RB * 4 * (CB_UB / 8);     // chunks of the own slice
#pragma unroll
    for (int q = threadIdx.x; q < OWN; q += CB_NT) {
      const int row = q / (4 * (CB_UB / 8)), rem = q - row * (4 * (CB_UB / 8));
      const int g = rem / (CB_UB / 8), c8 = rem - g * (CB_UB / 8);
      const int col = g * H + j * CB_UB + c8 * 8;
      const coop_v4u v = *(const coop_v4u*)(sA + cb_swz(row, col));
      const int b = b0 + row;
      if (b < B) *(coop_v4u*)(dxg + (((long)b * L + t) * 2 + dir) * CB_G4 + col) = v;
      if (more)
        __builtin_amdgcn_raw_buffer_store_b128(
            v, xrs, ((s & 1) * CB_RB * CB_G4 + row * CB_G4 + col) * 2, 0, COOP_SC1);
    }
    if (!more) break;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    // (debug flag COOP_DEBUG_DROP_PEER: workgroup 0 of direction 0 never signals, so its
    // peers' bounded waits must give up — tests/test_text_gpu.py)
    if (threadIdx.x == 0 && !((debug & COOP_DEBUG_DROP_PEER) && j == 0 && dir == 0))
      __hip_atomic_fetch_add(myctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    CB_STAMP(2);
    // 3. wait for the peers' slices of this step (monotonic: CB_NU per step published)
    if (threadIdx.x == 0) {
      const unsigned target = (unsigned)(CB_NU * (L - s));
      long spins = 0;
      int giveup = 0;
      while (__hip_atomic_load(myctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
        __builtin_amdgcn_s_sleep(1);
        ++spins;
        if (spins > spin_max) {
          __hip_atomic_store(status, 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          giveup = 1;
          break;
        }
        if ((spins & 255) == 0 &&
            __hip_atomic_load(status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) {
          giveup = 1;
          break;
        }
      }
      sgiveup = giveup;
    }
    __syncthreads();
    if (sgiveup) return;
    CB_STAMP(3);
    // peers' chunks (every chunk of the row block not owned here), loaded before any LDS write,
    // then the next step's operands (independent of the chain) behind them
    constexpr int ALL = CB_RB * CB_G4 / 8;           // chunks of the whole row block
    constexpr int PER = ALL / CB_NT;                 // per thread
    coop_v4u pv[PER];
    int pofs[PER];
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int q = threadIdx.x + i * CB_NT;
      const int row = q / (CB_G4 / 8), col = (q - row * (CB_G4 / 8)) * 8;
      const bool peer = ((col % H) / CB_UB) != j;
      pofs[i] = peer ? cb_swz(row, col) : -1;
      pv[i] = __builtin_amdgcn_raw_buffer_load_b128(
          xrs, peer ? ((s & 1) * CB_RB * CB_G4 + row * CB_G4 + col) * 2 : DMA_OOB, 0, COOP_SC1);
    }
    load_ops(s - 1);
#pragma unroll
    for (int i = 0; i < PER; ++i)
      if (pofs[i] >= 0) *(coop_v4u*)(sA + pofs[i]) = pv[i];
    __syncthreads();
    CB_STAMP(4);
    // 4. dh_next for this wave's 16 units
    f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < CB_NKS; ++ks) {
      const bf16x8 af = *(const bf16x8*)(sA + cb_swz(lane & 15, ks * 32 + (lane >> 4) * 8));
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, wf[ks], acc, 0, 0, 0);
    }
    dhn = acc;
    __syncthreads();   // the A image is rewritten by the next step's dG
    CB_STAMP(5);
  }
#undef CB_STAMP
}

template <typename T>
static int lstm_fwd_t(const void* xg, const void* whh, int B, int L, int H, void* hout,
                      float* cs, float* gs, hipStream_t st) {
  dim3 grid((B + LSTM_RB - 1) / LSTM_RB, 2);
  if (H == 256)
    hipLaunchKernelGGL((lstm_fwd_kernel<T, 256>), grid, dim3(LSTM_NW * 64), 0, st,
                       (const float*)xg, (const T*)whh, B, L, (T*)hout, cs, gs);
  else if (H == 128)
    hipLaunchKernelGGL((lstm_fwd_kernel<T, 128>), grid, dim3(LSTM_NW * 64), 0, st,
                       (const float*)xg, (const T*)whh, B, L, (T*)hout, cs, gs);
  else {
    mmdx_set_error("lstm: hidden size %d unsupported (128, 256)", H);
    return -22;
  }
  MMDX_LAUNCH_CHECK();
  return 0;
}

}  // namespace mmdx

using namespace mmdx;

// cooperative forward applies to bf16, H = 256, B <= 256
static bool coop_ok(int dtype, int B, int H) { return dtype == BF16 && H == COOP_H && B <= 256; }

extern "C" size_t mmdx_lstm_fwd_workspace_size(int dtype, int B, int L, int H) {
  (void)L;
  if (!coop_ok(dtype, B, H)) return 0;
  // h exchange [2 dir][2 parity][B][H] bf16 + counters ([2 dir][row groups], 64 B zeroed)
  return (size_t)2 * 2 * B * H * 2 + 256;
}

// debug_flags & COOP_DEBUG_TIMING (lab probe): the phase timestamps follow the workspace,
// [groups][2][COOP_NB][L][COOP_TS_PHASES] x u64 (the caller passes a larger workspace)
static size_t coop_timing_bytes(int B, int L) {
  const int groups = B <= 128 ? 1 : (B + 127) / 128;
  return (size_t)groups * 2 * COOP_NB * L * COOP_TS_PHASES * 8;
}

// The cooperative forward needs its 2 x COOP_NB x groups workgroups resident at once: one per
// CU (~140 KB of LDS each) on distinct CUs.  Checked once per device and kernel variant: the
// device must have at least that many CUs and the kernel must fit one block per CU.  The
// other streams' blocks cannot starve it: they always finish, and the spinning workgroups
// hold at most 2 x COOP_NB x 2 = 32 of the 256 CUs.
template <class K>
static bool coop_resident(K kernel, int threads, int groups) {
  // per device and kernel: the kernels are few, keyed by their address
  static std::atomic<int> ok[64][4];
  static std::atomic<const void*> keys[4];
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return false;
  int slot = -1;
  for (int i = 0; i < 4 && slot < 0; ++i) {
    const void* k = keys[i].load(std::memory_order_relaxed);
    if (k == (const void*)kernel) slot = i;
    else if (k == nullptr) {
      const void* expect = nullptr;
      if (keys[i].compare_exchange_strong(expect, (const void*)kernel) ||
          expect == (const void*)kernel)
        slot = i;
    }
  }
  if (slot < 0) return false;
  int v = ok[dev][slot].load(std::memory_order_relaxed);
  if (v == 0) {
    int per_cu = 0, cus = 0;
    const bool q =
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, threads, 0) == hipSuccess &&
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess;
    v = (q && per_cu >= 1) ? cus : -1;
    ok[dev][slot].store(v, std::memory_order_relaxed);
  }
  return v > 0 && v >= 2 * COOP_NB * groups;
}


extern "C" int mmdx_lstm_fwd(int dtype, const void* xg, const void* w_hh, int B, int L, int H,
                             void* h_out, float* c_save, float* gates_save, void* ws,
                             size_t ws_bytes, int* status, long spin_limit, int debug_flags,
                             void* stream) {
  MMDX_CHECK_ARG(dtype != F16, "mmdx_lstm_fwd: fp16 is the C5 path only");
  MMDX_CHECK_ARG(B > 0 && L > 0 && c_save && gates_save, "lstm fwd: bad args");
  hipStream_t st = (hipStream_t)stream;
  const size_t need = mmdx_lstm_fwd_workspace_size(dtype, B, L, H);
  if (need && ws && ws_bytes >= need) {
    MMDX_CHECK_ARG(status, "lstm fwd: the cooperative path needs a device status word");
    bf16* hx = (bf16*)ws;
    unsigned* ctr = (unsigned*)((char*)ws + (size_t)2 * 2 * B * H * 2);
    const long spin_max = spin_limit > 0 ? spin_limit : COOP_SPIN_MAX;
    unsigned long long* tst = nullptr;
    if (debug_flags & COOP_DEBUG_TIMING) {
      MMDX_CHECK_ARG(ws_bytes >= need + coop_timing_bytes(B, L),
                     "lstm fwd: the timing probe needs %zu more workspace bytes",
                     coop_timing_bytes(B, L));
      tst = (unsigned long long*)((char*)ws + need);
    }
    hipLaunchKernelGGL(lstm_coop_ctr_zero_kernel, dim3(1), dim3(64), 0, st, ctr, 16);
    // B > 128: independent groups of 128 rows (grid z), each with W_hh in LDS (RT = 2)
    const int groups = B <= 128 ? 1 : (B + 127) / 128;
    const dim3 grid(COOP_NB, 2, groups);
#define COOP_LAUNCH(KERNEL, RT, NT)                                                          \
  do {                                                                                       \
    MMDX_CHECK_ARG(coop_resident(KERNEL<RT>, NT, groups),                                    \
                   "lstm fwd: the cooperative recurrence cannot be co-resident here");       \
    hipLaunchKernelGGL(KERNEL<RT>, grid, dim3(NT), 0, st, (const float*)xg,                  \
                       (const bf16*)w_hh, B, L, (bf16*)h_out, c_save, gates_save, hx, ctr,   \
                       status, spin_max, debug_flags, tst);                                  \
  } while (0)
    if (B <= 64)
      COOP_LAUNCH(lstm_fwd_coop_kernel, 1, 512);
    else
      COOP_LAUNCH(lstm_fwd_coop_kernel, 2, 512);
#undef COOP_LAUNCH
    MMDX_LAUNCH_CHECK();
    return 0;
  }
  if (dtype == BF16) return lstm_fwd_t<bf16>(xg, w_hh, B, L, H, h_out, c_save, gates_save, st);
  return lstm_fwd_t<float>(xg, w_hh, B, L, H, h_out, c_save, gates_save, st);
}

// The cooperative backward applies to bf16, H = 256, B <= 16 * CB_MAX_GROUPS when the caller
// passes a status word; its 2 x CB_NU x ceil(B / 16) workgroups must fit the device at once.
template <int Dummy = 0>
static bool coop_bwd_resident(int groups) {
  static std::atomic<int> ok[64];
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return false;
  int v = ok[dev].load(std::memory_order_relaxed);
  if (v == 0) {
    int per_cu = 0, cus = 0;
    const bool q =
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, lstm_bwd_coop_kernel, CB_NT, 0) ==
            hipSuccess &&
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess;
    v = (q && per_cu >= 1) ? cus : -1;
    ok[dev].store(v, std::memory_order_relaxed);
  }
  return v > 0 && v >= 2 * CB_NU * groups;
}

static bool coop_bwd_ok(int dtype, int B, int H) {
  return dtype == BF16 && H == COOP_H && B <= CB_RB * CB_MAX_GROUPS;
}

static size_t lstm_bwd_base_bytes(int dtype, int B, int L, int H) {
  const size_t es = dtype == BF16 ? 2 : 4;
  // fragment-packed W_hh + shifted hidden states + dW_hh GEMM split-K scratch
  return 2 * (size_t)4 * H * H * es + 2 * (size_t)B * L * H * es +
         2 * mmdx_gemm_workspace_size(dtype, 4 * H, H, B * L) + 256;
}

extern "C" size_t mmdx_lstm_workspace_size(int dtype, int B, int L, int H) {
  size_t n = lstm_bwd_base_bytes(dtype, B, L, H);
  if (coop_bwd_ok(dtype, B, H)) {
    // + the cooperative backward's dG exchange [2 dir][groups][2 parity][16][4H] bf16 and
    //   its step counters [2 dir][groups]
    const size_t groups = (B + CB_RB - 1) / CB_RB;
    n = ((n + 255) & ~(size_t)255) + 2 * groups * 2 * CB_RB * CB_G4 * 2 + 256;
  }
  return n;
}

extern "C" int mmdx_lstm_bwd(int dtype, const void* w_hh, const void* h_out, const float* c_save,
                             const float* gates_save, const void* dh_out, int B, int L, int H,
                             void* dxg, float* dw_hh, void* ws, size_t ws_bytes, int* status,
                             long spin_limit, int debug_flags, void* stream) {
  MMDX_CHECK_ARG(dtype != F16, "mmdx_lstm_bwd: fp16 is the C5 path only");
  MMDX_CHECK_ARG(H == 128 || H == 256, "lstm bwd: hidden size %d unsupported", H);
  MMDX_CHECK_ARG(B > 0 && L > 0, "lstm bwd: bad args");
  MMDX_CHECK_ARG(ws && ws_bytes >= mmdx_lstm_workspace_size(dtype, B, L, H),
                 "lstm bwd: workspace too small");
  hipStream_t st = (hipStream_t)stream;
  const size_t es = dtype == BF16 ? 2 : 4;
  char* w = (char*)ws;
  void* whp = w;
  w += 2 * (size_t)4 * H * H * es;
  void* hprev = w;
  w += 2 * (size_t)B * L * H * es;
  w = (char*)(((uintptr_t)w + 255) & ~(uintptr_t)255);
  const size_t gws = mmdx_gemm_workspace_size(dtype, 4 * H, H, B * L);
  const long tw = 2L * 4 * H * H;
  const int tb = (int)std::min<long>((tw + 255) / 256, 4096);
  const int groups = (B + CB_RB - 1) / CB_RB;
  if (status && coop_bwd_ok(dtype, B, H)) {
    MMDX_CHECK_ARG(coop_bwd_resident(groups),
                   "lstm bwd: the cooperative recurrence cannot be co-resident here");
    char* x = (char*)ws + ((lstm_bwd_base_bytes(dtype, B, L, H) + 255) & ~(size_t)255);
    bf16* xbuf = (bf16*)x;
    unsigned* ctr = (unsigned*)(x + 2 * (size_t)groups * 2 * CB_RB * CB_G4 * 2);
    const long spin_max = spin_limit > 0 ? spin_limit : COOP_SPIN_MAX;
    hipLaunchKernelGGL(lstm_pack_whh_kernel<bf16>, dim3(tb), dim3(256), 0, st,
                       (const bf16*)w_hh, H, (bf16*)whp);
    hipLaunchKernelGGL(lstm_coop_ctr_zero_kernel, dim3(1), dim3(64), 0, st, ctr, 2 * groups);
    // lab probe (tools/lab/lstm_probe.py): MMDX_LSTM_BWD_PROBE=1 stamps the phases into the
    // [groups][2][CB_NU][L][8] u64 that follow the workspace (the caller passes them)
    unsigned long long* tst = nullptr;
    if (knobs().lstm_bwd_probe) {
      const size_t tb2 = (size_t)groups * 2 * CB_NU * L * COOP_TS_PHASES * 8;
      MMDX_CHECK_ARG(ws_bytes >= mmdx_lstm_workspace_size(dtype, B, L, H) + tb2,
                     "lstm bwd: the timing probe needs %zu more workspace bytes", tb2);
      tst = (unsigned long long*)((char*)ws + mmdx_lstm_workspace_size(dtype, B, L, H));
    }
    hipLaunchKernelGGL(lstm_bwd_coop_kernel, dim3(CB_NU, 2, groups), dim3(CB_NT), 0, st,
                       (const bf16*)whp, (const bf16*)h_out, c_save, gates_save,
                       (const bf16*)dh_out, B, L, (bf16*)dxg, (bf16*)hprev, xbuf, ctr, status,
                       spin_max, tst, debug_flags & COOP_DEBUG_DROP_PEER);
  } else {
    dim3 grid((B + LSTM_RB - 1) / LSTM_RB, 2);
#define LSTM_BWD(T, HH)                                                                         \
  hipLaunchKernelGGL(lstm_pack_whh_kernel<T>, dim3(tb), dim3(256), 0, st, (const T*)w_hh, HH,  \
                     (T*)whp);                                                                  \
  hipLaunchKernelGGL((lstm_bwd_kernel<T, HH>), grid, dim3(LSTM_NW * 64), 0, st,                 \
                     (const T*)whp, (const T*)h_out, c_save, gates_save, (const T*)dh_out, B,  \
                     L, (T*)dxg, (T*)hprev)
    if (dtype == BF16) {
      if (H == 256) { LSTM_BWD(bf16, 256); } else { LSTM_BWD(bf16, 128); }
    } else {
      if (H == 256) { LSTM_BWD(float, 256); } else { LSTM_BWD(float, 128); }
    }
#undef LSTM_BWD
  }
  MMDX_LAUNCH_CHECK();
  // dW_hh[d] = sum_rows dG[:, d]^T hprev[d]   ([4H] x [H] over B*L rows)
  for (int d = 0; d < 2; ++d) {
    const char* dg = (const char*)dxg + (size_t)d * 4 * H * es;
    const char* hp = (const char*)hprev + (size_t)d * B * L * H * es;
    int rc = mmdx_gemm(dtype, 4 * H, H, B * L, dg, 8L * H, 0, hp, H, 0,
                       dw_hh + (size_t)d * 4 * H * H, H, F32, nullptr, nullptr, ACT_NONE, 1.f,
                       0.f, nullptr, w, gws, stream);
    if (rc) return rc;
  }
  return 0;
}
