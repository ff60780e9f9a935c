// GEMM main-loop lab: bf16 C[M,N] = A[M,K] . B[N,K]^T (both k-major), fp32 accumulate.
// Variants of the LDS-DMA (global_load_lds_dwordx4) pipeline, timed against each other on
// conv-shaped problems before the winning structure goes into csrc/igemm.h.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/lab/gemm_lab.hip -o gemm_lab && ./gemm_lab
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      exit(1);                                                                       \
    }                                                                                \
  } while (0)

typedef __bf16 bf16;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(1))) void gbl_void;

__device__ __attribute__((aligned(16))) int4 g_zero16[4];

constexpr int BK = 64;  // k per stage: one 128-B row per tile row

__device__ __forceinline__ int xcd_swizzle(int orig, int nwg) {
  const int q = nwg / 8, r = nwg % 8, xcd = orig % 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / 8;
}

// One operand tile [ROWS][64] bf16 per stage, XOR-swizzled 16-B chunks:
// logical chunk c of row r lives at slot c ^ (r & 7).  Filled by LDS-DMA: wave instruction j
// of wave w writes rows (j*NW + w)*8 .. +7 (1 KiB, lane-linear), each lane fetching the
// global chunk that belongs at its slot.
template <int ROWS, int NW>
struct DmaOperand {
  static constexpr int INSTR = ROWS / (8 * NW);  // glds per wave per stage
  static_assert(ROWS % (8 * NW) == 0, "rows per wave");
  const bf16* src[INSTR];
  __device__ void init(const bf16* base, long ld, int row0, int nrows, int wid, int lane) {
    const int rr = lane >> 3, slot = lane & 7;
#pragma unroll
    for (int j = 0; j < INSTR; ++j) {
      const int row = (j * NW + wid) * 8 + rr;
      const int c = slot ^ (row & 7);
      src[j] = row0 + row < nrows ? base + (long)(row0 + row) * ld + c * 8 : nullptr;
    }
  }
  __device__ void issue(char* lds_stage, int k0, int wid) const {
#pragma unroll
    for (int j = 0; j < INSTR; ++j) {
      const void* g = src[j] ? (const void*)(src[j] + k0) : (const void*)g_zero16;
      __builtin_amdgcn_global_load_lds((gbl_void*)g,
                                       (lds_void*)(lds_stage + (j * NW + wid) * 8 * 128), 16, 0,
                                       0);
    }
  }
  // 16x32 fragment (16 rows from r16, k = ks..ks+31): lane gets row r16+(lane&15),
  // 8 k at ks + 8*(lane>>4).
  __device__ static bf16x8 frag(const char* lds_stage, int r16, int ks, int lane) {
    const int row = r16 + (lane & 15);
    const int c = (ks >> 3) + (lane >> 4);
    return *(const bf16x8*)(lds_stage + row * 128 + ((c ^ (row & 7)) << 4));
  }
};

template <int BM, int BN, int WM, int WN, int STAGES>
__global__ __launch_bounds__(64 * WM * WN) void gemm_dma(const bf16* __restrict__ A,
                                                          const bf16* __restrict__ B,
                                                          bf16* __restrict__ C, int M, int N,
                                                          int K) {
  constexpr int NW = WM * WN, NT = 64 * NW;
  constexpr int WTM = BM / WM, WTN = BN / WN, RM = WTM / 16, RN = WTN / 16;
  constexpr int A_BYTES = BM * 128, B_BYTES = BN * 128, STAGE = A_BYTES + B_BYTES;
  constexpr int LDC = BN + 4;
  constexpr int EPI = BM * LDC * 4;
  constexpr int OPS = STAGES * STAGE;
  constexpr int PR = EPI <= OPS ? BM : (OPS / (LDC * 4) >= 128 ? 128 : OPS / (LDC * 4) >= 64 ? 64 : 32);
  constexpr int LDS = OPS > PR * LDC * 4 ? OPS : PR * LDC * 4;
  __shared__ __attribute__((aligned(1024))) char lds[LDS];
  typedef DmaOperand<BM, NW> OA;
  typedef DmaOperand<BN, NW> OB;
  constexpr int L = OA::INSTR + OB::INSTR;  // glds per wave per stage

  const int tiles_n = (N + BN - 1) / BN, tiles_m = (M + BM - 1) / BM;
  const int tile = xcd_swizzle(blockIdx.x, tiles_m * tiles_n);
  const int tm = tile / tiles_n, tn = tile - tm * tiles_n;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int wm = wid / WN, wn = wid % WN;
  OA oa;
  OB ob;
  oa.init(A, K, tm * BM, M, wid, lane);
  ob.init(B, K, tn * BN, N, wid, lane);
  const int nt = K / BK;

  f32x4 acc[RM][RN];
#pragma unroll
  for (int i = 0; i < RM; ++i)
#pragma unroll
    for (int j = 0; j < RN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int s = 0; s < STAGES - 1; ++s)
    if (s < nt) {
      oa.issue(lds + s * STAGE, s * BK, wid);
      ob.issue(lds + s * STAGE + A_BYTES, s * BK, wid);
    }
  for (int t = 0; t < nt; ++t) {
    // tile t landed (this wave's DMAs), then every wave's: counted wait + raw barrier
    const int ahead = min(STAGES - 2, nt - 1 - t);  // tiles issued beyond t, may stay in flight
    if (ahead >= 2)
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * L) : "memory");
    else if (ahead == 1)
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(L) : "memory");
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    const int tn_ = t + STAGES - 1;
    if (tn_ < nt) {
      char* st = lds + (tn_ % STAGES) * STAGE;
      oa.issue(st, tn_ * BK, wid);
      ob.issue(st + A_BYTES, tn_ * BK, wid);
    }
    const char* as = lds + (t % STAGES) * STAGE;
    const char* bs = as + A_BYTES;
#pragma unroll
    for (int ks = 0; ks < BK; ks += 32) {
      bf16x8 af[RM], bfr[RN];
#pragma unroll
      for (int i = 0; i < RM; ++i) af[i] = OA::frag(as, wm * WTM + i * 16, ks, lane);
#pragma unroll
      for (int j = 0; j < RN; ++j) bfr[j] = OB::frag(bs, wn * WTN + j * 16, ks, lane);
#pragma unroll
      for (int i = 0; i < RM; ++i)
#pragma unroll
        for (int j = 0; j < RN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  // epilogue through LDS in row passes of PR rows (fp32 staging of the whole tile may not fit)
  float* cst = (float*)lds;
  constexpr int C4 = BN / 4;
#pragma unroll
  for (int p0 = 0; p0 < BM; p0 += PR) {
#pragma unroll
    for (int i = 0; i < RM; ++i) {
      const int rb = wm * WTM + i * 16;
      if (rb < p0 || rb >= p0 + PR) continue;
#pragma unroll
      for (int j = 0; j < RN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          cst[(rb - p0 + (lane >> 4) * 4 + r) * LDC + wn * WTN + j * 16 + (lane & 15)] =
              acc[i][j][r];
    }
    __syncthreads();
    for (int c = threadIdx.x; c < PR * C4; c += NT) {
      const int row = c / C4, col = (c - row * C4) * 4;
      const int m = tm * BM + p0 + row, n = tn * BN + col;
      if (m >= M || n >= N) continue;
      const f32x4 v = *(const f32x4*)(cst + row * LDC + col);
      typedef __attribute__((ext_vector_type(4))) __bf16 b4;
      b4 o;
      for (int j = 0; j < 4; ++j) o[j] = (bf16)v[j];
      *(b4*)(C + (long)m * N + n) = o;
    }
    __syncthreads();
  }
}

__global__ void ref_gemm(const bf16* A, const bf16* B, float* C, int M, int N, int K) {
  const int m = blockIdx.y, n = blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= N) return;
  float s = 0.f;
  for (int k = 0; k < K; ++k) s += (float)A[(long)m * K + k] * (float)B[(long)n * K + k];
  C[(long)m * N + n] = s;
}

__global__ void init_rand(bf16* p, long n, unsigned seed) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    unsigned h = (unsigned)i * 2654435761u ^ seed;
    h ^= h >> 13; h *= 0x5bd1e995u; h ^= h >> 15;
    p[i] = (bf16)((h & 0xffff) / 32768.f - 1.f);
  }
}

template <int BM, int BN, int WM, int WN, int S>
struct Variant {
  static const char* name() {
    static char buf[64];
    snprintf(buf, sizeof buf, "dma %dx%d w%dx%d s%d", BM, BN, WM, WN, S);
    return buf;
  }
  static void run(const bf16* A, const bf16* B, bf16* C, int M, int N, int K) {
    const int nwg = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
    hipLaunchKernelGGL((gemm_dma<BM, BN, WM, WN, S>), dim3(nwg), dim3(64 * WM * WN), 0, 0, A, B,
                       C, M, N, K);
  }
};

template <class V>
void bench(int M, int N, int K, bf16* A, bf16* B, bf16* C, float* R, bool check) {
  if (check) {
    V::run(A, B, C, M, N, K);
    CK(hipDeviceSynchronize());
    std::vector<bf16> c((size_t)M * N);
    std::vector<float> r((size_t)M * N);
    CK(hipMemcpy(c.data(), C, c.size() * 2, hipMemcpyDeviceToHost));
    CK(hipMemcpy(r.data(), R, r.size() * 4, hipMemcpyDeviceToHost));
    double err = 0, mx = 0;
    for (size_t i = 0; i < c.size(); ++i) {
      err = fmax(err, fabs((double)(float)c[i] - r[i]));
      mx = fmax(mx, fabs((double)r[i]));
    }
    printf("  check %-22s rel err %.3e %s\n", V::name(), err / mx, err / mx < 1e-2 ? "OK" : "FAIL");
    return;
  }
  hipEvent_t s, e;
  CK(hipEventCreate(&s));
  CK(hipEventCreate(&e));
  for (int i = 0; i < 3; ++i) V::run(A, B, C, M, N, K);
  const int reps = 20;
  CK(hipEventRecord(s));
  for (int i = 0; i < reps; ++i) V::run(A, B, C, M, N, K);
  CK(hipEventRecord(e));
  CK(hipEventSynchronize(e));
  float ms;
  CK(hipEventElapsedTime(&ms, s, e));
  ms /= reps;
  printf("  %-22s %7dx%5dx%5d %8.1fus %7.1f TF\n", V::name(), M, N, K, ms * 1e3,
         2.0 * M * N * K / ms / 1e9);
}

template <class... Vs>
void all(int M, int N, int K, bf16* A, bf16* B, bf16* C, float* R, bool check) {
  (bench<Vs>(M, N, K, A, B, C, R, check), ...);
}

#define VARIANTS                                                                          \
  Variant<128, 128, 2, 2, 2>, Variant<128, 128, 2, 2, 3>, Variant<256, 128, 4, 2, 2>,    \
      Variant<256, 128, 2, 2, 2>, Variant<128, 256, 2, 2, 2>, Variant<128, 128, 2, 2, 4>, \
      Variant<256, 256, 2, 4, 2>

int main() {
  const long maxA = 401408L * 1152, maxB = 8192L * 8192, maxC = 401408L * 512;
  bf16 *A, *B, *C;
  float* R;
  CK(hipMalloc(&A, maxA * 2));
  CK(hipMalloc(&B, maxB * 2));
  CK(hipMalloc(&C, maxC * 2));
  CK(hipMalloc(&R, 1024L * 1024 * 4));
  hipLaunchKernelGGL(init_rand, dim3(4096), dim3(256), 0, 0, A, maxA, 1u);
  hipLaunchKernelGGL(init_rand, dim3(4096), dim3(256), 0, 0, B, maxB, 2u);
  {
    const int M = 300, N = 200, K = 320;  // ragged M/N, checks the zero-row path
    hipLaunchKernelGGL(ref_gemm, dim3((N + 63) / 64, M), dim3(64), 0, 0, A, B, R, M, N, K);
    CK(hipDeviceSynchronize());
    all<VARIANTS>(M, N, K, A, B, C, R, true);
  }
  const int shapes[][3] = {{4096, 4096, 4096}, {8192, 8192, 8192}, {25088, 256, 2304},
                           {100352, 128, 1152}, {6272, 512, 4608}, {25088, 1024, 256},
                           {100352, 512, 128},  {6272, 2048, 512}, {401408, 256, 64}};
  for (auto& s : shapes) {
    printf("shape %dx%dx%d\n", s[0], s[1], s[2]);
    all<VARIANTS>(s[0], s[1], s[2], A, B, C, R, false);
  }
  return 0;
}
