// Store-bandwidth probe for the conv epilogue's write pattern (lab only, not product code):
// an [M][256] bf16 output written as 128 x 128 tiles by 512-thread blocks, one 16-B store per
// lane per row chunk (16 lanes per 256-B row segment, rows 512 B apart) — the epilogue_pass
// layout of the 8-wave 128 x 128 conv tiles — with plain stores, nontemporal stores, and a
// fully linear pattern for reference.  Prints GB/s per variant.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef __attribute__((ext_vector_type(4))) unsigned u32x4;

template <int MODE>
__global__ __launch_bounds__(512) void store_tiles(u32x4* out, int M, int N) {
  const int tiles_n = N / 128;
  const int tm = blockIdx.x / tiles_n, tn = blockIdx.x % tiles_n;
  const u32x4 v = {threadIdx.x, blockIdx.x, 7u, 9u};
  if (MODE == 2) {  // linear: the block's 32 KB as one contiguous range
    u32x4* base = out + (long)blockIdx.x * 2048;
#pragma unroll
    for (int it = 0; it < 4; ++it) base[threadIdx.x + it * 512] = v;
    return;
  }
#pragma unroll
  for (int it = 0; it < 4; ++it) {
    const int idx = threadIdx.x + it * 512;
    const int row = idx / 16, c8 = idx % 16;
    const long m = (long)tm * 128 + row;
    if (m >= M) continue;
    u32x4* p = out + (m * N + tn * 128 + c8 * 8) / 8;
    if (MODE == 1) __builtin_nontemporal_store(v, p);
    else *p = v;
  }
}

int main() {
  const int M = 401408, N = 256;
  u32x4* out;
  hipMalloc(&out, (size_t)M * N * 2);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int grid = (M / 128) * (N / 128);
  for (int mode = 0; mode < 3; ++mode) {
    for (int rep = 0; rep < 2; ++rep) {
      hipEventRecord(e0);
      for (int i = 0; i < 50; ++i) {
        if (mode == 0) store_tiles<0><<<grid, 512>>>(out, M, N);
        else if (mode == 1) store_tiles<1><<<grid, 512>>>(out, M, N);
        else store_tiles<2><<<grid, 512>>>(out, M, N);
      }
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      const double us = ms * 1e3 / 50;
      printf("mode %d (%s): %.1f us per 205 MB, %.0f GB/s\n", mode,
             mode == 0 ? "tile, plain" : mode == 1 ? "tile, nontemporal" : "linear, plain", us,
             (double)M * N * 2 / us / 1e3);
    }
  }
  hipFree(out);
  return 0;
}
