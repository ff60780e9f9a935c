// Does an out-of-range raw buffer load to LDS (LDS-DMA) write zeros or leave LDS untouched?
#include <hip/hip_runtime.h>
#include <cstdio>
typedef __attribute__((address_space(3))) void lds_void;
typedef int v4i __attribute__((ext_vector_type(4)));

__device__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, (int)bytes, 0x00020000);
}

__global__ void k(const int* src, int* out, unsigned nbytes) {
  __shared__ int lds[64 * 4 * 2];
  for (int i = threadIdx.x; i < 512; i += 64) lds[i] = 0x7eadbeef;
  __syncthreads();
  const __amdgpu_buffer_rsrc_t rs = make_rsrc(src, nbytes);
  // lane l loads 16 B at byte offset l*16: lanes past nbytes are out of range
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void*)lds, 16, threadIdx.x * 16, 0, 0, 0);
  // second instruction: all lanes out of range via a huge voffset
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void*)(lds + 256), 16, 0x80000000u, 0, 0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int i = threadIdx.x; i < 512; i += 64) out[i] = lds[i];
}

int main() {
  int *src, *out;
  hipMalloc(&src, 4096);
  hipMalloc(&out, 2048);
  int h[1024];
  for (int i = 0; i < 1024; ++i) h[i] = i + 1;
  hipMemcpy(src, h, 4096, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, src, out, 32 * 16);  // lanes 32..63 OOB
  int o[512];
  hipMemcpy(o, out, 2048, hipMemcpyDeviceToHost);
  printf("lane 0: %x %x %x %x\n", o[0], o[1], o[2], o[3]);
  printf("lane 31: %x   lane 32: %x %x   lane 63: %x\n", o[31 * 4], o[32 * 4], o[32 * 4 + 3], o[63 * 4]);
  printf("all-OOB instr: %x %x %x\n", o[256], o[300], o[511]);
  return 0;
}
