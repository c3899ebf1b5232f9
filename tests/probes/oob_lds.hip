// Probe: does an out-of-range buffer_load ... lds write zeros into LDS, or leave it untouched?
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef __attribute__((address_space(3))) void lds_void;
__global__ void k(const int* __restrict__ g, int* out) {
  __shared__ __attribute__((aligned(16))) int lds[256];
  lds[threadIdx.x * 4 + 0] = 0x11111111; lds[threadIdx.x * 4 + 1] = 0x22222222;
  lds[threadIdx.x * 4 + 2] = 0x33333333; lds[threadIdx.x * 4 + 3] = 0x44444444;
  __syncthreads();
  __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)g, (short)0, 1024, 0x00020000);
  int off = (threadIdx.x & 1) ? 0x80000000 : threadIdx.x * 16;
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void*)lds, 16, off, 0, 0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  for (int j = 0; j < 4; ++j) out[threadIdx.x * 4 + j] = lds[threadIdx.x * 4 + j];
}
int main() {
  int h[1024], *dg, *dout, o[256];
  for (int i = 0; i < 1024; ++i) h[i] = i + 1;
  hipMalloc(&dg, 4096); hipMalloc(&dout, 1024);
  hipMemcpy(dg, h, 4096, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, dg, dout);
  hipMemcpy(o, dout, 1024, hipMemcpyDeviceToHost);
  printf("lane0: %x %x %x %x  lane1(OOB): %x %x %x %x  lane2: %x\n", o[0], o[1], o[2], o[3], o[4], o[5], o[6], o[7], o[8]);
  return 0;
}
