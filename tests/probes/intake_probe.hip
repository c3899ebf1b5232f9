// L2 -> CU intake microbenchmark (development probe, not part of the library).
// How many bytes per clock can one CU pull from an L2-resident operand, by the
// two paths a conv tile can stage through: LDS-DMA (buffer_load ... lds, tile 16's
// path) and global_load_dwordx4 into VGPRs. The access pattern is tile 16's: a
// wave-instruction reads 8 rows x 128 B at a fixed row stride (an NHWC channel
// slab or a packed weight row block), 32 KiB per 512-thread block per step.
//   hipcc --offload-arch=gfx950 -O3 -shared -fPIC intake_probe.hip -o build/intake_probe.so
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((ext_vector_type(4))) unsigned u32x4;

__device__ __forceinline__ void dma16(const void* base, int nbytes, int voff, void* lds) {
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, nbytes, 0x00020000);
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void*)lds, 16, voff, 0, 0, 0);
}

// MODE 0: LDS-DMA, INFL steps of 4 DMAs per wave in flight (vmcnt(4 (INFL - 1)) after each step's issue)
// MODE 1: global_load_dwordx4 to VGPRs, the same addresses, xor-reduced
// BAR: an s_barrier per step (tile 16 has one)
template <int MODE, int LDSB, int INFL, bool BAR>
__global__ void __launch_bounds__(512) intake(const char* src, int src_mask, int row_stride, int steps,
                                              unsigned* sink) {
  __shared__ __attribute__((aligned(1024))) char smem[LDSB];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int lrow = lane >> 3, lch = lane & 7;
  unsigned acc = 0;
  const int src_bytes = src_mask + 1;
  for (int s = 0; s < steps; ++s) {
    const int step_row = (blockIdx.x * 131 + s) * 256;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = step_row + (wid * 4 + i) * 8 + lrow;
      const int off = (int)(((unsigned)row * (unsigned)row_stride) & (unsigned)src_mask & ~127u) + lch * 16;
      if (MODE == 0) {
        char* dst = smem + (((s * 32768) + (wid * 4 + i) * 1024) & (LDSB - 1));
        dma16(src, src_bytes, off, dst);
      } else {
        const u32x4 v = *reinterpret_cast<const u32x4*>(src + off);
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
      }
    }
    if (MODE == 0) {
      if (INFL == 1) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      else if (INFL == 2) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      else if (INFL == 3) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
    }
    if (BAR) __builtin_amdgcn_s_barrier();
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (MODE == 1 && acc == 0x12345678u) sink[0] = acc;
  if (MODE == 0 && threadIdx.x == 0 && smem[lane] == 123) sink[1] = 1;
}

// plain global loads kept in registers (no xor between issue and the next step's loads)
template <int LDSB>
__global__ void __launch_bounds__(512) intake_vgpr4(const char* src, int src_mask, int row_stride, int steps,
                                                    unsigned* sink) {
  __shared__ char smem[LDSB];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int lrow = lane >> 3, lch = lane & 7;
  u32x4 acc = {0, 0, 0, 0};
  for (int s = 0; s < steps; ++s) {
    const int step_row = (blockIdx.x * 131 + s) * 256;
    u32x4 v[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = step_row + (wid * 4 + i) * 8 + lrow;
      const int off = (int)(((unsigned)row * (unsigned)row_stride) & (unsigned)src_mask & ~127u) + lch * 16;
      v[i] = *reinterpret_cast<const u32x4*>(src + off);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) acc ^= v[i];
  }
  if (acc.x == 0x12345678u) sink[0] = acc.y;
  if (threadIdx.x == 0 && smem[lane] == 123) sink[1] = 1;
}

extern "C" int intake_probe(int mode, int lds_kb, int infl, int bar, const void* src, int src_mask, int row_stride,
                            int steps, int blocks, unsigned* sink, void* stream) {
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const char* s = reinterpret_cast<const char*>(src);
#define L0(LB, IF, B) hipLaunchKernelGGL((intake<0, LB, IF, B>), dim3(blocks), dim3(512), 0, st, s, src_mask, row_stride, steps, sink)
#define L1(LB, B) hipLaunchKernelGGL((intake<1, LB, 1, B>), dim3(blocks), dim3(512), 0, st, s, src_mask, row_stride, steps, sink)
  if (mode == 0) {
    if (lds_kb == 64) {
      if (infl == 1) { if (bar) L0(65536, 1, true); else L0(65536, 1, false); }
      else if (infl == 2) { if (bar) L0(65536, 2, true); else L0(65536, 2, false); }
      else if (infl == 3) { if (bar) L0(65536, 3, true); else L0(65536, 3, false); }
      else { if (bar) L0(65536, 4, true); else L0(65536, 4, false); }
    } else if (lds_kb == 32) {
      if (infl == 1) { if (bar) L0(32768, 1, true); else L0(32768, 1, false); }
      else if (infl == 2) { if (bar) L0(32768, 2, true); else L0(32768, 2, false); }
      else if (infl == 3) { if (bar) L0(32768, 3, true); else L0(32768, 3, false); }
      else { if (bar) L0(32768, 4, true); else L0(32768, 4, false); }
    } else {
      if (infl == 1) L0(131072, 1, false); else if (infl == 2) L0(131072, 2, false);
      else if (infl == 3) L0(131072, 3, false); else L0(131072, 4, false);
    }
  } else if (mode == 1) {
    if (lds_kb == 64) { if (bar) L1(65536, true); else L1(65536, false); }
    else if (lds_kb == 32) { if (bar) L1(32768, true); else L1(32768, false); }
    else L1(131072, false);
  } else {
    if (lds_kb == 64) hipLaunchKernelGGL((intake_vgpr4<65536>), dim3(blocks), dim3(512), 0, st, s, src_mask, row_stride, steps, sink);
    else if (lds_kb == 32) hipLaunchKernelGGL((intake_vgpr4<32768>), dim3(blocks), dim3(512), 0, st, s, src_mask, row_stride, steps, sink);
    else hipLaunchKernelGGL((intake_vgpr4<131072>), dim3(blocks), dim3(512), 0, st, s, src_mask, row_stride, steps, sink);
  }
  return (int)hipGetLastError();
}
