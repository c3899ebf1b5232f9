// Store-pattern microbenchmark (development probe, not part of the library):
// writes a [rows][512 B] bf16 image the ways a conv epilogue can.
//   hipcc --offload-arch=gfx950 -O3 -shared -fPIC store_probe.hip -o build/store_probe.so
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(2))) float f32x2;

// pattern 0: 16 B per lane, a wave writes 1 KiB contiguous (fill)
// pattern 1: 8 B per lane, lane l -> row (l & 15), bytes 8 (l >> 4) + 32 i : MFMA-fragment epilogue,
//            one wave instruction covers 16 rows x 32 B; FM x FN instructions per wave per tile
// pattern 2: 16 B per lane, 32 lanes per 512-B row (whole rows per instruction)
template <int PAT>
__global__ void __launch_bounds__(512) store_kernel(char* y, int rows, int tiles_per_block) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const f32x4 v4 = {1.f, 2.f, 3.f, 4.f};
  for (int tt = 0; tt < tiles_per_block; ++tt) {
    const int tile = blockIdx.x * tiles_per_block + tt;  // 64 rows x 512 B = 32 KiB per tile
    const long base = (long)tile * 64 * 512;
    if ((long)tile * 64 >= rows) return;
    if (PAT == 0) {
#pragma unroll
      for (int u = 0; u < 4; ++u) *reinterpret_cast<f32x4*>(y + base + (u * 8 + wid) * 1024 + lane * 16) = v4;
    } else if (PAT == 1) {
      // wave wid owns bytes 64 wid .. +63 of each row (32 channels), 4 row groups of 16 x 2 channel halves
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int i = 0; i < 2; ++i)
          *reinterpret_cast<f32x2*>(y + base + (16 * j + (lane & 15)) * 512 + 64 * wid + 32 * i + 8 * (lane >> 4)) =
              f32x2{1.f, 2.f};
    } else {
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int e = (u * 8 + wid) * 64 + lane, row = e >> 5, ch = e & 31;
        *reinterpret_cast<f32x4*>(y + base + row * 512 + ch * 16) = v4;
      }
    }
  }
}

extern "C" int store_probe(int pat, void* y, int rows, int blocks, int tiles_per_block, void* stream) {
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (pat == 0) hipLaunchKernelGGL(store_kernel<0>, dim3(blocks), dim3(512), 0, st, (char*)y, rows, tiles_per_block);
  if (pat == 1) hipLaunchKernelGGL(store_kernel<1>, dim3(blocks), dim3(512), 0, st, (char*)y, rows, tiles_per_block);
  if (pat == 2) hipLaunchKernelGGL(store_kernel<2>, dim3(blocks), dim3(512), 0, st, (char*)y, rows, tiles_per_block);
  return hipGetLastError();
}
