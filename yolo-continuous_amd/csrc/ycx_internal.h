// Internal helpers shared by the libycx_hip.so translation units.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "ycx.h"

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
typedef __attribute__((ext_vector_type(4))) float f32x4;

#define YCX_CHECK_ARG(cond) \
  do {                      \
    if (!(cond)) return YCX_ERR_BAD_ARG; \
  } while (0)
#define YCX_CHECK_SUPPORTED(cond) \
  do {                            \
    if (!(cond)) return YCX_ERR_UNSUPPORTED; \
  } while (0)

static inline ycx_status ycx_launch_status() {
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? YCX_OK : YCX_ERR_LAUNCH;
}

static inline unsigned ycx_cdiv(long long a, long long b) { return (unsigned)((a + b - 1) / b); }

// Activation applied in the conv epilogues (Conv.act, nets/common.py:103).
// FAST (bf16 outputs): the raw v_exp_f32 (2^x, no range fix-up: overflow to
// inf gives rcp 0, i.e. silu -> 0) and v_rcp_f32, ~1 ulp fp32, far below bf16
// rounding; otherwise the IEEE division of torch's silu for the f32 parity mode.
template <bool FAST>
__device__ __forceinline__ float ycx_act(float v, int act, float slope) {
  if (act == YCX_ACT_SILU)  // x*sigmoid(x)
    return FAST ? v * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(v * -1.44269504f))
                : v / (1.0f + expf(-v));
  if (act == YCX_ACT_LEAKY) return v > 0.0f ? v : v * slope;
  return v;
}

// The same with the act code as a template argument (no per-element branch).
template <int ACT>
__device__ __forceinline__ float act_t(float v, float slope) {
  if constexpr (ACT == YCX_ACT_SILU) return v * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(v * -1.44269504f));
  else if constexpr (ACT == YCX_ACT_LEAKY) return v > 0.0f ? v : v * slope;
  else return v;
}

// XCD-aware bijective remap of a 1-D block id (guide §5 "XCD swizzle must be
// bijective"): consecutive logical ids land on the same XCD (blocks b, b+8, ...
// share one), so blocks that share an activation tile share an L2.
__device__ __forceinline__ int ycx_xcd_remap(int bid, int nwg) {
  int q = nwg >> 3, r = nwg & 7, xcd = bid & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
}
