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

// Kernel-side bounds checks (`make debug` -> libycx_hip_dbg.so, built with
// -DYCX_DEBUG_BOUNDS): every guarded global store first tests its element range
// against the buffer extent the descriptor implies; a store outside it is skipped and
// counted (first offending source line kept) instead of faulting, and
// ycx_debug_bounds() returns the count. Release builds compile the test away.
// One counter per translation unit (no relocatable device code); the host side sums them.
#ifdef YCX_DEBUG_BOUNDS
static __device__ unsigned int g_ycx_oob[2];  // [0] violations, [1] first line
__device__ __forceinline__ bool ycx_bounds_ok(bool ok, int line) {
  if (!ok && atomicAdd(&g_ycx_oob[0], 1u) == 0) atomicExch(&g_ycx_oob[1], (unsigned)line);
  return ok;
}
#define YCX_BOUNDS_OK(lo, n, lim) ycx_bounds_ok((long long)(lo) >= 0 && (long long)(lo) + (n) <= (long long)(lim), __LINE__)
// host: read (and optionally reset) this unit's counters
#define YCX_DEFINE_BOUNDS_READER(fn)                                              \
  ycx_status fn(unsigned* out, int reset) {                                      \
    unsigned v[2] = {0, 0};                                                      \
    if (hipMemcpyFromSymbol(v, HIP_SYMBOL(g_ycx_oob), sizeof v) != hipSuccess)   \
      return YCX_ERR_LAUNCH;                                                     \
    out[0] += v[0];                                                              \
    if (v[0] && !out[1]) out[1] = v[1];                                          \
    if (reset) {                                                                 \
      const unsigned z[2] = {0, 0};                                              \
      if (hipMemcpyToSymbol(HIP_SYMBOL(g_ycx_oob), z, sizeof z) != hipSuccess)   \
        return YCX_ERR_LAUNCH;                                                   \
    }                                                                            \
    return YCX_OK;                                                               \
  }
#else
#define YCX_BOUNDS_OK(lo, n, lim) true
#endif

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
  if (act == YCX_ACT_SILU_PS)  // v = -log2(e) c (pre-scaled weights): c / (1 + 2^v)
    return v * __builtin_amdgcn_rcpf(__builtin_fmaf(__builtin_amdgcn_exp2f(v), -1.44269504f, -1.44269504f));
  return v;
}

// The same with the act code as a template argument (no per-element branch).
template <int ACT>
__device__ __forceinline__ float act_t(float v, float slope) {
  if constexpr (ACT == YCX_ACT_SILU) return v * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(v * -1.44269504f));
  else if constexpr (ACT == YCX_ACT_LEAKY) return v > 0.0f ? v : v * slope;
  else if constexpr (ACT == YCX_ACT_SILU_PS)
    return v * __builtin_amdgcn_rcpf(__builtin_fmaf(__builtin_amdgcn_exp2f(v), -1.44269504f, -1.44269504f));
  else return v;
}

// XCD-aware bijective remap of a 1-D block id (guide §5 "XCD swizzle must be
// bijective"): consecutive logical ids land on the same XCD (blocks b, b+8, ...
// share one), so blocks that share an activation tile share an L2.
__host__ __device__ __forceinline__ int ycx_xcd_remap(int bid, int nwg) {
  int q = nwg >> 3, r = nwg & 7, xcd = bid & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
}

// Logical block L (after ycx_xcd_remap: each XCD holds a contiguous range of L)
// -> (output-channel tile ct, pixel tile pt) of an n_ct x n_pt tile grid.
// gc <= 1: ct fastest (every XCD walks every ct over its 1/8 of the pixel tiles,
// i.e. streams the whole weight tensor through its L2). gc in {2, 4, 8} with
// n_ct % gc == 0: the grid is cut into 8 regions, gc channel groups x 8/gc pixel
// groups, enumerated region by region (ct fastest inside a region), so the
// region an XCD's range covers reads 1/gc of the weights and gc/8 of the
// pixels: weights are re-read 8/gc times instead of 8, activations gc times.
// Bijective by construction (an ordering of all tiles).
__host__ __device__ __forceinline__ void ycx_tile_of(int L, int n_ct, int n_pt, int gc, int& ct, int& pt) {
  if (gc <= 1 || n_ct % gc) {
    ct = L % n_ct;
    pt = L / n_ct;
    return;
  }
  const int gp = 8 / gc, nct_r = n_ct / gc;
  int pg = 0;  // largest pg with n_ct * pt_lo(pg) <= L, pt_lo(pg) = pg * n_pt / gp
  const int q = L / n_ct;
  while (pg + 1 < gp && (pg + 1) * n_pt / gp <= q) ++pg;
  const int lo = pg * n_pt / gp, npt = (pg + 1) * n_pt / gp - lo;
  const int rem = L - n_ct * lo, cg = rem / (nct_r * npt), r2 = rem - cg * (nct_r * npt);
  ct = cg * nct_r + r2 % nct_r;
  pt = lo + r2 / nct_r;
}

// torch.sigmoid as the decode kernels evaluate it (detect.py:53, 1/(1+e^-v),
// IEEE division, no contraction possible). One definition for every kernel
// that must produce bit-identical candidates.
__device__ __forceinline__ float ycx_sigmoid(float v) { return 1.0f / (1.0f + expf(-v)); }

// The class scan of detect.py:109-110 (torch.max over sigmoid(class logits),
// first index on ties) as the sequential strict-'>' scan defines it, with one
// pass of compares over the logits and two sigmoids instead of nc sigmoids.
// logit(k) returns class k's raw logit. ycx_sigmoid is monotone
// non-decreasing over every float (checked exhaustively on the device:
// ycx_check_sigmoid_monotone, tests/test_gpu_post.py). With m the largest
// non-NaN logit, bi its first index and pm the largest logit before bi: the
// scan's maximum is sm = sigmoid(m), and a class before bi can tie it only
// with a logit in [lo, m), where sigmoid(lo) < sm; so unless pm >= lo (a
// saturated or one-ulp tie, rare) the answer is bi. A NaN at class 0 sticks
// (the scan's 'sv > NaN' never holds); other NaNs never win.
// Logits m in [kClassFastLo, kClassFastHi]: the device sigmoid separates m from
// m - max(|m|, 1) 2^-12 (sigmoid(m) - sigmoid(m - tau) is >= 60 ulps there; past
// ~8 the sigmoid saturates towards 1, below ~-87 towards the denormals).
constexpr float kClassFastLo = -80.0f, kClassFastHi = 6.0f;
// Running (m, first index b, largest logit before b) over classes [k0, k1).
// Start from m = -inf, b = -1 (empty) or from class 0's logit (m = l0, b = 0).
template <class F>
__device__ __forceinline__ void ycx_class_scan(F&& logit, int k0, int k1, float& m, float& pm, int& b) {
  int k = k0;
  for (; k + 8 <= k1; k += 8) {
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = logit(k + u);
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const bool up = v[u] > m;  // false for NaN
      pm = up ? m : pm;
      b = up ? k + u : b;
      m = up ? v[u] : m;
    }
  }
  for (; k < k1; ++k) {
    const float v = logit(k);
    const bool up = v > m;
    pm = up ? m : pm;
    b = up ? k : b;
    m = up ? v : m;
  }
}

// (m, pm, b) of a lower part [0, c) and an upper part [c, nc) -> those of [0, nc).
__device__ __forceinline__ void ycx_class_merge(float& m, float& pm, int& b, float m2, float pm2, int b2) {
  if (m2 > m) {  // the upper part's maximum is larger: everything below c precedes it
    pm = fmaxf(m, pm2);
    m = m2;
    b = b2;
  }
}

// From the scan state of all classes (l0 not NaN) to the sequential scan's answer.
template <class F>
__device__ __forceinline__ void ycx_class_finish(F&& logit, float m, float pm, int b, float& best, int& bi) {
  const float sm = ycx_sigmoid(m);
  best = sm;
  bi = b;
  // nothing before bi can reach sm -- unless sm is 0: then an earlier -inf ties it
  if (pm == -INFINITY && sm > 0.0f) return;
  float tau = fmaxf(fabsf(m), 1.0f) * 0x1p-12f, lo = m < INFINITY ? m - tau : -INFINITY;
  // r06 fast path: for m in [kClassFastLo, kClassFastHi] sigmoid(lo) < sm holds (checked for every
  // such float by ycx_check_sigmoid_monotone), so the widening loop below would leave lo as it is
  // and pm < lo decides alone: no sigmoid of lo for the common row (the fused head: 11 of 78 us)
#ifndef YCX_NO_CLASS_FAST  // development A/B only
  if (m >= kClassFastLo && m <= kClassFastHi && pm < lo) return;
#endif
  for (int i = 0; i < 6 && ycx_sigmoid(lo) == sm; ++i) {  // saturated: widen until sigmoid drops
    tau *= 16.0f;
    lo = m - tau;
  }
  if (ycx_sigmoid(lo) == sm) lo = -INFINITY;  // still tied: every class is a candidate
  if (!(pm >= lo)) return;
  for (int k = 0; k < b; ++k) {  // rare: a class before bi whose sigmoid rounds to sm
    const float v = logit(k);
    if (v >= lo && ycx_sigmoid(v) == sm) {
      bi = k;
      return;
    }
  }
}

// Both halves of the classes as two independent chains (twice the ILP of one scan).
template <class F>
__device__ __forceinline__ void ycx_class_scan2(F&& logit, int nc, float& m, float& pm, int& b) {
  const int c = nc >> 1;
  float m2 = -INFINITY, pm2 = -INFINITY;
  int b2 = -1, k = 1, k2 = c;
  m = logit(0);
  pm = -INFINITY;
  b = 0;
  for (; k + 4 <= c && k2 + 4 <= nc; k += 4, k2 += 4) {
    float v[4], w[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      v[u] = logit(k + u);
      w[u] = logit(k2 + u);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const bool up = v[u] > m, up2 = w[u] > m2;
      pm = up ? m : pm;
      b = up ? k + u : b;
      m = up ? v[u] : m;
      pm2 = up2 ? m2 : pm2;
      b2 = up2 ? k2 + u : b2;
      m2 = up2 ? w[u] : m2;
    }
  }
  ycx_class_scan(logit, k, c, m, pm, b);
  ycx_class_scan(logit, k2, nc, m2, pm2, b2);
  ycx_class_merge(m, pm, b, m2, pm2, b2);
}

template <class F>
__device__ __forceinline__ void ycx_class_argmax(F&& logit, int nc, float& best, int& bi) {
  const float l0 = logit(0);
  if (l0 != l0) {
    best = l0;
    bi = 0;
    return;
  }
  float m, pm;
  int b;
  ycx_class_scan2(logit, nc, m, pm, b);
  ycx_class_finish(logit, m, pm, b, best, bi);
}
