// Implicit-GEMM convolution for gfx950 (CDNA4), NHWC activations.
//
// Replaces Conv.forward = act(bn(conv2d(x))) (nets/common.py:97-109), the
// re-parameterised RepConv (nets/common.py:477-495) and the Detect / IDetect
// 1x1 head convs (nets/detect.py:27-38, nets/idetect.py:26-31). BN, RepConv
// branches and ImplicitA/M are folded into (weight, bias) by the host prepack.
//
// GEMM view: D[co][px] = sum_k Wt[co][k] * X[px][k], k = (ky*kw + kx)*cin + ci.
//   A operand = packed weights  [cout_pad][kh*kw*cin]  (K contiguous)
//   B operand = NHWC activations, im2col-on-the-fly     (K contiguous per tap)
// Both operands are K-major, which is exactly the lane layout of
// v_mfma_f32_16x16x32_bf16 (lane l holds 8 consecutive k of row l&15), so
// every LDS fragment read is one ds_read_b128.
//
// bf16 path: 256 threads = 4 waves, tile BM(co) x BN(px) x BK, register-staged
// double-buffered LDS with an XOR swizzle (conflict-free ds_read_b128, checked
// by brute force), one barrier per K step, XCD-aware block remap, fp32
// accumulate, epilogue = bias + act (+ residual), staged through LDS as fp32 and
// written with 16-byte coalesced stores into a channel slice of the consumer's
// concat buffer (Concat is never materialised).
//
// f32 path ("parity mode"): same structure on v_mfma_f32_16x16x4_f32 (exact
// fp32 FMA chain), used to prove the 1e-3 relative bound vs the fp32 CPU
// reference.
#include <stdlib.h>
#include <algorithm>
#include <type_traits>
#include "ycx_internal.h"

// The 16-bit element type of the MFMA conv kernels. This file is compiled twice:
// as is (bf16: YCX_DT_BF16, and the fp32 / e4m3 paths) and with -DYCX_ELT_F16
// (IEEE half: YCX_DT_F16, same kernels on v_mfma_f32_16x16x32_f16, which runs at
// the bf16 rate with three more mantissa bits). The fp16 build's entry points carry
// an _f16 suffix and are reached through the bf16 build's dtype dispatch.
#ifdef YCX_ELT_F16
typedef _Float16 elt_t;
#define YCX_MFMA16 __builtin_amdgcn_mfma_f32_16x16x32_f16
#define YCX_DT_ELT YCX_DT_F16
#define YCX_SFX(name) name##_f16
#else
typedef __bf16 elt_t;
#define YCX_MFMA16 __builtin_amdgcn_mfma_f32_16x16x32_bf16
#define YCX_DT_ELT YCX_DT_BF16
#define YCX_SFX(name) name
#endif
typedef __attribute__((ext_vector_type(8))) elt_t eltx8;
typedef __attribute__((ext_vector_type(4))) elt_t eltx4;

namespace {

struct ConvArgs {
  const void* x;
  const void* w;
  const float* bias;
  void* y;
  const void* res;
  int N, H, W, Cin, in_coff, in_cs;
  int Ho, Wo, Cout, Cout_pad, out_coff, out_cs;
  int KH, KW, S, P;
  int act;
  float slope;
  int out_layout;
  int res_coff, res_cs;
  int M, HoWo, Ktot, nsteps, n_ct, nwg;
  float out_scale, res_scale;  // YCX_DT_FP8 only
  int pool;                    // x is the (2H, 2W) map of a fused k2 s2 max-pool (ycx_conv_desc.in_pool)
  int gc;                      // LDS-DMA tiles: channel groups of the XCD region map (ycx_tile_of)
  long long out_bytes;         // extent of y the descriptor implies (YCX_DEBUG_BOUNDS store checks)
  int ks;                      // split-K ranges (ycx_conv_desc.k_split; 1: none)
  float* part;                 // ks > 1: fp32 partials [ks][M][Cout_pad] (the caller's workspace)
};
// a store of nb bytes at ptr inside the output extent of args A (always true in release builds)
#define YCX_OUT_OK(A, ptr, nb) \
  YCX_BOUNDS_OK(reinterpret_cast<const char*>(ptr) - reinterpret_cast<const char*>((A).y), (nb), (A).out_bytes)

template <int BK>
__device__ __forceinline__ int swz(int row) {
  if constexpr (BK == 64) return (row >> 1) & 7;
  else return (-(row >> 2)) & 3;
}

// Writes 8 consecutive output channels of pixel p (fp32 values v) to the
// output, NHWC or NHWC-upsampled-x2, adding the residual first if present.
template <typename T>
__device__ __forceinline__ void store8(const ConvArgs& a, int p, int co, float v[8]) {
  if (a.res) {
    const T* r = reinterpret_cast<const T*>(a.res) + (size_t)p * a.res_cs + a.res_coff + co;
    if constexpr (sizeof(T) == 2) {
      eltx8 rv = *reinterpret_cast<const eltx8*>(r);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] += (float)rv[j];
    } else {
      f32x4 r0 = *reinterpret_cast<const f32x4*>(r), r1 = *reinterpret_cast<const f32x4*>(r + 4);
#pragma unroll
      for (int j = 0; j < 4; ++j) { v[j] += r0[j]; v[4 + j] += r1[j]; }
    }
  }
  T* base = reinterpret_cast<T*>(a.y);
  auto put = [&](size_t pix) {
    T* o = base + pix * a.out_cs + a.out_coff + co;
    if constexpr (sizeof(T) == 2) {
      eltx8 ov;
#pragma unroll
      for (int j = 0; j < 8; ++j) ov[j] = (elt_t)v[j];
      if (YCX_OUT_OK(a, o, sizeof(eltx8))) *reinterpret_cast<eltx8*>(o) = ov;
    } else {
      if (YCX_OUT_OK(a, o, sizeof(f32x4))) *reinterpret_cast<f32x4*>(o) = f32x4{v[0], v[1], v[2], v[3]};
      if (YCX_OUT_OK(a, o + 4, sizeof(f32x4))) *reinterpret_cast<f32x4*>(o + 4) = f32x4{v[4], v[5], v[6], v[7]};
    }
  };
  if (a.out_layout == YCX_OUT_NHWC_UP2) {
    int n = p / a.HoWo, rem = p - n * a.HoWo, oy = rem / a.Wo, ox = rem - oy * a.Wo;
    size_t W2 = 2 * (size_t)a.Wo;
    size_t b0 = ((size_t)n * 2 * a.Ho + 2 * oy) * W2 + 2 * ox;
    put(b0); put(b0 + 1); put(b0 + W2); put(b0 + W2 + 1);
  } else {
    put((size_t)p);
  }
}

// Writes 4 consecutive bf16 output channels of pixel p straight from an MFMA
// accumulator (8-byte store; the 4 lane groups of a 16x16 tile complete 32
// contiguous bytes per pixel and L2 merges the lines), residual added first.
__device__ __forceinline__ void store4_bf16(const ConvArgs& a, int p, int co, float v[4]) {
  if (a.res) {
    const eltx4 rv = *reinterpret_cast<const eltx4*>(reinterpret_cast<const elt_t*>(a.res) +
                                                       (size_t)p * a.res_cs + a.res_coff + co);
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] += (float)rv[j];
  }
  eltx4 ov;
#pragma unroll
  for (int j = 0; j < 4; ++j) ov[j] = (elt_t)v[j];
  elt_t* base = reinterpret_cast<elt_t*>(a.y) + a.out_coff + co;
  if (a.out_layout == YCX_OUT_NHWC_UP2) {
    const int n = p / a.HoWo, rem = p - n * a.HoWo, oy = rem / a.Wo, ox = rem - oy * a.Wo;
    const size_t W2 = 2 * (size_t)a.Wo;
    const size_t b0 = ((size_t)n * 2 * a.Ho + 2 * oy) * W2 + 2 * ox;
    if (YCX_OUT_OK(a, base + b0 * a.out_cs, sizeof(eltx4))) *reinterpret_cast<eltx4*>(base + b0 * a.out_cs) = ov;
    if (YCX_OUT_OK(a, base + (b0 + 1) * a.out_cs, sizeof(eltx4))) *reinterpret_cast<eltx4*>(base + (b0 + 1) * a.out_cs) = ov;
    if (YCX_OUT_OK(a, base + (b0 + W2) * a.out_cs, sizeof(eltx4))) *reinterpret_cast<eltx4*>(base + (b0 + W2) * a.out_cs) = ov;
    if (YCX_OUT_OK(a, base + (b0 + W2 + 1) * a.out_cs, sizeof(eltx4))) *reinterpret_cast<eltx4*>(base + (b0 + W2 + 1) * a.out_cs) = ov;
  } else {
    if (YCX_OUT_OK(a, base + (size_t)p * a.out_cs, sizeof(eltx4))) *reinterpret_cast<eltx4*>(base + (size_t)p * a.out_cs) = ov;
  }
}

// -------------------------------------------------------------------------
// bf16 MFMA kernel
// -------------------------------------------------------------------------
template <int BM, int BN, int BK, int WM, int WN>
__global__ void __launch_bounds__(256) conv_bf16_kernel(ConvArgs a) {
  static_assert(WM * WN == 4, "4 waves");
  constexpr int TM = BM / WM, TN = BN / WN;  // per-wave tile (co x px)
  constexpr int FM = TM / 16, FN = TN / 16;  // 16x16 MFMA tiles per wave
  constexpr int CPR = BK / 8;                // 16-byte chunks per LDS row
  constexpr int RPP = 256 / CPR;             // rows covered by one pass of 256 threads
  constexpr int ACH = (BM + RPP - 1) / RPP;  // A chunks per thread
  constexpr int BCH = (BN + RPP - 1) / RPP;  // B chunks per thread
  constexpr int A_EL = BM * BK, B_EL = BN * BK;
  constexpr int STAGE_BYTES = 2 * (A_EL + B_EL) * 2;
  constexpr int CP = BM + 4;                 // fp32 C staging pitch (floats)
  constexpr int C_BYTES = BN * CP * 4;
  constexpr int LDS_BYTES = STAGE_BYTES > C_BYTES ? STAGE_BYTES : C_BYTES;
  __shared__ __attribute__((aligned(16))) char smem[LDS_BYTES];
  elt_t* As = reinterpret_cast<elt_t*>(smem);  // [2][BM*BK]
  elt_t* Bs = As + 2 * A_EL;                    // [2][BN*BK]

  const elt_t* __restrict__ X = reinterpret_cast<const elt_t*>(a.x);
  const elt_t* __restrict__ Wt = reinterpret_cast<const elt_t*>(a.w);

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;
  const int L = ycx_xcd_remap(blockIdx.x, a.nwg);
  const int ct = L % a.n_ct, pt = L / a.n_ct;
  const int co0 = ct * BM, px0 = pt * BN;
  const int ch = tid % CPR;

  // Per-thread B rows: output pixel -> top-left input position.
  int b_iy0[BCH], b_ix0[BCH], b_nh[BCH];
  bool b_ok[BCH];
#pragma unroll
  for (int i = 0; i < BCH; ++i) {
    int row = tid / CPR + i * RPP;
    int p = px0 + row;
    bool ok = (row < BN) && (p < a.M);
    int pp = ok ? p : 0;
    int n = pp / a.HoWo, rem = pp - n * a.HoWo;
    int oy = rem / a.Wo, ox = rem - oy * a.Wo;
    b_iy0[i] = oy * a.S - a.P;
    b_ix0[i] = ox * a.S - a.P;
    b_nh[i] = n * a.H;
    b_ok[i] = ok;
  }

  eltx8 ra[ACH], rb[BCH];
  const eltx8 zero8 = {};
  auto gload = [&](int s, int ky, int kx, int cblk) {
#pragma unroll
    for (int i = 0; i < ACH; ++i) {
      int row = tid / CPR + i * RPP;
      if (row < BM)
        ra[i] = *reinterpret_cast<const eltx8*>(Wt + (size_t)(co0 + row) * a.Ktot + s * BK + ch * 8);
    }
#pragma unroll
    for (int i = 0; i < BCH; ++i) {
      int iy = b_iy0[i] + ky, ix = b_ix0[i] + kx;
      bool ok = b_ok[i] && (unsigned)iy < (unsigned)a.H && (unsigned)ix < (unsigned)a.W;
      rb[i] = ok ? *reinterpret_cast<const eltx8*>(
                       X + ((size_t)(b_nh[i] + iy) * a.W + ix) * a.in_cs + a.in_coff + cblk + ch * 8)
                 : zero8;
    }
  };
  auto lstore = [&](int buf) {
    elt_t* A = As + buf * A_EL;
    elt_t* B = Bs + buf * B_EL;
#pragma unroll
    for (int i = 0; i < ACH; ++i) {
      int row = tid / CPR + i * RPP;
      if (row < BM) *reinterpret_cast<eltx8*>(A + row * BK + ((ch ^ swz<BK>(row)) << 3)) = ra[i];
    }
#pragma unroll
    for (int i = 0; i < BCH; ++i) {
      int row = tid / CPR + i * RPP;
      if (row < BN) *reinterpret_cast<eltx8*>(B + row * BK + ((ch ^ swz<BK>(row)) << 3)) = rb[i];
    }
  };

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto compute = [&](int buf) {
    const elt_t* A = As + buf * A_EL;
    const elt_t* B = Bs + buf * B_EL;
#pragma unroll
    for (int kk = 0; kk < BK / 32; ++kk) {
      const int c = kk * 4 + (lane >> 4);
      eltx8 af[FM], bfr[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        int row = wm * TM + i * 16 + (lane & 15);
        af[i] = *reinterpret_cast<const eltx8*>(A + row * BK + ((c ^ swz<BK>(row)) << 3));
      }
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        int row = wn * TN + j * 16 + (lane & 15);
        bfr[j] = *reinterpret_cast<const eltx8*>(B + row * BK + ((c ^ swz<BK>(row)) << 3));
      }
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = YCX_MFMA16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
  };

  // K loop: step s <-> (tap (ky,kx), channel block cblk).
  int ky = 0, kx = 0, cblk = 0;
  gload(0, 0, 0, 0);
  lstore(0);
  __syncthreads();
  for (int s = 0; s < a.nsteps; ++s) {
    const bool more = s + 1 < a.nsteps;
    if (more) {
      cblk += BK;
      if (cblk == a.Cin) {
        cblk = 0;
        if (++kx == a.KW) { kx = 0; ++ky; }
      }
      gload(s + 1, ky, kx, cblk);
    }
    compute(s & 1);
    if (more) lstore((s + 1) & 1);
    __syncthreads();
  }

  // ---------------- epilogue ----------------
  if (a.out_layout == YCX_OUT_NCHW_F32) {
    float* Y = reinterpret_cast<float*>(a.y);
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        int p = px0 + wn * TN + j * 16 + (lane & 15);
        if (p >= a.M) continue;
        int n = p / a.HoWo, rem = p - n * a.HoWo;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          int co = co0 + wm * TM + i * 16 + (lane >> 4) * 4 + r;
          if (co < a.Cout) {
            float v = ycx_act<true>(acc[i][j][r] + a.bias[co], a.act, a.slope);
            if (YCX_OUT_OK(a, &Y[((size_t)n * a.out_cs + a.out_coff + co) * a.HoWo + rem], sizeof(Y[0]))) Y[((size_t)n * a.out_cs + a.out_coff + co) * a.HoWo + rem] = v;
          }
        }
      }
    return;
  }
  float* Cs = reinterpret_cast<float*>(smem);  // [BN][CP]
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    int col = wm * TM + i * 16 + (lane >> 4) * 4;
    f32x4 bv = *reinterpret_cast<const f32x4*>(a.bias + co0 + col);
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      int row = wn * TN + j * 16 + (lane & 15);
      f32x4 v;
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = ycx_act<true>(acc[i][j][r] + bv[r], a.act, a.slope);
      *reinterpret_cast<f32x4*>(Cs + row * CP + col) = v;
    }
  }
  __syncthreads();
  constexpr int CCH = BM / 8;
  for (int idx = tid; idx < BN * CCH; idx += 256) {
    int row = idx / CCH, c8 = idx - row * CCH;
    int p = px0 + row, co = co0 + c8 * 8;
    if (p >= a.M || co >= a.Cout) continue;
    f32x4 v0 = *reinterpret_cast<const f32x4*>(Cs + row * CP + c8 * 8);
    f32x4 v1 = *reinterpret_cast<const f32x4*>(Cs + row * CP + c8 * 8 + 4);
    float v[8] = {v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
    store8<elt_t>(a, p, co, v);
  }
}

// Epilogue from MFMA accumulators (D[co][px]: px = lane & 15, co = 4(lane>>4) + r
// within each 16x16 fragment): bias + act (+ residual, x2 upsample, fp32 NCHW
// heads) stored straight from registers.
template <int FM, int FN>
__device__ __forceinline__ void epilogue_regs(const ConvArgs& a, const f32x4 (&acc)[FM][FN], int cob, int pxb,
                                              int lane) {
  if (a.out_layout == YCX_OUT_NCHW_F32) {
    float* Y = reinterpret_cast<float*>(a.y);
    f32x4 bb[FM];  // all bias loads first (bias is [cout_pad]): one round trip, not one per element
#pragma unroll
    for (int i = 0; i < FM; ++i) bb[i] = *reinterpret_cast<const f32x4*>(a.bias + cob + i * 16 + (lane >> 4) * 4);
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        int p = pxb + j * 16 + (lane & 15);
        if (p >= a.M) continue;
        int n = p / a.HoWo, rem = p - n * a.HoWo;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          int co = cob + i * 16 + (lane >> 4) * 4 + r;
          if (co < a.Cout)
            if (YCX_OUT_OK(a, &Y[((size_t)n * a.out_cs + a.out_coff + co) * a.HoWo + rem], sizeof(Y[0]))) Y[((size_t)n * a.out_cs + a.out_coff + co) * a.HoWo + rem] =
                ycx_act<true>(acc[i][j][r] + bb[i][r], a.act, a.slope);
        }
      }
    return;
  }
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    const int co = cob + i * 16 + (lane >> 4) * 4;
    if (co >= a.Cout) continue;  // cout % 8 == 0, co % 4 == 0: the 4 channels are all valid
    const f32x4 bv = *reinterpret_cast<const f32x4*>(a.bias + co);
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int p = pxb + j * 16 + (lane & 15);
      if (p >= a.M) continue;
      float v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = ycx_act<true>(acc[i][j][r] + bv[r], a.act, a.slope);
      store4_bf16(a, p, co, v);
    }
  }
}

// act_t over four values with the SiLU's multiplies and add as packed fp32 (v_pk_mul_f32 /
// v_pk_add_f32, two values per instruction): the same IEEE operations in the same order as
// act_t, so bit-identical, with half the plain VALU issues beside the exp / rcp. nl2e is
// -log2(e) held in a VGPR (silu_nl2e()): a packed multiply takes no 32-bit literal.
__device__ __forceinline__ float silu_nl2e() {
  float k = -1.44269504f;
  asm volatile("" : "+v"(k));
  return k;
}

template <int ACT>
__device__ __forceinline__ f32x4 act4_t(f32x4 v, float slope, float nl2e) {
  if constexpr (ACT == YCX_ACT_SILU) {
    const f32x4 t = v * nl2e;
    f32x4 d;
#pragma unroll
    for (int q = 0; q < 4; ++q) d[q] = __builtin_amdgcn_exp2f(t[q]);
    d = 1.0f + d;
#pragma unroll
    for (int q = 0; q < 4; ++q) d[q] = __builtin_amdgcn_rcpf(d[q]);
    return v * d;
  } else if constexpr (ACT == YCX_ACT_SILU_PS) {  // v = k c with k = nl2e (pre-scaled weights): c / (1 + 2^v)
    f32x4 d;
#pragma unroll
    for (int q = 0; q < 4; ++q) d[q] = __builtin_amdgcn_exp2f(v[q]);
    const f32x4 kk = f32x4{nl2e, nl2e, nl2e, nl2e};
    d = __builtin_elementwise_fma(d, kk, kk);
#pragma unroll
    for (int q = 0; q < 4; ++q) d[q] = __builtin_amdgcn_rcpf(d[q]);
    return v * d;
  } else {
    f32x4 r;
#pragma unroll
    for (int q = 0; q < 4; ++q) r[q] = act_t<ACT>(v[q], slope);
    return r;
  }
}

// act4_t with the act code at run time (one uniform branch per call)
__device__ __forceinline__ f32x4 act4(f32x4 v, int act, float slope, float nl2e) {
  if (act == YCX_ACT_SILU_PS) return act4_t<YCX_ACT_SILU_PS>(v, slope, nl2e);
  if (act == YCX_ACT_SILU) return act4_t<YCX_ACT_SILU>(v, slope, nl2e);
  if (act == YCX_ACT_LEAKY) return act4_t<YCX_ACT_LEAKY>(v, slope, nl2e);
  return v;
}

// bias8_prefetch loads the bias of these channels (bias is [cout_pad]: always in bounds)
// before the K loop, so the epilogue does not wait on a load round trip per fragment pair.
template <int FM>
__device__ __forceinline__ void bias8_prefetch(const ConvArgs& a, int cob, int lane, f32x4 (&bp)[FM]) {
#pragma unroll
  for (int k = 0; k < FM / 2; ++k) {
    const int co = cob + 32 * k + 8 * (lane >> 4);
    bp[2 * k] = *reinterpret_cast<const f32x4*>(a.bias + co);
    bp[2 * k + 1] = *reinterpret_cast<const f32x4*>(a.bias + co + 4);
  }
}

// epilogue_regs8 for fragments whose 16 pixels start at arbitrary pixel indices pxf[j].
template <int FM, int FN>
__device__ __forceinline__ void epilogue_frag8(const ConvArgs& a, const f32x4 (&acc)[FM][FN], int cob,
                                               const int (&pxf)[FN], int lane, const f32x4 (&bp)[FM]) {
  const float nl2e = silu_nl2e();
#pragma unroll
  for (int k = 0; k < FM / 2; ++k) {
    const int co = cob + 32 * k + 8 * (lane >> 4);
    if (co >= a.Cout) continue;
    const f32x4 b0 = bp[2 * k], b1 = bp[2 * k + 1];
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const f32x4 x0 = act4(acc[2 * k][j] + b0, a.act, a.slope, nl2e);
      const f32x4 x1 = act4(acc[2 * k + 1][j] + b1, a.act, a.slope, nl2e);
      float v[8];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        v[r] = x0[r];
        v[4 + r] = x1[r];
      }
      store8<elt_t>(a, pxf[j] + (lane & 15), co, v);
    }
  }
}

// NHWC epilogue for permuted A rows (conv_bf16_glds): fragments 2k, 2k+1 hold channels
// cob + 32k + 8g .. +7 in C rows 4g..4g+3 (g = lane >> 4): one 16-byte store per lane and pixel
// (store8: residual and x2 upsample included).

template <int FM, int FN>
__device__ __forceinline__ void epilogue_regs8(const ConvArgs& a, const f32x4 (&acc)[FM][FN], int cob, int pxb,
                                               int lane, const f32x4 (&bp)[FM]) {
  const float nl2e = silu_nl2e();
#pragma unroll
  for (int k = 0; k < FM / 2; ++k) {
    const int co = cob + 32 * k + 8 * (lane >> 4);
    if (co >= a.Cout) continue;  // cout % 8 == 0: the 8 channels are all valid
    const f32x4 b0 = bp[2 * k], b1 = bp[2 * k + 1];
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int p = pxb + j * 16 + (lane & 15);
      if (p >= a.M) continue;
      // bias add and activation as packed fp32 (act4: bit-identical to ycx_act<true>)
      const f32x4 x0 = act4(acc[2 * k][j] + b0, a.act, a.slope, nl2e);
      const f32x4 x1 = act4(acc[2 * k + 1][j] + b1, a.act, a.slope, nl2e);
      float v[8];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        v[r] = x0[r];
        v[4 + r] = x1[r];
      }
      store8<elt_t>(a, p, co, v);
    }
  }
}

// Same, for fragments whose 16 pixels start at arbitrary pixel indices pxf[j].
template <int FM, int FN>
__device__ __forceinline__ void epilogue_frag(const ConvArgs& a, const f32x4 (&acc)[FM][FN], int cob,
                                              const int (&pxf)[FN], int lane) {
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    const int co = cob + i * 16 + (lane >> 4) * 4;
    if (co >= a.Cout) continue;
    const f32x4 bv = *reinterpret_cast<const f32x4*>(a.bias + co);
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      float v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = ycx_act<true>(acc[i][j][r] + bv[r], a.act, a.slope);
      store4_bf16(a, pxf[j] + (lane & 15), co, v);
    }
  }
}

// -------------------------------------------------------------------------
// bf16 MFMA kernel v2: 512 threads (8 waves), BK = 64, 3-stage LDS-DMA
// pipeline. Tiles are filled by global_load_lds_dwordx4 (no VGPR staging, no
// ds_write): each wave-instruction writes 1 KiB = 8 rows x 128 B linearly, so
// the XOR swizzle of the LDS image is applied on the per-lane SOURCE address
// (lane -> physical chunk p, fetches logical chunk p ^ swz(row)) and again on
// the fragment read (guide rule 21). Out-of-image taps and tail rows fetch a
// zero page instead of being masked. Two stages stay in flight: each K step
// waits with a counted vmcnt (never 0 inside the loop) and a raw s_barrier.
// -------------------------------------------------------------------------
typedef __attribute__((address_space(3))) void lds_void;

// 16-byte LDS-DMA through a raw buffer descriptor built from uniform values.
__device__ __forceinline__ void buf_lds16(const void* base, int nbytes, int voff, int soff, void* lds) {
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, nbytes, 0x00020000);
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void*)lds, 16, voff, soff, 0, 0);
}

#ifdef YCX_GLDS_STAMP
// Development build only: per-phase cycle sums of the glds main loop. Each
// stamp is an s_memtime whose result is consumed only at the end of the step
// (one lgkmcnt(0) there, after the MFMAs already waited for the fragments).
__device__ unsigned long long g_glds_stamp[16 * 8 + 1];
__device__ __forceinline__ unsigned long long stamp_issue() {
  unsigned long long v;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memtime %0" : "=s"(v));
  __builtin_amdgcn_sched_barrier(0);
  return v;
}
__device__ __forceinline__ void stamp_sync() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
#define STAMP(k) unsigned long long st_t##k = stamp_issue()
#else
#define STAMP(k) do { } while (0)
#endif

// Fused Detect-head epilogue (tile 38, ycx_conv2d_head): the workgroup holds
// all na * no channels of BN pixels; the biased fp32 logits go through LDS and
// one thread per (pixel, anchor) applies decode_box + the candidate filter of
// detect.py:29-121 with the float operations of ycx_post.hip's
// decode_filter_kernel, in the same order (FMA contraction off here too), so
// the candidates are bit-identical to the unfused path. Optional raw fp32 NCHW
// stores (the compat Model.forward output) are coalesced along pixels.
struct HeadArgs {
  ycx_head_desc h;
  ycx_cand* cand;
  int* rows_out;
  int* counts;
  float* heads;
  int* status;  // nullable: set to YCX_HEAD_NONFINITE when a logit of the tile is inf / NaN
};

// The fp16 range guard (ycx_conv2d_head's status): an activation past the fp16 range
// becomes inf at its producer's store, and inf / NaN reach the heads through every
// later conv. A lane that saw a non-finite logit stores the flag (same value from
// every writer; the flag is only ever set, never cleared, on the device).
__device__ __forceinline__ bool ycx_nonfinite(float v) {
  return (__float_as_uint(v) & 0x7f800000u) == 0x7f800000u;
}
__device__ __forceinline__ void head_flag(const HeadArgs& hd, bool bad) {
  if (bad && hd.status) *reinterpret_cast<volatile int*>(hd.status) = YCX_HEAD_NONFINITE;
}

__device__ __forceinline__ float head_sigmoid(float v) { return ycx_sigmoid(v); }

template <int BN>
__device__ void head_decode_tile(const ConvArgs& a, const HeadArgs& hd, const float* T, int ldt, int px0) {
#pragma clang fp contract(off)
  const ycx_head_desc& h = hd.h;
  const int tid = threadIdx.x, lane = tid & 63;
  const int HW = a.HoWo, W = a.Wo, H = a.Ho;
  if (hd.heads) {  // raw logits, fp32 NCHW: 64 consecutive pixels of one channel per wave-instruction
    for (int e = tid; e < a.Cout * BN; e += blockDim.x) {
      const int c = e / BN, px = e - c * BN, p = px0 + px;
      if (p < a.M) {
        const int n = p / HW, cell = p - n * HW;
        hd.heads[((size_t)n * a.Cout + c) * HW + cell] = T[c * ldt + px];
      }
    }
  }
  // One thread per row an * BN + px (kSplit, measured slower on MI355X: lanes l and l + 32
  // scan the lower and upper half of one row's classes, the lower lane finishes the row).
#ifdef YCX_HEAD_SPLIT
  constexpr bool kSplit = true;
#else
  constexpr bool kSplit = false;
#endif
  const int wid = tid >> 6, upper = kSplit ? lane >> 5 : 0, nrows = h.na * BN;
  const int per = kSplit ? blockDim.x / 2 : blockDim.x;
  const int n0 = px0 / HW;
  const bool two = min(px0 + BN, a.M) - 1 < (n0 + 2) * HW;  // the tile spans one or two images
  const float inv_w = 1.0f / (float)W;
  int* s_cnt = reinterpret_cast<int*>(const_cast<float*>(T) + a.Cout_pad * ldt);  // [16][2] + [2], past the tile
  for (int r0 = 0; r0 < nrows; r0 += per) {  // uniform trip count
    const int r = r0 + (kSplit ? wid * 32 + (lane & 31) : tid);
    const int an = r / BN, px = r - an * BN, p = px0 + px;
    const bool valid = r < nrows && p < a.M;
    int n = 0, cell = 0;
    if (valid) {
      n = p >= (n0 + 1) * HW ? (two ? n0 + 1 : p / HW) : n0;
      cell = p - n * HW;
    }
    const float* L = T + (size_t)(an * h.no) * ldt + px;
    const float obj = valid ? head_sigmoid(L[4 * ldt]) : 0.0f;
    const bool want = valid && obj >= h.conf_thres;  // obj * cls <= obj: otherwise the row cannot pass
    auto logit = [&](int k) { return L[(5 + k) * ldt]; };
    const int c = kSplit ? h.nc >> 1 : h.nc;
    float m = -INFINITY, pm = -INFINITY;
    int b = -1;
    if (want) {
      if (kSplit && upper) {
        ycx_class_scan(logit, c, h.nc, m, pm, b);
      } else if (kSplit) {
        m = logit(0);
        b = 0;
        ycx_class_scan(logit, 1, c, m, pm, b);
      } else {
#if defined(YCX_HEAD_ABL) && YCX_HEAD_ABL == 2  // development timing only: class 0 alone
        m = logit(0);
        b = 0;
#else
        ycx_class_scan2(logit, h.nc, m, pm, b);
#endif
      }
    }
    float m2 = -INFINITY, pm2 = -INFINITY;
    int b2 = -1;
    if constexpr (kSplit) {
      m2 = __shfl_xor(m, 32);
      pm2 = __shfl_xor(pm, 32);
      b2 = __shfl_xor(b, 32);
    }
    bool pass = false;
    ycx_cand cd;
    if (want && !upper) {
      float best;
      int bi;
      if (m != m) {  // NaN at class 0 sticks (the sequential scan's 'sv > NaN' never holds)
        best = m;
        bi = 0;
      } else {
        ycx_class_merge(m, pm, b, m2, pm2, b2);
#if defined(YCX_HEAD_ABL) && YCX_HEAD_ABL == 3  // development timing only: finish = one sigmoid
        best = head_sigmoid(m);
        bi = b;
#else
        ycx_class_finish(logit, m, pm, b, best, bi);
#endif
      }
      const float score = obj * best;
      if (score >= h.conf_thres) {
        int iy = (int)((float)cell * inv_w);  // cell / W: exact after the +-1 fix-up (cell < 2^24)
        iy -= iy * W > cell ? 1 : 0;
        iy += (iy + 1) * W <= cell ? 1 : 0;
        const float gx = (float)(cell - iy * W), gy = (float)iy;
        const float px_ = head_sigmoid(L[0]), py = head_sigmoid(L[ldt]);
        const float pw = head_sigmoid(L[2 * ldt]), ph = head_sigmoid(L[3 * ldt]);
        const float bx = ((px_ * 2.0f) - 0.5f + gx) / (float)W;
        const float by = ((py * 2.0f) - 0.5f + gy) / (float)H;
        const float tw = pw * 2.0f, th = ph * 2.0f;
        const float bw = (tw * tw * h.anchors_scaled[2 * an]) / (float)W;
        const float bhh = (th * th * h.anchors_scaled[2 * an + 1]) / (float)H;
        pass = true;
        cd = ycx_cand{bx - bw / 2.0f, by - bhh / 2.0f, bx + bw / 2.0f, by + bhh / 2.0f, obj, best, bi,
                      h.row_off + an * HW + cell};
      }
    }
#if defined(YCX_HEAD_ABL) && YCX_HEAD_ABL == 4  // development timing only: no append
    if (cd.row == -7) hd.cand[0] = cd;
    continue;
#endif
    if (two) {  // one atomic per (block, image) instead of one per (wave, image)
      const int k = n - n0;
      const unsigned long long q0 = __ballot(pass && k == 0), q1 = __ballot(pass && k == 1);
      if (lane == 0) {
        s_cnt[2 * wid] = __popcll(q0);
        s_cnt[2 * wid + 1] = __popcll(q1);
      }
      __syncthreads();
      if (tid < 2) {
        int tot = 0;
        for (int w = 0; w < (int)(blockDim.x >> 6); ++w) tot += s_cnt[2 * w + tid];
        s_cnt[32 + tid] = tot ? atomicAdd(hd.counts + n0 + tid, tot) : 0;
      }
      __syncthreads();
      if (pass) {
        int slot = s_cnt[32 + k] + __popcll((k ? q1 : q0) & ((1ull << lane) - 1ull));
        for (int w = 0; w < wid; ++w) slot += s_cnt[2 * w + k];
        hd.cand[(size_t)n * h.rows_total + cd.row] = cd;
        if (slot < h.rows_total) hd.rows_out[(size_t)n * h.rows_total + slot] = cd.row;  // counts not reset: no overrun
      }
      __syncthreads();  // s_cnt is reused by the next pass
      continue;
    }
    // tiny maps (a tile over three or more images): wave-aggregated append per image
    unsigned long long rem = __ballot(pass);
    while (rem) {
      const int leader = __ffsll((long long)rem) - 1;
      const int nl = __shfl(n, leader);
      const bool mine = pass && n == nl;
      const unsigned long long q = __ballot(mine);
      int base = 0;
      if (lane == leader) base = atomicAdd(hd.counts + nl, __popcll(q));
      base = __shfl(base, leader);
      if (mine) {
        const int slot = base + __popcll(q & ((1ull << lane) - 1ull));
        hd.cand[(size_t)nl * h.rows_total + cd.row] = cd;
        if (slot < h.rows_total) hd.rows_out[(size_t)nl * h.rows_total + slot] = cd.row;
      }
      rem &= ~q;
    }
  }
}

// TT (two taps per K step) serves Cin == 32: one 64-wide K step spans taps
// 2s and 2s+1, and each lane's logical chunk c = pch ^ swz(row) (constant per
// lane across steps) selects tap 2s + (c >> 2) and channels 8(c & 3). The
// weights stay linear in k, so only the activation side changes; an odd last
// tap fetches zeros on the activation side (its weight chunk is finite).
// NST = 2 halves the LDS so two workgroups share a CU: one block's prologue
// and epilogue then overlap the other's MFMA loop (short-K layers).
// POOL (1x1 / s1 / p0 only): the activation operand is MP's k2 s2 max-pool of the
// (2H, 2W) map x (nets/common.py:25-31), formed while staging: step t issues the
// weight DMA of t + 1 and four 16-byte global loads per pixel row (the 2x2 window),
// and after step t's MFMAs takes their max and writes it to the LDS slot where the
// activation DMA would have put it. The pooled map never reaches HBM.
// SK (split-K, ycx_conv_desc.k_split, r06): gridDim = tiles x a.ks; workgroup (slice, tile) runs
// K steps [slice nsteps / ks, (slice + 1) nsteps / ks) of its tile and stores the raw fp32 sums
// to a.part[slice][M][Cout_pad]; splitk_reduce adds the slices in order, then bias / act /
// residual / store. Logical ids are slice-major, so an XCD's range is mostly one slice.
template <int BM, int BN, int WM, int WN, bool TT, int NST, int NSB = NST, bool HEAD = false, bool POOL = false,
          bool KCM = false, bool SK = false>
__global__ void __launch_bounds__(WM * WN * 64) conv_bf16_glds(ConvArgs a, HeadArgs hd) {
  constexpr int NW = WM * WN;
  static_assert(NW == 4 || NW == 8, "4 or 8 waves");
  static_assert(NST == 2 || NST == 3, "pipeline depth");
  static_assert(NSB == NST || (NST == 2 && NSB == 3), "B ring: as deep as A's, or one deeper (2 / 3)");
  constexpr int BK = 64;
  constexpr int TM = BM / WM, TN = BN / WN;
  constexpr int FM = TM / 16, FN = TN / 16;
  constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2, STAGE = A_BYTES + B_BYTES;
  constexpr int A_PW = BM / (8 * NW), B_PW = BN / (8 * NW);  // wave-instructions (8 rows each) per wave per stage
  constexpr int LPS = A_PW + B_PW;                 // vmcnt per stage per wave
  // NSB == NST: NST stages of [A | B]. NSB > NST (split rings): the activation ring runs one
  // K step further ahead than the weight ring (weights are L2-resident, activations come
  // from HBM / the Infinity Cache): A ring [NST][A_BYTES] then B ring [NSB][B_BYTES].
  constexpr bool SPLIT = NSB != NST;
  constexpr int LDS_BYTES = SPLIT ? NST * A_BYTES + NSB * B_BYTES : NST * STAGE;
  static_assert(A_PW >= 1 && B_PW >= 1 && BM % (8 * NW) == 0 && BN % (8 * NW) == 0, "tile rows per wave");
  constexpr int HEAD_LDT = BN + 1;  // HEAD: fp32 logits [BM][BN + 1] (odd stride: conflict-free writes)
  static_assert(!HEAD || BM * HEAD_LDT * 4 + 34 * 4 <= LDS_BYTES, "head tile (+ append counts) fits the stages");
  static_assert(!HEAD || NW <= 16, "head append counts: 16 waves");
  static_assert(!POOL || (NST == 2 && !SPLIT && !TT && !HEAD), "pooled operand: two-stage [A | B] ring");
  __shared__ __attribute__((aligned(1024))) char smem[LDS_BYTES];

  const elt_t* __restrict__ X = reinterpret_cast<const elt_t*>(a.x);
  const elt_t* __restrict__ Wt = reinterpret_cast<const elt_t*>(a.w);
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
#ifdef YCX_GLDS_STAMP
  unsigned long long st_sum[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  const unsigned long long st_start = stamp_issue();
#endif
  const int wm = wid / WN, wn = wid % WN;
  static_assert(!SK || (!TT && !POOL && !HEAD), "split-K: plain im2col steps");
  int L = ycx_xcd_remap(blockIdx.x, SK ? (int)gridDim.x : a.nwg), slice = 0;
  if constexpr (SK) {
    slice = L / a.nwg;
    L -= slice * a.nwg;
  }
  int ct, pt;
  ycx_tile_of(L, a.n_ct, a.nwg / a.n_ct, a.gc, ct, pt);
  const int co0 = ct * BM, px0 = pt * BN;
  // this workgroup's K steps [s_lo, s_lo + nt)
  const int s_lo = SK ? slice * a.nsteps / a.ks : 0;
  const int lrow = lane >> 3, pch = lane & 7;  // row within the 8-row wave slab, physical chunk

  // Buffer descriptors (raw, stride 0): 32-bit byte offsets, and an offset past
  // num_records makes the LDS-DMA write zeros (measured on gfx950) — the
  // padding taps and the pixel tail cost no branch and no zero page.
  const int w_bytes = a.Cout_pad * a.Ktot * 2, x_bytes = a.N * a.H * a.W * a.in_cs * 2;
  // NHWC outputs with an even fragment count: LDS row wm TM + 16 f + m holds channel
  // wm TM + 32 (f >> 1) + 8 (m >> 2) + 4 (f & 1) + (m & 3), so C rows 4g..4g+3 of fragments 2k and
  // 2k+1 are 8 consecutive channels and the epilogue stores 16 bytes per lane and pixel
  const bool perm = (FM % 2 == 0) && a.out_layout != YCX_OUT_NCHW_F32;
  int a_off[A_PW];
#pragma unroll
  for (int i = 0; i < A_PW; ++i) {
    const int row = 8 * (wid + NW * i) + lrow;
    const int f = (row % TM) >> 4, m = row & 15;
    const int ch = perm ? (row / TM) * TM + 32 * (f >> 1) + 8 * (m >> 2) + 4 * (f & 1) + (m & 3) : row;
    a_off[i] = ((co0 + ch) * a.Ktot + ((pch ^ swz<BK>(row)) << 3)) * 2;
  }
  int b_iy0[B_PW], b_ix0[B_PW], b_base[B_PW];
#pragma unroll
  for (int i = 0; i < B_PW; ++i) {
    const int row = 8 * (wid + NW * i) + lrow;
    const int p = px0 + row;
    const bool ok = p < a.M;
    const int pp = ok ? p : 0;
    const int n = pp / a.HoWo, rem = pp - n * a.HoWo;
    const int oy = rem / a.Wo, ox = rem - oy * a.Wo;
    b_iy0[i] = ok ? oy * a.S - a.P : -(1 << 20);  // tail rows fail the bounds test
    b_ix0[i] = ox * a.S - a.P;
    const int lch = pch ^ swz<BK>(row);  // logical chunk this lane fetches
    if constexpr (POOL)  // element offset of the window's top-left pixel; -1: tail row (zeros)
      b_base[i] = ok ? ((n * 2 * a.H + 2 * oy) * 2 * a.W + 2 * ox) * a.in_cs + a.in_coff + (lch << 3) : -1;
    else
      b_base[i] = (((n * a.H + b_iy0[i]) * a.W + b_ix0[i]) * a.in_cs + a.in_coff + ((TT ? lch & 3 : lch) << 3)) * 2;
  }
  // swz<64>(row) = (4 wid + lrow / 2) & 7 for every i: one tap select per lane.
  const bool sel1 = TT && ((pch ^ swz<BK>(8 * wid + lrow)) >> 2);

  int i_ky = 0, i_kx = 0, i_cb = 0;  // K position (first tap) of the next stage to issue
  const int ntaps = a.KH * a.KW;
  int i_tap = 0;
  if constexpr (SK) {
    if (!KCM) {
      const int cpt = a.Cin / BK, tap = s_lo / cpt;
      i_cb = (s_lo - tap * cpt) * BK;
      i_ky = tap / a.KW;
      i_kx = tap - i_ky * a.KW;
    }
  }
  // Stride-2 3x3s (Cin % 64 == 0) walk K channel-chunk-major with the taps that read the same
  // input pixels next to each other: (ky, kx) = (0,0) (0,2) (0,1) (2,0) (2,2) (2,1) (1,0) (1,2) (1,1)
  // (kx 0 / 2 of neighbouring output pixels share the odd input columns, ky 0 / 2 of neighbouring
  // output rows the odd input rows). In (tap, chunk) order a tap's re-read of a pixel came 4-12 K
  // steps after its first read at Cin 128 (up to 48 at Cin 512), long enough for the concurrent
  // tiles of an XCD to evict it from the 4 MB L2: 1.9-2.5x the input bytes came from beyond the
  // L2 (tests/probes/pmc_s2.sh). Step s is chunk s / 9, tap kTapS2[s % 9]; A follows the same K.
  // A template instance (KCM, launched for 3x3/s2 at Cin 128 only): as a runtime test it cost
  // every tile-16 launch up to 8 % (the uniform branches in both issue paths).
  constexpr bool kcm = KCM;
  static_assert(!KCM || (!TT && !POOL && !HEAD), "K order for plain 3x3/s2 steps");
  constexpr unsigned long long kTapS2 = 0x453786201ull;  // 4 bits per position: taps 0 2 1 6 8 7 3 5 4
  auto k_of = [&](int s) {  // K element offset of step s_lo + s in the packed weight row
    s += s_lo;
    if (!kcm) return s * BK;
    const int c = s / 9, tp = (int)((kTapS2 >> (4 * (s - 9 * c))) & 15);
    return tp * a.Cin + c * BK;
  };
  int i_s = s_lo;  // kcm: B steps issued (absolute)
  auto a_slot = [&](int buf) { return SPLIT ? smem + buf * A_BYTES : smem + buf * STAGE; };
  auto b_slot = [&](int buf) { return SPLIT ? smem + NST * A_BYTES + buf * B_BYTES : smem + buf * STAGE + A_BYTES; };
  auto issueA = [&](int s, int buf) {
    char* base = a_slot(buf);
#pragma unroll
    for (int i = 0; i < A_PW; ++i) buf_lds16(Wt, w_bytes, a_off[i], k_of(s) * 2, base + (wid + NW * i) * 1024);
  };
  auto issueB = [&](int buf) {  // the next K step in (tap, channel) order (kcm: k_of's order)
    char* base = b_slot(buf);
    int ky = i_ky, kx = i_kx;
    if (!TT && !POOL && kcm) {
      const int c = i_s / 9, tp = (int)((kTapS2 >> (4 * (i_s - 9 * c))) & 15);
      ky = tp / 3;
      kx = tp - 3 * ky;
      i_cb = c * BK;
      ++i_s;
    }
    if (TT) {
      // second tap of the pair; past the last tap it can never pass the bounds test
      int ky1 = i_ky, kx1 = i_kx + 1;
      if (kx1 == a.KW) { kx1 = 0; ++ky1; }
      if (i_tap + 1 >= ntaps) ky1 = -(1 << 22);
      ky = sel1 ? ky1 : ky;
      kx = sel1 ? kx1 : kx;
    }
    const int tap = ((ky * a.W + kx) * a.in_cs + i_cb) * 2;
#pragma unroll
    for (int i = 0; i < B_PW; ++i) {
      const bool ok = (unsigned)(b_iy0[i] + ky) < (unsigned)a.H && (unsigned)(b_ix0[i] + kx) < (unsigned)a.W;
      buf_lds16(X, x_bytes, ok ? b_base[i] + tap : 0x7FFFFFF0, 0, base + (wid + NW * i) * 1024);
    }
    if (TT) {
      i_tap += 2;
      i_kx += 2;
      while (i_kx >= a.KW) { i_kx -= a.KW; ++i_ky; }
    } else {
      i_cb += BK;
      if (i_cb == a.Cin) {
        i_cb = 0;
        if (++i_kx == a.KW) { i_kx = 0; ++i_ky; }
      }
    }
  };
  auto issue = [&](int s, int buf) {
    issueA(s, buf);
    issueB(buf);
  };
  // POOL: the window's four rows of the next K step in flight in registers (no VALU on
  // them before the MFMAs, which would wait for the loads), pooled into LDS after them
  eltx8 pw[POOL ? B_PW : 1][4];
  auto loadB = [&]() {
    const int cs = a.in_cs, rs = 2 * a.W * a.in_cs;
#pragma unroll
    for (int i = 0; i < B_PW; ++i) {
      const elt_t* src = X + (b_base[i] < 0 ? 0 : b_base[i] + i_cb);
      pw[i][0] = *reinterpret_cast<const eltx8*>(src);
      pw[i][1] = *reinterpret_cast<const eltx8*>(src + cs);
      pw[i][2] = *reinterpret_cast<const eltx8*>(src + rs);
      pw[i][3] = *reinterpret_cast<const eltx8*>(src + rs + cs);
    }
    i_cb += BK;
  };
  auto writeB = [&](int buf) {
    char* base = b_slot(buf);
#pragma unroll
    for (int i = 0; i < B_PW; ++i) {
      eltx8 v;
#pragma unroll
      for (int j = 0; j < 8; ++j)
        v[j] = (elt_t)fmaxf(fmaxf((float)pw[i][0][j], (float)pw[i][1][j]), fmaxf((float)pw[i][2][j], (float)pw[i][3][j]));
      if (b_base[i] < 0) v = eltx8{};
      *reinterpret_cast<eltx8*>(base + (wid + NW * i) * 1024 + lane * 16) = v;
    }
    // the next raw s_barrier does not wait for LDS stores by itself (gfx950 back-off
    // barrier): complete them here so no wave reads the stage before they land
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  };

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // epilogue bias in registers before the K loop (a load round trip per fragment pair otherwise)
  f32x4 bpre[FM];
  if constexpr (HEAD) {
#pragma unroll
    for (int i = 0; i < FM; ++i) bpre[i] = *reinterpret_cast<const f32x4*>(a.bias + co0 + wm * TM + i * 16 + (lane >> 4) * 4);
  } else if constexpr (FM % 2 == 0 && !POOL) {  // POOL: no registers to spare, loaded after the loop
    if (perm) bias8_prefetch<FM>(a, co0 + wm * TM, lane, bpre);
  }
  const int nt = SK ? (slice + 1) * a.nsteps / a.ks - s_lo : a.nsteps;
  if constexpr (POOL) {
    issueA(0, 0);
    loadB();
    writeB(0);
  } else if constexpr (SPLIT) {
    // prologue A0, B0, B1; step t issues A(t+1) then B(t+2), so at the top of step t the
    // wave's youngest outstanding DMA is B(t+1) (issued after A(t)): vmcnt(B_PW)
    issueA(0, 0);
    issueB(0);
    if (nt > 1) issueB(1);
  } else {
    issue(0, 0);
    if (NST == 3 && nt > 1) issue(1, 1);
  }
#ifdef YCX_GLDS_STAMP
  unsigned long long st_prev = stamp_issue();
  stamp_sync();
  st_sum[0] = st_prev - st_start;
#endif
  for (int t = 0; t < nt; ++t) {
    if constexpr (SPLIT) {
      if (t + 1 < nt) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(B_PW) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
      if (NST == 3 && t + 1 < nt) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(LPS) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    STAMP(1);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    STAMP(2);
    if constexpr (SPLIT) {
      if (t + 1 < nt) issueA(t + 1, (t + 1) % NST);
      if (t + 2 < nt) issueB((t + 2) % NSB);
    } else if constexpr (POOL) {
      if (t + 1 < nt) {
        issueA(t + 1, (t + 1) % NST);
        loadB();
      }
    } else {
      // DMA issued first thing after the barrier: issuing it after the fragment reads or
      // between the MFMA halves measured 4-19 % slower (latency, not issue cost, binds)
      if (t + NST - 1 < nt) issue(t + NST - 1, (t + NST - 1) % NST);
    }
    STAMP(3);
    const elt_t* A = reinterpret_cast<const elt_t*>(a_slot(t % NST));
    const elt_t* B = reinterpret_cast<const elt_t*>(b_slot(t % NSB));
    // all of the stage's fragments are requested before the first MFMA (left to
    // itself the compiler re-reads fragments between MFMAs to save registers,
    // exposing an LDS latency every two MFMAs)
    eltx8 af[BK / 32][FM], bfr[BK / 32][FN];
#pragma unroll
    for (int kk = 0; kk < BK / 32; ++kk) {
      const int c = kk * 4 + (lane >> 4);
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        const int row = wm * TM + i * 16 + (lane & 15);
        af[kk][i] = *reinterpret_cast<const eltx8*>(A + row * BK + ((c ^ swz<BK>(row)) << 3));
      }
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int row = wn * TN + j * 16 + (lane & 15);
        bfr[kk][j] = *reinterpret_cast<const eltx8*>(B + row * BK + ((c ^ swz<BK>(row)) << 3));
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    STAMP(4);
#ifndef YCX_GLDS_NO_SETPRIO  // MFMA phase at raised wave priority (concurrent bench +0.6-1.2 %)
    __builtin_amdgcn_s_setprio(1);
#endif
#pragma unroll
    for (int kk = 0; kk < BK / 32; ++kk)
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = YCX_MFMA16(af[kk][i], bfr[kk][j], acc[i][j], 0, 0, 0);
#ifndef YCX_GLDS_NO_SETPRIO
    __builtin_amdgcn_s_setprio(0);
#endif
    __builtin_amdgcn_sched_barrier(0);
    // slot (t + 1) % 2 held step t - 1, which every wave finished before this step's barrier
    if constexpr (POOL)
      if (t + 1 < nt) writeB((t + 1) % NST);
    STAMP(5);
#ifdef YCX_GLDS_STAMP
    stamp_sync();
    st_sum[1] += st_t1 - st_prev;
    st_sum[2] += st_t2 - st_t1;
    st_sum[3] += st_t3 - st_t2;
    st_sum[4] += st_t4 - st_t3;
    st_sum[5] += st_t5 - st_t4;
    st_prev = st_t5;
#endif
  }
  bool done = false;
  if constexpr (SK) {  // raw fp32 sums: 8 consecutive channels of one pixel per lane and fragment pair
    static_assert(FM % 2 == 0, "split-K partials use the permuted rows");
    float* P = a.part + (size_t)slice * a.M * a.Cout_pad;
#pragma unroll
    for (int k = 0; k < FM / 2; ++k) {
      const int co = co0 + wm * TM + 32 * k + 8 * (lane >> 4);
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int p = px0 + wn * TN + j * 16 + (lane & 15);
        if (p < a.M) {
          float* q = P + (size_t)p * a.Cout_pad + co;
          *reinterpret_cast<f32x4*>(q) = acc[2 * k][j];
          *reinterpret_cast<f32x4*>(q + 4) = acc[2 * k + 1][j];
        }
      }
    }
    done = true;
  }
  if constexpr (HEAD) {
    // every wave is past its last fragment read: the stages become the logit tile
    __syncthreads();
    float* T = reinterpret_cast<float*>(smem);
    const int cob = wm * TM, pxb = wn * TN;
    bool bad = false;
#pragma unroll
    for (int i = 0; i < FM; ++i) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int co = cob + i * 16 + (lane >> 4) * 4 + r;
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          const float v = acc[i][j][r] + bpre[i][r];
          bad |= ycx_nonfinite(v);
          T[co * HEAD_LDT + pxb + j * 16 + (lane & 15)] = v;
        }
      }
    }
    head_flag(hd, bad);
    __syncthreads();
#if defined(YCX_HEAD_ABL) && YCX_HEAD_ABL == 1  // development timing only: the decode skipped
    if (px0 < 0)
#endif
    head_decode_tile<BN>(a, hd, T, HEAD_LDT, px0);
    done = true;
  }
  if constexpr (FM % 2 == 0 && !HEAD && !SK) {
    if (perm) {
      if constexpr (POOL) bias8_prefetch<FM>(a, co0 + wm * TM, lane, bpre);
      epilogue_regs8<FM, FN>(a, acc, co0 + wm * TM, px0 + wn * TN, lane, bpre);
      done = true;
    }
  }
  if constexpr (!HEAD && !SK)
    if (!done) epilogue_regs<FM, FN>(a, acc, co0 + wm * TM, px0 + wn * TN, lane);
#ifdef YCX_GLDS_STAMP
  {
    const unsigned long long e = stamp_issue();
    stamp_sync();
    st_sum[6] = e - st_prev;
    st_sum[7] = e - st_start;
  }
  if (lane < 8) {
    unsigned long long v = 0;
#pragma unroll
    for (int b = 0; b < 8; ++b) v = lane == b ? st_sum[b] : v;
    atomicAdd(&g_glds_stamp[(wid & 15) * 8 + lane], v);
  }
  if (tid == 0) atomicAdd(&g_glds_stamp[128], 1ull);
#endif
}

// Split-K combine (r06): the a.ks fp32 partial sums of every (pixel, 8 channels) added in
// slice order, then bias + act (+ residual, x2 upsample) and the 16-byte store of the
// unsplit epilogue (store8). One thread per (pixel, 8-channel group): consecutive threads
// read consecutive 32-byte runs of a partial row.
template <int ACT>
__global__ void __launch_bounds__(256) splitk_reduce(ConvArgs a) {
  const int ng = a.Cout >> 3;  // cout % 8 == 0
  const long long total = (long long)a.M * ng, slab = (long long)a.M * a.Cout_pad;
  const float nl2e = silu_nl2e();
  for (long long e = (long long)blockIdx.x * 256 + threadIdx.x; e < total; e += (long long)gridDim.x * 256) {
    const int p = (int)(e / ng), co = (int)(e - (long long)p * ng) * 8;
    const float* q = a.part + (size_t)p * a.Cout_pad + co;
    f32x4 s0 = *reinterpret_cast<const f32x4*>(q), s1 = *reinterpret_cast<const f32x4*>(q + 4);
    for (int k = 1; k < a.ks; ++k) {
      q += slab;
      s0 += *reinterpret_cast<const f32x4*>(q);
      s1 += *reinterpret_cast<const f32x4*>(q + 4);
    }
    const f32x4 x0 = act4_t<ACT>(s0 + *reinterpret_cast<const f32x4*>(a.bias + co), a.slope, nl2e);
    const f32x4 x1 = act4_t<ACT>(s1 + *reinterpret_cast<const f32x4*>(a.bias + co + 4), a.slope, nl2e);
    float v[8];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      v[r] = x0[r];
      v[4 + r] = x1[r];
    }
    store8<elt_t>(a, p, co, v);
  }
}

// -------------------------------------------------------------------------
// fp8 (OCP e4m3fn) implicit-GEMM conv on the CDNA4 block-scaled MFMA
// v_mfma_scale_f32_16x16x128_f8f6f4 with unit block scales (E8M0 127): twice
// the bf16 MFMA rate, and half the HBM / LDS bytes per MAC. Same pipeline as
// conv_bf16_glds (two-stage LDS-DMA ring, two workgroups per CU): one K step
// is one 128-byte row per operand = 128 channels, so the LDS image, its
// chunk swizzle and the DMA slabs are the bf16 kernel's byte for byte; a K
// step is ONE MFMA per fragment pair (K = 128) instead of two (K = 2 x 32).
// TPS taps per K step serve cin = 128 / TPS < 128 (64: 2 taps, 32: 4 taps):
// lane chunk lch selects tap TPS*s + lch / (8 / TPS) and bytes 16 (lch % (8 / TPS));
// a tap past the last fetches zeros, and the weight rows are zero-padded to a
// multiple of 128 bytes (ycx.h), so the tail step adds exact zeros.
// Fragments: lane l holds 32 bytes (logical chunks 2(l>>4), 2(l>>4)+1) of row
// l&15 for A (weights) and B (pixels): the same (lane, byte) -> k map on both
// operands, so the contraction pairs equal k whatever the hardware's k order.
// Epilogue: v = act(acc * dq[co] + bias[co]) (+ residual * res_scale), stored
// as e4m3(clamp(v * out_scale, +-448)) (4 bytes per lane), or fp32 NCHW heads.
// -------------------------------------------------------------------------
typedef __attribute__((ext_vector_type(8))) int i32x8;
typedef __attribute__((ext_vector_type(4))) int i32x4;

__device__ __forceinline__ float f8_sat(float v) { return fminf(fmaxf(v, -448.0f), 448.0f); }

// Four fp32 -> four e4m3fn bytes (round to nearest even, saturated first).
__device__ __forceinline__ uint32_t f8x4_pack(float a, float b, float c, float d) {
  int w = __builtin_amdgcn_cvt_pk_fp8_f32(f8_sat(a), f8_sat(b), 0, false);
  w = __builtin_amdgcn_cvt_pk_fp8_f32(f8_sat(c), f8_sat(d), w, true);
  return (uint32_t)w;
}

// Row swizzle of the fp8 128-B LDS rows. An fp8 fragment read takes two
// consecutive 16-B chunks per lane (2g, 2g + 1 of its row, g = lane >> 4), and
// with this swizzle every ds_read_b128 lane group hits 16 distinct bank
// granules for any 16-row-aligned fragment (brute-forced over the four lane
// groups and both reads; the bf16 kernels' swz<64> is 2-way there). The DMA
// slab rows 8 (w + NW i) + lrow give swz8 = f(lrow, w & 1): one logical chunk per lane.
__device__ __forceinline__ int swz8(int row) { return ((row >> 1) & 1) | (((row >> 3) & 1) << 2); }

// 4 consecutive fp8 output channels of pixel p (residual added first, then scaled).
__device__ __forceinline__ void store4_f8(const ConvArgs& a, int p, int co, float v[4]) {
  if (a.res) {
    const int rv = *reinterpret_cast<const int*>(reinterpret_cast<const uint8_t*>(a.res) + (size_t)p * a.res_cs +
                                                 a.res_coff + co);
    v[0] += __builtin_amdgcn_cvt_f32_fp8(rv, 0) * a.res_scale;
    v[1] += __builtin_amdgcn_cvt_f32_fp8(rv, 1) * a.res_scale;
    v[2] += __builtin_amdgcn_cvt_f32_fp8(rv, 2) * a.res_scale;
    v[3] += __builtin_amdgcn_cvt_f32_fp8(rv, 3) * a.res_scale;
  }
  const float s = a.out_scale;
  const uint32_t o = f8x4_pack(v[0] * s, v[1] * s, v[2] * s, v[3] * s);
  uint8_t* base = reinterpret_cast<uint8_t*>(a.y) + a.out_coff + co;
  if (a.out_layout == YCX_OUT_NHWC_UP2) {
    const int n = p / a.HoWo, rem = p - n * a.HoWo, oy = rem / a.Wo, ox = rem - oy * a.Wo;
    const size_t W2 = 2 * (size_t)a.Wo;
    const size_t b0 = ((size_t)n * 2 * a.Ho + 2 * oy) * W2 + 2 * ox;
    if (YCX_OUT_OK(a, base + b0 * a.out_cs, sizeof(uint32_t))) *reinterpret_cast<uint32_t*>(base + b0 * a.out_cs) = o;
    if (YCX_OUT_OK(a, base + (b0 + 1) * a.out_cs, sizeof(uint32_t))) *reinterpret_cast<uint32_t*>(base + (b0 + 1) * a.out_cs) = o;
    if (YCX_OUT_OK(a, base + (b0 + W2) * a.out_cs, sizeof(uint32_t))) *reinterpret_cast<uint32_t*>(base + (b0 + W2) * a.out_cs) = o;
    if (YCX_OUT_OK(a, base + (b0 + W2 + 1) * a.out_cs, sizeof(uint32_t))) *reinterpret_cast<uint32_t*>(base + (b0 + W2 + 1) * a.out_cs) = o;
  } else {
    if (YCX_OUT_OK(a, base + (size_t)p * a.out_cs, sizeof(uint32_t))) *reinterpret_cast<uint32_t*>(base + (size_t)p * a.out_cs) = o;
  }
}

// 8 consecutive fp8 output channels of pixel p (residual added first, then scaled): 8-byte stores.
__device__ __forceinline__ void store8_f8(const ConvArgs& a, int p, int co, float v[8]) {
  if (a.res) {
    const uint2 rv = *reinterpret_cast<const uint2*>(reinterpret_cast<const uint8_t*>(a.res) + (size_t)p * a.res_cs +
                                                     a.res_coff + co);
    v[0] += __builtin_amdgcn_cvt_f32_fp8((int)rv.x, 0) * a.res_scale;
    v[1] += __builtin_amdgcn_cvt_f32_fp8((int)rv.x, 1) * a.res_scale;
    v[2] += __builtin_amdgcn_cvt_f32_fp8((int)rv.x, 2) * a.res_scale;
    v[3] += __builtin_amdgcn_cvt_f32_fp8((int)rv.x, 3) * a.res_scale;
    v[4] += __builtin_amdgcn_cvt_f32_fp8((int)rv.y, 0) * a.res_scale;
    v[5] += __builtin_amdgcn_cvt_f32_fp8((int)rv.y, 1) * a.res_scale;
    v[6] += __builtin_amdgcn_cvt_f32_fp8((int)rv.y, 2) * a.res_scale;
    v[7] += __builtin_amdgcn_cvt_f32_fp8((int)rv.y, 3) * a.res_scale;
  }
  const float s = a.out_scale;
  const uint2 o = make_uint2(f8x4_pack(v[0] * s, v[1] * s, v[2] * s, v[3] * s),
                             f8x4_pack(v[4] * s, v[5] * s, v[6] * s, v[7] * s));
  uint8_t* base = reinterpret_cast<uint8_t*>(a.y) + a.out_coff + co;
  if (a.out_layout == YCX_OUT_NHWC_UP2) {
    const int n = p / a.HoWo, rem = p - n * a.HoWo, oy = rem / a.Wo, ox = rem - oy * a.Wo;
    const size_t W2 = 2 * (size_t)a.Wo;
    const size_t b0 = ((size_t)n * 2 * a.Ho + 2 * oy) * W2 + 2 * ox;
    if (YCX_OUT_OK(a, base + b0 * a.out_cs, sizeof(uint2))) *reinterpret_cast<uint2*>(base + b0 * a.out_cs) = o;
    if (YCX_OUT_OK(a, base + (b0 + 1) * a.out_cs, sizeof(uint2))) *reinterpret_cast<uint2*>(base + (b0 + 1) * a.out_cs) = o;
    if (YCX_OUT_OK(a, base + (b0 + W2) * a.out_cs, sizeof(uint2))) *reinterpret_cast<uint2*>(base + (b0 + W2) * a.out_cs) = o;
    if (YCX_OUT_OK(a, base + (b0 + W2 + 1) * a.out_cs, sizeof(uint2))) *reinterpret_cast<uint2*>(base + (b0 + W2 + 1) * a.out_cs) = o;
  } else {
    if (YCX_OUT_OK(a, base + (size_t)p * a.out_cs, sizeof(uint2))) *reinterpret_cast<uint2*>(base + (size_t)p * a.out_cs) = o;
  }
}

// NHWC fp8 epilogue for permuted A rows: fragments 2k, 2k+1 hold channels cob + 32k + 8g .. +7.
template <int FM, int FN>
__device__ __forceinline__ void epilogue_f8x8(const ConvArgs& a, const f32x4 (&acc)[FM][FN], int cob, int pxb,
                                              int lane) {
  const float* dq = a.bias + a.Cout_pad;
  const float nl2e = silu_nl2e();
  // every bias / dq vector first (bias is [2 cout_pad]: in bounds), one load round trip in all
  f32x4 bb[FM], qq[FM];
#pragma unroll
  for (int k = 0; k < FM / 2; ++k) {
    const int co = cob + 32 * k + 8 * (lane >> 4);
    bb[2 * k] = *reinterpret_cast<const f32x4*>(a.bias + co);
    bb[2 * k + 1] = *reinterpret_cast<const f32x4*>(a.bias + co + 4);
    qq[2 * k] = *reinterpret_cast<const f32x4*>(dq + co);
    qq[2 * k + 1] = *reinterpret_cast<const f32x4*>(dq + co + 4);
  }
#pragma unroll
  for (int k = 0; k < FM / 2; ++k) {
    const int co = cob + 32 * k + 8 * (lane >> 4);
    if (co >= a.Cout) continue;  // cout % 8 == 0
    const f32x4 b0 = bb[2 * k], b1 = bb[2 * k + 1], q0 = qq[2 * k], q1 = qq[2 * k + 1];
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int p = pxb + j * 16 + (lane & 15);
      if (p >= a.M) continue;
      // dequant-fma and activation as packed fp32 (v_pk_fma_f32, act4): bit-identical
      const f32x4 x0 = act4(__builtin_elementwise_fma(acc[2 * k][j], q0, b0), a.act, a.slope, nl2e);
      const f32x4 x1 = act4(__builtin_elementwise_fma(acc[2 * k + 1][j], q1, b1), a.act, a.slope, nl2e);
      float v[8];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        v[r] = x0[r];
        v[4 + r] = x1[r];
      }
      store8_f8(a, p, co, v);
    }
  }
}

template <int FM, int FN>
__device__ __forceinline__ void epilogue_f8(const ConvArgs& a, const f32x4 (&acc)[FM][FN], int cob, int pxb,
                                            int lane) {
  const float* dq = a.bias + a.Cout_pad;
  if (a.out_layout == YCX_OUT_NCHW_F32) {
    float* Y = reinterpret_cast<float*>(a.y);
    f32x4 bb[FM], qq[FM];  // all loads first (bias is [2 cout_pad]): one round trip, not one per element
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const int co = cob + i * 16 + (lane >> 4) * 4;
      bb[i] = *reinterpret_cast<const f32x4*>(a.bias + co);
      qq[i] = *reinterpret_cast<const f32x4*>(dq + co);
    }
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int p = pxb + j * 16 + (lane & 15);
        if (p >= a.M) continue;
        const int n = p / a.HoWo, rem = p - n * a.HoWo;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int co = cob + i * 16 + (lane >> 4) * 4 + r;
          if (co < a.Cout)
            if (YCX_OUT_OK(a, &Y[((size_t)n * a.out_cs + a.out_coff + co) * a.HoWo + rem], sizeof(Y[0]))) Y[((size_t)n * a.out_cs + a.out_coff + co) * a.HoWo + rem] =
                ycx_act<true>(fmaf(acc[i][j][r], qq[i][r], bb[i][r]), a.act, a.slope);
        }
      }
    return;
  }
  const float nl2e = silu_nl2e();
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    const int co = cob + i * 16 + (lane >> 4) * 4;
    if (co >= a.Cout) continue;  // cout % 8 == 0, co % 4 == 0: the 4 channels are all valid
    const f32x4 bv = *reinterpret_cast<const f32x4*>(a.bias + co);
    const f32x4 qv = *reinterpret_cast<const f32x4*>(dq + co);
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int p = pxb + j * 16 + (lane & 15);
      if (p >= a.M) continue;
      // packed fma + act4: bit-identical to fmaf + ycx_act<true>
      const f32x4 x = act4(__builtin_elementwise_fma(acc[i][j], qv, bv), a.act, a.slope, nl2e);
      float v[4] = {x[0], x[1], x[2], x[3]};
      store4_f8(a, p, co, v);
    }
  }
}

// POOL (1x1 / s1 / p0, cin % 128 == 0): the activation operand is MP's k2 s2 max-pool of the
// (2H, 2W) map x, formed while staging as in conv_bf16_glds: step t issues the weight DMA of
// t + 1 and four 16-byte loads per pixel row (the 2x2 window, 16 channels per lane), and after
// step t's MFMAs takes the max in fp32 in ycx_maxpool's window order and writes the re-encoded
// bytes (exact: the max is one of the inputs) where the activation DMA would have put them.
template <int BM, int BN, int WM, int WN, int TPS, bool HEAD = false, bool POOL = false>
__global__ void __launch_bounds__(WM * WN * 64, POOL ? 4 : 1) conv_f8_glds(ConvArgs a, HeadArgs hd) {  // POOL: 2 blocks / CU
  constexpr int NW = WM * WN, NST = 2;
  static_assert(NW == 4 || NW == 8, "4 or 8 waves");
  static_assert(TPS == 0 || TPS == 1 || TPS == 2 || TPS == 4, "taps per K step (0: any cin % 16 == 0)");
  static_assert(!POOL || (TPS == 1 && !HEAD), "pooled operand: one tap of 128 channels per K step");
  constexpr int RB = 128;                   // bytes per operand row per K step
  constexpr int TM = BM / WM, TN = BN / WN;
  constexpr int FM = TM / 16, FN = TN / 16;
  constexpr int A_BYTES = BM * RB, B_BYTES = BN * RB, STAGE = A_BYTES + B_BYTES;
  constexpr int A_PW = BM / (8 * NW), B_PW = BN / (8 * NW);
  constexpr int CPT = TPS ? 8 / TPS : 1;    // 16-byte chunks per tap
  static_assert(A_PW >= 1 && B_PW >= 1 && BM % (8 * NW) == 0 && BN % (8 * NW) == 0, "tile rows per wave");
  __shared__ __attribute__((aligned(1024))) char smem[NST * STAGE];

  const uint8_t* __restrict__ X = reinterpret_cast<const uint8_t*>(a.x);
  const uint8_t* __restrict__ Wt = reinterpret_cast<const uint8_t*>(a.w);
  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / WN, wn = wid % WN;
  const int L = ycx_xcd_remap(blockIdx.x, a.nwg);
  int ct, pt;
  ycx_tile_of(L, a.n_ct, a.nwg / a.n_ct, a.gc, ct, pt);
  const int co0 = ct * BM, px0 = pt * BN;
  const int lrow = lane >> 3, pch = lane & 7;

  const int w_bytes = a.Cout_pad * a.Ktot, x_bytes = a.N * a.H * a.W * a.in_cs;
  // NHWC outputs: permuted A rows as in conv_bf16_glds (8 channels, 8 bytes per lane and pixel)
  const bool perm = a.out_layout != YCX_OUT_NCHW_F32;
  int a_off[A_PW];
#pragma unroll
  for (int i = 0; i < A_PW; ++i) {
    const int row = 8 * (wid + NW * i) + lrow;
    const int f = (row % TM) >> 4, m = row & 15;
    const int ch = perm ? (row / TM) * TM + 32 * (f >> 1) + 8 * (m >> 2) + 4 * (f & 1) + (m & 3) : row;
    a_off[i] = (co0 + ch) * a.Ktot + ((pch ^ swz8(row)) << 4);
  }
  // swz8(8 (wid + NW i) + lrow) depends on lrow and wid & 1 only (NW even): the logical
  // chunk (so the tap select) of a lane is the same in all its slabs.
  const int lch = pch ^ swz8(8 * wid + lrow);
  // TPS 0: lane chunk k = 128 s + 16 lch -> (tap, channel) = divmod(k, cin), tracked per lane
  const int tsel = TPS == 1 ? 0 : TPS == 0 ? (16 * lch) / a.Cin : lch / CPT;
  const int cbyte = TPS == 0 ? 0 : (TPS == 1 ? lch : lch % CPT) << 4;
  int b_iy0[B_PW], b_ix0[B_PW], b_base[B_PW];
#pragma unroll
  for (int i = 0; i < B_PW; ++i) {
    const int row = 8 * (wid + NW * i) + lrow;
    const int p = px0 + row;
    const bool ok = p < a.M;
    const int pp = ok ? p : 0;
    const int n = pp / a.HoWo, rem = pp - n * a.HoWo;
    const int oy = rem / a.Wo, ox = rem - oy * a.Wo;
    b_iy0[i] = ok ? oy * a.S - a.P : -(1 << 20);  // tail rows fail the bounds test
    b_ix0[i] = ox * a.S - a.P;
    if constexpr (POOL)  // byte offset of the window's top-left pixel; -1: tail row (zeros)
      b_base[i] = ok ? ((n * 2 * a.H + 2 * oy) * 2 * a.W + 2 * ox) * a.in_cs + a.in_coff + cbyte : -1;
    else
      b_base[i] = ((n * a.H + b_iy0[i]) * a.W + b_ix0[i]) * a.in_cs + a.in_coff + cbyte;
  }
  // this lane's tap for the next stage to issue (TPS > 1), or the block-wide
  // (tap, channel block) position (TPS == 1)
  const int ntaps = a.KH * a.KW;
  int l_tap = tsel, ky = tsel / a.KW, kx = tsel - (tsel / a.KW) * a.KW;
  int cb = TPS == 0 ? 16 * lch - tsel * a.Cin : 0;
  auto issueA = [&](int s, int buf) {
    char* base = smem + buf * STAGE;
    if constexpr (POOL) {  // the weight-row offsets rebuilt per step from an opaque lane id, as the fragment addresses
      int l = lane;
      asm volatile("" : "+v"(l));
      const int lr = l >> 3, pc = l & 7;
#pragma unroll
      for (int i = 0; i < A_PW; ++i) {
        const int row = 8 * (wid + NW * i) + lr;
        const int f = (row % TM) >> 4, m = row & 15;
        const int ch = perm ? (row / TM) * TM + 32 * (f >> 1) + 8 * (m >> 2) + 4 * (f & 1) + (m & 3) : row;
        buf_lds16(Wt, w_bytes, (co0 + ch) * a.Ktot + ((pc ^ swz8(row)) << 4), s * RB, base + (wid + NW * i) * 1024);
      }
    } else {
#pragma unroll
      for (int i = 0; i < A_PW; ++i) buf_lds16(Wt, w_bytes, a_off[i], s * RB, base + (wid + NW * i) * 1024);
    }
  };
  // POOL: the window's four 16-byte rows of the next K step in flight in registers, pooled
  // into LDS after the MFMAs (no VALU on them before, which would wait for the loads)
  int4 pw[POOL ? B_PW : 1][4];
  int pcb = 0;  // channel byte of the next pooled K step
  auto loadB = [&]() {
    const int cs = a.in_cs, rs = 2 * a.W * a.in_cs;
#pragma unroll
    for (int i = 0; i < B_PW; ++i) {
      const uint8_t* src = X + (b_base[i] < 0 ? 0 : b_base[i] + pcb);
      pw[i][0] = *reinterpret_cast<const int4*>(src);
      pw[i][1] = *reinterpret_cast<const int4*>(src + cs);
      pw[i][2] = *reinterpret_cast<const int4*>(src + rs);
      pw[i][3] = *reinterpret_cast<const int4*>(src + rs + cs);
    }
    pcb += RB;
  };
  auto writeB = [&](int buf) {
    char* base = smem + buf * STAGE + A_BYTES;
#pragma unroll
    for (int i = 0; i < B_PW; ++i) {
      int o[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int w0 = q == 0 ? pw[i][0].x : q == 1 ? pw[i][0].y : q == 2 ? pw[i][0].z : pw[i][0].w;
        const int w1 = q == 0 ? pw[i][1].x : q == 1 ? pw[i][1].y : q == 2 ? pw[i][1].z : pw[i][1].w;
        const int w2 = q == 0 ? pw[i][2].x : q == 1 ? pw[i][2].y : q == 2 ? pw[i][2].z : pw[i][2].w;
        const int w3 = q == 0 ? pw[i][3].x : q == 1 ? pw[i][3].y : q == 2 ? pw[i][3].z : pw[i][3].w;
        // ycx_maxpool's order: (0,0), (0,1), (1,0), (1,1), from -inf
#define YCX_F8_MAX4(J)                                                                     \
  fmaxf(fmaxf(fmaxf(fmaxf(-INFINITY, __builtin_amdgcn_cvt_f32_fp8(w0, J)),               \
                    __builtin_amdgcn_cvt_f32_fp8(w1, J)), __builtin_amdgcn_cvt_f32_fp8(w2, J)), \
        __builtin_amdgcn_cvt_f32_fp8(w3, J))
        o[q] = b_base[i] < 0 ? 0 : (int)f8x4_pack(YCX_F8_MAX4(0), YCX_F8_MAX4(1), YCX_F8_MAX4(2), YCX_F8_MAX4(3));
#undef YCX_F8_MAX4
      }
      *reinterpret_cast<int4*>(base + (wid + NW * i) * 1024 + lane * 16) = int4{o[0], o[1], o[2], o[3]};
    }
    // the next raw s_barrier does not wait for LDS stores by itself: complete them here
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  };
  auto issue = [&](int s, int buf) {
    issueA(s, buf);
    char* base = smem + buf * STAGE;
    const bool tap_ok = TPS == 1 || l_tap < ntaps;
    const int tap = (ky * a.W + kx) * a.in_cs + cb;
#pragma unroll
    for (int i = 0; i < B_PW; ++i) {
      const bool ok = tap_ok && (unsigned)(b_iy0[i] + ky) < (unsigned)a.H &&
                      (unsigned)(b_ix0[i] + kx) < (unsigned)a.W;
      buf_lds16(X, x_bytes, ok ? b_base[i] + tap : 0x7FFFFFF0, 0, base + A_BYTES + (wid + NW * i) * 1024);
    }
    if (TPS == 1) {
      cb += RB;
      if (cb == a.Cin) {
        cb = 0;
        if (++kx == a.KW) { kx = 0; ++ky; }
      }
    } else if (TPS == 0) {
      cb += RB;
      while (cb >= a.Cin) {
        cb -= a.Cin;
        ++l_tap;
        if (++kx == a.KW) { kx = 0; ++ky; }
      }
    } else {
      l_tap += TPS;
      kx += TPS;
      while (kx >= a.KW) { kx -= a.KW; ++ky; }
    }
  };

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nt = a.nsteps;
  if constexpr (POOL) {
    issueA(0, 0);
    loadB();
    writeB(0);
  } else {
    issue(0, 0);
  }
  for (int t = 0; t < nt; ++t) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (POOL) {
      if (t + 1 < nt) {
        issueA(t + 1, (t + 1) & 1);
        loadB();
      }
    } else {
      if (t + 1 < nt) issue(t + 1, (t + 1) & 1);
    }
    const char* A = smem + (t & 1) * STAGE;
    const char* B = A + A_BYTES;
    // POOL keeps the next step's window rows (8 B_PW VGPRs) live across the MFMAs: there the A
    // fragments come in two halves, the second half's LDS reads issued behind the first half's
    // MFMAs, so the loop fits the 128 VGPRs of two blocks per CU
    constexpr int AH = POOL ? 2 : 1, FMH = FM / AH;
    static_assert(FM % AH == 0, "A fragment halves");
    // POOL: the fragment addresses rebuilt per step from an opaque lane id (hoisted out of the
    // loop they are a dozen more live VGPRs)
    int ln = lane;
    if constexpr (POOL) asm volatile("" : "+v"(ln));
    const int c0 = 2 * (ln >> 4);
    auto load_a = [&](int i) {
      const int row = wm * TM + i * 16 + (ln & 15);
      const i32x4 lo = *reinterpret_cast<const i32x4*>(A + row * RB + ((c0 ^ swz8(row)) << 4));
      const i32x4 hi = *reinterpret_cast<const i32x4*>(A + row * RB + (((c0 + 1) ^ swz8(row)) << 4));
      return i32x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    };
    i32x8 af[FMH], bfr[FN];
#pragma unroll
    for (int i = 0; i < FMH; ++i) af[i] = load_a(i);
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int row = wn * TN + j * 16 + (ln & 15);
      const i32x4 lo = *reinterpret_cast<const i32x4*>(B + row * RB + ((c0 ^ swz8(row)) << 4));
      const i32x4 hi = *reinterpret_cast<const i32x4*>(B + row * RB + (((c0 + 1) ^ swz8(row)) << 4));
      bfr[j] = i32x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int h = 0; h < AH; ++h) {
      if (h > 0) {
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int i = 0; i < FMH; ++i) af[i] = load_a(FMH * h + i);
        __builtin_amdgcn_sched_barrier(0);
      }
#pragma unroll
      for (int i = 0; i < FMH; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[FMH * h + i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(af[i], bfr[j], acc[FMH * h + i][j], 0,
                                                                                0, 0, 127, 0, 127);
    }
    __builtin_amdgcn_sched_barrier(0);
    // slot (t + 1) & 1 held step t - 1, which every wave finished before this step's barrier
    if constexpr (POOL)
      if (t + 1 < nt) writeB((t + 1) & 1);
  }
  static_assert(FM % 2 == 0, "fragment pairs");
  if constexpr (HEAD) {
    // Detect head (tile 39): the fp32 logits act(acc * dq + bias) of all BM channels of BN
    // pixels to LDS (the unfused epilogue_f8's expression, so the candidates are the same),
    // then the decode + filter of conv_bf16_glds's head tile
    constexpr int HEAD_LDT = BN + 1;
    static_assert(BM * HEAD_LDT * 4 + 34 * 4 <= NST * STAGE, "head tile (+ append counts) fits the stages");
    const float* dq = a.bias + a.Cout_pad;
    f32x4 bb[FM], qq[FM];
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const int co = co0 + wm * TM + i * 16 + (lane >> 4) * 4;
      bb[i] = *reinterpret_cast<const f32x4*>(a.bias + co);
      qq[i] = *reinterpret_cast<const f32x4*>(dq + co);
    }
    __syncthreads();  // every wave is past its last fragment read: the stages become the logit tile
    float* T = reinterpret_cast<float*>(smem);
    bool bad = false;
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int co = wm * TM + i * 16 + (lane >> 4) * 4 + r;
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          const float v = fmaf(acc[i][j][r], qq[i][r], bb[i][r]);
          bad |= ycx_nonfinite(v);
          T[co * HEAD_LDT + wn * TN + j * 16 + (lane & 15)] = v;
        }
      }
    head_flag(hd, bad);
    __syncthreads();
    head_decode_tile<BN>(a, hd, T, HEAD_LDT, px0);
  } else {
    if (perm) epilogue_f8x8<FM, FN>(a, acc, co0 + wm * TM, px0 + wn * TN, lane);
    else epilogue_f8<FM, FN>(a, acc, co0 + wm * TM, px0 + wn * TN, lane);
  }
}

// -------------------------------------------------------------------------
// 3x3 stride-1 conv from an LDS halo tile. A block owns a 16x16 output tile of
// one image and BM output channels. Per 64-channel input chunk the (16+2)^2
// halo (41.5 KB) is DMA'd into LDS ONCE and all nine taps build their B
// fragments from it (the im2col path re-fetches every input pixel nine
// times); the weights of one (tap, chunk) step, BM x 64, stream through
// NSTA LDS-DMA stages. Halo pixel h keeps its 16-B channel chunk q at slot
// q ^ (h & 7): the MFMA B reads (16 consecutive pixels x 4 chunk groups) hit
// 16 distinct bank slots per LDS cycle (brute-forced over every halo offset).
// Requires H == Ho, W == Wo, Ho % 16 == Wo % 16 == 0, Cin % 64 == 0.
// -------------------------------------------------------------------------
// -------------------------------------------------------------------------
// 3x3/s1 conv, 64 -> 64 channels, weight-stationary (yolov7's 320^2 / 160^2
// ELAN 3x3s): the per-tile halo kernel above pulls all nine taps of weights
// (72 KB) into LDS for every 16x16 tile, more bytes than the tile's halo
// (41.5 KB); at 320^2 that is 0.94 GB of L2 -> LDS traffic per layer. Here
// one 512-thread block per CU loads the weights into LDS once ([tap][co] rows
// of 128 B, chunk-swizzled as the im2col tiles' A image) and walks a
// contiguous range of tiles; the halo of tile i + 1 is DMA'd into the second
// of two halo buffers while tile i computes (no barrier inside a tile). Wave
// (wm, wn): channels 32 wm .. +31, tile rows 4 wn .. +3. The epilogue's
// FM x FN stores per wave are counted into the next tile's wait.
// Requires Cin == Cout_pad == 64, H == Ho, W == Wo, both % 16 == 0, NHWC bf16
// output without residual.
// -------------------------------------------------------------------------
template <int ACT>
__global__ void __launch_bounds__(512) conv3x3_ws64(ConvArgs a) {
  constexpr int NW = 8, TH = 16, TW = 16, HW = TW + 2, HP = (TH + 2) * HW;  // 324 halo pixels
  constexpr int HPIECES = (HP + 7) / 8, HPW = (HPIECES + NW - 1) / NW;     // 1-KB DMA pieces (8 pixels)
  constexpr int HBUF = HPIECES * 1024, WBYTES = 9 * 64 * 128;
  constexpr int FM = 2, FN = 4;
  __shared__ __attribute__((aligned(1024))) char smem[WBYTES + 2 * HBUF];
  const float nl2e = silu_nl2e();
  char* const wl = smem;
  const elt_t* __restrict__ X = reinterpret_cast<const elt_t*>(a.x);
  const elt_t* __restrict__ Wt = reinterpret_cast<const elt_t*>(a.w);
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 2, wn = wid & 3;
  const int lrow = lane >> 3, pch = lane & 7;
  const int tx_n = a.Wo / TW, tpi = (a.Ho / TH) * tx_n, ntiles = a.N * tpi;
  const int blk = ycx_xcd_remap(blockIdx.x, gridDim.x);
  const int tb = (int)((long long)blk * ntiles / gridDim.x), te = (int)((long long)(blk + 1) * ntiles / gridDim.x);
  if (tb >= te) return;
  const int w_bytes = a.Cout_pad * a.Ktot * 2, x_bytes = a.N * a.H * a.W * a.in_cs * 2;

  // weights: LDS row R = 64 tap + co (128 B), logical chunk q at q ^ swz(co); 72 pieces, 9 per wave.
  // LDS row co holds channel 32 (co >> 5) + 8 (m >> 2) + 4 f + (m & 3) (f = co >> 4 & 1, m = co & 15):
  // C rows 4g..4g+3 of the two fragments are channels 32 wm + 8g .. +7, one 16-byte store per lane
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    const int R = 8 * (wid + NW * i) + lrow, t = R >> 6, co = R & 63, m = co & 15;
    const int ch = (co & 32) + 8 * (m >> 2) + 4 * ((co >> 4) & 1) + (m & 3);
    buf_lds16(Wt, w_bytes, (ch * a.Ktot + t * 64 + ((pch ^ swz<64>(co)) << 3)) * 2, 0, wl + (wid + NW * i) * 1024);
  }
  // halo of a tile into buffer b: halo pixel h keeps its chunk q at q ^ (h & 7)
  auto issue_h = [&](int tile, int b) {
    const int n = tile / tpi, ti = tile - n * tpi;
    const int oy0 = (ti / tx_n) * TH, ox0 = (ti % tx_n) * TW;
#pragma unroll
    for (int i = 0; i < HPW; ++i) {
      const int piece = wid + NW * i;
      if (piece >= HPIECES) break;  // uniform
      const int h = 8 * piece + lrow, hy = h / HW, hx = h - hy * HW;
      const int iy = oy0 - 1 + hy, ix = ox0 - 1 + hx;
      const bool ok = h < HP && (unsigned)iy < (unsigned)a.H && (unsigned)ix < (unsigned)a.W;
      buf_lds16(X, x_bytes, ok ? (((n * a.H + iy) * a.W + ix) * a.in_cs + a.in_coff + ((pch ^ (h & 7)) << 3)) * 2
                               : 0x7FFFFFF0, 0, smem + WBYTES + b * HBUF + piece * 1024);
    }
  };
  issue_h(tb, 0);
  f32x4 bv[FM];
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    const int co = 32 * wm + 8 * (lane >> 4) + 4 * i;
    bv[i] = co < a.Cout ? *reinterpret_cast<const f32x4*>(a.bias + co) : f32x4{0.f, 0.f, 0.f, 0.f};
  }
  const bool exact = a.Cout == 64;  // then every tile stores FN times per wave
  elt_t* __restrict__ Y = reinterpret_cast<elt_t*>(a.y) + a.out_coff;

  for (int tile = tb; tile < te; ++tile) {
    const int b = (tile - tb) & 1;
    if (tile > tb && exact) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(FN) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();  // this tile's halo (and the weights) landed; the other buffer is free
    if (tile + 1 < te) issue_h(tile + 1, b ^ 1);
    const char* halo = smem + WBYTES + b * HBUF;
    f32x4 acc[FM][FN];
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[i][j] = bv[i];
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int ky = t / 3, kx = t - 3 * ky;
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        const int lc = kk * 4 + (lane >> 4);
        eltx8 af[FM], bfr[FN];
#pragma unroll
        for (int i = 0; i < FM; ++i) {
          const int co = 32 * wm + 16 * i + (lane & 15);
          af[i] = *reinterpret_cast<const eltx8*>(wl + (t * 64 + co) * 128 + ((lc ^ swz<64>(co)) << 4));
        }
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          const int h = (wn * FN + j + ky) * HW + (lane & 15) + kx;
          bfr[j] = *reinterpret_cast<const eltx8*>(halo + h * 128 + ((lc ^ (h & 7)) << 4));
        }
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j)
            acc[i][j] = YCX_MFMA16(af[i], bfr[j], acc[i][j], 0, 0, 0);
      }
    }
    // epilogue: act, 16-byte stores from registers (no global loads: they would drain vmcnt)
    const int n = tile / tpi, ti = tile - n * tpi;
    const int oy0 = (ti / tx_n) * TH, ox0 = (ti % tx_n) * TW;
    const int co = 32 * wm + 8 * (lane >> 4);
    if (co < a.Cout) {  // cout % 8 == 0: the 8 channels are all valid
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int p = n * a.HoWo + (oy0 + wn * FN + j) * a.Wo + ox0 + (lane & 15);
        eltx8 ov;
#pragma unroll
        for (int i = 0; i < FM; ++i) {
          const f32x4 x = act4_t<ACT>(acc[i][j], a.slope, nl2e);
#pragma unroll
          for (int q = 0; q < 4; ++q) ov[4 * i + q] = (elt_t)x[q];
        }
        if (YCX_OUT_OK(a, Y + (size_t)p * a.out_cs + co, sizeof(eltx8))) *reinterpret_cast<eltx8*>(Y + (size_t)p * a.out_cs + co) = ov;
      }
    }
  }
}

// -------------------------------------------------------------------------
// 3x3/s2 conv, 64 -> <= 128 channels, weights in VGPRs (tile 50: yolov7's 320^2 -> 160^2
// 64 -> 128 downsample). The im2col tile 16 pulls every input pixel through LDS ~2.25
// times plus the whole 147 KB weight tensor per 128-pixel tile (~2.3 KB of LDS-DMA per
// output pixel). Here one 512-thread block per CU keeps each wave's 32 output channels x
// 576 K of weights in registers (36 A fragments) across a contiguous range of TH x 16
// output tiles and DMAs only each tile's (2 TH + 1) x 33 input halo (594 B per output pixel
// at TH = 4),
// double-buffered as in conv3x3_ws64. Halo columns are stored split by parity (the 17
// even columns, then the 16 odd ones), so at every tap a fragment's 16 output pixels
// read 16 consecutive halo slots; slot h keeps chunk q at q ^ (h & 7).
// Wave (wm, wn): channels 32 wm .. +31, tile rows TH / 2 * wn .. +TH / 2. TH = 4 keeps the
// 144 weight VGPRs, 16 accumulators and 8 B fragments under the 256 registers of two waves
// per SIMD (TH = 8 spills).
// Requires Cin == 64, Cout_pad == 128, pad 1, Ho % TH == Wo % 16 == 0, NHWC output
// without residual.
// -------------------------------------------------------------------------
// s_waitcnt vmcnt(n) for a wave-uniform runtime n (the largest case <= n; I is the cap)
template <int I>
__device__ __forceinline__ void vm_wait_le(int n) {
  if constexpr (I > 0) {
    if (n >= I) {
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(I) : "memory");
      return;
    }
    vm_wait_le<I - 1>(n);
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
}

template <int ACT, int TH, int NB>
__global__ void __launch_bounds__(512) conv3x3s2_wsr(ConvArgs a) {
  constexpr int NW = 8, TW = 16, HC = 2 * TW + 1, HP = (2 * TH + 1) * HC;  // 17 x 33 halo pixels
  constexpr int HEVEN = TW + 1;                                                   // even columns: slots 0..16
  constexpr int HPIECES = (HP + 7) / 8, HPW = (HPIECES + NW - 1) / NW;           // 1-KB DMA pieces (8 pixels)
  constexpr int HBUF = HPIECES * 1024;
  constexpr int FM = 2, FN = TH / 2;
  static_assert(NB >= 2 && NB * HBUF <= 160 * 1024, "halo ring in LDS");
  __shared__ __attribute__((aligned(1024))) char smem[NB * HBUF];
  const float nl2e = silu_nl2e();
  const elt_t* __restrict__ X = reinterpret_cast<const elt_t*>(a.x);
  const elt_t* __restrict__ Wt = reinterpret_cast<const elt_t*>(a.w);
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int nh = (HPIECES - wid + NW - 1) / NW;  // this wave's halo DMAs per tile
  const int lrow = lane >> 3, pch = lane & 7;
  const int tx_n = a.Wo / TW, tpi = (a.Ho / TH) * tx_n, ntiles = a.N * tpi;
  const int blk = ycx_xcd_remap(blockIdx.x, gridDim.x);
  const int tb = (int)((long long)blk * ntiles / gridDim.x), te = (int)((long long)(blk + 1) * ntiles / gridDim.x);
  if (tb >= te) return;
  const int x_bytes = a.N * a.H * a.W * a.in_cs * 2;

  auto issue_h = [&](int tile, int b) {
    const int n = tile / tpi, ti = tile - n * tpi;
    const int iy0 = 2 * (ti / tx_n) * TH - 1, ix0 = 2 * (ti % tx_n) * TW - 1;
#pragma unroll
    for (int i = 0; i < HPW; ++i) {
      const int piece = wid + NW * i;
      if (piece >= HPIECES) break;  // uniform
      const int h = 8 * piece + lrow, hy = h / HC, s = h - hy * HC;
      const int iy = iy0 + hy, ix = ix0 + (s < HEVEN ? 2 * s : 2 * (s - HEVEN) + 1);
      const bool ok = h < HP && (unsigned)iy < (unsigned)a.H && (unsigned)ix < (unsigned)a.W;
      buf_lds16(X, x_bytes, ok ? (((n * a.H + iy) * a.W + ix) * a.in_cs + a.in_coff + ((pch ^ (h & 7)) << 3)) * 2
                               : 0x7FFFFFF0, 0, smem + b * HBUF + piece * 1024);
    }
  };
  issue_h(tb, 0);
  // A fragments of all nine taps: row m of fragment i is channel 32 wm + 8 (m >> 2) + 4 i + (m & 3),
  // so C rows 4g..4g+3 of the two fragments are channels 32 wm + 8g .. +7 (one 16-byte store per lane)
  eltx8 wf[9][2][FM];
  {
    const int m = lane & 15;
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const elt_t* wr = Wt + (size_t)(32 * wm + 8 * (m >> 2) + 4 * i + (m & 3)) * a.Ktot + 8 * (lane >> 4);
#pragma unroll
      for (int t = 0; t < 9; ++t)
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) wf[t][kk][i] = *reinterpret_cast<const eltx8*>(wr + t * 64 + 32 * kk);
    }
  }
  f32x4 bv[FM];
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    const int co = 32 * wm + 8 * (lane >> 4) + 4 * i;
    bv[i] = co < a.Cout ? *reinterpret_cast<const f32x4*>(a.bias + co) : f32x4{0.f, 0.f, 0.f, 0.f};
  }
  const bool exact = a.Cout == 128;  // then every tile stores FN times per wave
  elt_t* __restrict__ Y = reinterpret_cast<elt_t*>(a.y) + a.out_coff;
  for (int q = 1; q < NB - 1; ++q)
    if (tb + q < te) issue_h(tb + q, q);

  // a tile's epilogue runs beside the next tile's MFMAs (as conv1x1_wres's PIPE): accp holds the
  // previous tile's sums, its stores follow this tile's MFMAs
  f32x4 accp[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) accp[i][j] = bv[i];
  const int co = 32 * wm + 8 * (lane >> 4);
  auto finish = [&](const f32x4 (&s)[FM][FN], eltx8 (&ov)[FN]) {
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        const f32x4 x = act4_t<ACT>(s[i][j], a.slope, nl2e);
#pragma unroll
        for (int q = 0; q < 4; ++q) ov[j][4 * i + q] = (elt_t)x[q];
      }
  };
  auto store = [&](int tile, const eltx8 (&ov)[FN]) {
    const int n = tile / tpi, ti = tile - n * tpi;
    const int oy0 = (ti / tx_n) * TH, ox0 = (ti % tx_n) * TW;
    if (co < a.Cout) {  // cout % 8 == 0: the 8 channels are all valid
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int p = n * a.HoWo + (oy0 + wn * FN + j) * a.Wo + ox0 + (lane & 15);
        if (YCX_OUT_OK(a, Y + (size_t)p * a.out_cs + co, sizeof(eltx8))) *reinterpret_cast<eltx8*>(Y + (size_t)p * a.out_cs + co) = ov[j];
      }
    }
  };
  for (int tile = tb; tile < te; ++tile) {
    const int k = tile - tb, b = k % NB;
    // in flight behind this tile's halo: the halos of the next min(NB - 2, te - 1 - tile) tiles,
    // then (exact) the FN stores of tiles max(0, k - NB) .. k - 2 (tile j's go out in tile j + 1,
    // after the halo of j + NB); the weights came before them
    const int ahead = min(NB - 2, te - 1 - tile);
    const int nsb = exact ? max(0, k - 1 - max(0, k - NB)) : 0;
    vm_wait_le<(NB - 2) * HPW + (NB - 1) * FN>(ahead * nh + nsb * FN);
    __syncthreads();  // this tile's halo landed; every wave is done with the previous tile's buffer
    if (tile + NB - 1 < te) issue_h(tile + NB - 1, (k + NB - 1) % NB);
    const char* halo = smem + b * HBUF;
    // the fragment addresses are rebuilt per tile from two opaque values: hoisted out of the
    // tile loop they would take 72 VGPRs next to the 144 of weights
    int h0 = 2 * wn * FN * HC + (lane & 15), g = lane >> 4;
    asm volatile("" : "+v"(h0), "+v"(g));
    f32x4 acc[FM][FN];
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[i][j] = bv[i];
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int ky = t / 3, kx = t - 3 * ky;
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        const int lc = kk * 4 + g;
        eltx8 bfr[FN];
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          const int h = h0 + (2 * j + ky) * HC + (kx & 1) * HEVEN + (kx >> 1);
          bfr[j] = *reinterpret_cast<const eltx8*>(halo + h * 128 + ((lc ^ (h & 7)) << 4));
        }
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j) acc[i][j] = YCX_MFMA16(wf[t][kk][i], bfr[j], acc[i][j], 0, 0, 0);
      }
    }
    {  // the previous tile's epilogue beside this tile's MFMAs (one basic block)
      eltx8 ov[FN];
      finish(accp, ov);
#pragma unroll
      for (int j = 0; j < FN; ++j) {  // pinned here: otherwise sunk into the conditional stores below
        const int4 w = __builtin_bit_cast(int4, ov[j]);
        asm volatile("" ::"v"(w.x), "v"(w.y), "v"(w.z), "v"(w.w));
      }
      __builtin_amdgcn_sched_barrier(0);
      if (k > 0) store(tile - 1, ov);
    }
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) accp[i][j] = acc[i][j];
  }
  eltx8 ov[FN];
  finish(accp, ov);
  store(te - 1, ov);
}

// TH x TW output tiles. TW = 16: a fragment is one tile row. Band mode (TW != 16, r03): TW is
// the map's full width (40 at the 40^2 layers), so a tile is TH whole rows whose pixels are
// consecutive in NHWC; fragment f covers band pixels 16 f .. +15, each lane finds its own
// (row, column) in the halo, and the epilogue stores 16 consecutive pixels per fragment.
// tests/probes/conv_bench.py: see DESIGN.md §6 for the band tile against tile 16.
template <int BM, int WM, int WN, int NSTA, int TH = 16, int TW = 16>
__global__ void __launch_bounds__(WM * WN * 64) conv3x3_halo(ConvArgs a) {
  constexpr int NW = WM * WN;
  constexpr bool BAND = TW != 16;
  constexpr int HW = TW + 2, HP = (TH + 2) * HW;  // halo pixels (324 for 16 x 16)
  constexpr int HPIECES = (HP + 7) / 8;           // 1-KB DMA pieces (8 pixels)
  constexpr int HPW = (HPIECES + NW - 1) / NW;    // pieces per wave
  constexpr int TM = BM / WM, FM = TM / 16;
  constexpr int FN = TH * TW / 16 / WN;  // 16-pixel fragments per wave
  static_assert(TH * TW % (16 * WN) == 0, "whole fragments per wave");
  constexpr int A_BYTES = BM * 64 * 2, A_PW = BM / (8 * NW);
  static_assert(A_PW >= 1 && BM % (8 * NW) == 0, "A rows per wave");
  __shared__ __attribute__((aligned(1024))) char smem[NSTA * A_BYTES + HPIECES * 1024];
  char* halo = smem + NSTA * A_BYTES;

  const elt_t* __restrict__ X = reinterpret_cast<const elt_t*>(a.x);
  const elt_t* __restrict__ Wt = reinterpret_cast<const elt_t*>(a.w);
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;
  const int L = ycx_xcd_remap(blockIdx.x, a.nwg);
  const int ct = L % a.n_ct, rest = L / a.n_ct;
  const int tx_n = a.Wo / TW, tpi = (a.Ho / TH) * tx_n;
  const int n = rest / tpi, ti = rest - n * tpi;
  const int oy0 = (ti / tx_n) * TH, ox0 = (ti % tx_n) * TW, co0 = ct * BM;
  const int lrow = lane >> 3, pch = lane & 7;
  const int w_bytes = a.Cout_pad * a.Ktot * 2, x_bytes = a.N * a.H * a.W * a.in_cs * 2;
  // band mode: halo pixel of fragment j's lane at tap (0, 0)
  int hb[BAND ? FN : 1];
#pragma unroll
  for (int j = 0; j < (BAND ? FN : 1); ++j) {
    const int q = 16 * (wn * FN + j) + (lane & 15);
    hb[j] = (q / TW) * HW + q % TW;
  }

  // permuted A rows as in conv_bf16_glds: 16-byte epilogue stores
  int a_off[A_PW];
#pragma unroll
  for (int i = 0; i < A_PW; ++i) {
    const int row = 8 * (wid + NW * i) + lrow;
    const int f = (row % TM) >> 4, m = row & 15;
    const int ch = FM % 2 == 0 ? (row / TM) * TM + 32 * (f >> 1) + 8 * (m >> 2) + 4 * (f & 1) + (m & 3) : row;
    a_off[i] = ((co0 + ch) * a.Ktot + ((pch ^ swz<64>(row)) << 3)) * 2;
  }
  int h_off[HPW];  // halo piece i of this wave: byte offset of the lane's chunk (chunk 0 of the tap), or -1
#pragma unroll
  for (int i = 0; i < HPW; ++i) {
    const int h = 8 * (wid + NW * i) + lrow;
    const int hy = h / HW, hx = h - hy * HW;
    const int iy = oy0 - 1 + hy, ix = ox0 - 1 + hx;
    const bool ok = h < HP && (unsigned)iy < (unsigned)a.H && (unsigned)ix < (unsigned)a.W;
    h_off[i] = ok ? (((n * a.H + iy) * a.W + ix) * a.in_cs + a.in_coff + ((pch ^ (h & 7)) << 3)) * 2 : -1;
  }
  const int nchunk = a.Cin / 64, total = 9 * nchunk;
  auto issue_a = [&](int s) {
    const int c = s / 9, t = s - 9 * c;
    char* base = smem + (s % NSTA) * A_BYTES;
#pragma unroll
    for (int i = 0; i < A_PW; ++i)
      buf_lds16(Wt, w_bytes, a_off[i], (t * a.Cin + 64 * c) * 2, base + (wid + NW * i) * 1024);
  };
  auto issue_h = [&](int c) {
#pragma unroll
    for (int i = 0; i < HPW; ++i)
      if (wid + NW * i < HPIECES)
        buf_lds16(X, x_bytes, h_off[i] >= 0 ? h_off[i] + 128 * c : 0x7FFFFFF0, 0, halo + (wid + NW * i) * 1024);
  };

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  issue_h(0);
#pragma unroll
  for (int q = 0; q < NSTA - 1; ++q)
    if (q < total) issue_a(q);
  for (int s = 0; s < total; ++s) {
    const int c = s / 9, t = s - 9 * c;
    if (t == 0 && c > 0) {
      // next input chunk: every wave is past the previous chunk's last tap, then one halo refill
      __builtin_amdgcn_s_barrier();
      issue_h(c);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else if (NSTA == 3 && s + 1 < total) {
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(A_PW) : "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    if (s + NSTA - 1 < total) issue_a(s + NSTA - 1);
    const char* As = smem + (s % NSTA) * A_BYTES;
    const int ky = t / 3, kx = t - 3 * ky;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int lc = kk * 4 + (lane >> 4);
      eltx8 af[FM], bfr[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        const int row = wm * TM + i * 16 + (lane & 15);
        af[i] = *reinterpret_cast<const eltx8*>(As + row * 128 + ((lc ^ swz<64>(row)) << 4));
      }
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int h = BAND ? hb[j] + ky * HW + kx : (wn * FN + j + ky) * HW + (lane & 15) + kx;
        bfr[j] = *reinterpret_cast<const eltx8*>(halo + h * 128 + ((lc ^ (h & 7)) << 4));
      }
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = YCX_MFMA16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    __builtin_amdgcn_sched_barrier(0);
  }
  int pxf[FN];
#pragma unroll
  for (int j = 0; j < FN; ++j)
    pxf[j] = BAND ? n * a.HoWo + oy0 * a.Wo + 16 * (wn * FN + j) : n * a.HoWo + (oy0 + wn * FN + j) * a.Wo + ox0;
  if constexpr (FM % 2 == 0) {
    f32x4 bpre[FM];  // loaded here: prefetched before the K loop it cost this kernel 8-15 %
    bias8_prefetch<FM>(a, co0 + wm * TM, lane, bpre);
    epilogue_frag8<FM, FN>(a, acc, co0 + wm * TM, pxf, lane, bpre);
  }
  else epilogue_frag<FM, FN>(a, acc, co0 + wm * TM, pxf, lane);
}

// -------------------------------------------------------------------------
// fp32 parity kernel: 64x64 tile, BK=16, v_mfma_f32_16x16x4_f32.
// -------------------------------------------------------------------------
__global__ void __launch_bounds__(256) conv_f32_kernel(ConvArgs a) {
  constexpr int BM = 64, BN = 64, BK = 16, TM = 32, TN = 32, FM = 2, FN = 2;
  __shared__ __attribute__((aligned(16))) float As[2][BM * BK];
  __shared__ __attribute__((aligned(16))) float Bs[2][BN * BK];
  const float* __restrict__ X = reinterpret_cast<const float*>(a.x);
  const float* __restrict__ Wt = reinterpret_cast<const float*>(a.w);
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int L = ycx_xcd_remap(blockIdx.x, a.nwg);
  const int ct = L % a.n_ct, pt = L / a.n_ct;
  const int co0 = ct * BM, px0 = pt * BN;
  const int ch = tid & 3, row = tid >> 2;  // one 16-B chunk of A and of B per thread
  auto sw = [](int r) { return (r >> 1) & 3; };

  int p = px0 + row;
  bool pok = p < a.M;
  int pp = pok ? p : 0;
  int n = pp / a.HoWo, rem = pp - n * a.HoWo, oy = rem / a.Wo, ox = rem - oy * a.Wo;
  int iy0 = oy * a.S - a.P, ix0 = ox * a.S - a.P, nh = n * a.H;

  f32x4 ra, rb;
  auto gload = [&](int s, int ky, int kx, int cblk) {
    ra = *reinterpret_cast<const f32x4*>(Wt + (size_t)(co0 + row) * a.Ktot + s * BK + ch * 4);
    int iy = iy0 + ky, ix = ix0 + kx;
    bool ok = pok && (unsigned)iy < (unsigned)a.H && (unsigned)ix < (unsigned)a.W;
    rb = ok ? *reinterpret_cast<const f32x4*>(X + ((size_t)(nh + iy) * a.W + ix) * a.in_cs + a.in_coff +
                                              cblk + ch * 4)
            : f32x4{0.f, 0.f, 0.f, 0.f};
  };
  auto lstore = [&](int buf) {
    *reinterpret_cast<f32x4*>(&As[buf][row * BK + ((ch ^ sw(row)) << 2)]) = ra;
    *reinterpret_cast<f32x4*>(&Bs[buf][row * BK + ((ch ^ sw(row)) << 2)]) = rb;
  };
  f32x4 acc[FM][FN];
  for (int i = 0; i < FM; ++i)
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  int ky = 0, kx = 0, cblk = 0;
  gload(0, 0, 0, 0);
  lstore(0);
  __syncthreads();
  for (int s = 0; s < a.nsteps; ++s) {
    const bool more = s + 1 < a.nsteps;
    if (more) {
      cblk += BK;
      if (cblk == a.Cin) {
        cblk = 0;
        if (++kx == a.KW) { kx = 0; ++ky; }
      }
      gload(s + 1, ky, kx, cblk);
    }
    const int buf = s & 1;
#pragma unroll
    for (int kk = 0; kk < BK / 4; ++kk) {  // k = kk*4 + (lane>>4): chunk kk, element lane>>4
      float af[FM], bf[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        int r = wm * TM + i * 16 + (lane & 15);
        af[i] = As[buf][r * BK + ((kk ^ sw(r)) << 2) + (lane >> 4)];
      }
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        int r = wn * TN + j * 16 + (lane & 15);
        bf[j] = Bs[buf][r * BK + ((kk ^ sw(r)) << 2) + (lane >> 4)];
      }
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[i], bf[j], acc[i][j], 0, 0, 0);
    }
    if (more) lstore((s + 1) & 1);
    __syncthreads();
  }

  // Epilogue: lane holds 4 consecutive output channels of one pixel per tile.
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      int pe = px0 + wn * TN + j * 16 + (lane & 15);
      int cb = co0 + wm * TM + i * 16 + (lane >> 4) * 4;
      if (pe >= a.M) continue;
      float v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = ycx_act<false>(acc[i][j][r] + a.bias[cb + r], a.act, a.slope);
      if (a.out_layout == YCX_OUT_NCHW_F32) {
        int n2 = pe / a.HoWo, rem2 = pe - n2 * a.HoWo;
        float* Y = reinterpret_cast<float*>(a.y);
        for (int r = 0; r < 4; ++r)
          if (cb + r < a.Cout) if (YCX_OUT_OK(a, &Y[((size_t)n2 * a.out_cs + a.out_coff + cb + r) * a.HoWo + rem2], sizeof(Y[0]))) Y[((size_t)n2 * a.out_cs + a.out_coff + cb + r) * a.HoWo + rem2] = v[r];
        continue;
      }
      if (cb >= a.Cout) continue;
      if (a.res) {
        f32x4 rv = *reinterpret_cast<const f32x4*>(reinterpret_cast<const float*>(a.res) +
                                                    (size_t)pe * a.res_cs + a.res_coff + cb);
        for (int r = 0; r < 4; ++r) v[r] += rv[r];
      }
      float* Y = reinterpret_cast<float*>(a.y);
      f32x4 ov = {v[0], v[1], v[2], v[3]};
      if (a.out_layout == YCX_OUT_NHWC_UP2) {
        int n2 = pe / a.HoWo, rem2 = pe - n2 * a.HoWo, oy2 = rem2 / a.Wo, ox2 = rem2 - oy2 * a.Wo;
        size_t W2 = 2 * (size_t)a.Wo;
        size_t b0 = ((size_t)n2 * 2 * a.Ho + 2 * oy2) * W2 + 2 * ox2;
        size_t q[4] = {b0, b0 + 1, b0 + W2, b0 + W2 + 1};
        for (int t = 0; t < 4; ++t) if (YCX_OUT_OK(a, Y + q[t] * a.out_cs + a.out_coff + cb, sizeof(f32x4))) *reinterpret_cast<f32x4*>(Y + q[t] * a.out_cs + a.out_coff + cb) = ov;
      } else {
        if (YCX_OUT_OK(a, Y + (size_t)pe * a.out_cs + a.out_coff + cb, sizeof(f32x4))) *reinterpret_cast<f32x4*>(Y + (size_t)pe * a.out_cs + a.out_coff + cb) = ov;
      }
    }
}

// -------------------------------------------------------------------------
// Stem: first conv on the fp32 NCHW model input (cin <= 4). VALU direct conv,
// one thread per output pixel, folded weights broadcast from LDS.
// -------------------------------------------------------------------------
template <int KH, int KW, int CIN, typename OutT>
__global__ void __launch_bounds__(256) stem_kernel(ConvArgs a) {
  extern __shared__ __attribute__((aligned(16))) float ws[];  // [KH*KW*CIN][Cout_pad] + bias
  constexpr int NT = KH * KW * CIN;
  const float* Wt = reinterpret_cast<const float*>(a.w);
  const int wn = NT * a.Cout_pad;
  for (int i = threadIdx.x; i < wn; i += blockDim.x) ws[i] = Wt[i];
  for (int i = threadIdx.x; i < a.Cout_pad; i += blockDim.x) ws[wn + i] = a.bias[i];
  __syncthreads();
  const int pr = blockIdx.x * blockDim.x + threadIdx.x;
  const bool pv = pr < a.M;  // tail threads compute a duplicate pixel and store nothing
  const int p = pv ? pr : a.M - 1;
  const int n = p / a.HoWo, rem = p - n * a.HoWo, oy = rem / a.Wo, ox = rem - oy * a.Wo;
  const float* X = reinterpret_cast<const float*>(a.x);
  float patch[NT];
#pragma unroll
  for (int ky = 0; ky < KH; ++ky)
#pragma unroll
    for (int kx = 0; kx < KW; ++kx) {
      int iy = oy * a.S - a.P + ky, ix = ox * a.S - a.P + kx;
      bool ok = (unsigned)iy < (unsigned)a.H && (unsigned)ix < (unsigned)a.W;
#pragma unroll
      for (int ci = 0; ci < CIN; ++ci)
        patch[(ky * KW + kx) * CIN + ci] =
            ok ? X[(((size_t)n * a.in_cs + a.in_coff + ci) * a.H + iy) * a.W + ix] : 0.0f;
    }
  for (int c0 = 0; c0 < a.Cout; c0 += 8) {
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = 0.0f;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      f32x4 w0 = *reinterpret_cast<const f32x4*>(ws + t * a.Cout_pad + c0);
      f32x4 w1 = *reinterpret_cast<const f32x4*>(ws + t * a.Cout_pad + c0 + 4);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        v[j] = fmaf(patch[t], w0[j], v[j]);
        v[4 + j] = fmaf(patch[t], w1[j], v[4 + j]);
      }
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = ycx_act<sizeof(OutT) <= 2>(v[j] + ws[wn + c0 + j], a.act, a.slope);
    if constexpr (sizeof(OutT) == 1) {
      if (pv) {
        store4_f8(a, p, c0, v);
        store4_f8(a, p, c0 + 4, v + 4);
      }
    } else {
      if (pv) store8<OutT>(a, p, c0, v);
    }
  }
}

// -------------------------------------------------------------------------
// MFMA stem (bf16): K = KH*KW*CIN <= 32 is ONE v_mfma_f32_16x16x32_bf16 step.
// A = folded weights held in registers for the whole kernel; B = im2col
// gathered straight from the fp32 NCHW image (lane l: pixel l&15 of a
// 16-pixel run, k = 8(l>>4) + j), converted to bf16 in registers. A wave
// owns whole 16-pixel runs of one output row (Wo % 16 == 0), so the pixel ->
// (n, oy, ox) split is scalar and each gather is one add from a per-lane tap
// offset. A-rows are permuted so that the two MFMAs of a pair leave 8
// consecutive channels in each lane: one 16-byte store per lane, a wave
// writes 16 pixels x 32 channels as one contiguous KiB.
// -------------------------------------------------------------------------
__device__ __forceinline__ int stem_ch(int t, int m) {  // MFMA t, A-row m -> output channel
  return 32 * (t >> 1) + 8 * (m >> 2) + 4 * (t & 1) + (m & 3);
}

template <int KH, int KW, int CIN, int CT, bool F8 = false>  // F8: e4m3 output (x out_scale)
__global__ void __launch_bounds__(256) stem_mfma(ConvArgs a) {
  constexpr int KT = KH * KW * CIN;
  static_assert(KT <= 32 && CT % 2 == 0, "one MFMA K step, channel pairs");
  const int lane = threadIdx.x & 63, lx = lane & 15, kq = lane >> 4;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const float* Wt = reinterpret_cast<const float*>(a.w);  // [KT][Cout_pad]
  const float* __restrict__ X = reinterpret_cast<const float*>(a.x);
  const int HW = a.H * a.W;
  eltx8 af[CT];
  int dy[8], dx[8], toff[8];
  bool kv[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int k = 8 * kq + j;
    kv[j] = k < KT;
    const int kk = kv[j] ? k : 0, tap = kk / CIN, dc = kk - tap * CIN;
    dy[j] = tap / KW;
    dx[j] = tap - dy[j] * KW;
    toff[j] = dc * HW + dy[j] * a.W + dx[j];
#pragma unroll
    for (int t = 0; t < CT; ++t) af[t][j] = (elt_t)(kv[j] ? Wt[kk * a.Cout_pad + stem_ch(t, lx)] : 0.0f);
  }
  float bias[CT][4];
#pragma unroll
  for (int t = 0; t < CT; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) bias[t][r] = a.bias[stem_ch(t, 4 * kq + r)];
  const int ngroups = a.M / 16;
  char* __restrict__ Y = reinterpret_cast<char*>(a.y);
  // Each workgroup owns a contiguous run of 16-pixel groups, and consecutive
  // runs sit on one XCD (bijective remap): the three input rows a run reads
  // are fetched into one L2 instead of every XCD's.
  const int per = (ngroups + (int)gridDim.x - 1) / (int)gridDim.x;
  const int g0 = ycx_xcd_remap(blockIdx.x, gridDim.x) * per;
  const int g1 = min(ngroups, g0 + per);
  for (int g = g0 + wv; g < g1; g += 4) {
    const int p0 = g * 16;  // scalar: the run lies in one output row
    const int n = p0 / a.HoWo, rem = p0 - n * a.HoWo, oy = rem / a.Wo, ox0 = rem - oy * a.Wo;
    const float* Xn = X + (size_t)(n * a.in_cs + a.in_coff) * HW;
    const int iy0 = oy * a.S - a.P, ixl = (ox0 + lx) * a.S - a.P;
    const int base = iy0 * a.W + ixl;
    eltx8 b;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const bool ok = kv[j] && (unsigned)(iy0 + dy[j]) < (unsigned)a.H && (unsigned)(ixl + dx[j]) < (unsigned)a.W;
      b[j] = (elt_t)(ok ? Xn[base + toff[j]] : 0.0f);
    }
#pragma unroll
    for (int q = 0; q < CT / 2; ++q) {
      const f32x4 z = {0.f, 0.f, 0.f, 0.f};
      const f32x4 c0 = YCX_MFMA16(af[2 * q], b, z, 0, 0, 0);
      const f32x4 c1 = YCX_MFMA16(af[2 * q + 1], b, z, 0, 0, 0);
      const int ch0 = 32 * q + 8 * kq;
      if (ch0 < a.Cout) {
        float o[8];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          o[r] = ycx_act<true>(c0[r] + bias[2 * q][r], a.act, a.slope);
          o[4 + r] = ycx_act<true>(c1[r] + bias[2 * q + 1][r], a.act, a.slope);
        }
        if constexpr (F8) {
          const float sc = a.out_scale;
          const uint32_t lo = f8x4_pack(o[0] * sc, o[1] * sc, o[2] * sc, o[3] * sc);
          const uint32_t hi = f8x4_pack(o[4] * sc, o[5] * sc, o[6] * sc, o[7] * sc);
          if (YCX_OUT_OK(a, Y + (size_t)(p0 + lx) * a.out_cs + a.out_coff + ch0, sizeof(uint2))) *reinterpret_cast<uint2*>(Y + (size_t)(p0 + lx) * a.out_cs + a.out_coff + ch0) = make_uint2(lo, hi);
        } else {
          eltx8 ob;
#pragma unroll
          for (int r = 0; r < 8; ++r) ob[r] = (elt_t)o[r];
          if (YCX_OUT_OK(a, Y + ((size_t)(p0 + lx) * a.out_cs + a.out_coff + ch0) * 2, sizeof(eltx8))) *reinterpret_cast<eltx8*>(Y + ((size_t)(p0 + lx) * a.out_cs + a.out_coff + ch0) * 2) = ob;
        }
      }
    }
  }
}

// -------------------------------------------------------------------------
// Stem + stride-2 conv, fused (yolov7's layers 0-1: 3x3 3->32, 3x3/s2 32->64).
// Persistent 256-thread blocks (two per CU) walk a contiguous range of 4 x 32
// tiles of the second conv's output, all its (<= 64) channels. Per block, once:
// the second conv's weights (9 taps x this wave's 32 channels, 72 VGPRs) and
// the stem's folded weights into registers. Per tile:
//  (0) the fp32 image patch under the tile's 9 x 65 stem pixels (3 x 11 x 67
//      floats at stem stride 1) sits in LDS, loaded into registers during the
//      previous tile (row per wave-instruction, lane = column) and written
//      after it; the patch rows / planes are padded (RS, CPS) so the stem's
//      B gathers hit 2.5 instead of 4 LDS cycles per read;
//  (1) the stem pixels are computed by MFMA (K = 27 <= 32, one instruction per
//      16 pixels x 16 channels), fully unrolled so a wave keeps several
//      gathers / MFMAs / SiLUs in flight, and kept in LDS as bf16, 64 B per
//      pixel, zero outside the stem map (the second conv's padding); even and
//      odd stem columns live in separate planes so the B fragments of 16
//      consecutive output pixels are 16 consecutive slots;
//  (2) the second conv: one tap = one 32-deep MFMA step, B from the stem tile.
// The 32-channel stem map (839 MB at bs = 32, 640^2) never touches HBM.
// tests/probes/stem2_bench.py (bs 32, 640^2): 0.67 ms for the per-tile blocks
// (stem phase alone 0.36: one dependent gather -> MFMA -> SiLU chain per wave).
// -------------------------------------------------------------------------
constexpr int kS2TH = 4, kS2TW = 32;                       // output tile
constexpr int kS2R = 2 * kS2TH + 1, kS2C = 2 * kS2TW + 1;  // 9 x 65 stem pixels
constexpr int kS2Even = (kS2C + 1) / 2, kS2Odd = kS2C / 2;
constexpr int kS2Dump = kS2R * kS2C;  // one slot past the tile: writes of the pixels past it

__device__ __forceinline__ int s2_slot(int r, int c) {
  return (c & 1) ? kS2R * kS2Even + r * kS2Odd + (c >> 1) : r * kS2Even + (c >> 1);
}
// 16-B chunk q of a stem pixel in plane column col lives at chunk q ^ s2_swz(col):
// the stem phase's 16-B writes drop from 32 to 14 LDS cycles and the conv
// phase's B reads from 8 to 4 (bank simulation over every access; the swizzle
// depends on col & 7 only, so per conv lane it is one of two constants).
__device__ __forceinline__ int s2_swz(int col) { return (col ^ ((col >> 1) & 2)) & 3; }

constexpr int s2_pad(int v, int m) { return v + ((m - v % 32) + 32) % 32; }  // smallest >= v, == m mod 32

template <int SS, int ACT1, int ACT2, bool F8 = false>  // stem stride, stem / conv act, e4m3 output
__global__ void __launch_bounds__(256, SS == 1 ? 2 : 1) stem2_fused(ConvArgs sa, ConvArgs ca) {  // SS 2: 100 KB of LDS, one block per CU
  constexpr int NPIX = kS2R * kS2C, NGRP = (NPIX + 15) / 16, GPW = (NGRP + 3) / 4;
  constexpr int IR = (kS2R - 1) * SS + 3, IC = (kS2C - 1) * SS + 3;  // image patch rows / cols
  constexpr int RS = s2_pad(IC, 7), CPS = s2_pad(IR * RS, 23);         // padded row / plane strides
  constexpr int NROW = 3 * IR, RPW = (NROW + 3) / 4, NCH = (IC + 63) / 64;  // patch rows, per wave, 64-col chunks
  constexpr int FM = 2, FN = 4;  // per wave: 32 output channels x 64 pixels (2 rows x 32)
  constexpr int STEM_BYTES = (((NPIX + 1) * 64) + 255) & ~255;  // + the dump slot
  constexpr int IMGB = (3 * CPS * 4 + 255) & ~255;                  // one image patch buffer
  __shared__ __attribute__((aligned(1024))) char smem[STEM_BYTES + 2 * IMGB];
  const int tid = threadIdx.x, lane = tid & 63, lx = lane & 15, kq = lane >> 4;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wv & 1, wn = wv >> 1;  // 32-channel half, 2-row half
  // tiles run down a column of the image (ty fastest: 0.394 vs 0.415 ms with the packed SiLU;
  // keeping the shared stem row in LDS for the next tile down measured no faster)
  const int tx_n = ca.Wo / kS2TW, ty_n = ca.Ho / kS2TH, tpi = ty_n * tx_n, ntiles = ca.N * tpi;
  const int blk = ycx_xcd_remap(blockIdx.x, gridDim.x);
  const int tb = (int)((long long)blk * ntiles / gridDim.x), te = (int)((long long)(blk + 1) * ntiles / gridDim.x);
  if (tb >= te) return;

  // second conv weights, all taps, this wave's 32 channels (A lane: row lx of fragment i is channel
  // 32 wm + 8 (lx >> 2) + 4 i + (lx & 3), k = 32 t + 8 kq ..: C rows 4 kq .. +3 of the two fragments
  // are channels 32 wm + 8 kq .. +7, one 16-byte (e4m3: 8-byte) store per lane and pixel)
  static_assert(FM == 2, "channel pairs");
  const elt_t* __restrict__ Wc = reinterpret_cast<const elt_t*>(ca.w);  // [Cout_pad][3][3][32]
  eltx8 aw[9][FM];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int i = 0; i < FM; ++i)
      aw[t][i] = *reinterpret_cast<const eltx8*>(Wc + (size_t)(32 * wm + 8 * (lx >> 2) + 4 * i + (lx & 3)) * ca.Ktot +
                                                  32 * t + 8 * kq);
  f32x4 bvc[FM];
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    const int co = 32 * wm + 8 * kq + 4 * i;
    bvc[i] = co < ca.Cout ? *reinterpret_cast<const f32x4*>(ca.bias + co) : f32x4{0.f, 0.f, 0.f, 0.f};
  }
  // stem weights / bias / gather offsets (k = 8 kq + j -> tap k / 3, channel k % 3; k >= 27 gathers
  // what lane kq = 2 gathers, a broadcast, and weighs it 0)
  constexpr int KT = 27, CIN = 3;
  eltx8 af[2];
  int toff[8];
  {
    const float* Ws = reinterpret_cast<const float*>(sa.w);  // [KT][Cout_pad]
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int k = 8 * kq + j, kv = k < KT, kk = kv ? k : 16 + j;
      const int tap = kk / CIN, dc = kk - tap * CIN, dy = tap / 3, dx = tap - dy * 3;
      toff[j] = dc * CPS + dy * RS + dx;
#pragma unroll
      for (int t = 0; t < 2; ++t) af[t][j] = (elt_t)(kv ? Ws[kk * sa.Cout_pad + stem_ch(t, lx)] : 0.0f);
    }
  }
  f32x4 bias_s[2];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) bias_s[t][r] = sa.bias[stem_ch(t, 4 * kq + r)];
  // conv B reads: the chunk swizzle of plane column cc + d (d = kx / 2 on the even plane) is
  // that of lx + d, 16 (j & 1) being a multiple of 8
  const int swb0 = 16 * (kq ^ s2_swz(lx)), swb1 = 16 * (kq ^ s2_swz(lx + 1));

  // image patch fetch: 4-byte LDS-DMA straight into one of two patch buffers
  // (row q = (channel, row) per wave-instruction, lane = column); an element
  // outside the image reads the descriptor's out-of-range zero
  const int HWi = sa.H * sa.W;
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
      (void*)sa.x, (short)0, sa.N * sa.in_cs * HWi * 4, 0x00020000);
  auto fetch = [&](int tile, int buf) {
    const int n = tile / tpi, ti = tile - n * tpi, tx = ti / ty_n, ty = ti - tx * ty_n;
    const int iy0 = (2 * ty * kS2TH - 1) * SS - sa.P, ix0 = (2 * tx * kS2TW - 1) * SS - sa.P;
    const int nb = (n * sa.in_cs + sa.in_coff) * HWi;
    char* base = smem + STEM_BYTES + buf * IMGB;
#pragma unroll
    for (int u = 0; u < RPW; ++u) {
      const int q = wv + 4 * u, c = q / IR, r = q - c * IR, iy = iy0 + r;
      if (q >= NROW) break;  // uniform
      const bool rok = (unsigned)iy < (unsigned)sa.H;
      const int rowb = nb + c * HWi + iy * sa.W;
#pragma unroll
      for (int h = 0; h < NCH; ++h) {
        const int col = 64 * h + lane, ix = ix0 + col;
        const bool ok = rok && (unsigned)ix < (unsigned)sa.W;
        if (64 * h + 64 <= IC || col < IC)
          __builtin_amdgcn_raw_ptr_buffer_load_lds(xr, (lds_void*)(base + (c * CPS + r * RS + 64 * h) * 4), 4,
                                                   ok ? (rowb + ix) * 4 : 0x7FFFFFF0, 0, 0, 0);
      }
    }
  };
  // stem phase addresses, the same for every tile: group g = wv + 4 u, pixel
  // p = 16 g + lx -> image offset (floats) and stem-tile byte address (swizzled
  // chunk kq); the pixels past the tile (p >= NPIX, last group) write a dump slot
  int s_img[GPW], s_dst[GPW];
#pragma unroll
  for (int u = 0; u < GPW; ++u) {
    const int p = 16 * (wv + 4 * u) + lx, ok = p < NPIX, pp = ok ? p : 0;
    const int r = pp / kS2C, c = pp - r * kS2C;
    s_img[u] = (r * SS) * RS + c * SS;
    s_dst[u] = ok ? s2_slot(r, c) * 64 + 16 * (kq ^ s2_swz(c >> 1)) : kS2Dump * 64 + 16 * kq;
  }
  fetch(tb, 0);
  const float nl2e = silu_nl2e();
  elt_t* __restrict__ Y = reinterpret_cast<elt_t*>(ca.y) + ca.out_coff;
  // the previous tile's epilogue issued exactly FM x FN stores per wave after
  // this tile's fetch when every channel is stored (vmcnt counts in issue order)
  const bool exact = ca.Cout == FM * 32;

  for (int tile = tb; tile < te; ++tile) {
    const int n = tile / tpi, ti = tile - n * tpi, tx = ti / ty_n, ty = ti - tx * ty_n;
    const int oy0 = ty * kS2TH, ox0 = tx * kS2TW;
    const int sy0 = 2 * oy0 - 1, sx0 = 2 * ox0 - 1;  // stem pixel of tile slot (0, 0)
    const float* img = reinterpret_cast<const float*>(smem + STEM_BYTES + ((tile - tb) & 1) * IMGB);
    if (tile > tb && exact) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(FM * FN) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();  // patch landed (every wave's share); stem tile free
    if (tile + 1 < te) fetch(tile + 1, (tile + 1 - tb) & 1);

    // (1) stem tile: group g = wv + 4 u covers pixels 16 g .. +15; the MFMA
    //     accumulates onto the bias; branch-free so the unrolled groups overlap
#ifdef YCX_S2_NOSTEM  // development timing only: the stem phase skipped
    if (tile < 0)
#endif
#pragma unroll
    for (int u = 0; u < GPW; ++u) {
      if (u == GPW - 1 && wv + 4 * u >= NGRP) break;  // uniform: the last group is one wave's
      const float* ip = img + s_img[u];  // tap (0, 0), channel 0
      eltx8 bq;
#pragma unroll
      for (int j = 0; j < 8; ++j) bq[j] = (elt_t)ip[toff[j]];
      const f32x4 c0 = YCX_MFMA16(af[0], bq, bias_s[0], 0, 0, 0);
      const f32x4 c1 = YCX_MFMA16(af[1], bq, bias_s[1], 0, 0, 0);
      eltx8 o;
#ifdef YCX_S2_NOACT1  // development timing only (tests/probes/stem2_bench.py): stem without its activation
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        o[q] = (elt_t)c0[q];
        o[4 + q] = (elt_t)c1[q];
      }
#else
      const f32x4 a0 = act4_t<ACT1>(c0, sa.slope, nl2e), a1 = act4_t<ACT1>(c1, sa.slope, nl2e);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        o[q] = (elt_t)a0[q];
        o[4 + q] = (elt_t)a1[q];
      }
#endif
      *reinterpret_cast<eltx8*>(smem + s_dst[u]) = o;
      if (u & 1) __builtin_amdgcn_sched_barrier(0);  // two groups in flight: bounded registers
    }
    // border tiles: stem pixels outside the stem map are the second conv's zero padding
    const bool top = sy0 < 0, bottom = sy0 + kS2R > sa.Ho, left = sx0 < 0, right = sx0 + kS2C > sa.Wo;
    if (top || bottom || left || right) {
      __syncthreads();
      const eltx8 z8 = {};
      for (int e = tid; e < (kS2R + kS2C) * 2 * 4; e += 256) {  // (row or column, pixel, 16-B chunk)
        const int ch = e & 3, k = e >> 2;
        int r = -1, c = -1;
        if (k < kS2C) { r = top ? 0 : -1; c = k; }
        else if (k < 2 * kS2C) { r = bottom ? sa.Ho - sy0 : -1; c = k - kS2C; }
        else if (k < 2 * kS2C + kS2R) { c = left ? 0 : -1; r = k - 2 * kS2C; }
        else { c = right ? sa.Wo - sx0 : -1; r = k - 2 * kS2C - kS2R; }
        if (r >= 0 && c >= 0 && r < kS2R && c < kS2C)
          *reinterpret_cast<eltx8*>(smem + s2_slot(r, c) * 64 + 16 * (ch ^ s2_swz(c >> 1))) = z8;
      }
    }
    __syncthreads();  // stem tile complete; patch free

    // (2) second conv: wave (wm, wn) -> channels 32 wm.., output rows 2 wn, 2 wn + 1
    //     (fragment j: row rr = 2 wn + (j >> 1), cols cc = 16 (j & 1) + lx). Its
    //     stem pixel for tap (ky, kx) is (2 rr + ky, 2 cc + kx): even kx in the
    //     even plane at slot (2 rr + ky) E + cc + kx/2, odd kx in the odd plane at
    //     R E + (2 rr + ky) O + cc — per-lane bases plus per-tap constants.
    f32x4 acc[FM][FN];  // accumulates onto the bias
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[i][j] = bvc[i];
#ifdef YCX_S2_NOCONV  // development timing only: the conv phase's LDS reads and MFMAs skipped
    if (tile < 0)
#endif
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int ky = t / 3, kx = t - 3 * ky;
      eltx8 bfr[FN];
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int rr = 2 * wn + (j >> 1), cc = 16 * (j & 1) + lx;
        const int slot = (kx & 1) ? kS2R * kS2Even + (2 * rr + ky) * kS2Odd + cc : (2 * rr + ky) * kS2Even + cc + kx / 2;
        bfr[j] = *reinterpret_cast<const eltx8*>(smem + slot * 64 + (kx == 2 ? swb1 : swb0));
      }
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = YCX_MFMA16(aw[t][i], bfr[j], acc[i][j], 0, 0, 0);
    }
    // epilogue: bias (in the accumulators) + act, 8 channels of one pixel per lane
    const int co = 32 * wm + 8 * kq;
    if (co < ca.Cout) {  // cout % 8 == 0: the 8 channels are all valid
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int p = n * ca.HoWo + (oy0 + 2 * wn + (j >> 1)) * ca.Wo + ox0 + 16 * (j & 1) + lx;
        float v[8];
#pragma unroll
        for (int i = 0; i < FM; ++i) {
#ifdef YCX_S2_NOACT2  // development timing only
          const f32x4 av = acc[i][j];
#else
          const f32x4 av = act4_t<ACT2>(acc[i][j], ca.slope, nl2e);
#endif
#pragma unroll
          for (int q = 0; q < 4; ++q) v[4 * i + q] = av[q];
        }
        if constexpr (F8) {  // the stem map and this conv run in bf16; only the output is e4m3
          const float sc = ca.out_scale;
          if (YCX_OUT_OK(ca, reinterpret_cast<uint8_t*>(ca.y) + ca.out_coff + (size_t)p * ca.out_cs + co, sizeof(uint2))) *reinterpret_cast<uint2*>(reinterpret_cast<uint8_t*>(ca.y) + ca.out_coff + (size_t)p * ca.out_cs + co) =
              make_uint2(f8x4_pack(v[0] * sc, v[1] * sc, v[2] * sc, v[3] * sc),
                         f8x4_pack(v[4] * sc, v[5] * sc, v[6] * sc, v[7] * sc));
        } else {
          eltx8 ov;
#pragma unroll
          for (int q = 0; q < 8; ++q) ov[q] = (elt_t)v[q];
          if (YCX_OUT_OK(ca, Y + (size_t)p * ca.out_cs + co, sizeof(eltx8))) *reinterpret_cast<eltx8*>(Y + (size_t)p * ca.out_cs + co) = ov;
        }
      }
    }
  }
}

// -------------------------------------------------------------------------
// 1x1 conv with the weights resident in registers (memory-bound pointwise
// layers: K = Cin <= 512). A block of WCO x WPX waves is persistent over a
// contiguous range of PT-pixel tiles; wave (wc, wp) owns output channels
// 32 wc .. +31 of the block's channel group and pixels TPW wp .. +TPW-1 of
// every tile, and holds those 32 rows of W (K/4 VGPRs) for the whole launch.
// Activations stream HBM -> LDS once per tile through an NS-stage LDS-DMA
// ring; a stage (one barrier step) is SUB 64-channel slabs of PT rows x 128 B,
// each XOR-swizzled as in conv_bf16_glds, read by all the block's waves. The
// MFMA A operand never touches LDS, and no block re-reads weight tiles (the
// im2col kernels pull every weight tile into LDS once per block: for
// 256 x 256 at 160^2 that doubles the bytes moved into LDS). The ring runs
// across tile boundaries: a full tile's epilogue issues exactly FM x FN
// eltx4 stores per wave and those enter the following counted vmcnt waits
// (loads, stores and LDS-DMA retire in issue order on gfx950), so the
// epilogue never drains the ring.
// Requires 1x1/s1/p0, Cin = 64 KC, NHWC bf16 output without residual.
// -------------------------------------------------------------------------

// s_waitcnt vmcnt(BASE + nb) lgkmcnt(0) for a uniform runtime nb in [LO, HI]
// (the count is an immediate: binary search over the encodable values; a
// count above 63 waits for 63, i.e. for more than needed, which is safe).
template <int BASE, int LO, int HI>
__device__ __forceinline__ void wait_vm_counted(int nb) {
  if constexpr (LO >= HI || BASE + LO >= 63) {
    asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(BASE + LO < 63 ? BASE + LO : 63) : "memory");
  } else {
    constexpr int MID = (LO + HI) / 2;
    if (nb > MID) wait_vm_counted<BASE, MID + 1, HI>(nb);
    else wait_vm_counted<BASE, LO, MID>(nb);
  }
}

// PIPE (KC <= 4, where 32 more accumulator VGPRs fit): a tile's epilogue (bias, activation,
// bf16 pack) runs in the first K step of the next tile, beside that step's MFMAs (the
// activation is a template argument so the two share one basic block and the scheduler can
// interleave them), and its stores follow that step's MFMAs. In tile order the eight waves'
// epilogues otherwise ran together with no MFMA on the CU (10-15 % of the launch at
// cout >= 256, tests/probes/conv_bench.py CONV_ACT=0 against 1).
template <int WCO, int WPX, int TPW, int KC, int NS, int SUB, int ACT>
__global__ void __launch_bounds__(WCO * WPX * 64) conv1x1_wres(ConvArgs a) {
  constexpr bool PIPE = KC <= 4;
  constexpr int NW = WCO * WPX, PT = TPW * WPX, FM = 2, FN = TPW / 16, BCO = WCO * 32;
  constexpr int KS = KC / SUB, SLAB = PT * 128, STAGE = SUB * SLAB, A_PW = PT / (8 * NW);
  constexpr int NSTO = FN;  // 16-byte stores per wave per tile (A rows permuted: 8 channels per lane)
  constexpr int VM_RING = A_PW * SUB * (NS - 2);
  static_assert(KC % SUB == 0, "slabs per stage");
  static_assert(A_PW >= 1 && PT % (8 * NW) == 0 && TPW % 16 == 0, "tile rows per wave");
  __shared__ __attribute__((aligned(1024))) char smem[NS * STAGE];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wc = wid % WCO, wp = wid / WCO;
  const int G = a.n_ct;
  const int L = ycx_xcd_remap(blockIdx.x, a.nwg);
  const int g = L % G, r = L / G, R = a.nwg / G;
  const int T = (a.M + PT - 1) / PT;
  const int t0 = (int)((long long)r * T / R), t1 = (int)((long long)(r + 1) * T / R);
  if (t0 >= t1) return;  // whole block: no barrier is left waiting
  const int cob = g * BCO + wc * 32;

  // this wave's weights (A fragments: row m = lane & 15 of fragment i is channel
  // cob + 8 (m >> 2) + 4 i + (m & 3), k = 32 kq + 8 (lane >> 4) ..): the C rows 4g .. 4g+3 of
  // fragments 0 and 1 are then channels 8g .. 8g+7, one 16-byte store per lane and pixel
  const elt_t* __restrict__ Wt = reinterpret_cast<const elt_t*>(a.w);
  eltx8 af[2 * KC][FM];
  const int m16 = lane & 15;
#pragma unroll
  for (int kq = 0; kq < 2 * KC; ++kq)
#pragma unroll
    for (int i = 0; i < FM; ++i)
      af[kq][i] = *reinterpret_cast<const eltx8*>(Wt + (size_t)(cob + 8 * (m16 >> 2) + 4 * i + (m16 & 3)) * a.Ktot +
                                                   32 * kq + 8 * (lane >> 4));
  f32x4 bv[FM];
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    const int co = cob + 8 * (lane >> 4) + 4 * i;
    bv[i] = co < a.Cout ? *reinterpret_cast<const f32x4*>(a.bias + co) : f32x4{0.f, 0.f, 0.f, 0.f};
  }

  // LDS-DMA: wave-instruction (wid + NW i) fills rows 8 (wid + NW i) .. +7 of a slab
  const elt_t* __restrict__ X = reinterpret_cast<const elt_t*>(a.x);
  const int x_bytes = a.M * a.in_cs * 2;
  const int lrow = lane >> 3, pch = lane & 7;
  int rrow[A_PW], roff[A_PW];
#pragma unroll
  for (int i = 0; i < A_PW; ++i) {
    rrow[i] = 8 * (wid + NW * i) + lrow;
    roff[i] = (rrow[i] * a.in_cs + a.in_coff + ((pch ^ swz<64>(rrow[i])) << 3)) * 2;
  }
  const int nst = (t1 - t0) * KS;
  auto issue = [&](int s) {
    const int tl = s / KS, ks = s - tl * KS;
    const int px0 = (t0 + tl) * PT;
    char* base = smem + (s % NS) * STAGE;
#pragma unroll
    for (int sb = 0; sb < SUB; ++sb)
#pragma unroll
      for (int i = 0; i < A_PW; ++i) {
        const int off = px0 + rrow[i] < a.M ? px0 * a.in_cs * 2 + roff[i] + (ks * SUB + sb) * 128 : 0x7FFFFFF0;
        buf_lds16(X, x_bytes, off, 0, base + sb * SLAB + (wid + NW * i) * 1024);
      }
  };
  for (int s = 0; s < NS - 1 && s < nst; ++s) issue(s);

  const bool exact = a.Cout == a.Cout_pad;  // then every full tile stores exactly NSTO times per wave
  elt_t* __restrict__ Y = reinterpret_cast<elt_t*>(a.y) + a.out_coff;
  const float nl2e = silu_nl2e();  // act4_t: the packed form of ycx_act<true>, bit-identical
  const int co = cob + 8 * (lane >> 4);  // channels co .. co+7 (cout % 8 == 0: all valid or none)
  // tile tl's outputs from its sums: 8 channels of one pixel per lane and fragment column
  auto finish = [&](const f32x4 (&s)[FM][FN], eltx8 (&ov)[FN]) {
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        const f32x4 v = act4_t<ACT>(s[i][j] + bv[i], a.slope, nl2e);
#pragma unroll
        for (int q = 0; q < 4; ++q) ov[j][4 * i + q] = (elt_t)v[q];
      }
  };
  auto store = [&](int tl, const eltx8 (&ov)[FN]) {
    const int pb = (t0 + tl) * PT + wp * TPW + (lane & 15);
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int p = pb + 16 * j;
      if (p < a.M && co < a.Cout) if (YCX_OUT_OK(a, Y + (size_t)p * a.out_cs + co, sizeof(eltx8))) *reinterpret_cast<eltx8*>(Y + (size_t)p * a.out_cs + co) = ov[j];
    }
  };
  f32x4 acc[FM][FN], accp[FM][FN];  // accp (PIPE): the previous tile's sums
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  int t = 0;
  for (int tl = 0; tl < t1 - t0; ++tl) {
#pragma unroll
    for (int ks = 0; ks < KS; ++ks, ++t) {
      // wait for stage t: younger than its loads are the NS-2 later stages and the store
      // batches issued in steps t-NS+1 .. t-1 (a tile's batch: in its last step, or with PIPE
      // in the next tile's first step)
      if (t + NS - 2 >= nst) {
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
      } else if constexpr (PIPE) {
        const int lo = t - NS + 1 > KS ? t - NS + 1 : KS;  // batches: steps i KS, i >= 1
        const int nb = exact && t - 1 >= lo ? (t - 1) / KS - (lo + KS - 1) / KS + 1 : 0;
        wait_vm_counted<VM_RING, 0, (NS + KS - 2) / KS * NSTO>(nb > 0 ? nb * NSTO : 0);
      } else {
        const int lo = t - NS + 1 > 0 ? t - NS + 1 : 0;  // tile ends: steps i KS + KS - 1
        const int nb = exact && t >= KS ? (t - 1 - (KS - 1)) / KS - (lo + KS - 1 - (KS - 1)) / KS + 1 : 0;
        wait_vm_counted<VM_RING, 0, (NS + KS - 2) / KS * NSTO>(nb * NSTO);
      }
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      if (t + NS - 1 < nst) issue(t + NS - 1);
      if (ks == 0) {
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j) {
            if constexpr (PIPE) accp[i][j] = acc[i][j];
            acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
          }
      }
      const char* B = smem + (t % NS) * STAGE;
#pragma unroll
      for (int kk = 0; kk < 2 * SUB; ++kk) {
        const int c = (kk & 1) * 4 + (lane >> 4);
        const char* Bs = B + (kk >> 1) * SLAB;
        eltx8 bfr[FN];
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          const int row = wp * TPW + j * 16 + (lane & 15);
          bfr[j] = *reinterpret_cast<const eltx8*>(Bs + row * 128 + ((c ^ swz<64>(row)) << 4));
        }
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j)
            acc[i][j] = YCX_MFMA16(af[2 * SUB * ks + kk][i], bfr[j], acc[i][j], 0, 0, 0);
      }
      if constexpr (PIPE) {
        if (ks == 0) {  // the previous tile's epilogue beside this step's MFMAs (same basic block)
          eltx8 ov[FN];
          finish(accp, ov);
#pragma unroll
          for (int j = 0; j < FN; ++j) {  // pinned here: otherwise sunk into the conditional stores below
            const int4 w = __builtin_bit_cast(int4, ov[j]);
            asm volatile("" ::"v"(w.x), "v"(w.y), "v"(w.z), "v"(w.w));
          }
          __builtin_amdgcn_sched_barrier(0);
          if (tl > 0) store(tl - 1, ov);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    if constexpr (!PIPE) {
      // epilogue from registers: no global loads here (one would make the compiler drain vmcnt)
      eltx8 ov[FN];
      finish(acc, ov);
      store(tl, ov);
    }
  }
  if constexpr (PIPE) {
    eltx8 ov[FN];
    finish(acc, ov);
    store(t1 - t0 - 1, ov);
  }
}

// -------------------------------------------------------------------------
// Two chained 1x1 convs in one launch (tile 55, ycx_conv2d_pair): y1 = act(W1 x + b1)
// (cin 64 KC -> 256) and y2 = act(W2 y1 + b2) (256 -> CO2), where the second conv reads
// nothing but the first one's output (yolov7's 160^2 ELAN exit: layer 11, 256 -> 256,
// feeding layer 14, 256 -> 128; layer 11's map also goes to the MP branch, so y1 is
// still stored when the caller gives an output for it). conv1x1_wres's pipeline for
// the first conv (eight waves, 32 output channels each, W1 rows resident in VGPRs,
// 64-pixel tiles of x through the LDS-DMA ring); its epilogue also writes the
// tile's bf16 y1 (64 pixels x 256 channels, the ring's swizzled slab layout) into
// LDS, and after one barrier every wave runs the second conv on it with its own W2
// rows in VGPRs (CO2 = 128: 32 channels x 32 pixels per wave; 256: 32 x 64). The
// 64-pixel y1 tile never makes the HBM round trip of the unfused pair (at yolov7
// bs 32: 419 MB less read). Both epilogues apply the same float operations as
// conv1x1_wres's, so y1 and y2 are bit-identical to the two unfused launches.
// The ring's counted vmcnt waits include both conversions' stores.
// -------------------------------------------------------------------------
template <int KC, int NS, int SUB, int CO2>
__global__ void __launch_bounds__(512) conv1x1_wres_pair(ConvArgs a, ConvArgs b) {
  constexpr int NW = 8, PT = 64, FM = 2, FN = 4, KS = KC / SUB, SLAB = PT * 128, STAGE = SUB * SLAB;
  constexpr int A_PW = PT / (8 * NW);
  constexpr int K2 = 256, FN2 = CO2 == 128 ? 2 : 4;  // second conv: K = 256, pixels per wave 16 FN2
  static_assert(CO2 == 128 || CO2 == 256, "second conv: 128 or 256 output channels");
  static_assert(KC % SUB == 0 && A_PW == 1, "slabs per stage");
  constexpr int VM_RING = A_PW * SUB * (NS - 2);
  constexpr int Y1_BYTES = (K2 / 64) * SLAB;  // y1 tile: 4 slabs of 64 pixels x 128 B
  __shared__ __attribute__((aligned(1024))) char smem[NS * STAGE + Y1_BYTES];
  char* const y1s = smem + NS * STAGE;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int L = ycx_xcd_remap(blockIdx.x, a.nwg);
  const int R = a.nwg;
  const int T = (a.M + PT - 1) / PT;
  const int t0 = (int)((long long)L * T / R), t1 = (int)((long long)(L + 1) * T / R);
  if (t0 >= t1) return;  // whole block: no barrier is left waiting
  const int m16 = lane & 15;

  // first conv: this wave's 32 output channels (rows permuted as conv1x1_wres)
  const int cob = wid * 32;
  const elt_t* __restrict__ W1 = reinterpret_cast<const elt_t*>(a.w);
  eltx8 af[2 * KC][FM];
#pragma unroll
  for (int kq = 0; kq < 2 * KC; ++kq)
#pragma unroll
    for (int i = 0; i < FM; ++i)
      af[kq][i] = *reinterpret_cast<const eltx8*>(W1 + (size_t)(cob + 8 * (m16 >> 2) + 4 * i + (m16 & 3)) * a.Ktot +
                                                   32 * kq + 8 * (lane >> 4));
  f32x4 bv[FM];
#pragma unroll
  for (int i = 0; i < FM; ++i) bv[i] = *reinterpret_cast<const f32x4*>(a.bias + cob + 8 * (lane >> 4) + 4 * i);
  // second conv: channels cob2 .. +31, pixels 16 FN2 h2 .. of every tile
  const int cob2 = CO2 == 128 ? (wid & 3) * 32 : wid * 32, h2 = CO2 == 128 ? wid >> 2 : 0;
  const elt_t* __restrict__ W2 = reinterpret_cast<const elt_t*>(b.w);
  eltx8 af2[K2 / 32][FM];
#pragma unroll
  for (int kq = 0; kq < K2 / 32; ++kq)
#pragma unroll
    for (int i = 0; i < FM; ++i)
      af2[kq][i] = *reinterpret_cast<const eltx8*>(W2 + (size_t)(cob2 + 8 * (m16 >> 2) + 4 * i + (m16 & 3)) * b.Ktot +
                                                    32 * kq + 8 * (lane >> 4));
  f32x4 bv2[FM];
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    const int co = cob2 + 8 * (lane >> 4) + 4 * i;
    bv2[i] = co < b.Cout ? *reinterpret_cast<const f32x4*>(b.bias + co) : f32x4{0.f, 0.f, 0.f, 0.f};
  }

  // LDS-DMA of x: wave-instruction wid fills rows 8 wid .. +7 of a slab
  const elt_t* __restrict__ X = reinterpret_cast<const elt_t*>(a.x);
  const int x_bytes = a.M * a.in_cs * 2;
  const int lrow = lane >> 3, pch = lane & 7;
  const int rrow = 8 * wid + lrow;
  const int roff = (rrow * a.in_cs + a.in_coff + ((pch ^ swz<64>(rrow)) << 3)) * 2;
  const int nst = (t1 - t0) * KS;
  auto issue = [&](int s) {
    const int tl = s / KS, ks = s - tl * KS;
    const int px0 = (t0 + tl) * PT;
    char* base = smem + (s % NS) * STAGE;
#pragma unroll
    for (int sb = 0; sb < SUB; ++sb) {
      const int off = px0 + rrow < a.M ? px0 * a.in_cs * 2 + roff + (ks * SUB + sb) * 128 : 0x7FFFFFF0;
      buf_lds16(X, x_bytes, off, 0, base + sb * SLAB + wid * 1024);
    }
  };
  for (int s = 0; s < NS - 1 && s < nst; ++s) issue(s);

  // every full tile stores exactly NSTO 16-byte vectors per wave (both outputs whole)
  const bool store1 = a.y != nullptr;
  constexpr int NSTO_MAX = FN + FN2;
  const int nsto = (store1 ? FN : 0) + FN2;
  const bool exact = b.Cout == b.Cout_pad;  // a.Cout == a.Cout_pad == 256 (host check)
  elt_t* __restrict__ Y1 = store1 ? reinterpret_cast<elt_t*>(a.y) + a.out_coff : nullptr;
  elt_t* __restrict__ Y2 = reinterpret_cast<elt_t*>(b.y) + b.out_coff;
  int t = 0;
  for (int tl = 0; tl < t1 - t0; ++tl) {
    f32x4 acc[FM][FN];
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < KS; ++ks, ++t) {
      if (t + NS - 2 >= nst) {
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
      } else {
        const int lo = t - NS + 1 > 0 ? t - NS + 1 : 0;  // tile ends: steps i KS + KS - 1
        const int nb = exact && t >= KS ? (t - 1 - (KS - 1)) / KS - (lo + KS - 1 - (KS - 1)) / KS + 1 : 0;
        if (exact) wait_vm_counted<VM_RING, 0, (NS + KS - 2) / KS * NSTO_MAX>(nb * nsto);
        else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
      }
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      if (t + NS - 1 < nst) issue(t + NS - 1);
      const char* B = smem + (t % NS) * STAGE;
#pragma unroll
      for (int kk = 0; kk < 2 * SUB; ++kk) {
        const int c = (kk & 1) * 4 + (lane >> 4);
        const char* Bs = B + (kk >> 1) * SLAB;
        eltx8 bfr[FN];
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          const int row = j * 16 + (lane & 15);
          bfr[j] = *reinterpret_cast<const eltx8*>(Bs + row * 128 + ((c ^ swz<64>(row)) << 4));
        }
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j)
            acc[i][j] = YCX_MFMA16(af[2 * SUB * ks + kk][i], bfr[j], acc[i][j], 0, 0, 0);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    // epilogue 1: y1 to HBM (when stored) and, as the second conv's B operand, to LDS.
    // The previous tile's second-conv reads of y1s finished before this tile's ring barriers.
    const int pt0 = (t0 + tl) * PT;
    const int co = cob + 8 * (lane >> 4);  // channels co .. co+7
    const int s1 = co >> 6, c1 = (co >> 3) & 7;
    const float nl2e = silu_nl2e();  // act4: the packed form of ycx_act<true>, bit-identical
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      eltx8 ov;
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        const f32x4 v = act4(acc[i][j] + bv[i], a.act, a.slope, nl2e);
#pragma unroll
        for (int q = 0; q < 4; ++q) ov[4 * i + q] = (elt_t)v[q];
      }
      const int row = j * 16 + (lane & 15), p = pt0 + row;
      if (store1 && p < a.M)
        if (YCX_OUT_OK(a, Y1 + (size_t)p * a.out_cs + co, sizeof(eltx8))) *reinterpret_cast<eltx8*>(Y1 + (size_t)p * a.out_cs + co) = ov;
      *reinterpret_cast<eltx8*>(y1s + s1 * SLAB + row * 128 + ((c1 ^ swz<64>(row)) << 4)) = ov;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the raw s_barrier does not wait for LDS stores
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    // second conv on the y1 tile
    f32x4 acc2[FM][FN2];
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN2; ++j) acc2[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kk = 0; kk < K2 / 32; ++kk) {
      const int c = (kk & 1) * 4 + (lane >> 4);
      const char* Bs = y1s + (kk >> 1) * SLAB;
      eltx8 bfr[FN2];
#pragma unroll
      for (int j = 0; j < FN2; ++j) {
        const int row = h2 * 16 * FN2 + j * 16 + (lane & 15);
        bfr[j] = *reinterpret_cast<const eltx8*>(Bs + row * 128 + ((c ^ swz<64>(row)) << 4));
      }
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN2; ++j) acc2[i][j] = YCX_MFMA16(af2[kk][i], bfr[j], acc2[i][j], 0, 0, 0);
    }
    __builtin_amdgcn_sched_barrier(0);
    const int co2 = cob2 + 8 * (lane >> 4);
#pragma unroll
    for (int j = 0; j < FN2; ++j) {
      eltx8 ov;
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        const f32x4 v = act4(acc2[i][j] + bv2[i], b.act, b.slope, nl2e);
#pragma unroll
        for (int q = 0; q < 4; ++q) ov[4 * i + q] = (elt_t)v[q];
      }
      const int p = pt0 + h2 * 16 * FN2 + j * 16 + (lane & 15);
      if (p < b.M && co2 < b.Cout)
        if (YCX_OUT_OK(b, Y2 + (size_t)p * b.out_cs + co2, sizeof(eltx8))) *reinterpret_cast<eltx8*>(Y2 + (size_t)p * b.out_cs + co2) = ov;
    }
  }
}

// -------------------------------------------------------------------------
// fp8 weight-resident 1x1 conv (tile 36): conv1x1_wres's structure on the
// block-scaled e4m3 MFMA. Wave (wc, wp) holds the e4m3 rows of output channels
// 32 wc .. +31 of its group for all of K in registers (K/4 VGPRs: 64 at
// cin 512) and streams PT-pixel tiles of activations HBM -> LDS once each
// through an NS-stage LDS-DMA ring of 128-channel slabs (PT rows x 128 B,
// XOR-swizzled as in conv_f8_glds); one ring step = one 16x16x128 MFMA per
// fragment pair. The ring runs across tiles: a full tile's epilogue issues
// exactly FM x FN dword stores per wave, counted into the next waits.
// Requires 1x1/s1/p0, cin = 128 KC (KC = 1, 2, 4), NHWC e4m3 output without residual.
// -------------------------------------------------------------------------
// The epilogue runs beside the next tile's first-step MFMAs as in conv1x1_wres (PIPE there).
template <int WCO, int WPX, int TPW, int KC, int NS, int ACT>
__global__ void __launch_bounds__(WCO * WPX * 64) conv1x1_wres_f8(ConvArgs a) {
  constexpr int NW = WCO * WPX, PT = TPW * WPX, FM = 2, FN = TPW / 16, BCO = WCO * 32;
  constexpr int STAGE = PT * 128, A_PW = PT / (8 * NW);
  constexpr int NSTO = FN;  // 8-byte stores per wave per tile (A rows permuted: 8 channels per lane)
  constexpr int VM_RING = A_PW * (NS - 2);
  static_assert(A_PW >= 1 && PT % (8 * NW) == 0 && TPW % 16 == 0, "tile rows per wave");
  __shared__ __attribute__((aligned(1024))) char smem[NS * STAGE];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wc = wid % WCO, wp = wid / WCO;
  const int G = a.n_ct;
  const int L = ycx_xcd_remap(blockIdx.x, a.nwg);
  const int g = L % G, r = L / G, R = a.nwg / G;
  const int T = (a.M + PT - 1) / PT;
  const int t0 = (int)((long long)r * T / R), t1 = (int)((long long)(r + 1) * T / R);
  if (t0 >= t1) return;  // whole block: no barrier is left waiting
  const int cob = g * BCO + wc * 32;
  const int c0 = 2 * (lane >> 4);

  // this wave's weights: A fragment (slab s, i) = bytes 128 s + 16 c0 .. +31 of the weight row of
  // channel cob + 8 (m >> 2) + 4 i + (m & 3), m = lane & 15: the C rows 4g .. 4g+3 of fragments 0
  // and 1 are then channels 8g .. 8g+7 of the wave's 32, one 8-byte e4m3 store per lane and pixel
  const uint8_t* __restrict__ Wt = reinterpret_cast<const uint8_t*>(a.w);
  i32x8 af[KC][FM];
#pragma unroll
  for (int s = 0; s < KC; ++s)
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const int m = lane & 15;
      const uint8_t* w = Wt + (size_t)(cob + 8 * (m >> 2) + 4 * i + (m & 3)) * a.Ktot + 128 * s + 16 * c0;
      const i32x4 lo = *reinterpret_cast<const i32x4*>(w), hi = *reinterpret_cast<const i32x4*>(w + 16);
      af[s][i] = i32x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    }
  f32x4 bv[FM], qv[FM];
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    const int co = cob + 8 * (lane >> 4) + 4 * i;
    const bool ok = co < a.Cout;
    bv[i] = ok ? *reinterpret_cast<const f32x4*>(a.bias + co) : f32x4{0.f, 0.f, 0.f, 0.f};
    qv[i] = ok ? *reinterpret_cast<const f32x4*>(a.bias + a.Cout_pad + co) : f32x4{0.f, 0.f, 0.f, 0.f};
  }

  // LDS-DMA: wave-instruction (wid + NW i) fills rows 8 (wid + NW i) .. +7 of a slab
  const uint8_t* __restrict__ X = reinterpret_cast<const uint8_t*>(a.x);
  const int x_bytes = a.M * a.in_cs;
  const int lrow = lane >> 3, pch = lane & 7;
  int rrow[A_PW], roff[A_PW];
#pragma unroll
  for (int i = 0; i < A_PW; ++i) {
    rrow[i] = 8 * (wid + NW * i) + lrow;
    roff[i] = rrow[i] * a.in_cs + a.in_coff + ((pch ^ swz8(rrow[i])) << 4);
  }
  const int nst = (t1 - t0) * KC;
  auto issue = [&](int s) {
    const int tl = s / KC, ks = s - tl * KC;
    const int px0 = (t0 + tl) * PT;
    char* base = smem + (s % NS) * STAGE;
#pragma unroll
    for (int i = 0; i < A_PW; ++i) {
      const int off = px0 + rrow[i] < a.M ? px0 * a.in_cs + roff[i] + ks * 128 : 0x7FFFFFF0;
      buf_lds16(X, x_bytes, off, 0, base + (wid + NW * i) * 1024);
    }
  };
  for (int s = 0; s < NS - 1 && s < nst; ++s) issue(s);

  const bool exact = a.Cout == a.Cout_pad;  // then every full tile stores exactly NSTO times per wave
  uint8_t* __restrict__ Y = reinterpret_cast<uint8_t*>(a.y) + a.out_coff;
  const float osc = a.out_scale;
  const float nl2e = silu_nl2e();  // act4_t and a packed fma: bit-identical to fmaf + ycx_act<true>
  const int co = cob + 8 * (lane >> 4);  // channels co .. co+7 (cout % 8 == 0: all valid or none)
  auto finish = [&](const f32x4 (&s)[FM][FN], uint2 (&ov)[FN]) {
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      f32x4 x[FM];
#pragma unroll
      for (int i = 0; i < FM; ++i) x[i] = act4_t<ACT>(__builtin_elementwise_fma(s[i][j], qv[i], bv[i]), a.slope, nl2e) * osc;
      ov[j] = make_uint2(f8x4_pack(x[0][0], x[0][1], x[0][2], x[0][3]), f8x4_pack(x[1][0], x[1][1], x[1][2], x[1][3]));
    }
  };
  auto store = [&](int tl, const uint2 (&ov)[FN]) {
    const int pb = (t0 + tl) * PT + wp * TPW + (lane & 15);
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int p = pb + 16 * j;
      if (p < a.M && co < a.Cout) if (YCX_OUT_OK(a, Y + (size_t)p * a.out_cs + co, sizeof(uint2))) *reinterpret_cast<uint2*>(Y + (size_t)p * a.out_cs + co) = ov[j];
    }
  };
  static_assert(FM == 2, "two fragments: 8 channels per lane");
  f32x4 acc[FM][FN], accp[FM][FN];  // accp: the previous tile's sums
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  int t = 0;
  for (int tl = 0; tl < t1 - t0; ++tl) {
#pragma unroll
    for (int ks = 0; ks < KC; ++ks, ++t) {
      // wait for stage t: younger than its loads are the NS-2 later stages and the store
      // batches issued in steps t-NS+1 .. t-1 (a tile's batch in the next tile's first step)
      if (t + NS - 2 >= nst) {
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
      } else {
        const int lo = t - NS + 1 > KC ? t - NS + 1 : KC;  // batches: steps i KC, i >= 1
        const int nb = exact && t - 1 >= lo ? (t - 1) / KC - (lo + KC - 1) / KC + 1 : 0;
        wait_vm_counted<VM_RING, 0, (NS + KC - 2) / KC * NSTO>(nb > 0 ? nb * NSTO : 0);
      }
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      if (t + NS - 1 < nst) issue(t + NS - 1);
      if (ks == 0) {
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j) {
            accp[i][j] = acc[i][j];
            acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
          }
      }
      const char* B = smem + (t % NS) * STAGE;
      i32x8 bfr[FN];
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int row = wp * TPW + j * 16 + (lane & 15);
        const i32x4 lo = *reinterpret_cast<const i32x4*>(B + row * 128 + ((c0 ^ swz8(row)) << 4));
        const i32x4 hi = *reinterpret_cast<const i32x4*>(B + row * 128 + (((c0 + 1) ^ swz8(row)) << 4));
        bfr[j] = i32x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      }
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(af[ks][i], bfr[j], acc[i][j], 0, 0, 0, 127,
                                                                       0, 127);
      if (ks == 0) {  // the previous tile's epilogue beside this step's MFMAs (same basic block)
        uint2 ov[FN];
        finish(accp, ov);
#pragma unroll
        for (int j = 0; j < FN; ++j) asm volatile("" ::"v"(ov[j].x), "v"(ov[j].y));  // not sunk into the stores
        __builtin_amdgcn_sched_barrier(0);
        if (tl > 0) store(tl - 1, ov);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  {
    uint2 ov[FN];
    finish(acc, ov);
    store(t1 - t0 - 1, ov);
  }
}

// -------------------------------------------------------------------------
// fp8 weight-stationary 3x3 64 -> 64 (tile 37): conv3x3_ws64 on the e4m3
// block-scaled MFMA. One K step of 128 = two taps x 64 channels, so the nine
// taps are five steps (the tenth tap's weights are the zero padding of the
// 640-byte weight rows, its B operand any finite pixel). Persistent 512-thread
// block per CU: all five 128-byte weight slices of the 64 output channels in
// LDS (40 KB, chunk q of row (step, co) at q ^ swz(co)); 16x16 output tiles
// whose 18x18 halo (64 B per pixel) is LDS-DMA'd into the second buffer while
// the current tile computes. Halo chunk q of pixel h lives at q ^ ((h >> 2) & 1):
// with the 16x16x128 B-fragment lane map (lane -> pixel l & 15, chunk pair of
// group l >> 4) every ds_read_b128 lane group then hits 16 distinct 16-B bank
// granules at any halo offset (brute-forced over all offsets). Epilogue:
// act(acc * dq + bias) * out_scale -> e4m3, 4 B per lane; the stores enter the
// next tile's counted vmcnt wait.
// -------------------------------------------------------------------------
template <int ACT>
__global__ void __launch_bounds__(512) conv3x3_ws64_f8(ConvArgs a) {
  constexpr int NW = 8, TH = 16, TW = 16, HW = TW + 2, HP = (TH + 2) * HW;  // 324 halo pixels
  constexpr int HPIECES = (HP + 15) / 16, HPW = (HPIECES + NW - 1) / NW;    // 1-KB DMA pieces (16 pixels)
  constexpr int HBUF = HPIECES * 1024, WBYTES = 5 * 64 * 128;
  constexpr int FM = 2, FN = 4;
  __shared__ __attribute__((aligned(1024))) char smem[WBYTES + 2 * HBUF];
  char* const wl = smem;
  const uint8_t* __restrict__ X = reinterpret_cast<const uint8_t*>(a.x);
  const uint8_t* __restrict__ Wt = reinterpret_cast<const uint8_t*>(a.w);
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 2, wn = wid & 3;
  const int lrow = lane >> 3, pch = lane & 7;
  const int tx_n = a.Wo / TW, tpi = (a.Ho / TH) * tx_n, ntiles = a.N * tpi;
  const int blk = ycx_xcd_remap(blockIdx.x, gridDim.x);
  const int tb = (int)((long long)blk * ntiles / gridDim.x), te = (int)((long long)(blk + 1) * ntiles / gridDim.x);
  if (tb >= te) return;
  const int w_bytes = a.Cout_pad * a.Ktot, x_bytes = a.N * a.H * a.W * a.in_cs;

  // weights: LDS row R = 64 step + co (128 B), logical chunk q at q ^ swz(co); 40 pieces, 5 per wave.
  // Row co holds channel 32 (co >> 5) + 8 (m >> 2) + 4 f + (m & 3) (f = co >> 4 & 1, m = co & 15), as in
  // conv3x3_ws64: C rows 4g..4g+3 of the two fragments are channels 32 wm + 8g .. +7, one 8-byte store
  // per lane and pixel
#pragma unroll
  for (int i = 0; i < 5; ++i) {
    const int R = 8 * (wid + NW * i) + lrow, st = R >> 6, co = R & 63, m = co & 15;
    const int ch = (co & 32) + 8 * (m >> 2) + 4 * ((co >> 4) & 1) + (m & 3);
    buf_lds16(Wt, w_bytes, ch * a.Ktot + st * 128 + ((pch ^ swz8(co)) << 4), 0, wl + (wid + NW * i) * 1024);
  }
  // halo of a tile into buffer b: a 1-KB piece is 16 pixels; lane -> pixel (lane >> 2), physical chunk lane & 3
  auto issue_h = [&](int tile, int b) {
    const int n = tile / tpi, ti = tile - n * tpi;
    const int oy0 = (ti / tx_n) * TH, ox0 = (ti % tx_n) * TW;
#pragma unroll
    for (int i = 0; i < HPW; ++i) {
      const int piece = wid + NW * i;
      if (piece >= HPIECES) break;  // uniform
      const int h = 16 * piece + (lane >> 2), hy = h / HW, hx = h - hy * HW;
      const int iy = oy0 - 1 + hy, ix = ox0 - 1 + hx;
      const bool ok = h < HP && (unsigned)iy < (unsigned)a.H && (unsigned)ix < (unsigned)a.W;
      const int lc = (lane & 3) ^ ((h >> 2) & 1);  // logical chunk this lane fetches
      buf_lds16(X, x_bytes, ok ? ((n * a.H + iy) * a.W + ix) * a.in_cs + a.in_coff + (lc << 4) : 0x7FFFFFF0, 0,
                smem + WBYTES + b * HBUF + piece * 1024);
    }
  };
  issue_h(tb, 0);
  f32x4 bv[FM], qv[FM];
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    const int co = 32 * wm + 8 * (lane >> 4) + 4 * i;
    const bool ok = co < a.Cout;
    bv[i] = ok ? *reinterpret_cast<const f32x4*>(a.bias + co) : f32x4{0.f, 0.f, 0.f, 0.f};
    qv[i] = ok ? *reinterpret_cast<const f32x4*>(a.bias + a.Cout_pad + co) : f32x4{0.f, 0.f, 0.f, 0.f};
  }
  const float nl2e = silu_nl2e();
  const bool exact = a.Cout == 64;  // then every tile stores FN times per wave
  uint8_t* __restrict__ Y = reinterpret_cast<uint8_t*>(a.y) + a.out_coff;
  const float osc = a.out_scale;
  const int g = lane >> 4, c0 = 2 * g;   // A: chunk pair of the 128-B row
  const int hc2 = 2 * (g & 1);            // B: channel half (chunk pair) of the tap

  for (int tile = tb; tile < te; ++tile) {
    const int b = (tile - tb) & 1;
    if (tile > tb && exact) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(FN) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();  // this tile's halo (and the weights) landed; the other buffer is free
    if (tile + 1 < te) issue_h(tile + 1, b ^ 1);
    const char* halo = smem + WBYTES + b * HBUF;
    f32x4 acc[FM][FN];
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 1
    for (int st = 0; st < 5; ++st) {  // not unrolled: hoisting 5 steps' lane addresses spills
      int t = 2 * st + (g >> 1);
      t = t > 8 ? 8 : t;  // the tenth tap: zero weights, any finite pixel
      const int ky = t / 3, kx = t - 3 * ky;
      i32x8 af[FM], bfr[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        const int co = 32 * wm + 16 * i + (lane & 15);
        const char* row = wl + (st * 64 + co) * 128;
        const i32x4 lo = *reinterpret_cast<const i32x4*>(row + ((c0 ^ swz8(co)) << 4));
        const i32x4 hi = *reinterpret_cast<const i32x4*>(row + (((c0 + 1) ^ swz8(co)) << 4));
        af[i] = i32x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      }
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int h = (wn * FN + j + ky) * HW + (lane & 15) + kx;
        const int sw = (h >> 2) & 1;
        const char* px = halo + h * 64;
        const i32x4 lo = *reinterpret_cast<const i32x4*>(px + ((hc2 ^ sw) << 4));
        const i32x4 hi = *reinterpret_cast<const i32x4*>(px + (((hc2 + 1) ^ sw) << 4));
        bfr[j] = i32x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      }
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(af[i], bfr[j], acc[i][j], 0, 0, 0, 127, 0, 127);
      __builtin_amdgcn_sched_barrier(0);  // one step's fragments live at a time
    }
    // epilogue: e4m3 8-byte stores (8 consecutive channels per lane and pixel) from registers
    // (no global loads: they would drain vmcnt); dequant-fma and act as packed fp32
    const int n = tile / tpi, ti = tile - n * tpi;
    const int oy0 = (ti / tx_n) * TH, ox0 = (ti % tx_n) * TW;
    const int co = 32 * wm + 8 * (lane >> 4);
    if (co < a.Cout) {  // cout % 8 == 0: the 8 channels are all valid
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int p = n * a.HoWo + (oy0 + wn * FN + j) * a.Wo + ox0 + (lane & 15);
        const f32x4 x0 = act4_t<ACT>(__builtin_elementwise_fma(acc[0][j], qv[0], bv[0]), a.slope, nl2e) * osc;
        const f32x4 x1 = act4_t<ACT>(__builtin_elementwise_fma(acc[1][j], qv[1], bv[1]), a.slope, nl2e) * osc;
        if (YCX_OUT_OK(a, Y + (size_t)p * a.out_cs + co, sizeof(uint2)))
          *reinterpret_cast<uint2*>(Y + (size_t)p * a.out_cs + co) =
              make_uint2(f8x4_pack(x0[0], x0[1], x0[2], x0[3]), f8x4_pack(x1[0], x1[1], x1[2], x1[3]));
      }
    }
  }
}

ConvArgs make_args(const ycx_conv_desc* d, const void* x, const void* w, const float* bias, void* y,
                   const void* res) {
  ConvArgs a;
  a.x = x; a.w = w; a.bias = bias; a.y = y; a.res = res;
  a.N = d->n; a.H = d->h; a.W = d->w; a.Cin = d->cin; a.in_coff = d->in_c_off; a.in_cs = d->in_c_stride;
  a.Ho = d->ho; a.Wo = d->wo; a.Cout = d->cout; a.Cout_pad = d->cout_pad;
  a.out_coff = d->out_c_off; a.out_cs = d->out_c_stride;
  a.KH = d->kh; a.KW = d->kw; a.S = d->stride; a.P = d->pad;
  a.act = d->act; a.slope = d->leaky_slope; a.out_layout = d->out_layout;
  a.res_coff = d->res_c_off; a.res_cs = d->res_c_stride;
  a.M = d->n * d->ho * d->wo; a.HoWo = d->ho * d->wo; a.Ktot = d->kh * d->kw * d->cin;
  if (d->dtype == YCX_DT_FP8) a.Ktot = (a.Ktot + 127) / 128 * 128;  // padded weight row (bytes)
  a.nsteps = 0; a.n_ct = 0; a.nwg = 0; a.gc = 0;
  a.out_scale = d->out_scale; a.res_scale = d->res_scale;
  a.pool = d->in_pool;
  a.ks = d->k_split > 1 ? d->k_split : 1;
  a.part = nullptr;
  {
    const long long es = d->dtype == YCX_DT_F32 ? 4 : d->dtype == YCX_DT_FP8 ? 1 : 2;
    const long long px = (long long)d->n * d->ho * d->wo * (d->out_layout == YCX_OUT_NHWC_UP2 ? 4 : 1);
    a.out_bytes = px * d->out_c_stride * (d->out_layout == YCX_OUT_NCHW_F32 ? 4 : es);
  }
  return a;
}

struct TileInfo {
  int bm, bn, bk;
  const char* name;
};
// Tile ids (ycx_conv_desc.tile): 1..N. Keep in sync with launch_bf16 below.
const TileInfo kTiles[] = {
    {0, 0, 0, "auto"},
    {128, 128, 64, "bf16_co128_px128_k64"},
    {64, 256, 64, "bf16_co64_px256_k64"},
    {64, 128, 64, "bf16_co64_px128_k64"},
    {128, 64, 64, "bf16_co128_px64_k64"},
    {32, 256, 32, "bf16_co32_px256_k32"},
    {64, 256, 32, "bf16_co64_px256_k32"},
    {128, 128, 32, "bf16_co128_px128_k32"},
    {64, 64, 16, "f32_co64_px64_k16"},
    {128, 256, 64, "glds_co128_px256_k64"},
    {64, 256, 64, "glds_co64_px256_k64"},
    {256, 128, 64, "glds_co256_px128_k64"},
    {128, 128, 64, "glds_co128_px128_k64"},
    {64, 256, 32, "glds2_co64_px256_k32x2"},
    {128, 256, 32, "glds2_co128_px256_k32x2"},
    {64, 256, 64, "glds_co64_px256_k64_s2"},
    {128, 128, 64, "glds_co128_px128_k64_s2"},
    {64, 256, 32, "glds2_co64_px256_k32x2_s2"},
    {64, 128, 64, "glds_co64_px128_k64_s2"},
    {64, 256, 64, "halo3x3_co64_t16x16"},
    {128, 256, 64, "halo3x3_co128_t16x16_s2"},
    {128, 256, 64, "halo3x3_co128_t16x16_s3"},
    {32, 64, 64, "wres1x1"},
    {64, 256, 64, "halo3x3_ws_co64"},
    {256, 256, 64, "glds_co256_px256_k64_s2"},
    {256, 128, 64, "glds_co256_px128_k64_s2"},
    {128, 256, 64, "glds_co128_px256_k64_s2"},
    {256, 256, 64, "retired_p8_co256_px256"},     // 27-33: retired experiments, kept in
    {128, 256, 64, "retired_p8_co128_px256"},     // tools/experiments/pingpong_p8_tiles27_33.patch
    {256, 128, 64, "retired_p8_co256_px128"},
    {256, 256, 64, "retired_p8i_co256_px256"},
    {128, 256, 64, "retired_p8i_co128_px256"},
    {128, 128, 64, "retired_glds4w_co128_px128"},
    {64, 128, 64, "retired_glds4w_co64_px128"},
    {128, 128, 16, "f8_co128_px128_k128_s2"},
    {64, 128, 16, "f8_co64_px128_k128_s2"},
    {32, 64, 128, "f8_wres1x1"},
    {64, 256, 64, "f8_halo3x3_ws_co64"},
    {256, 64, 64, "head_co256_px64_decode"},
    {256, 64, 128, "f8_head_co256_px64_decode"},
    {256, 256, 32, "retired_big_co256_px256_k32_s4"},  // 40-47: retired (tools/experiments/conv_bigt_tiles40_47.patch)
    {256, 128, 32, "retired_big_co256_px128_k32_s3"},
    {128, 256, 32, "retired_big_co128_px256_k32_s3"},
    {128, 128, 32, "retired_big_co128_px128_k32_s4"},
    {256, 128, 32, "retired_big_co256_px128_k32_s3_dma_after_reads"},
    {256, 128, 32, "retired_big_co256_px128_k32_s3_dma_mid_mfma"},
    {256, 128, 32, "retired_big_co256_px128_k32_s3_dma_after_mfma"},
    {256, 256, 32, "retired_big_co256_px256_k32_s4_dma_after_mfma"},
    {64, 320, 64, "halo3x3_band_co64_8x40_s2"},
    {128, 160, 64, "halo3x3_band_co128_4x40_s2"},
    {128, 128, 64, "halo3x3s2_wsr_co128"},
    {256, 128, 64, "retired_glds16w_co256_px128_s2"},  // 51-54: 16-wave tiles, measured slower
    {128, 256, 64, "retired_glds16w_co128_px256_s2"},
    {256, 128, 64, "retired_glds16w_co256_px128_s3"},
    {128, 256, 64, "retired_glds16w_co128_px256_s3"},
    {256, 64, 64, "wres1x1_pair"},  // 55: ycx_conv2d_pair only (two chained 1x1 convs)
    {64, 128, 64, "glds_co64_px128_k64_s3"},  // 56: tile 18 with a three-stage ring (r06)
    {128, 128, 64, "retired_wsp_co128_px128_k64_ns4"},  // 57: tools/experiments/wsp_tile57.patch (r06)
};
constexpr int kNumTiles = sizeof(kTiles) / sizeof(kTiles[0]);

template <int BM, int BN, int BK, int WM, int WN>
ycx_status launch_bf16(ConvArgs a, hipStream_t st) {
  a.nsteps = a.KH * a.KW * (a.Cin / BK);
  a.n_ct = a.Cout_pad / BM;
  int n_pt = (a.M + BN - 1) / BN;
  a.nwg = a.n_ct * n_pt;
  hipLaunchKernelGGL((conv_bf16_kernel<BM, BN, BK, WM, WN>), dim3(a.nwg), dim3(256), 0, st, a);
  return ycx_launch_status();
}

// Persistent grids (r06): the fewest blocks that keep a full grid's largest per-block tile count,
// ceil(T / ceil(T / cap)) for T balanced tiles on at most cap blocks: the same time for this launch,
// and the CUs it leaves run the other batches in flight (80^2 ws64: 800 tiles, 256 -> 200 blocks).
inline long long even_grid(long long T, long long cap) {
  if (T <= cap) return T;
  const long long per = (T + cap - 1) / cap;
  return (T + per - 1) / per;
}

bool ws64_ok(const ConvArgs& a) {
  return a.KH == 3 && a.KW == 3 && a.S == 1 && a.P == 1 && a.H == a.Ho && a.W == a.Wo && a.Ho % 16 == 0 &&
         a.Wo % 16 == 0 && a.Cin == 64 && a.Cout_pad == 64 && a.out_layout == YCX_OUT_NHWC && !a.res &&
         (long long)a.N * a.H * a.W * a.in_cs * 2 < (1LL << 31) - 64;
}

// tile 23: one persistent block per CU
ycx_status launch_ws64(ConvArgs a, hipStream_t st) {
  if (!ws64_ok(a)) return YCX_ERR_UNSUPPORTED;
  const long long ntiles = (long long)a.N * (a.Ho / 16) * (a.Wo / 16);
#ifndef YCX_WS64_BLOCKS  // development A/B knob: the persistent grid's block cap
#define YCX_WS64_BLOCKS 256
#endif
  const dim3 g((unsigned)even_grid(ntiles, YCX_WS64_BLOCKS)), b(512);
  switch (a.act) {
    case YCX_ACT_SILU_PS: hipLaunchKernelGGL((conv3x3_ws64<YCX_ACT_SILU_PS>), g, b, 0, st, a); break;
    case YCX_ACT_SILU: hipLaunchKernelGGL((conv3x3_ws64<YCX_ACT_SILU>), g, b, 0, st, a); break;
    case YCX_ACT_LEAKY: hipLaunchKernelGGL((conv3x3_ws64<YCX_ACT_LEAKY>), g, b, 0, st, a); break;
    default: hipLaunchKernelGGL((conv3x3_ws64<YCX_ACT_NONE>), g, b, 0, st, a); break;
  }
  return ycx_launch_status();
}

bool s2wsr_ok(const ConvArgs& a) {
  return a.KH == 3 && a.KW == 3 && a.S == 2 && a.P == 1 && a.Ho % 4 == 0 && a.Wo % 16 == 0 && a.Cin == 64 &&
         a.Cout_pad == 128 && a.out_layout == YCX_OUT_NHWC && !a.res && !a.pool &&
         (long long)a.N * a.H * a.W * a.in_cs * 2 < (1LL << 31) - 64;
}

// tile 50: one persistent block per CU; NB halo buffers (NB - 1 tiles in flight)
#ifndef YCX_S2WSR_NB
#define YCX_S2WSR_NB 2
#endif
ycx_status launch_s2wsr(ConvArgs a, hipStream_t st) {
  if (!s2wsr_ok(a)) return YCX_ERR_UNSUPPORTED;
  const long long ntiles = (long long)a.N * (a.Ho / 4) * (a.Wo / 16);
  const dim3 g((unsigned)even_grid(ntiles, 256)), b(512);
  switch (a.act) {
    case YCX_ACT_SILU_PS: hipLaunchKernelGGL((conv3x3s2_wsr<YCX_ACT_SILU_PS, 4, YCX_S2WSR_NB>), g, b, 0, st, a); break;
    case YCX_ACT_SILU: hipLaunchKernelGGL((conv3x3s2_wsr<YCX_ACT_SILU, 4, YCX_S2WSR_NB>), g, b, 0, st, a); break;
    case YCX_ACT_LEAKY: hipLaunchKernelGGL((conv3x3s2_wsr<YCX_ACT_LEAKY, 4, YCX_S2WSR_NB>), g, b, 0, st, a); break;
    default: hipLaunchKernelGGL((conv3x3s2_wsr<YCX_ACT_NONE, 4, YCX_S2WSR_NB>), g, b, 0, st, a); break;
  }
  return ycx_launch_status();
}

template <int BM, int WM, int WN, int NSTA, int TH = 16, int TW = 16>
ycx_status launch_halo(ConvArgs a, hipStream_t st) {
  constexpr bool BAND = TW != 16;
  if (a.KH != 3 || a.KW != 3 || a.S != 1 || a.P != 1 || a.H != a.Ho || a.W != a.Wo || a.Ho % TH ||
      (BAND ? a.Wo != TW : a.Wo % TW != 0) || a.Cin % 64 || a.Cout_pad % BM || a.out_layout == YCX_OUT_NCHW_F32)
    return YCX_ERR_UNSUPPORTED;
  a.n_ct = a.Cout_pad / BM;
  a.nwg = a.n_ct * a.N * (a.Ho / TH) * (a.Wo / TW);
  hipLaunchKernelGGL((conv3x3_halo<BM, WM, WN, NSTA, TH, TW>), dim3(a.nwg), dim3(WM * WN * 64), 0, st, a);
  return ycx_launch_status();
}

// Channel groups of the XCD region map (ycx_tile_of) for an LDS-DMA tile launch: 0 (plain
// bijective XCD remap). The region map (gc 2 / 4) measured slower in the concurrent bench
// (DESIGN.md §6 r03); -DYCX_GLDS_GC=<g> builds it for an A/B.
#ifndef YCX_GLDS_GC
#define YCX_GLDS_GC 0
#endif
static inline int glds_gc(const ConvArgs&) { return YCX_GLDS_GC; }

template <int BM, int BN, int WM, int WN, bool TT = false, int NST = 3, int NSB = NST>
ycx_status launch_glds(ConvArgs a, hipStream_t st) {
  if (TT && a.Cin != 32) return YCX_ERR_UNSUPPORTED;
  if (!TT && a.Cin % 64 != 0) return YCX_ERR_UNSUPPORTED;
  a.nsteps = TT ? (a.KH * a.KW + 1) / 2 : a.KH * a.KW * (a.Cin / 64);
  a.n_ct = a.Cout_pad / BM;
  a.nwg = a.n_ct * ((a.M + BN - 1) / BN);
  a.gc = glds_gc(a);
  if constexpr (!TT && NST == 2 && NSB == 2 && BN == 128) {  // tiles 16, 18, 25
    if (a.pool) {
      if (a.KH != 1 || a.KW != 1 || a.S != 1 || a.P != 0) return YCX_ERR_UNSUPPORTED;
      hipLaunchKernelGGL((conv_bf16_glds<BM, BN, WM, WN, false, 2, 2, false, true>), dim3(a.nwg), dim3(WM * WN * 64),
                         0, st, a, HeadArgs{});
      return ycx_launch_status();
    }
  }
  if (a.pool) return YCX_ERR_UNSUPPORTED;
  if constexpr (!TT && NSB == NST && BN == 128 && (BM == 128 || BM == 64)) {  // tiles 16, 18, 56: split-K
    if (a.ks > 1) {
      if (!a.part || a.out_layout == YCX_OUT_NCHW_F32 || a.ks > a.nsteps) return YCX_ERR_UNSUPPORTED;
      const dim3 g(a.nwg * a.ks), b(WM * WN * 64);
      if (a.S == 2 && a.KH == 3 && a.KW == 3 && a.Cin == 128 && BM == 128 && NST == 2)
        hipLaunchKernelGGL((conv_bf16_glds<BM, BN, WM, WN, false, NST, NST, false, false, true, true>), g, b, 0, st, a,
                           HeadArgs{});
      else
        hipLaunchKernelGGL((conv_bf16_glds<BM, BN, WM, WN, false, NST, NST, false, false, false, true>), g, b, 0, st,
                           a, HeadArgs{});
      ycx_status s = ycx_launch_status();
      if (s != YCX_OK) return s;
      const long long total = (long long)a.M * (a.Cout >> 3);
      const dim3 rg((unsigned)std::min<long long>((total + 255) / 256, 4096)), rb(256);
      switch (a.act) {
        case YCX_ACT_SILU_PS: hipLaunchKernelGGL(splitk_reduce<YCX_ACT_SILU_PS>, rg, rb, 0, st, a); break;
        case YCX_ACT_SILU: hipLaunchKernelGGL(splitk_reduce<YCX_ACT_SILU>, rg, rb, 0, st, a); break;
        case YCX_ACT_LEAKY: hipLaunchKernelGGL(splitk_reduce<YCX_ACT_LEAKY>, rg, rb, 0, st, a); break;
        default: hipLaunchKernelGGL(splitk_reduce<YCX_ACT_NONE>, rg, rb, 0, st, a); break;
      }
      return ycx_launch_status();
    }
  }
  if (a.ks > 1) return YCX_ERR_UNSUPPORTED;
  if constexpr (!TT && NST == 2 && NSB == 2 && BM == 128 && BN == 128) {  // tile 16 on a 3x3/s2 at Cin 128
    if (a.S == 2 && a.KH == 3 && a.KW == 3 && a.Cin == 128) {  // Cin 256 / 512: slower
      hipLaunchKernelGGL((conv_bf16_glds<BM, BN, WM, WN, false, 2, 2, false, false, true>), dim3(a.nwg),
                         dim3(WM * WN * 64), 0, st, a, HeadArgs{});
      return ycx_launch_status();
    }
  }
  hipLaunchKernelGGL((conv_bf16_glds<BM, BN, WM, WN, TT, NST, NSB>), dim3(a.nwg), dim3(WM * WN * 64), 0, st, a,
                     HeadArgs{});
  return ycx_launch_status();
}

// tile 38 (bf16) / 39 (e4m3): Detect head conv (all <= 256 channels of BN = 64 pixels per
// workgroup) + decode + filter
ycx_status launch_head(ConvArgs a, const HeadArgs& hd, hipStream_t st, bool f8) {
  if (f8) {  // one 128-channel K step per tap (cin % 128 == 0), weight rows of whole K steps
    if (a.Cin % 128 || a.Cout_pad != 256 || a.Cout > 256 || a.Ktot != a.Cin) return YCX_ERR_UNSUPPORTED;
    a.nsteps = a.Cin / 128;
    a.n_ct = 1;
    a.nwg = (a.M + 63) / 64;
    hipLaunchKernelGGL((conv_f8_glds<256, 64, 4, 2, 1, true>), dim3(a.nwg), dim3(512), 0, st, a, hd);
    return ycx_launch_status();
  }
  if (a.Cin % 64 || a.Cout_pad != 256 || a.Cout > 256) return YCX_ERR_UNSUPPORTED;
  a.nsteps = a.KH * a.KW * (a.Cin / 64);
  a.n_ct = 1;
  a.nwg = (a.M + 63) / 64;
  hipLaunchKernelGGL((conv_bf16_glds<256, 64, 4, 2, false, 2, 2, true>), dim3(a.nwg), dim3(512), 0, st, a, hd);
  return ycx_launch_status();
}

// fp8 tiles 34-35: cin 32 / 64 run 4 / 2 taps per 128-channel K step; other
// cin % 16 == 0 (not 128k) walk k = (tap, channel) per lane (TPS 0).
template <int BM, int BN, int WM, int WN>
ycx_status launch_f8(ConvArgs a, hipStream_t st) {
  const int tps = a.Cin == 32 ? 4 : a.Cin == 64 ? 2 : a.Cin % 128 == 0 ? 1 : 0;
  if (tps == 0 && a.Cin % 16 != 0) return YCX_ERR_UNSUPPORTED;
  if (a.Cout_pad % BM != 0) return YCX_ERR_UNSUPPORTED;
  const int ntaps = a.KH * a.KW;
  a.nsteps = (ntaps * a.Cin + 127) / 128;
  if (a.nsteps * 128 != a.Ktot) return YCX_ERR_UNSUPPORTED;  // weight rows padded to whole K steps
  a.n_ct = a.Cout_pad / BM;
  a.nwg = a.n_ct * ((a.M + BN - 1) / BN);
  a.gc = glds_gc(a);
  const dim3 g(a.nwg), b(WM * WN * 64);
  if (a.pool) {  // fused MP (ycx_conv_desc.in_pool): one 128-channel tap per K step
    if (tps != 1) return YCX_ERR_UNSUPPORTED;
    hipLaunchKernelGGL((conv_f8_glds<BM, BN, WM, WN, 1, false, true>), g, b, 0, st, a, HeadArgs{});
    return ycx_launch_status();
  }
  if (tps == 4) hipLaunchKernelGGL((conv_f8_glds<BM, BN, WM, WN, 4>), g, b, 0, st, a, HeadArgs{});
  else if (tps == 2) hipLaunchKernelGGL((conv_f8_glds<BM, BN, WM, WN, 2>), g, b, 0, st, a, HeadArgs{});
  else if (tps == 1) hipLaunchKernelGGL((conv_f8_glds<BM, BN, WM, WN, 1>), g, b, 0, st, a, HeadArgs{});
  else hipLaunchKernelGGL((conv_f8_glds<BM, BN, WM, WN, 0>), g, b, 0, st, a, HeadArgs{});
  return ycx_launch_status();
}

template <int WCO, int WPX, int TPW, int NS, int SUB, int ACT>
ycx_status launch_wres_cin(const ConvArgs& a, dim3 g, dim3 b, hipStream_t st) {
  switch (a.Cin) {
    case 64: hipLaunchKernelGGL((conv1x1_wres<WCO, WPX, TPW, 1, NS, 1, ACT>), g, b, 0, st, a); break;
    case 128: hipLaunchKernelGGL((conv1x1_wres<WCO, WPX, TPW, 2, NS, SUB, ACT>), g, b, 0, st, a); break;
    case 256: hipLaunchKernelGGL((conv1x1_wres<WCO, WPX, TPW, 4, NS, SUB, ACT>), g, b, 0, st, a); break;
    case 512: hipLaunchKernelGGL((conv1x1_wres<WCO, WPX, TPW, 8, NS, SUB, ACT>), g, b, 0, st, a); break;
    default: return YCX_ERR_UNSUPPORTED;
  }
  return ycx_launch_status();
}

// Weight-resident 1x1 (tile 22): the wave split follows cout_pad, the K unroll Cin.
template <int WCO, int WPX, int TPW, int NS, int SUB>
ycx_status launch_wres_k(ConvArgs a, hipStream_t st) {
  a.n_ct = a.Cout_pad / (WCO * 32);
  const int T = (a.M + TPW * WPX - 1) / (TPW * WPX);
  const int R = std::max(1, (int)even_grid(T, 256 / a.n_ct));
  a.nwg = R * a.n_ct;
  dim3 g(a.nwg), b(WCO * WPX * 64);
  switch (a.act) {
    case YCX_ACT_SILU_PS: return launch_wres_cin<WCO, WPX, TPW, NS, SUB, YCX_ACT_SILU_PS>(a, g, b, st);
    case YCX_ACT_SILU: return launch_wres_cin<WCO, WPX, TPW, NS, SUB, YCX_ACT_SILU>(a, g, b, st);
    case YCX_ACT_LEAKY: return launch_wres_cin<WCO, WPX, TPW, NS, SUB, YCX_ACT_LEAKY>(a, g, b, st);
    default: return launch_wres_cin<WCO, WPX, TPW, NS, SUB, YCX_ACT_NONE>(a, g, b, st);
  }
}

bool wres_ok(const ConvArgs& a) {
  return a.KH == 1 && a.KW == 1 && a.S == 1 && a.P == 0 && a.H == a.Ho && a.W == a.Wo && !a.res &&
         a.out_layout == YCX_OUT_NHWC && (a.Cin == 64 || a.Cin == 128 || a.Cin == 256 || a.Cin == 512) &&
         (a.Cout_pad == 64 || a.Cout_pad == 128 || a.Cout_pad % 256 == 0) &&
         (long long)a.M * a.in_cs * 2 < (1LL << 31) - 64;
}

// tests/probes/conv_bench.py (bs 32): 160^2 256->256 0.30 -> 0.22 ms, 80^2 512->512 0.24 -> 0.16 ms,
// 160^2 256->128 0.17 -> 0.13 ms against tile 16
ycx_status launch_wres(ConvArgs a, hipStream_t st) {
  if (!wres_ok(a)) return YCX_ERR_UNSUPPORTED;
#ifndef YCX_WRES_NS  // ring depth of the 256-channel-group variant (development A/B knob)
#define YCX_WRES_NS 5
#endif
#ifndef YCX_WRES_TPW
#define YCX_WRES_TPW 64
#endif
  if (a.Cout_pad % 256 == 0) return launch_wres_k<8, 1, YCX_WRES_TPW, YCX_WRES_NS, 2>(a, st);  // 16 KB stages
  if (a.Cout_pad == 128) return launch_wres_k<4, 2, 64, 6, 1>(a, st);
  return launch_wres_k<2, 4, 32, 6, 1>(a, st);
}

// tile 55: two chained 1x1 convs (conv1x1_wres_pair), one persistent block per CU
template <int KC, int NS, int SUB>
ycx_status launch_wres_pair_k(ConvArgs a, ConvArgs b, hipStream_t st) {
  const int T = (a.M + 63) / 64;
  a.nwg = std::max(1, (int)even_grid(T, 256));
  if (b.Cout_pad == 128)
    hipLaunchKernelGGL((conv1x1_wres_pair<KC, NS, SUB, 128>), dim3(a.nwg), dim3(512), 0, st, a, b);
  else
    hipLaunchKernelGGL((conv1x1_wres_pair<KC, NS, SUB, 256>), dim3(a.nwg), dim3(512), 0, st, a, b);
  return ycx_launch_status();
}

ycx_status launch_wres_pair(ConvArgs a, ConvArgs b, hipStream_t st) {
  switch (a.Cin) {
    case 64: return launch_wres_pair_k<1, 5, 1>(a, b, st);
    case 128: return launch_wres_pair_k<2, 5, 2>(a, b, st);
    case 256: return launch_wres_pair_k<4, YCX_WRES_NS, 2>(a, b, st);
    default: return YCX_ERR_UNSUPPORTED;
  }
}

bool wres_f8_ok(const ConvArgs& a) {
  return a.KH == 1 && a.KW == 1 && a.S == 1 && a.P == 0 && a.H == a.Ho && a.W == a.Wo && !a.res &&
         a.out_layout == YCX_OUT_NHWC && (a.Cin == 128 || a.Cin == 256 || a.Cin == 512) && a.Ktot == a.Cin &&
         (a.Cout_pad == 64 || a.Cout_pad == 128 || a.Cout_pad % 256 == 0) &&
         (long long)a.M * a.in_cs < (1LL << 31) - 64;
}

template <int WCO, int WPX, int TPW, int NS, int ACT>
ycx_status launch_wres_f8_cin(const ConvArgs& a, dim3 g, dim3 b, hipStream_t st) {
  switch (a.Cin) {
    case 128: hipLaunchKernelGGL((conv1x1_wres_f8<WCO, WPX, TPW, 1, NS, ACT>), g, b, 0, st, a); break;
    case 256: hipLaunchKernelGGL((conv1x1_wres_f8<WCO, WPX, TPW, 2, NS, ACT>), g, b, 0, st, a); break;
    case 512: hipLaunchKernelGGL((conv1x1_wres_f8<WCO, WPX, TPW, 4, NS, ACT>), g, b, 0, st, a); break;
    default: return YCX_ERR_UNSUPPORTED;
  }
  return ycx_launch_status();
}

template <int WCO, int WPX, int TPW, int NS>
ycx_status launch_wres_f8_k(ConvArgs a, hipStream_t st) {
  a.n_ct = a.Cout_pad / (WCO * 32);
  const int T = (a.M + TPW * WPX - 1) / (TPW * WPX);
  const int R = std::max(1, (int)even_grid(T, 256 / a.n_ct));
  a.nwg = R * a.n_ct;
  dim3 g(a.nwg), b(WCO * WPX * 64);
  switch (a.act) {
    case YCX_ACT_SILU_PS: return launch_wres_f8_cin<WCO, WPX, TPW, NS, YCX_ACT_SILU_PS>(a, g, b, st);
    case YCX_ACT_SILU: return launch_wres_f8_cin<WCO, WPX, TPW, NS, YCX_ACT_SILU>(a, g, b, st);
    case YCX_ACT_LEAKY: return launch_wres_f8_cin<WCO, WPX, TPW, NS, YCX_ACT_LEAKY>(a, g, b, st);
    default: return launch_wres_f8_cin<WCO, WPX, TPW, NS, YCX_ACT_NONE>(a, g, b, st);
  }
}

// tile 37: fp8 weight-stationary 3x3 64 -> 64, one persistent block per CU
ycx_status launch_ws64_f8(ConvArgs a, hipStream_t st) {
  if (!(a.KH == 3 && a.KW == 3 && a.S == 1 && a.P == 1 && a.H == a.Ho && a.W == a.Wo && a.Ho % 16 == 0 &&
        a.Wo % 16 == 0 && a.Cin == 64 && a.Cout_pad == 64 && a.Ktot == 640 && a.out_layout == YCX_OUT_NHWC &&
        !a.res && (long long)a.N * a.H * a.W * a.in_cs < (1LL << 31) - 64))
    return YCX_ERR_UNSUPPORTED;
  const long long ntiles = (long long)a.N * (a.Ho / 16) * (a.Wo / 16);
  const dim3 g((unsigned)even_grid(ntiles, 256)), b(512);
  switch (a.act) {
    case YCX_ACT_SILU_PS: hipLaunchKernelGGL((conv3x3_ws64_f8<YCX_ACT_SILU_PS>), g, b, 0, st, a); break;
    case YCX_ACT_SILU: hipLaunchKernelGGL((conv3x3_ws64_f8<YCX_ACT_SILU>), g, b, 0, st, a); break;
    case YCX_ACT_LEAKY: hipLaunchKernelGGL((conv3x3_ws64_f8<YCX_ACT_LEAKY>), g, b, 0, st, a); break;
    default: hipLaunchKernelGGL((conv3x3_ws64_f8<YCX_ACT_NONE>), g, b, 0, st, a); break;
  }
  return ycx_launch_status();
}

// tile 36: the fp8 weight-resident 1x1 (persistent, one block per CU and channel group)
ycx_status launch_wres_f8(ConvArgs a, hipStream_t st) {
  if (!wres_f8_ok(a)) return YCX_ERR_UNSUPPORTED;
#ifndef YCX_F8W_NS
#define YCX_F8W_NS 5
#endif
#ifndef YCX_F8W_NS2
#define YCX_F8W_NS2 6
#endif
#ifndef YCX_F8W_TPW
#define YCX_F8W_TPW 64
#endif
  if (a.Cout_pad % 256 == 0) return launch_wres_f8_k<8, 1, YCX_F8W_TPW, YCX_F8W_NS>(a, st);
  if (a.Cout_pad == 128) return launch_wres_f8_k<4, 2, 64, YCX_F8W_NS2>(a, st);
  return launch_wres_f8_k<2, 4, 32, YCX_F8W_NS2>(a, st);
}

}  // namespace

#ifndef YCX_ELT_F16  // dtype-independent entry points: once, in the bf16 build
extern "C" const char* ycx_conv_tile_name(int32_t tile) {
  if (tile < 0 || tile >= kNumTiles) return "invalid";
  return kTiles[tile].name;
}
#endif

// Tile heuristic: pick the largest tile that still gives >= ~2 waves of blocks
// on 256 CUs, with BK = 32 only where cin is not a multiple of 64.
static int32_t pick_tile(const ycx_conv_desc* d, bool allow_wres) {  // allow_wres: no residual (tiles 22, 23)
  if (d->dtype == YCX_DT_F32) return 8;
  const long long M = (long long)d->n * d->ho * d->wo;
  if (d->in_pool) {  // the pooled-operand variants of the two-stage LDS-DMA tiles
    const bool big = d->cout_pad % 128 == 0 && (d->cout_pad / 128) * ((M + 127) / 128) >= 256;
    if (d->dtype == YCX_DT_FP8) return big ? 34 : 35;
    return d->cout_pad % 128 == 0 && (d->cout_pad / 128) * ((M + 127) / 128) >= 64 ? 16 : 18;
  }
  if (d->dtype == YCX_DT_FP8) {
    // pointwise layers with cin in {128, 256, 512} and >= 8 pixel tiles per persistent block:
    // weights resident in registers (tile 36)
    if (allow_wres && d->kh == 1 && d->kw == 1 && d->stride == 1 && d->pad == 0 && d->out_layout == YCX_OUT_NHWC &&
        (d->cin == 128 || d->cin == 256 || d->cin == 512) &&
        (d->cout_pad == 64 || d->cout_pad == 128 || d->cout_pad % 256 == 0)) {
      const long long pt = d->cout_pad >= 256 ? 64 : 128, groups = d->cout_pad >= 256 ? d->cout_pad / 256 : 1;
#ifndef YCX_WRES_F8_MIN_TILES  // pixel tiles per persistent block (r06: 8 -> 4, as the bf16 tile 22)
#define YCX_WRES_F8_MIN_TILES 4
#endif
      if (M >= YCX_WRES_F8_MIN_TILES * pt * (256 / groups)) return 36;
    }
    // 3x3 / s1 64 -> 64 'same' convs on 16-aligned maps with >= 2 tiles per block: weights in LDS (tile 37)
    if (allow_wres && d->kh == 3 && d->kw == 3 && d->stride == 1 && d->pad == 1 && d->h == d->ho &&
        d->w == d->wo && d->ho % 16 == 0 && d->wo % 16 == 0 && d->cin == 64 && d->cout_pad == 64 &&
        d->out_layout == YCX_OUT_NHWC && (long long)d->n * (d->ho / 16) * (d->wo / 16) >= 512)
      return 37;
    return d->cout_pad % 128 == 0 && (d->cout_pad / 128) * ((M + 127) / 128) >= 256 ? 34 : 35;
  }
  const bool k64 = (d->cin % 64) == 0;
  if (d->cout_pad % 64 != 0) return 5;  // cout 32: co32 x px256, BK 32 (cin % 32 == 0)
  // The 512-thread LDS-DMA kernels' buffer descriptors address < 2 GiB per operand.
  const bool fits = (long long)d->n * d->h * d->w * d->in_c_stride * 2 < (1LL << 31) &&
                    (long long)d->cout_pad * d->kh * d->kw * d->cin * 2 < (1LL << 31);
  // Two-stage LDS-DMA tiles (two workgroups per CU) wherever they fill the chip
  // (tests/probes/conv_bench.py: 10-40 % over the 3-stage one-per-CU tiles).
  if (d->cin == 32 && fits) {  // two taps per 64-wide K step
    if ((d->cout_pad / 64) * ((M + 255) / 256) >= 256) return 17;
  }
  if (!k64) {
    if (d->cout_pad % 128 == 0 && d->cout_pad >= 128) return 7;
    if (d->cout_pad % 64 == 0) return 6;
    return 5;
  }
  if (!fits) return d->cout_pad % 128 == 0 ? 1 : 2;
  // Pointwise layers with K <= 512 and >= 8 pixel tiles per persistent block:
  // weights resident in registers (tile 22; the 160^2 / 80^2 yolov7 1x1s)
  if (allow_wres && d->kh == 1 && d->kw == 1 && d->stride == 1 && d->pad == 0 &&
      d->out_layout == YCX_OUT_NHWC && d->cin <= 512 && (d->cin & (d->cin - 1)) == 0 &&
      (d->cout_pad == 64 || d->cout_pad == 128 || d->cout_pad % 256 == 0)) {
    const long long pt = d->cout_pad >= 256 ? 64 : 128, groups = d->cout_pad >= 256 ? d->cout_pad / 256 : 1;
#ifndef YCX_WRES_MIN_TILES  // pixel tiles per persistent block (r06: 8 -> 4, the 40^2 512->512 and 80^2
#define YCX_WRES_MIN_TILES 4  // 512->128 1x1s 50 -> 45-46 and 68 -> 66 us; 2 or 1 take slower 40^2 / 20^2 ones)
#endif
    if (M >= YCX_WRES_MIN_TILES * pt * (256 / groups)) return 22;
  }
  // 3x3 stride-1 'same' convs on 16-aligned maps: LDS halo tiles (tests/probes/conv_bench.py:
  // +14-18 % over the im2col tiles at 80^2 with >= 128 output channels, +18 % at 320^2 x 64)
  if (d->kh == 3 && d->kw == 3 && d->stride == 1 && d->pad == 1 && d->h == d->ho && d->w == d->wo &&
      d->ho % 16 == 0 && d->wo % 16 == 0 && d->out_layout != YCX_OUT_NCHW_F32) {
    // 64 -> 64: weights resident in LDS across a persistent block's tiles (tile 23:
    // 320^2 0.43 -> 0.28 ms, 160^2 0.10 -> 0.06 ms at bs 32); needs >= 2 tiles per block
    if (allow_wres && d->cin == 64 && d->cout_pad == 64 && d->out_layout == YCX_OUT_NHWC &&
        (long long)d->n * (d->ho / 16) * (d->wo / 16) >= 512)
      return 23;
    if (d->cout_pad % 128 == 0) return 20;
    if (d->cout_pad == 64 && d->ho >= 160) return 19;
  }
  // 3x3/s2 64 -> 128 downsample with >= 4 output tiles per persistent block: weights in
  // registers, input halo in LDS (tile 50)
  if (allow_wres && d->kh == 3 && d->kw == 3 && d->stride == 2 && d->pad == 1 && d->cin == 64 &&
      d->cout_pad == 128 && d->out_layout == YCX_OUT_NHWC && d->ho % 4 == 0 && d->wo % 16 == 0 &&
      (long long)d->n * (d->ho / 4) * (d->wo / 16) >= 2048) {
#ifndef YCX_NO_S2WSR  // -DYCX_NO_S2WSR: the im2col tiles instead, for an A/B build
    return 50;
#endif
  }
  // 40-wide maps (not 16-aligned): the 8 x 40 band halo tile where it has >= 2.5 waves of
  // workgroups (40^2 bs 32 256->512: 0.113 vs 0.124 ms; with fewer workgroups it loses to tile 16,
  // profiles/r03/band_halo_40.txt)
  if (d->kh == 3 && d->kw == 3 && d->stride == 1 && d->pad == 1 && d->h == d->ho && d->w == d->wo && d->wo == 40 &&
      d->ho % 8 == 0 && d->out_layout != YCX_OUT_NCHW_F32 && (long long)(d->cout_pad / 64) * d->n * (d->ho / 8) >= 1280)
    return 48;
  if (d->cout_pad % 128 == 0) {
    // Tile 16 down to a quarter wave of workgroups (r06): at 20^2 x bs 32 (200 workgroups) it takes
    // within 1-2 us of tile 18's time with half the workgroups, and the other batches in flight
    // run in the CU slots it leaves (concurrent bench +1.3 %, profiles/r06/tile_pick/). Below
    // that (small batches, latency) the co64 x px128 blocks, two per CU.
    if ((d->cout_pad / 128) * ((M + 127) / 128) >= 64) return 16;
    return 18;
  }
  if ((M + 255) / 256 >= 512) return 15;  // tests/probes/conv_bench.py: 80^2 x bs 32 128->64 3x3 48.7 vs 52.3 us (t18)
  if ((d->cout_pad / 64) * ((M + 127) / 128) >= 256) return 18;
  return 3;
}

#ifndef YCX_ELT_F16
extern "C" int32_t ycx_conv_tile_of(int32_t bid, int32_t nwg, int32_t n_ct, int32_t gc) {
  if (nwg <= 0 || n_ct <= 0 || nwg % n_ct || bid < 0 || bid >= nwg || nwg / n_ct >= 65536) return -1;
  int ct, pt;
  ycx_tile_of(ycx_xcd_remap(bid, nwg), n_ct, nwg / n_ct, gc, ct, pt);
  return ct * 65536 + pt;
}

extern "C" int32_t ycx_conv_pick_tile(const ycx_conv_desc* d) {
  if (!d) return 0;
  return pick_tile(d, d->res_c_stride == 0);  // res_c_stride > 0: the call will pass a residual
}

// the fp16 build's entry points (ycx_conv.hip compiled with -DYCX_ELT_F16)
extern "C" ycx_status ycx_conv2d_ws_f16(const ycx_conv_desc*, const void*, const void*, const float*, void*,
                                        const void*, void*, size_t, void*);
extern "C" ycx_status ycx_conv2d_head_f16(const ycx_conv_desc*, const ycx_head_desc*, const void*, const void*,
                                          const float*, float*, ycx_cand*, int32_t*, int32_t*, int32_t*, void*);
extern "C" ycx_status ycx_stem_conv_f16(const ycx_conv_desc*, const float*, const float*, const float*, void*,
                                        void*);
extern "C" ycx_status ycx_conv2d_pair_f16(const ycx_conv_desc*, const ycx_conv_desc*, const void*, const void*,
                                          const float*, void*, const void*, const float*, void*, void*);
extern "C" ycx_status ycx_stem_conv2_f16(const ycx_conv_desc*, const ycx_conv_desc*, const float*, const float*,
                                         const float*, const void*, const float*, void*, void*);
#define YCX_TO_F16(cond, call) \
  do {                         \
    if (cond) return call;     \
  } while (0)
#else
#define YCX_TO_F16(cond, call) \
  do {                         \
  } while (0)
#endif

#ifndef YCX_ELT_F16
extern "C" size_t ycx_conv_workspace_size(const ycx_conv_desc* d) {
  if (!d || d->k_split <= 1 || d->n <= 0 || d->ho <= 0 || d->wo <= 0 || d->cout_pad <= 0) return 0;
  return (size_t)d->k_split * d->n * d->ho * d->wo * d->cout_pad * sizeof(float);
}

// Split-K pick (r06): none by default; -DYCX_KSPLIT_AUTO builds the
// heuristic under test (LDS-DMA tiles 16 / 18 with fewer than YCX_KSPLIT_AUTO workgroups
// and >= 16 K steps: split so the grid reaches that many).
extern "C" int32_t ycx_conv_pick_ksplit(const ycx_conv_desc* d) {
  if (!d || (d->dtype != YCX_DT_BF16 && d->dtype != YCX_DT_F16) || d->in_pool || d->out_layout == YCX_OUT_NCHW_F32)
    return 1;
#ifdef YCX_KSPLIT_AUTO
  const int tile = d->tile ? d->tile : pick_tile(d, d->res_c_stride == 0);
  if (tile != 16 && tile != 18 && tile != 56) return 1;
  const int bm = kTiles[tile].bm;
  const long long nwg = (long long)(d->cout_pad / bm) * ((long long)d->n * d->ho * d->wo + 127) / 128;
  const int nsteps = d->kh * d->kw * (d->cin / 64);
  int ks = 1;
  while (nwg * (ks + 1) <= YCX_KSPLIT_AUTO && nsteps / (ks + 1) >= 8 && ks < 4) ++ks;
  if (nwg * ks < YCX_KSPLIT_AUTO / 2 && nsteps >= 32) ks = std::max(ks, 2);
  return nsteps >= 16 ? ks : 1;
#else
  return 1;
#endif
}
#endif

extern "C" ycx_status YCX_SFX(ycx_conv2d_ws)(const ycx_conv_desc*, const void*, const void*, const float*, void*,
                                             const void*, void*, size_t, void*);
extern "C" ycx_status YCX_SFX(ycx_conv2d)(const ycx_conv_desc* d, const void* x, const void* w, const float* bias,
                                          void* y, const void* residual, void* stream) {
  return YCX_SFX(ycx_conv2d_ws)(d, x, w, bias, y, residual, nullptr, 0, stream);
}

extern "C" ycx_status YCX_SFX(ycx_conv2d_ws)(const ycx_conv_desc* d, const void* x, const void* w, const float* bias,
                                             void* y, const void* residual, void* workspace, size_t workspace_bytes,
                                             void* stream) {
  YCX_TO_F16(d && d->dtype == YCX_DT_F16,
             ycx_conv2d_ws_f16(d, x, w, bias, y, residual, workspace, workspace_bytes, stream));
  YCX_CHECK_ARG(d && x && w && bias && y);
  YCX_CHECK_ARG(d->k_split >= 0);
  YCX_CHECK_ARG(d->n > 0 && d->h > 0 && d->w > 0 && d->cin > 0 && d->cout > 0 && d->ho > 0 && d->wo > 0);
  YCX_CHECK_ARG(d->kh > 0 && d->kw > 0 && d->stride > 0 && d->pad >= 0);
  YCX_CHECK_ARG(d->cout_pad >= d->cout && d->in_c_off >= 0 && d->in_c_off + d->cin <= d->in_c_stride);
  YCX_CHECK_ARG(d->ho == (d->h + 2 * d->pad - d->kh) / d->stride + 1);
  YCX_CHECK_ARG(d->wo == (d->w + 2 * d->pad - d->kw) / d->stride + 1);
  YCX_CHECK_ARG(d->out_c_off >= 0);
  YCX_CHECK_ARG(d->out_layout == YCX_OUT_NCHW_F32 || d->out_c_off + d->cout <= d->out_c_stride);
  YCX_CHECK_SUPPORTED(d->dtype == YCX_DT_ELT || d->dtype == YCX_DT_F32 || d->dtype == YCX_DT_FP8);
  YCX_CHECK_SUPPORTED(d->out_layout >= YCX_OUT_NHWC && d->out_layout <= YCX_OUT_NHWC_UP2);
  YCX_CHECK_SUPPORTED(d->act >= YCX_ACT_NONE && d->act <= YCX_ACT_SILU_PS);
  YCX_CHECK_SUPPORTED(d->act != YCX_ACT_SILU_PS || d->dtype != YCX_DT_F32);  // fp32 parity mode: plain SiLU
  YCX_CHECK_SUPPORTED(!residual || d->out_layout == YCX_OUT_NHWC);
  const int vec = d->dtype == YCX_DT_ELT ? 8 : d->dtype == YCX_DT_FP8 ? 16 : 4;  // 16-byte DMA chunks
  YCX_CHECK_SUPPORTED(d->in_c_off % vec == 0 && d->in_c_stride % vec == 0);
  if (d->out_layout != YCX_OUT_NCHW_F32)
    YCX_CHECK_SUPPORTED(d->cout % 8 == 0 && d->out_c_off % 8 == 0 && d->out_c_stride % 8 == 0);
  if (residual) YCX_CHECK_SUPPORTED(d->res_c_off % 8 == 0 && d->res_c_stride % 8 == 0);
  // The 32-bit index math inside the kernels.
  YCX_CHECK_SUPPORTED((long long)d->n * d->ho * d->wo < (1LL << 31));
  YCX_CHECK_SUPPORTED((long long)d->cout_pad * d->kh * d->kw * d->cin < (1LL << 31));
  if (d->in_pool) {  // fused MP: 16-bit or fp8 (cin % 128 == 0) pointwise over a (2h, 2w) map
    YCX_CHECK_ARG(d->in_pool == 1);
    YCX_CHECK_SUPPORTED((d->dtype == YCX_DT_ELT || (d->dtype == YCX_DT_FP8 && d->cin % 128 == 0)) && d->kh == 1 &&
                        d->kw == 1 && d->stride == 1 && d->pad == 0);
    YCX_CHECK_SUPPORTED((long long)d->n * 4 * d->h * d->w * d->in_c_stride * (d->dtype == YCX_DT_FP8 ? 1 : 2) <
                        (1LL << 31) - 64);
  }
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  ConvArgs a = make_args(d, x, w, bias, y, residual);

  int tile = d->tile ? d->tile : pick_tile(d, residual == nullptr);  // tile 22 stores no residual
  YCX_CHECK_SUPPORTED(tile > 0 && tile < kNumTiles);
  if (a.ks > 1) {  // split-K: the two-stage / three-stage LDS-DMA tiles, 16-bit, NHWC outputs
    YCX_CHECK_SUPPORTED(d->dtype == YCX_DT_ELT && !d->in_pool && d->out_layout != YCX_OUT_NCHW_F32 &&
                        (tile == 16 || tile == 18 || tile == 56) && d->cin % 64 == 0 && d->k_split <= 16);
    if (!workspace || workspace_bytes < ycx_conv_workspace_size(d)) return YCX_ERR_CAPACITY;
    YCX_CHECK_SUPPORTED((long long)d->k_split * d->n * d->ho * d->wo * d->cout_pad < (1LL << 31));
    a.part = reinterpret_cast<float*>(workspace);
  }
  YCX_CHECK_SUPPORTED(!d->in_pool || tile == 16 || tile == 18 || tile == 25 || tile == 34 || tile == 35);
  const TileInfo& t = kTiles[tile];
  YCX_CHECK_SUPPORTED(d->cin % t.bk == 0 && d->cout_pad % t.bm == 0);
  YCX_CHECK_SUPPORTED((d->dtype == YCX_DT_FP8) == (tile >= 34 && tile <= 37));
  if (d->dtype == YCX_DT_FP8) {
    YCX_CHECK_SUPPORTED((long long)d->cout_pad * a.Ktot < (1LL << 31) &&
                        (long long)d->n * d->h * d->w * d->in_c_stride < (1LL << 31) - 64);
    if (tile == 36) return launch_wres_f8(a, st);
    if (tile == 37) return launch_ws64_f8(a, st);
    return tile == 34 ? launch_f8<128, 128, 2, 4>(a, st) : launch_f8<64, 128, 1, 8>(a, st);
  }
  if (d->dtype == YCX_DT_F32) {
    YCX_CHECK_SUPPORTED(tile == 8);
    a.nsteps = a.KH * a.KW * (a.Cin / 16);
    a.n_ct = a.Cout_pad / 64;
    a.nwg = a.n_ct * ((a.M + 63) / 64);
    hipLaunchKernelGGL(conv_f32_kernel, dim3(a.nwg), dim3(256), 0, st, a);
    return ycx_launch_status();
  }
  switch (tile) {
    case 1: return launch_bf16<128, 128, 64, 2, 2>(a, st);
    case 2: return launch_bf16<64, 256, 64, 1, 4>(a, st);
    case 3: return launch_bf16<64, 128, 64, 2, 2>(a, st);
    case 4: return launch_bf16<128, 64, 64, 2, 2>(a, st);
    case 5: return launch_bf16<32, 256, 32, 1, 4>(a, st);
    case 6: return launch_bf16<64, 256, 32, 1, 4>(a, st);
    case 7: return launch_bf16<128, 128, 32, 2, 2>(a, st);
    case 9: return launch_glds<128, 256, 2, 4>(a, st);
    case 10: return launch_glds<64, 256, 1, 8>(a, st);
    case 11: return launch_glds<256, 128, 4, 2>(a, st);
    case 12: return launch_glds<128, 128, 2, 4>(a, st);
    case 13: return launch_glds<64, 256, 1, 8, true>(a, st);
    case 14: return launch_glds<128, 256, 2, 4, true>(a, st);
    case 15: return launch_glds<64, 256, 1, 8, false, 2>(a, st);
#ifdef YCX_T16_NSB3  // development A/B: activation ring one K step deeper
    case 16: return launch_glds<128, 128, 2, 4, false, 2, 3>(a, st);
#else
    case 16: return launch_glds<128, 128, 2, 4, false, 2>(a, st);
#endif
    case 17: return launch_glds<64, 256, 1, 8, true, 2>(a, st);
    case 18: return launch_glds<64, 128, 1, 8, false, 2>(a, st);
    case 19: return launch_halo<64, 1, 4, 3>(a, st);
    case 20: return launch_halo<128, 2, 4, 2>(a, st);
    case 21: return launch_halo<128, 2, 4, 3>(a, st);
    case 22: return launch_wres(a, st);
    case 23: return launch_ws64(a, st);
    case 24: return launch_glds<256, 256, 2, 4, false, 2>(a, st);
    case 25: return launch_glds<256, 128, 2, 4, false, 2>(a, st);
    case 26: return launch_glds<128, 256, 2, 4, false, 2>(a, st);
    case 48: return launch_halo<64, 2, 4, 2, 8, 40>(a, st);      // band halo tiles (40-wide maps)
    case 49: return launch_halo<128, 4, 2, 2, 4, 40>(a, st);
    case 50: return launch_s2wsr(a, st);
    case 56: return launch_glds<64, 128, 1, 8, false, 3>(a, st);
    default: return YCX_ERR_UNSUPPORTED;
  }
}

extern "C" ycx_status YCX_SFX(ycx_conv2d_head)(const ycx_conv_desc* d, const ycx_head_desc* h, const void* x,
                                               const void* w, const float* bias, float* heads, ycx_cand* cand,
                                               int32_t* cand_rows, int32_t* cand_counts, int32_t* status,
                                               void* stream) {
  YCX_TO_F16(d && d->dtype == YCX_DT_F16,
             ycx_conv2d_head_f16(d, h, x, w, bias, heads, cand, cand_rows, cand_counts, status, stream));
  YCX_CHECK_ARG(d && h && x && w && bias && cand && cand_rows && cand_counts);
  YCX_CHECK_ARG(d->n > 0 && d->h > 0 && d->w > 0 && d->cin > 0 && d->cout > 0 && d->ho == d->h && d->wo == d->w);
  YCX_CHECK_ARG(d->in_c_off >= 0 && d->in_c_off + d->cin <= d->in_c_stride && d->cout_pad >= d->cout);
  YCX_CHECK_ARG(h->na > 0 && h->na <= 8 && h->nc > 0 && h->no == h->nc + 5 && h->na * h->no == d->cout);
  YCX_CHECK_ARG(h->row_off >= 0 && h->row_off + h->na * d->ho * d->wo <= h->rows_total);
  const bool f8 = d->dtype == YCX_DT_FP8;
  YCX_CHECK_SUPPORTED((d->dtype == YCX_DT_ELT || f8) && d->kh == 1 && d->kw == 1 && d->stride == 1 && d->pad == 0);
  YCX_CHECK_SUPPORTED(d->act == YCX_ACT_NONE && d->out_layout == YCX_OUT_NCHW_F32 && d->cout_pad == 256);
  YCX_CHECK_SUPPORTED(!d->in_pool);
  YCX_CHECK_SUPPORTED(f8 ? (d->in_c_off % 16 == 0 && d->in_c_stride % 16 == 0)
                         : (d->in_c_off % 8 == 0 && d->in_c_stride % 8 == 0));
  YCX_CHECK_SUPPORTED((long long)d->n * d->h * d->w * d->in_c_stride * 2 < (1LL << 31));
  YCX_CHECK_SUPPORTED((long long)d->n * h->rows_total < (1LL << 31));
  ConvArgs a = make_args(d, x, w, bias, heads, nullptr);
  a.out_coff = 0;
  a.out_cs = d->cout;
  HeadArgs hd{*h, cand, cand_rows, cand_counts, heads, status};
  return launch_head(a, hd, reinterpret_cast<hipStream_t>(stream), f8);
}

extern "C" ycx_status YCX_SFX(ycx_conv2d_pair)(const ycx_conv_desc* da, const ycx_conv_desc* db, const void* x,
                                               const void* wa, const float* ba, void* ya, const void* wb,
                                               const float* bb, void* yb, void* stream) {
  YCX_TO_F16(da && da->dtype == YCX_DT_F16,
             ycx_conv2d_pair_f16(da, db, x, wa, ba, ya, wb, bb, yb, stream));
  YCX_CHECK_ARG(da && db && x && wa && ba && wb && bb && yb);
  YCX_CHECK_ARG(da->n > 0 && da->h > 0 && da->w > 0 && da->cin > 0 && da->cout > 0);
  YCX_CHECK_ARG(da->ho == da->h && da->wo == da->w && db->n == da->n && db->h == da->ho && db->w == da->wo &&
                db->ho == db->h && db->wo == db->w && db->cin == da->cout && db->cout > 0);
  YCX_CHECK_ARG(da->in_c_off >= 0 && da->in_c_off + da->cin <= da->in_c_stride && db->cout_pad >= db->cout);
  YCX_CHECK_ARG(db->out_c_off >= 0 && db->out_c_off + db->cout <= db->out_c_stride);
  YCX_CHECK_ARG(!ya || (da->out_c_off >= 0 && da->out_c_off + da->cout <= da->out_c_stride));
  YCX_CHECK_SUPPORTED(da->dtype == YCX_DT_ELT && db->dtype == YCX_DT_ELT);
  for (const ycx_conv_desc* d : {da, db}) {
    YCX_CHECK_SUPPORTED(d->kh == 1 && d->kw == 1 && d->stride == 1 && d->pad == 0 && !d->in_pool &&
                        d->out_layout == YCX_OUT_NHWC && d->act >= YCX_ACT_NONE && d->act <= YCX_ACT_SILU_PS);
    YCX_CHECK_SUPPORTED(d->out_c_off % 8 == 0 && d->out_c_stride % 8 == 0);
  }
  YCX_CHECK_SUPPORTED((da->cin == 64 || da->cin == 128 || da->cin == 256) && da->cout == 256 && da->cout_pad == 256);
  YCX_CHECK_SUPPORTED(da->in_c_off % 8 == 0 && da->in_c_stride % 8 == 0);
  YCX_CHECK_SUPPORTED(db->cin == 256 && (db->cout_pad == 128 || db->cout_pad == 256) && db->cout % 8 == 0);
  YCX_CHECK_SUPPORTED((long long)da->n * da->h * da->w * da->in_c_stride * 2 < (1LL << 31) - 64);
  ConvArgs a = make_args(da, x, wa, ba, ya, nullptr);
  ConvArgs b = make_args(db, nullptr, wb, bb, yb, nullptr);
  return launch_wres_pair(a, b, reinterpret_cast<hipStream_t>(stream));
}

extern "C" ycx_status YCX_SFX(ycx_stem_conv)(const ycx_conv_desc* d, const float* x, const float* w,
                                             const float* bias, void* y, void* stream) {
  YCX_TO_F16(d && d->dtype == YCX_DT_F16, ycx_stem_conv_f16(d, x, w, bias, y, stream));
  YCX_CHECK_ARG(d && x && w && bias && y);
  YCX_CHECK_ARG(d->n > 0 && d->h > 0 && d->w > 0 && d->cout > 0 && d->cout_pad >= d->cout);
  YCX_CHECK_ARG(d->ho == (d->h + 2 * d->pad - d->kh) / d->stride + 1);
  YCX_CHECK_ARG(d->wo == (d->w + 2 * d->pad - d->kw) / d->stride + 1);
  YCX_CHECK_ARG(d->in_c_off >= 0 && d->in_c_off + d->cin <= d->in_c_stride);
  YCX_CHECK_SUPPORTED(d->cout % 8 == 0 && d->cout_pad % 8 == 0 && d->out_c_off % 8 == 0 &&
                      d->out_c_stride % 8 == 0 && d->out_c_off + d->cout <= d->out_c_stride);
  YCX_CHECK_SUPPORTED(d->out_layout == YCX_OUT_NHWC || d->out_layout == YCX_OUT_NHWC_UP2);
  YCX_CHECK_SUPPORTED(d->dtype == YCX_DT_ELT || d->dtype == YCX_DT_F32 || d->dtype == YCX_DT_FP8);
  YCX_CHECK_SUPPORTED((long long)d->n * d->ho * d->wo < (1LL << 31) && !d->in_pool);
  YCX_CHECK_SUPPORTED(d->act >= YCX_ACT_NONE && d->act <= YCX_ACT_SILU_PS &&
                      (d->act != YCX_ACT_SILU_PS || d->dtype != YCX_DT_F32));
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  ConvArgs a = make_args(d, x, w, bias, y, nullptr);
  a.Ktot = d->kh * d->kw * d->cin;  // fp32 stem weights: no fp8 row padding
  const bool bf = d->dtype == YCX_DT_ELT, f8 = d->dtype == YCX_DT_FP8;
  if ((bf || f8) && d->out_layout == YCX_OUT_NHWC && (d->cout_pad == 32 || d->cout_pad == 64) && d->wo % 16 == 0) {
    const long long groups = (long long)a.M / 16;
    dim3 g((unsigned)std::min<long long>((groups + 3) / 4, 256LL * 16));
#define YCX_STEM_MFMA(KH_, KW_, CI_)                                                           \
    if (d->kh == KH_ && d->kw == KW_ && d->cin == CI_) {                                       \
      if (d->cout_pad == 32 && f8)                                                             \
        hipLaunchKernelGGL((stem_mfma<KH_, KW_, CI_, 2, true>), g, dim3(256), 0, st, a);       \
      else if (d->cout_pad == 32)                                                              \
        hipLaunchKernelGGL((stem_mfma<KH_, KW_, CI_, 2>), g, dim3(256), 0, st, a);             \
      else if (f8)                                                                             \
        hipLaunchKernelGGL((stem_mfma<KH_, KW_, CI_, 4, true>), g, dim3(256), 0, st, a);       \
      else                                                                                     \
        hipLaunchKernelGGL((stem_mfma<KH_, KW_, CI_, 4>), g, dim3(256), 0, st, a);             \
      return ycx_launch_status();                                                              \
    }
    YCX_STEM_MFMA(3, 3, 3)
    YCX_STEM_MFMA(3, 3, 1)
    YCX_STEM_MFMA(1, 1, 3)
    YCX_STEM_MFMA(5, 5, 1)
#undef YCX_STEM_MFMA
  }
  const size_t lds = ((size_t)d->kh * d->kw * d->cin * d->cout_pad + d->cout_pad) * sizeof(float);
  YCX_CHECK_SUPPORTED(lds <= 64 * 1024);
  dim3 grid(ycx_cdiv(a.M, 256));
#define YCX_STEM(KH_, KW_, CI_)                                                                  \
  if (d->kh == KH_ && d->kw == KW_ && d->cin == CI_) {                                           \
    if (bf)                                                                                      \
      hipLaunchKernelGGL((stem_kernel<KH_, KW_, CI_, elt_t>), grid, dim3(256), lds, st, a);     \
    else if (f8)                                                                                 \
      hipLaunchKernelGGL((stem_kernel<KH_, KW_, CI_, uint8_t>), grid, dim3(256), lds, st, a);    \
    else                                                                                         \
      hipLaunchKernelGGL((stem_kernel<KH_, KW_, CI_, float>), grid, dim3(256), lds, st, a);      \
    return ycx_launch_status();                                                                  \
  }
  YCX_STEM(3, 3, 3)
  YCX_STEM(3, 3, 1)
  YCX_STEM(3, 3, 4)
  YCX_STEM(1, 1, 3)
  YCX_STEM(5, 5, 3)
  YCX_STEM(6, 6, 3)
#undef YCX_STEM
  return YCX_ERR_UNSUPPORTED;
}

extern "C" ycx_status YCX_SFX(ycx_stem_conv2)(const ycx_conv_desc* sd, const ycx_conv_desc* cd, const float* x,
                                              const float* w_stem, const float* b_stem, const void* w_conv,
                                              const float* b_conv, void* y, void* stream) {
  YCX_TO_F16(cd && cd->dtype == YCX_DT_F16,
             ycx_stem_conv2_f16(sd, cd, x, w_stem, b_stem, w_conv, b_conv, y, stream));
  YCX_CHECK_ARG(sd && cd && x && w_stem && b_stem && w_conv && b_conv && y);
  YCX_CHECK_ARG(sd->n > 0 && sd->h > 0 && sd->w > 0 && cd->n == sd->n);
  YCX_CHECK_ARG(sd->ho == (sd->h + 2 * sd->pad - sd->kh) / sd->stride + 1);
  YCX_CHECK_ARG(sd->wo == (sd->w + 2 * sd->pad - sd->kw) / sd->stride + 1);
  YCX_CHECK_ARG(cd->h == sd->ho && cd->w == sd->wo && cd->cin == sd->cout);
  YCX_CHECK_ARG(cd->ho == (cd->h + 2 * cd->pad - cd->kh) / cd->stride + 1);
  YCX_CHECK_ARG(cd->wo == (cd->w + 2 * cd->pad - cd->kw) / cd->stride + 1);
  YCX_CHECK_ARG(sd->in_c_off >= 0 && sd->in_c_off + sd->cin <= sd->in_c_stride);
  YCX_CHECK_ARG(cd->cout_pad >= cd->cout && cd->out_c_off >= 0 && cd->out_c_off + cd->cout <= cd->out_c_stride);
  YCX_CHECK_SUPPORTED(sd->kh == 3 && sd->kw == 3 && sd->pad == 1 && (sd->stride == 1 || sd->stride == 2) &&
                      sd->cin == 3 && sd->cout == 32 && sd->cout_pad == 32);
  YCX_CHECK_SUPPORTED(cd->kh == 3 && cd->kw == 3 && cd->stride == 2 && cd->pad == 1 && cd->cin == 32 &&
                      cd->cout_pad == 64 && cd->cout % 8 == 0 && cd->out_c_off % 8 == 0 && cd->out_c_stride % 8 == 0);
  // FP8: the pair computes in bf16 (the stem map never leaves LDS); the output is e4m3 (cd->out_scale)
  YCX_CHECK_SUPPORTED(sd->dtype == cd->dtype && (cd->dtype == YCX_DT_ELT || cd->dtype == YCX_DT_FP8) &&
                      cd->out_layout == YCX_OUT_NHWC);
  YCX_CHECK_SUPPORTED(sd->act >= YCX_ACT_NONE && sd->act <= YCX_ACT_SILU_PS && cd->act >= YCX_ACT_NONE &&
                      cd->act <= YCX_ACT_SILU_PS);
  YCX_CHECK_SUPPORTED(cd->ho % kS2TH == 0 && cd->wo % kS2TW == 0);
  YCX_CHECK_SUPPORTED((long long)cd->n * cd->ho * cd->wo < (1LL << 31));
  ConvArgs sa = make_args(sd, x, w_stem, b_stem, nullptr, nullptr);
  ConvArgs ca = make_args(cd, nullptr, w_conv, b_conv, y, nullptr);
  const bool f8 = cd->dtype == YCX_DT_FP8;
  // both weight sets are unpadded (fp32 stem, bf16 conv) whatever the output dtype
  sa.Ktot = sd->kh * sd->kw * sd->cin;
  ca.Ktot = cd->kh * cd->kw * cd->cin;
  const long long ntiles = (long long)cd->n * (cd->ho / kS2TH) * (cd->wo / kS2TW);
#ifndef YCX_STEM2_BLOCKS  // development A/B knob: the persistent grid's block cap
#define YCX_STEM2_BLOCKS 512
#endif
  ca.nwg = (int)even_grid(ntiles, YCX_STEM2_BLOCKS);  // persistent: two blocks per CU
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const dim3 g(ca.nwg), b(256);
#define YCX_STEM2(SS_, A1_, A2_)                                                           \
  if (sd->stride == SS_ && sd->act == A1_ && cd->act == A2_) {                            \
    if (f8)                                                                               \
      hipLaunchKernelGGL((stem2_fused<SS_, A1_, A2_, true>), g, b, 0, st, sa, ca);        \
    else                                                                                  \
      hipLaunchKernelGGL((stem2_fused<SS_, A1_, A2_>), g, b, 0, st, sa, ca);              \
    return ycx_launch_status();                                                           \
  }
  YCX_STEM2(1, YCX_ACT_SILU_PS, YCX_ACT_SILU_PS)
  YCX_STEM2(1, YCX_ACT_SILU, YCX_ACT_SILU)
  YCX_STEM2(1, YCX_ACT_LEAKY, YCX_ACT_LEAKY)
  YCX_STEM2(1, YCX_ACT_NONE, YCX_ACT_NONE)
  YCX_STEM2(2, YCX_ACT_SILU_PS, YCX_ACT_SILU_PS)
  YCX_STEM2(2, YCX_ACT_SILU, YCX_ACT_SILU)
  YCX_STEM2(2, YCX_ACT_LEAKY, YCX_ACT_LEAKY)
  YCX_STEM2(2, YCX_ACT_NONE, YCX_ACT_NONE)
#undef YCX_STEM2
  return YCX_ERR_UNSUPPORTED;
}

#if defined(YCX_GLDS_STAMP) && !defined(YCX_ELT_F16)
extern "C" int ycx_debug_glds_stamps(unsigned long long* out, int reset) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_glds_stamp), sizeof(g_glds_stamp)) != hipSuccess) return 1;
  if (reset) {
    unsigned long long z[16 * 8 + 1] = {};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_glds_stamp), z, sizeof(z)) != hipSuccess) return 1;
  }
  return 0;
}
#endif

#ifdef YCX_DEBUG_BOUNDS
extern "C" YCX_DEFINE_BOUNDS_READER(YCX_SFX(ycx_dbg_bounds_conv))
#endif
