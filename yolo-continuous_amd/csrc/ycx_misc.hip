// Data-movement kernels of the YOLO layer graph (NHWC, HBM-bound):
//   max-pool  : MP (k2 s2), SP (k s1 pad k//2), SPPCSPC pools (nets/common.py:25-40, 257)
//   copy      : Concat fallback when a producer cannot write its slice directly,
//               and nn.Upsample(None, 2, 'nearest') (cfg/net/yolov7.yaml:71,85)
// plus the static-plan executor (ycx_run_ops) that replaces the Python layer
// loop of Model.forward (nets/yolo.py:143-153), and its HIP-graph capture.
//
// Each thread moves one 16-byte vector (8 bf16 or 4 fp32 channels); consecutive
// threads take consecutive channel chunks of one pixel, so every wave reads and
// writes whole contiguous channel rows.
#include <vector>
#include "ycx_internal.h"

namespace {

template <typename T>
struct Vec;
template <>
struct Vec<__bf16> {
  typedef bf16x8 type;
  static constexpr int N = 8;
};
template <>
struct Vec<float> {
  typedef f32x4 type;
  static constexpr int N = 4;
};

template <typename T>
__global__ void __launch_bounds__(256) maxpool_kernel(ycx_pool_desc d, const T* __restrict__ x,
                                                      T* __restrict__ y) {
  typedef typename Vec<T>::type V;
  constexpr int VN = Vec<T>::N;
  const int cv = d.c / VN;
  const long long total = (long long)d.n * d.ho * d.wo * cv;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    int c = (int)(i % cv);
    long long p = i / cv;
    int ox = (int)(p % d.wo);
    long long t = p / d.wo;
    int oy = (int)(t % d.ho);
    int n = (int)(t / d.ho);
    float m[VN];
#pragma unroll
    for (int j = 0; j < VN; ++j) m[j] = -INFINITY;
    const int y0 = oy * d.stride - d.pad, x0 = ox * d.stride - d.pad;
    const int ya = max(y0, 0), yb = min(y0 + d.k, d.h), xa = max(x0, 0), xb = min(x0 + d.k, d.w);
    for (int iy = ya; iy < yb; ++iy)
      for (int ix = xa; ix < xb; ++ix) {
        V v = *reinterpret_cast<const V*>(x + (((size_t)n * d.h + iy) * d.w + ix) * d.in_c_stride +
                                          d.in_c_off + c * VN);
#pragma unroll
        for (int j = 0; j < VN; ++j) m[j] = fmaxf(m[j], (float)v[j]);
      }
    V o;
#pragma unroll
    for (int j = 0; j < VN; ++j) o[j] = (T)m[j];
    *reinterpret_cast<V*>(y + (((size_t)n * d.ho + oy) * d.wo + ox) * d.out_c_stride + d.out_c_off +
                          c * VN) = o;
  }
}

template <typename T>
__global__ void __launch_bounds__(256) copy_kernel(ycx_copy_desc d, const T* __restrict__ x,
                                                   T* __restrict__ y) {
  typedef typename Vec<T>::type V;
  constexpr int VN = Vec<T>::N;
  const int cv = d.c / VN;
  const int ho = d.h * d.scale, wo = d.w * d.scale;
  const long long total = (long long)d.n * ho * wo * cv;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    int c = (int)(i % cv);
    long long p = i / cv;
    int ox = (int)(p % wo);
    long long t = p / wo;
    int oy = (int)(t % ho);
    int n = (int)(t / ho);
    int iy = oy / d.scale, ix = ox / d.scale;  // nearest: floor(out * in/out)
    V v = *reinterpret_cast<const V*>(x + (((size_t)n * d.h + iy) * d.w + ix) * d.in_c_stride +
                                      d.in_c_off + c * VN);
    if (d.out_layout == YCX_OUT_NCHW_F32) {
      float* yf = reinterpret_cast<float*>(y);
#pragma unroll
      for (int j = 0; j < VN; ++j)
        yf[(((size_t)n * d.out_c_stride + d.out_c_off + c * VN + j) * ho + oy) * wo + ox] = (float)v[j];
    } else {
      *reinterpret_cast<V*>(y + (((size_t)n * ho + oy) * wo + ox) * d.out_c_stride + d.out_c_off + c * VN) = v;
    }
  }
}

// ---- fp8 (OCP e4m3fn) variants: 8 channels = 8 bytes per thread ----
__device__ __forceinline__ void f8x8_unpack(uint2 v, float f[8]) {
  f[0] = __builtin_amdgcn_cvt_f32_fp8((int)v.x, 0); f[1] = __builtin_amdgcn_cvt_f32_fp8((int)v.x, 1);
  f[2] = __builtin_amdgcn_cvt_f32_fp8((int)v.x, 2); f[3] = __builtin_amdgcn_cvt_f32_fp8((int)v.x, 3);
  f[4] = __builtin_amdgcn_cvt_f32_fp8((int)v.y, 0); f[5] = __builtin_amdgcn_cvt_f32_fp8((int)v.y, 1);
  f[6] = __builtin_amdgcn_cvt_f32_fp8((int)v.y, 2); f[7] = __builtin_amdgcn_cvt_f32_fp8((int)v.y, 3);
}
__device__ __forceinline__ uint32_t f8x4_pack_sat(float a, float b, float c, float d) {
  int w = __builtin_amdgcn_cvt_pk_fp8_f32(fminf(fmaxf(a, -448.f), 448.f), fminf(fmaxf(b, -448.f), 448.f), 0, false);
  w = __builtin_amdgcn_cvt_pk_fp8_f32(fminf(fmaxf(c, -448.f), 448.f), fminf(fmaxf(d, -448.f), 448.f), w, true);
  return (uint32_t)w;
}

// Max over the window in fp32 of the decoded bytes; the max is one of the
// inputs, so re-encoding it is exact (input and output share the scale).
__global__ void __launch_bounds__(256) maxpool_f8_kernel(ycx_pool_desc d, const uint8_t* __restrict__ x,
                                                         uint8_t* __restrict__ y) {
  const int cv = d.c / 8;
  const long long total = (long long)d.n * d.ho * d.wo * cv;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    int c = (int)(i % cv);
    long long p = i / cv;
    int ox = (int)(p % d.wo);
    long long t = p / d.wo;
    int oy = (int)(t % d.ho);
    int n = (int)(t / d.ho);
    float m[8], f[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) m[j] = -INFINITY;
    const int y0 = oy * d.stride - d.pad, x0 = ox * d.stride - d.pad;
    const int ya = max(y0, 0), yb = min(y0 + d.k, d.h), xa = max(x0, 0), xb = min(x0 + d.k, d.w);
    for (int iy = ya; iy < yb; ++iy)
      for (int ix = xa; ix < xb; ++ix) {
        f8x8_unpack(*reinterpret_cast<const uint2*>(x + (((size_t)n * d.h + iy) * d.w + ix) * d.in_c_stride +
                                                    d.in_c_off + c * 8), f);
#pragma unroll
        for (int j = 0; j < 8; ++j) m[j] = fmaxf(m[j], f[j]);
      }
    *reinterpret_cast<uint2*>(y + (((size_t)n * d.ho + oy) * d.wo + ox) * d.out_c_stride + d.out_c_off + c * 8) =
        make_uint2(f8x4_pack_sat(m[0], m[1], m[2], m[3]), f8x4_pack_sat(m[4], m[5], m[6], m[7]));
  }
}

// Byte copy (same scale on both sides), or decode to fp32 NCHW x dequant.
__global__ void __launch_bounds__(256) copy_f8_kernel(ycx_copy_desc d, const uint8_t* __restrict__ x,
                                                      uint8_t* __restrict__ y) {
  const int cv = d.c / 8;
  const int ho = d.h * d.scale, wo = d.w * d.scale;
  const long long total = (long long)d.n * ho * wo * cv;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    int c = (int)(i % cv);
    long long p = i / cv;
    int ox = (int)(p % wo);
    long long t = p / wo;
    int oy = (int)(t % ho);
    int n = (int)(t / ho);
    int iy = oy / d.scale, ix = ox / d.scale;
    const uint2 v = *reinterpret_cast<const uint2*>(x + (((size_t)n * d.h + iy) * d.w + ix) * d.in_c_stride +
                                                    d.in_c_off + c * 8);
    if (d.out_layout == YCX_OUT_NCHW_F32) {
      float f[8];
      f8x8_unpack(v, f);
      float* yf = reinterpret_cast<float*>(y);
#pragma unroll
      for (int j = 0; j < 8; ++j)
        yf[(((size_t)n * d.out_c_stride + d.out_c_off + c * 8 + j) * ho + oy) * wo + ox] = f[j] * d.dequant;
    } else {
      *reinterpret_cast<uint2*>(y + (((size_t)n * ho + oy) * wo + ox) * d.out_c_stride + d.out_c_off + c * 8) = v;
    }
  }
}

__global__ void __launch_bounds__(256) quantize_f8_kernel(const float* __restrict__ x, uint8_t* __restrict__ y,
                                                          long long n, float scale) {
  for (long long i = (blockIdx.x * (long long)blockDim.x + threadIdx.x) * 4; i < n;
       i += (long long)gridDim.x * blockDim.x * 4) {
    float v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = i + j < n ? x[i + j] * scale : 0.0f;
    const uint32_t w = f8x4_pack_sat(v[0], v[1], v[2], v[3]);
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (i + j < n) y[i + j] = (uint8_t)(w >> (8 * j));
  }
}

unsigned grid_for(long long total) {
  long long b = (total + 255) / 256;
  if (b > 256LL * 16) b = 256LL * 16;  // grid-stride beyond 16 blocks per CU
  return (unsigned)(b < 1 ? 1 : b);
}

}  // namespace

extern "C" ycx_status ycx_maxpool(const ycx_pool_desc* d, const void* x, void* y, void* stream) {
  YCX_CHECK_ARG(d && x && y);
  YCX_CHECK_ARG(d->n > 0 && d->h > 0 && d->w > 0 && d->c > 0 && d->k > 0 && d->stride > 0 && d->pad >= 0);
  YCX_CHECK_ARG(d->ho == (d->h + 2 * d->pad - d->k) / d->stride + 1);
  YCX_CHECK_ARG(d->wo == (d->w + 2 * d->pad - d->k) / d->stride + 1);
  YCX_CHECK_ARG(d->pad * 2 <= d->k);  // torch: pad <= k/2
  YCX_CHECK_ARG(d->in_c_off + d->c <= d->in_c_stride && d->out_c_off + d->c <= d->out_c_stride);
  YCX_CHECK_SUPPORTED(d->dtype == YCX_DT_BF16 || d->dtype == YCX_DT_F32 || d->dtype == YCX_DT_FP8);
  const int vn = d->dtype == YCX_DT_F32 ? 4 : 8;
  YCX_CHECK_SUPPORTED(d->c % vn == 0 && d->in_c_off % vn == 0 && d->in_c_stride % vn == 0 &&
                      d->out_c_off % vn == 0 && d->out_c_stride % vn == 0);
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  long long total = (long long)d->n * d->ho * d->wo * (d->c / vn);
  if (d->dtype == YCX_DT_FP8)
    hipLaunchKernelGGL(maxpool_f8_kernel, dim3(grid_for(total)), dim3(256), 0, st, *d, (const uint8_t*)x,
                       (uint8_t*)y);
  else if (d->dtype == YCX_DT_BF16)
    hipLaunchKernelGGL(maxpool_kernel<__bf16>, dim3(grid_for(total)), dim3(256), 0, st, *d,
                       (const __bf16*)x, (__bf16*)y);
  else
    hipLaunchKernelGGL(maxpool_kernel<float>, dim3(grid_for(total)), dim3(256), 0, st, *d, (const float*)x,
                       (float*)y);
  return ycx_launch_status();
}

extern "C" ycx_status ycx_copy_channels(const ycx_copy_desc* d, const void* x, void* y, void* stream) {
  YCX_CHECK_ARG(d && x && y);
  YCX_CHECK_ARG(d->n > 0 && d->h > 0 && d->w > 0 && d->c > 0 && (d->scale == 1 || d->scale == 2));
  YCX_CHECK_ARG(d->in_c_off + d->c <= d->in_c_stride && d->out_c_off + d->c <= d->out_c_stride);
  YCX_CHECK_SUPPORTED(d->out_layout == YCX_OUT_NHWC || d->out_layout == YCX_OUT_NCHW_F32);
  YCX_CHECK_SUPPORTED(d->dtype == YCX_DT_BF16 || d->dtype == YCX_DT_F32 || d->dtype == YCX_DT_FP8);
  const int vn = d->dtype == YCX_DT_F32 ? 4 : 8;
  YCX_CHECK_SUPPORTED(d->c % vn == 0 && d->in_c_off % vn == 0 && d->in_c_stride % vn == 0 &&
                      d->out_c_off % vn == 0 && d->out_c_stride % vn == 0);
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  long long total = (long long)d->n * d->h * d->scale * d->w * d->scale * (d->c / vn);
  if (d->dtype == YCX_DT_FP8)
    hipLaunchKernelGGL(copy_f8_kernel, dim3(grid_for(total)), dim3(256), 0, st, *d, (const uint8_t*)x,
                       (uint8_t*)y);
  else if (d->dtype == YCX_DT_BF16)
    hipLaunchKernelGGL(copy_kernel<__bf16>, dim3(grid_for(total)), dim3(256), 0, st, *d, (const __bf16*)x,
                       (__bf16*)y);
  else
    hipLaunchKernelGGL(copy_kernel<float>, dim3(grid_for(total)), dim3(256), 0, st, *d, (const float*)x,
                       (float*)y);
  return ycx_launch_status();
}

extern "C" ycx_status ycx_quantize_fp8(const float* x, void* y, int64_t n, float scale, void* stream) {
  YCX_CHECK_ARG(n >= 0 && (n == 0 || (x && y)));
  if (n == 0) return YCX_OK;
  hipLaunchKernelGGL(quantize_f8_kernel, dim3(grid_for((n + 3) / 4)), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), x, (uint8_t*)y, (long long)n, scale);
  return ycx_launch_status();
}

// ---------------------------------------------------------------------------
// Static plan executor: Model.forward's interpreter loop (nets/yolo.py:145-151)
// becomes one native loop over pre-validated op descriptors.
// ---------------------------------------------------------------------------
static ycx_status run_one(const ycx_op& op, void* stream) {
  switch (op.kind) {
    case YCX_OP_CONV:
      return ycx_conv2d(&op.d.conv, op.in, op.weight, op.bias, op.out, op.residual, stream);
    case YCX_OP_STEM:
      return ycx_stem_conv(&op.d.conv, (const float*)op.in, (const float*)op.weight, op.bias, op.out, stream);
    case YCX_OP_POOL:
      return ycx_maxpool(&op.d.pool, op.in, op.out, stream);
    case YCX_OP_COPY:
      return ycx_copy_channels(&op.d.copy, op.in, op.out, stream);
    case YCX_OP_STEM2:
      return ycx_stem_conv2(&op.d.pair[0], &op.d.pair[1], (const float*)op.in, (const float*)op.weight, op.bias,
                            op.weight2, op.bias2, op.out, stream);
    case YCX_OP_HEAD:
      return ycx_conv2d_head(&op.d.head.conv, &op.d.head.head, op.in, op.weight, op.bias, (float*)op.out,
                             (ycx_cand*)op.cand, op.cand_rows, op.cand_counts, stream);
    default:
      return YCX_ERR_BAD_ARG;
  }
}

extern "C" ycx_status ycx_run_ops(const ycx_op* ops, int32_t n_ops, void* stream, void* const* events) {
  YCX_CHECK_ARG(ops && n_ops >= 0);
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  for (int32_t i = 0; i < n_ops; ++i) {
    if (events && hipEventRecord(reinterpret_cast<hipEvent_t>(events[i]), st) != hipSuccess)
      return YCX_ERR_LAUNCH;
    ycx_status s = run_one(ops[i], stream);
    if (s != YCX_OK) return s;
  }
  if (events && hipEventRecord(reinterpret_cast<hipEvent_t>(events[n_ops]), st) != hipSuccess)
    return YCX_ERR_LAUNCH;
  return YCX_OK;
}

extern "C" ycx_status ycx_graph_capture(const ycx_op* ops, int32_t n_ops, void* stream, void** graph_exec) {
  YCX_CHECK_ARG(ops && graph_exec && stream);
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  hipGraph_t g = nullptr;
  if (hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal) != hipSuccess) return YCX_ERR_LAUNCH;
  ycx_status s = ycx_run_ops(ops, n_ops, stream, nullptr);
  hipError_t e = hipStreamEndCapture(st, &g);
  if (s != YCX_OK) {
    if (g) (void)hipGraphDestroy(g);
    return s;
  }
  if (e != hipSuccess || !g) return YCX_ERR_LAUNCH;
  hipGraphExec_t ex = nullptr;
  e = hipGraphInstantiate(&ex, g, nullptr, nullptr, 0);
  (void)hipGraphDestroy(g);
  if (e != hipSuccess) return YCX_ERR_LAUNCH;
  *graph_exec = ex;
  return YCX_OK;
}

extern "C" ycx_status ycx_graph_launch(void* graph_exec, void* stream) {
  YCX_CHECK_ARG(graph_exec);
  return hipGraphLaunch(reinterpret_cast<hipGraphExec_t>(graph_exec), reinterpret_cast<hipStream_t>(stream)) ==
                 hipSuccess
             ? YCX_OK
             : YCX_ERR_LAUNCH;
}

extern "C" ycx_status ycx_graph_destroy(void* graph_exec) {
  YCX_CHECK_ARG(graph_exec);
  return hipGraphExecDestroy(reinterpret_cast<hipGraphExec_t>(graph_exec)) == hipSuccess ? YCX_OK
                                                                                         : YCX_ERR_LAUNCH;
}

extern "C" int ycx_abi_version(void) { return YCX_ABI_VERSION; }

extern "C" size_t ycx_struct_size(int32_t which) {
  switch (which) {
    case 0: return sizeof(ycx_conv_desc);
    case 1: return sizeof(ycx_pool_desc);
    case 2: return sizeof(ycx_copy_desc);
    case 3: return sizeof(ycx_decode_desc);
    case 4: return sizeof(ycx_cand);
    case 5: return sizeof(ycx_filter_desc);
    case 6: return sizeof(ycx_decode_filter_desc);
    case 7: return sizeof(ycx_nms_desc);
    case 8: return sizeof(ycx_op);
    case 9: return sizeof(ycx_letterbox_desc);
    case 10: return sizeof(ycx_correct_desc);
    case 11: return sizeof(ycx_head_desc);
    default: return 0;
  }
}

extern "C" const char* ycx_strerror(ycx_status s) {
  switch (s) {
    case YCX_OK: return "ok";
    case YCX_ERR_BAD_ARG: return "ycx: bad argument (null pointer or inconsistent shape)";
    case YCX_ERR_UNSUPPORTED: return "ycx: unsupported shape/dtype for the HIP kernels";
    case YCX_ERR_LAUNCH: return "ycx: HIP launch/runtime failure";
    case YCX_ERR_CAPACITY: return "ycx: workspace or output capacity too small";
    default: return "ycx: unknown status";
  }
}
