// Post-processing of the YOLO heads on gfx950: box decode, candidate filter,
// per-image sort and per-class greedy NMS.
//
//   ycx_decode          decode_box, one level              detect.py:29-87
//   ycx_filter_decoded  non_max_suppression :98-121         (xyxy in place, class max,
//                                                            obj*cls_conf >= conf_thres)
//   ycx_decode_filter   the two above fused, reading raw heads (fast path)
//   ycx_sort_nms        the per-class torchvision.ops.nms loop (detect.py:124-137):
//                       one workgroup per image, 64-bit key bitonic sort in LDS,
//                       greedy suppression with an LDS bitset
//
// Bit-exactness: the float expressions and their evaluation order restate the
// reference (and torchvision's CPU nms kernel) operation by operation; FMA
// contraction is disabled for this file so every product/sum rounds like the
// CPU code does.
#pragma clang fp contract(off)
#include "ycx_internal.h"

namespace {

__device__ __forceinline__ float sigmoidf_ref(float v) { return 1.0f / (1.0f + expf(-v)); }

// Wave-aggregated append: one atomic per wave (ballot + popcount + mbcnt).
__device__ __forceinline__ int wave_append(bool pass, int* counter) {
  const unsigned long long m = __ballot(pass);
  if (m == 0) return -1;
  const int lane = threadIdx.x & 63;
  const int leader = __ffsll((long long)m) - 1;
  int base = 0;
  if (lane == leader) base = atomicAdd(counter, __popcll(m));
  base = __shfl(base, leader);
  return pass ? base + __popcll(m & ((1ull << lane) - 1ull)) : -1;
}

// ---------------------------------------------------------------------------
// decode_box for one level: block = 64 consecutive grid cells of one (n, a).
// Reads the NCHW head channel by channel (coalesced over cells), transposes
// through LDS and writes the [64][no] output rows as one contiguous run.
// ---------------------------------------------------------------------------
constexpr int kDecCells = 64;

__global__ void __launch_bounds__(256) decode_kernel(ycx_decode_desc d, const float* __restrict__ head,
                                                     float* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) float tile[];  // [kDecCells][no]
  const int n = blockIdx.z, a = blockIdx.y;
  const int hw = d.h * d.w;
  const int cell0 = blockIdx.x * kDecCells;
  const int ncell = min(kDecCells, hw - cell0);
  const float aw = d.anchors_scaled[2 * a], ah = d.anchors_scaled[2 * a + 1];
  const float* hb = head + ((size_t)n * d.na * d.no + (size_t)a * d.no) * hw;
  for (int idx = threadIdx.x; idx < d.no * kDecCells; idx += blockDim.x) {
    const int o = idx / kDecCells, c = idx - o * kDecCells;
    if (c >= ncell) continue;
    const int cell = cell0 + c;
    float p = sigmoidf_ref(hb[(size_t)o * hw + cell]);
    float v;
    if (o == 0) {
      const float gx = (float)(cell % d.w);
      v = ((p * 2.0f) - 0.5f + gx) / (float)d.w;
    } else if (o == 1) {
      const float gy = (float)(cell / d.w);
      v = ((p * 2.0f) - 0.5f + gy) / (float)d.h;
    } else if (o == 2) {
      const float t = p * 2.0f;
      v = (t * t * aw) / (float)d.w;
    } else if (o == 3) {
      const float t = p * 2.0f;
      v = (t * t * ah) / (float)d.h;
    } else {
      v = p;
    }
    tile[c * d.no + o] = v;
  }
  __syncthreads();
  float* ob = out + ((size_t)n * d.rows_total + d.row_off + (size_t)a * hw + cell0) * d.no;
  for (int idx = threadIdx.x; idx < ncell * d.no; idx += blockDim.x) ob[idx] = tile[idx];
}

// Class max with torch.max(dim) semantics (first index of the maximum).
__device__ __forceinline__ void class_max(const float* row_cls, int nc, int stride, float& best, int& bi) {
  best = row_cls[0];
  bi = 0;
  for (int c = 1; c < nc; ++c) {
    float v = row_cls[(size_t)c * stride];
    if (v > best) { best = v; bi = c; }
  }
}

// ---------------------------------------------------------------------------
// Filter of a decoded [n][rows][no] tensor: detect.py:98-121.
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) filter_decoded_kernel(ycx_filter_desc d, float* __restrict__ pred,
                                                             ycx_cand* __restrict__ cand, int* __restrict__ rows_out,
                                                             int* __restrict__ counts) {
  const int n = blockIdx.y;
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  bool pass = false;
  ycx_cand c;
  if (r < d.rows) {
    float* p = pred + ((size_t)n * d.rows + r) * d.no;
    const float cx = p[0], cy = p[1], w = p[2], h = p[3];
    const float x1 = cx - w / 2.0f, y1 = cy - h / 2.0f, x2 = cx + w / 2.0f, y2 = cy + h / 2.0f;
    if (d.write_xyxy) { p[0] = x1; p[1] = y1; p[2] = x2; p[3] = y2; }
    // No early-out on obj here: the input is an arbitrary decoded tensor, so
    // cls_conf <= 1 cannot be assumed (the fused path below can assume it).
    const float obj = p[4];
    float best;
    int bi;
    class_max(p + 5, d.nc, 1, best, bi);
    const float score = obj * best;
    if (score >= d.conf_thres) {
      pass = true;
      c = ycx_cand{x1, y1, x2, y2, obj, best, bi, r};
    }
  }
  const int slot = wave_append(pass, counts + n);
  if (pass) {
    cand[(size_t)n * d.rows + r] = c;
    rows_out[(size_t)n * d.rows + slot] = r;
  }
}

// ---------------------------------------------------------------------------
// Fused decode + filter from the raw NCHW heads (fast path). Same float ops in
// the same order as decode_kernel followed by filter_decoded_kernel.
// ---------------------------------------------------------------------------
struct DecodeFilterArgs {
  ycx_decode_filter_desc d;
  const float* heads[4];
};

__global__ void __launch_bounds__(256) decode_filter_kernel(DecodeFilterArgs a, ycx_cand* __restrict__ cand,
                                                            int* __restrict__ rows_out, int* __restrict__ counts) {
  const ycx_decode_filter_desc& d = a.d;
  const int n = blockIdx.y;
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  bool pass = false;
  ycx_cand c;
  if (r < d.rows_total) {
    int l = 0;
    while (l + 1 < d.nl && r >= d.row_off[l + 1]) ++l;
    const int H = d.h[l], W = d.w[l], hw = H * W;
    const int local = r - d.row_off[l];
    const int an = local / hw, cell = local - an * hw;
    const float* hb = a.heads[l] + ((size_t)n * d.na * d.no + (size_t)an * d.no) * hw + cell;
    const float obj = sigmoidf_ref(hb[(size_t)4 * hw]);
    if (obj >= d.conf_thres) {
      float best = sigmoidf_ref(hb[(size_t)5 * hw]);
      int bi = 0;
      for (int k = 1; k < d.nc; ++k) {
        float v = sigmoidf_ref(hb[(size_t)(5 + k) * hw]);
        if (v > best) { best = v; bi = k; }
      }
      const float score = obj * best;
      if (score >= d.conf_thres) {
        const float gx = (float)(cell % W), gy = (float)(cell / W);
        const float px = sigmoidf_ref(hb[0]), py = sigmoidf_ref(hb[hw]);
        const float pw = sigmoidf_ref(hb[(size_t)2 * hw]), ph = sigmoidf_ref(hb[(size_t)3 * hw]);
        const float bx = ((px * 2.0f) - 0.5f + gx) / (float)W;
        const float by = ((py * 2.0f) - 0.5f + gy) / (float)H;
        const float tw = pw * 2.0f, th = ph * 2.0f;
        const float bw = (tw * tw * d.anchors_scaled[l][2 * an]) / (float)W;
        const float bh = (th * th * d.anchors_scaled[l][2 * an + 1]) / (float)H;
        pass = true;
        c = ycx_cand{bx - bw / 2.0f, by - bh / 2.0f, bx + bw / 2.0f, by + bh / 2.0f, obj, best, bi, r};
      }
    }
  }
  const int slot = wave_append(pass, counts + n);
  if (pass) {
    cand[(size_t)n * d.rows_total + r] = c;
    rows_out[(size_t)n * d.rows_total + slot] = r;
  }
}

// ---------------------------------------------------------------------------
// Sort + NMS: one 1024-thread workgroup per image.
// ---------------------------------------------------------------------------
constexpr int kNmsThreads = 1024;
constexpr int kLdsKeys = 8192;  // 64 KiB of 64-bit keys; larger sets sort in the workspace

struct NmsLayout {
  size_t keys_off, box_off, area_off, per_image;
  int p_max;
};

__host__ __device__ inline int next_pow2(int v) {
  int p = 1;
  while (p < v) p <<= 1;
  return p;
}
__host__ __device__ inline int row_bits(int rows) {
  int b = 1;
  while ((1 << b) < rows) ++b;
  return b;
}
__host__ __device__ inline NmsLayout nms_layout(int rows_total) {
  NmsLayout L;
  L.p_max = next_pow2(rows_total);
  L.keys_off = 0;
  L.box_off = (size_t)L.p_max * 8;
  L.area_off = L.box_off + (size_t)rows_total * 16;
  L.per_image = (L.area_off + (size_t)rows_total * 4 + 255) & ~(size_t)255;
  return L;
}

__device__ void bitonic_sort(unsigned long long* keys, int P) {
  for (int k = 2; k <= P; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = threadIdx.x; i < P; i += blockDim.x) {
        const int ixj = i ^ j;
        if (ixj > i) {
          const unsigned long long x = keys[i], y = keys[ixj];
          const bool up = (i & k) == 0;
          if ((x > y) == up) { keys[i] = y; keys[ixj] = x; }
        }
      }
      __syncthreads();
    }
  }
}

__global__ void __launch_bounds__(kNmsThreads) sort_nms_kernel(ycx_nms_desc d, const ycx_cand* __restrict__ cand,
                                                               const int* __restrict__ cand_rows,
                                                               const int* __restrict__ cand_counts, char* ws,
                                                               float* __restrict__ dets, int* __restrict__ keep_rows,
                                                               int* __restrict__ keep_counts) {
  __shared__ unsigned long long s_keys[kLdsKeys];
  __shared__ unsigned int s_removed[(kLdsKeys * 16) / 32];  // bitset for up to 131072 candidates
  const int img = blockIdx.x;
  const int tid = threadIdx.x;
  const NmsLayout L = nms_layout(d.rows_total);
  char* wsi = ws + (size_t)img * L.per_image;
  const int cnt = min(cand_counts[img], d.rows_total);
  const int rb = row_bits(d.rows_total);
  const ycx_cand* ci = cand + (size_t)img * d.rows_total;
  const int* cr = cand_rows + (size_t)img * d.rows_total;

  const int P = next_pow2(max(cnt, 1));
  unsigned long long* keys = P <= kLdsKeys ? s_keys : reinterpret_cast<unsigned long long*>(wsi + L.keys_off);
  for (int i = tid; i < P; i += blockDim.x) {
    unsigned long long k = ~0ull;
    if (i < cnt) {
      const int r = cr[i];
      const ycx_cand c = ci[r];
      const float score = c.obj * c.cls_conf;
      const unsigned int inv = 0xFFFFFFFFu - __float_as_uint(score);
      k = ((unsigned long long)(unsigned)c.cls << (32 + rb)) | ((unsigned long long)inv << rb) |
          (unsigned long long)(unsigned)r;
    }
    keys[i] = k;
  }
  const int nwords = (cnt + 31) >> 5;
  for (int i = tid; i < nwords; i += blockDim.x) s_removed[i] = 0u;
  __syncthreads();
  bitonic_sort(keys, P);

  // Gather sorted boxes + areas (areas = (x2-x1)*(y2-y1), torchvision nms).
  f32x4* sbox = reinterpret_cast<f32x4*>(wsi + L.box_off);
  float* sarea = reinterpret_cast<float*>(wsi + L.area_off);
  const unsigned long long rmask = (1ull << rb) - 1ull;
  for (int i = tid; i < cnt; i += blockDim.x) {
    const ycx_cand c = ci[(int)(keys[i] & rmask)];
    sbox[i] = f32x4{c.x1, c.y1, c.x2, c.y2};
    sarea[i] = (c.x2 - c.x1) * (c.y2 - c.y1);
  }
  __syncthreads();

  // Greedy per-class suppression in sorted order (class asc, score desc).
  int nkeep = 0;
  int i = 0;
  while (true) {
    // Skip to the next unsuppressed candidate (uniform: every lane reads the same words).
    while (i < cnt) {
      const unsigned int free_bits = ~s_removed[i >> 5] >> (i & 31);
      if (free_bits) { i += __builtin_ctz(free_bits); break; }
      i = (i | 31) + 1;
    }
    if (i >= cnt) break;
    const unsigned long long ki = keys[i];
    const int row_i = (int)(ki & rmask);
    if (nkeep < d.max_det && tid == 0) {
      const ycx_cand c = ci[row_i];
      float* o = dets + ((size_t)img * d.max_det + nkeep) * 7;
      o[0] = c.x1; o[1] = c.y1; o[2] = c.x2; o[3] = c.y2;
      o[4] = c.obj; o[5] = c.cls_conf; o[6] = (float)c.cls;
      keep_rows[(size_t)img * d.max_det + nkeep] = row_i;
    }
    ++nkeep;
    const unsigned long long cls_i = ki >> (32 + rb);
    const f32x4 bi = sbox[i];
    const float ai = sarea[i];
    for (int j = i + 1 + tid; j < cnt; j += blockDim.x) {
      if ((keys[j] >> (32 + rb)) != cls_i) break;  // sorted by class: the segment ended
      if ((s_removed[j >> 5] >> (j & 31)) & 1u) continue;
      const f32x4 bj = sbox[j];
      const float xx1 = fmaxf(bi[0], bj[0]), yy1 = fmaxf(bi[1], bj[1]);
      const float xx2 = fminf(bi[2], bj[2]), yy2 = fminf(bi[3], bj[3]);
      const float w = fmaxf(0.0f, xx2 - xx1), h = fmaxf(0.0f, yy2 - yy1);
      const float inter = w * h;
      const float ovr = inter / (ai + sarea[j] - inter);
      if ((double)ovr > d.iou_thres) atomicOr(&s_removed[j >> 5], 1u << (j & 31));
    }
    __syncthreads();
    ++i;
  }
  if (tid == 0) keep_counts[img] = nkeep;
  for (int k = nkeep + tid; k < d.max_det; k += blockDim.x) {
    keep_rows[(size_t)img * d.max_det + k] = -1;
    float* o = dets + ((size_t)img * d.max_det + k) * 7;
    for (int t = 0; t < 7; ++t) o[t] = 0.0f;
  }
}

}  // namespace

extern "C" ycx_status ycx_decode(const ycx_decode_desc* d, const float* head, float* out, void* stream) {
  YCX_CHECK_ARG(d && head && out);
  YCX_CHECK_ARG(d->n > 0 && d->h > 0 && d->w > 0 && d->na > 0 && d->no > 5);
  YCX_CHECK_ARG(d->row_off >= 0 && d->row_off + d->na * d->h * d->w <= d->rows_total);
  YCX_CHECK_SUPPORTED(d->na <= 8 && d->no <= 256);
  const size_t lds = (size_t)kDecCells * d->no * sizeof(float);
  dim3 grid(ycx_cdiv((long long)d->h * d->w, kDecCells), d->na, d->n);
  hipLaunchKernelGGL(decode_kernel, grid, dim3(256), lds, reinterpret_cast<hipStream_t>(stream), *d, head, out);
  return ycx_launch_status();
}

extern "C" ycx_status ycx_filter_decoded(const ycx_filter_desc* d, float* pred, ycx_cand* cand, int32_t* cand_rows,
                                         int32_t* cand_counts, void* stream) {
  YCX_CHECK_ARG(d && pred && cand && cand_rows && cand_counts);
  YCX_CHECK_ARG(d->n > 0 && d->rows > 0 && d->nc > 0 && d->no >= 5 + d->nc);
  dim3 grid(ycx_cdiv(d->rows, 256), d->n);
  hipLaunchKernelGGL(filter_decoded_kernel, grid, dim3(256), 0, reinterpret_cast<hipStream_t>(stream), *d, pred,
                     cand, cand_rows, cand_counts);
  return ycx_launch_status();
}

extern "C" ycx_status ycx_decode_filter(const ycx_decode_filter_desc* d, const float* const* heads, ycx_cand* cand,
                                        int32_t* cand_rows, int32_t* cand_counts, void* stream) {
  YCX_CHECK_ARG(d && heads && cand && cand_rows && cand_counts);
  YCX_CHECK_ARG(d->n > 0 && d->nl > 0 && d->nl <= 4 && d->na > 0 && d->na <= 8 && d->nc > 0 &&
                d->no == d->nc + 5);
  int rows = 0;
  for (int l = 0; l < d->nl; ++l) {
    YCX_CHECK_ARG(heads[l] && d->h[l] > 0 && d->w[l] > 0 && d->row_off[l] == rows);
    rows += d->na * d->h[l] * d->w[l];
  }
  YCX_CHECK_ARG(rows == d->rows_total);
  DecodeFilterArgs a;
  a.d = *d;
  for (int l = 0; l < 4; ++l) a.heads[l] = l < d->nl ? heads[l] : nullptr;
  dim3 grid(ycx_cdiv(d->rows_total, 256), d->n);
  hipLaunchKernelGGL(decode_filter_kernel, grid, dim3(256), 0, reinterpret_cast<hipStream_t>(stream), a, cand,
                     cand_rows, cand_counts);
  return ycx_launch_status();
}

extern "C" size_t ycx_nms_workspace_size(const ycx_nms_desc* d) {
  if (!d || d->n <= 0 || d->rows_total <= 0) return 0;
  return nms_layout(d->rows_total).per_image * (size_t)d->n;
}

extern "C" ycx_status ycx_sort_nms(const ycx_nms_desc* d, const ycx_cand* cand, const int32_t* cand_rows,
                                   const int32_t* cand_counts, void* workspace, size_t workspace_bytes, float* dets,
                                   int32_t* keep_rows, int32_t* keep_counts, void* stream) {
  YCX_CHECK_ARG(d && cand && cand_rows && cand_counts && workspace && dets && keep_rows && keep_counts);
  YCX_CHECK_ARG(d->n > 0 && d->rows_total > 0 && d->nc > 0 && d->max_det > 0);
  if (workspace_bytes < ycx_nms_workspace_size(d)) return YCX_ERR_CAPACITY;
  const int rb = row_bits(d->rows_total);
  YCX_CHECK_SUPPORTED(rb <= 17 && d->rows_total <= kLdsKeys * 16);
  YCX_CHECK_SUPPORTED((long long)d->nc <= (1LL << (32 - rb)));
  hipLaunchKernelGGL(sort_nms_kernel, dim3(d->n), dim3(kNmsThreads), 0, reinterpret_cast<hipStream_t>(stream), *d,
                     cand, cand_rows, cand_counts, (char*)workspace, dets, keep_rows, keep_counts);
  return ycx_launch_status();
}
