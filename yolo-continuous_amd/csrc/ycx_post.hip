// Post-processing of the YOLO heads on gfx950: box decode and candidate filter
// (the sort + per-class NMS that consumes the candidates is in ycx_nms.hip).
//
//   ycx_decode          decode_box, one level              detect.py:29-87
//   ycx_filter_decoded  non_max_suppression :98-121         (xyxy in place, class max,
//                                                            obj*cls_conf >= conf_thres)
//   ycx_decode_filter   the two above fused, reading raw heads (fast path)
//
// Bit-exactness: the float expressions and their evaluation order restate the
// reference (and torchvision's CPU nms kernel) operation by operation; FMA
// contraction is disabled for this file so every product/sum rounds like the
// CPU code does.
#pragma clang fp contract(off)
#include <stdlib.h>
#include <stdint.h>
#include "ycx_internal.h"

namespace {

__device__ __forceinline__ float sigmoidf_ref(float v) { return ycx_sigmoid(v); }

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

// ---------------------------------------------------------------------------
// IDetect eval branch for one level (nets/idetect.py:33-43, with the strides
// the reference leaves unset supplied by the caller): the raw map re-laid as
// (bs, na, ny, nx, no) and the decoded rows z (pixel units):
//   xy = (sigmoid * 2 - 0.5 + grid) * stride,  wh = (sigmoid * 2)^2 * anchor_grid
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) idetect_kernel(ycx_decode_desc d, float stride, const float* __restrict__ head,
                                                      float* __restrict__ z, float* __restrict__ xview) {
  extern __shared__ __attribute__((aligned(16))) float tile[];  // [kDecCells][2 * no]
  const int n = blockIdx.z, a = blockIdx.y;
  const int hw = d.h * d.w;
  const int cell0 = blockIdx.x * kDecCells;
  const int ncell = min(kDecCells, hw - cell0);
  const float aw = d.anchors_scaled[2 * a], ah = d.anchors_scaled[2 * a + 1];
  const float* hb = head + ((size_t)n * d.na * d.no + (size_t)a * d.no) * hw;
  float* raw = tile + kDecCells * d.no;
  for (int idx = threadIdx.x; idx < d.no * kDecCells; idx += blockDim.x) {
    const int o = idx / kDecCells, c = idx - o * kDecCells;
    if (c >= ncell) continue;
    const int cell = cell0 + c;
    const float r = hb[(size_t)o * hw + cell];
    const float p = sigmoidf_ref(r);
    float v;
    if (o == 0) {
      v = ((p * 2.0f) - 0.5f + (float)(cell % d.w)) * stride;
    } else if (o == 1) {
      v = ((p * 2.0f) - 0.5f + (float)(cell / d.w)) * stride;
    } else if (o == 2) {
      const float t = p * 2.0f;
      v = (t * t) * aw;
    } else if (o == 3) {
      const float t = p * 2.0f;
      v = (t * t) * ah;
    } else {
      v = p;
    }
    tile[c * d.no + o] = v;
    raw[c * d.no + o] = r;
  }
  __syncthreads();
  const size_t row0 = (size_t)a * hw + cell0;  // (a, y, x) order = view(bs, -1, no) of (bs, na, ny, nx, no)
  float* zb = z + ((size_t)n * d.rows_total + d.row_off + row0) * d.no;
  float* xb = xview + ((size_t)n * d.na * hw + row0) * d.no;
  for (int idx = threadIdx.x; idx < ncell * d.no; idx += blockDim.x) {
    zb[idx] = tile[idx];
    xb[idx] = raw[idx];
  }
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
    if (slot < d.rows) rows_out[(size_t)n * d.rows + slot] = r;  // counts not reset by the caller: no overrun
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
  const int lane = threadIdx.x & 63;
  bool pass = false;
  ycx_cand c;
  int l = 0, hw = 1, W = 1, H = 1, an = 0, cell = 0;
  const float* hb = nullptr;
  float obj = 0.0f;
  if (r < d.rows_total) {
    while (l + 1 < d.nl && r >= d.row_off[l + 1]) ++l;
    H = d.h[l];
    W = d.w[l];
    hw = H * W;
    const int local = r - d.row_off[l];
    an = local / hw;
    cell = local - an * hw;
    hb = a.heads[l] + ((size_t)n * d.na * d.no + (size_t)an * d.no) * hw + cell;
    obj = sigmoidf_ref(hb[(size_t)4 * hw]);
  }
  // obj * cls <= obj (cls <= 1, monotone rounding): a row below conf on obj alone
  // never passes, so its class logits are not read.
  const bool want = hb != nullptr && obj >= d.conf_thres;
  unsigned long long m = __ballot(want);
  float best = 0.0f;
  int bi = 0;
  if (__popcll(m) <= 8) {
    // Sparse wave (trained weights: ~1e2 candidates per image): the whole wave
    // scans one row's classes at a time (one memory round trip for nc <= 64 per
    // lane-class slot instead of nc / 8 per lane). The result equals the
    // sequential strict-> scan: non-NaN maximum, first index on ties, and a NaN
    // at class 0 sticks.
    while (m) {
      const int j = __ffsll(m) - 1;
      m &= m - 1;
      const float* hj = reinterpret_cast<const float*>(__shfl((long long)hb, j));
      const int hwj = __shfl(hw, j);
      float bv = 0.0f;
      int bk = 0x7fffffff;
      for (int k = lane; k < d.nc; k += 64) {
        const float sv = sigmoidf_ref(hj[(size_t)(5 + k) * hwj]);
        if (sv == sv && (bk == 0x7fffffff || sv > bv)) { bv = sv; bk = k; }
      }
      for (int o = 32; o; o >>= 1) {
        const float ov = __shfl_xor(bv, o);
        const int ok = __shfl_xor(bk, o);
        if (ok != 0x7fffffff && (bk == 0x7fffffff || ov > bv || (ov == bv && ok < bk))) { bv = ov; bk = ok; }
      }
      if (lane == j) {
        const float s0 = sigmoidf_ref(hb[(size_t)5 * hw]);
        if (s0 != s0) { best = s0; bi = 0; } else { best = bv; bi = bk; }
      }
    }
  } else if (want) {
    ycx_class_argmax([&](int k) { return hb[(size_t)(5 + k) * hw]; }, d.nc, best, bi);
  }
  if (want) {
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
  const int slot = wave_append(pass, counts + n);
  if (pass) {
    cand[(size_t)n * d.rows_total + r] = c;
    if (slot < d.rows_total) rows_out[(size_t)n * d.rows_total + slot] = r;  // (counts not reset: no overrun)
  }
}

// Four consecutive rows (cells of one level/anchor plane) per thread: every
// class plane is read with 16-byte loads, so a wave streams 1 KB runs of each
// plane instead of 256 B (the fp32 NCHW heads put a row's nc logits in nc
// planes). Same float ops per row as decode_filter_kernel. Needs h*w % 4 == 0
// on every level and 16-byte aligned heads (checked by the launcher).
__global__ void __launch_bounds__(256) decode_filter4_kernel(DecodeFilterArgs a, ycx_cand* __restrict__ cand,
                                                             int* __restrict__ rows_out, int* __restrict__ counts) {
  const ycx_decode_filter_desc& d = a.d;
  const int n = blockIdx.y;
  const int r0 = (blockIdx.x * blockDim.x + threadIdx.x) * 4;
  const int lane = threadIdx.x & 63;
  bool pass[4] = {false, false, false, false};
  ycx_cand c[4];
  int l = 0, H = 1, W = 1, hw = 4, an = 0, cell = 0;
  const float* hb = nullptr;
  float obj[4] = {0.0f, 0.0f, 0.0f, 0.0f};
  bool want[4] = {false, false, false, false};
  if (r0 < d.rows_total) {
    while (l + 1 < d.nl && r0 >= d.row_off[l + 1]) ++l;
    H = d.h[l];
    W = d.w[l];
    hw = H * W;
    const int local = r0 - d.row_off[l];
    an = local / hw;
    cell = local - an * hw;
    hb = a.heads[l] + ((size_t)n * d.na * d.no + (size_t)an * d.no) * hw + cell;
    const float4 o = *reinterpret_cast<const float4*>(hb + (size_t)4 * hw);
    const float ov[4] = {o.x, o.y, o.z, o.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      obj[i] = sigmoidf_ref(ov[i]);
      want[i] = obj[i] >= d.conf_thres;  // obj * cls <= obj: otherwise the row cannot pass
    }
  }
  unsigned long long wm[4];
  int nwant = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    wm[i] = __ballot(want[i]);
    nwant += __popcll(wm[i]);
  }
  float best[4] = {0.0f, 0.0f, 0.0f, 0.0f};
  int bi[4] = {0, 0, 0, 0};
  const bool any = want[0] || want[1] || want[2] || want[3];
  auto plane = [&](int ch) { return *reinterpret_cast<const float4*>(hb + (size_t)ch * hw); };
  if (nwant <= 8) {
    // Sparse wave (trained weights: ~1e2 candidates per image): the whole wave
    // scans one row's classes at a time, one memory round trip instead of nc / 4.
    // The wave argmax equals the sequential strict-> scan: non-NaN maximum, first
    // index on ties, and a NaN at class 0 sticks.
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      unsigned long long m = wm[i];
      while (m) {
        const int j = __ffsll(m) - 1;
        m &= m - 1;
        const float* hj = reinterpret_cast<const float*>(__shfl((long long)hb, j)) + i;
        const int hwj = __shfl(hw, j);
        float bv = 0.0f;
        int bk = 0x7fffffff;
        for (int k = lane; k < d.nc; k += 64) {
          const float sv = sigmoidf_ref(hj[(size_t)(5 + k) * hwj]);
          if (sv == sv && (bk == 0x7fffffff || sv > bv)) { bv = sv; bk = k; }
        }
        for (int o = 32; o; o >>= 1) {
          const float ov = __shfl_xor(bv, o);
          const int ok = __shfl_xor(bk, o);
          if (ok != 0x7fffffff && (bk == 0x7fffffff || ov > bv || (ov == bv && ok < bk))) { bv = ov; bk = ok; }
        }
        if (lane == j) {
          const float s0 = sigmoidf_ref(hb[(size_t)5 * hw + i]);
          if (s0 != s0) { best[i] = s0; bi[i] = 0; } else { best[i] = bv; bi[i] = bk; }
        }
      }
    }
  } else if (any) {
    const float4 c0 = plane(5);
    best[0] = sigmoidf_ref(c0.x);
    best[1] = sigmoidf_ref(c0.y);
    best[2] = sigmoidf_ref(c0.z);
    best[3] = sigmoidf_ref(c0.w);
    {
      int k = 1;
      for (; k + 4 <= d.nc; k += 4) {  // 16 logits in flight; compares in class order (first index on ties)
        float4 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = plane(5 + k + u);
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const float e[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const float sv = sigmoidf_ref(e[i]);
            if (sv > best[i]) { best[i] = sv; bi[i] = k + u; }
          }
        }
      }
      for (; k < d.nc; ++k) {
        const float4 v = plane(5 + k);
        const float e[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float sv = sigmoidf_ref(e[i]);
          if (sv > best[i]) { best[i] = sv; bi[i] = k; }
        }
      }
    }
  }
  if (any) {
    {
      const float4 b0 = plane(0), b1 = plane(1), b2 = plane(2), b3 = plane(3);
      const float lx[4] = {b0.x, b0.y, b0.z, b0.w}, ly[4] = {b1.x, b1.y, b1.z, b1.w};
      const float lw[4] = {b2.x, b2.y, b2.z, b2.w}, lh[4] = {b3.x, b3.y, b3.z, b3.w};
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float score = obj[i] * best[i];
        if (want[i] && score >= d.conf_thres) {
          const int ci = cell + i;
          const float gx = (float)(ci % W), gy = (float)(ci / W);
          const float px = sigmoidf_ref(lx[i]), py = sigmoidf_ref(ly[i]);
          const float pw = sigmoidf_ref(lw[i]), ph = sigmoidf_ref(lh[i]);
          const float bx = ((px * 2.0f) - 0.5f + gx) / (float)W;
          const float by = ((py * 2.0f) - 0.5f + gy) / (float)H;
          const float tw = pw * 2.0f, th = ph * 2.0f;
          const float bw = (tw * tw * d.anchors_scaled[l][2 * an]) / (float)W;
          const float bh = (th * th * d.anchors_scaled[l][2 * an + 1]) / (float)H;
          pass[i] = true;
          c[i] = ycx_cand{bx - bw / 2.0f, by - bh / 2.0f, bx + bw / 2.0f, by + bh / 2.0f, obj[i], best[i], bi[i],
                          r0 + i};
        }
      }
    }
  }
  // Wave-aggregated append of up to 4 rows per lane (rows stay ascending within the wave).
  const unsigned long long lt = (1ull << lane) - 1ull;
  int tot = 0, pre = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const unsigned long long m = __ballot(pass[i]);
    tot += __popcll(m);
    pre += __popcll(m & lt);
  }
  if (tot == 0) return;  // wave-uniform
  int base = 0;
  if (lane == 0) base = atomicAdd(counts + n, tot);
  int slot = __shfl(base, 0) + pre;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    if (pass[i]) {
      cand[(size_t)n * d.rows_total + r0 + i] = c[i];
      if (slot < d.rows_total) rows_out[(size_t)n * d.rows_total + slot] = r0 + i;
      ++slot;
    }
  }
}

}  // namespace

namespace {
// The premise of ycx_class_finish's fast path for one logit m: sigmoid(m - tau) < sigmoid(m)
// with tau and m - tau as ycx_class_finish forms them (1 = violated).
__device__ __forceinline__ unsigned sigmoid_gap_bad(float m, float sm) {
  if (!(m >= kClassFastLo && m <= kClassFastHi)) return 0u;
  const float tau = fmaxf(fabsf(m), 1.0f) * 0x1p-12f;
  return ycx_sigmoid(m - tau) < sm ? 0u : 1u;
}

// Every finite non-negative bit pattern b (and its negative) against b + 1;
// 256 consecutive patterns per thread, the previous sigmoid carried. Also the
// fast-path premise (sigmoid_gap_bad) at every one of those floats.
__global__ void __launch_bounds__(256) sigmoid_monotone_kernel(unsigned long long* bad) {
  constexpr unsigned kPer = 256, kEnd = 0x7F800000u;  // +inf
  const unsigned b0 = (blockIdx.x * 256u + threadIdx.x) * kPer;
  if (b0 >= kEnd) return;
  unsigned cnt = 0;
  const float x0 = __uint_as_float(b0), y0 = __uint_as_float(b0 | 0x80000000u);
  float pp = ycx_sigmoid(x0), pn = ycx_sigmoid(y0);
  cnt += sigmoid_gap_bad(x0, pp) + sigmoid_gap_bad(y0, pn);
  for (unsigned i = 1; i <= kPer && b0 + i <= kEnd; ++i) {
    const unsigned b = b0 + i;
    const float x = __uint_as_float(b), y = __uint_as_float(b | 0x80000000u);
    const float sp = ycx_sigmoid(x), sn = ycx_sigmoid(y);
    cnt += (sp < pp ? 1u : 0u) + (sn > pn ? 1u : 0u);  // +x rising, -x falling with b
    cnt += sigmoid_gap_bad(x, sp) + sigmoid_gap_bad(y, sn);
    pp = sp;
    pn = sn;
  }
  if (cnt) atomicAdd(bad, (unsigned long long)cnt);
}
}  // namespace

extern "C" ycx_status ycx_check_sigmoid_monotone(unsigned long long* violations, void* stream) {
  YCX_CHECK_ARG(violations != nullptr);
  const unsigned threads = 0x7F800000u / 256u;
  hipLaunchKernelGGL(sigmoid_monotone_kernel, dim3((threads + 255) / 256), dim3(256), 0, (hipStream_t)stream,
                     violations);
  return ycx_launch_status();
}

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

extern "C" ycx_status ycx_idetect_decode(const ycx_decode_desc* d, float stride, const float* head, float* z,
                                         float* xview, void* stream) {
  YCX_CHECK_ARG(d && head && z && xview);
  YCX_CHECK_ARG(d->n > 0 && d->h > 0 && d->w > 0 && d->na > 0 && d->no > 5);
  YCX_CHECK_ARG(d->row_off >= 0 && d->row_off + d->na * d->h * d->w <= d->rows_total);
  YCX_CHECK_SUPPORTED(d->na <= 8 && d->no <= 256);
  const size_t lds = (size_t)2 * kDecCells * d->no * sizeof(float);
  dim3 grid(ycx_cdiv((long long)d->h * d->w, kDecCells), d->na, d->n);
  hipLaunchKernelGGL(idetect_kernel, grid, dim3(256), lds, reinterpret_cast<hipStream_t>(stream), *d, stride, head, z,
                     xview);
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
  bool quad = true;  // the one-row-per-thread kernel covers ragged levels and unaligned heads
  for (int l = 0; l < d->nl; ++l)
    quad = quad && (d->h[l] * d->w[l]) % 4 == 0 && (reinterpret_cast<uintptr_t>(heads[l]) & 15) == 0;
  if (quad) {
    dim3 grid(ycx_cdiv(d->rows_total / 4, 256), d->n);
    hipLaunchKernelGGL(decode_filter4_kernel, grid, dim3(256), 0, reinterpret_cast<hipStream_t>(stream), a, cand,
                       cand_rows, cand_counts);
  } else {
    dim3 grid(ycx_cdiv(d->rows_total, 256), d->n);
    hipLaunchKernelGGL(decode_filter_kernel, grid, dim3(256), 0, reinterpret_cast<hipStream_t>(stream), a, cand,
                       cand_rows, cand_counts);
  }
  return ycx_launch_status();
}
