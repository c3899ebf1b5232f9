// Per-image, per-class greedy NMS with torchvision.ops.nms semantics — the
// loop of detect.py:124-137 (unique classes ascending, nms per class, results
// concatenated class by class) for the whole batch in three launches.
//
//  nms_prep    one 1024-thread workgroup per image:
//              class histogram (LDS atomics) + exclusive scan -> one bucket per
//              class; every wave pulls whole classes from an LDS counter and a
//              class of S <= 512 candidates is finished entirely in registers:
//              64*R keys (score desc, row asc: torchvision's stable descending
//              sort) bitonic-sorted across lanes (shfl_xor) and register slots,
//              boxes gathered, greedy suppression with removed/kept flags as
//              R-bit masks per lane and box i broadcast by readlane — no LDS,
//              no barrier. Larger classes are bitonic-sorted by the workgroup
//              (LDS keys up to 8192) and queued as tasks for nms_mask.
//  nms_mask    the whole GPU: one wave per (large class, 64-row strip) computes
//              the IoU > thr bitmask of its rows against every later column
//              (row-major words, j > i only) — the O(S^2) part, fully parallel.
//  nms_finish  one workgroup per image: one wave per large class runs the
//              serial greedy scan over the bitmask (removed words in LDS, one
//              64-bit OR per lane per kept row), then an exclusive scan of the
//              per-class kept counts places every kept row in class order.
//
// IoU is torchvision's fp32 expression inter / (area_i + area_j - inter),
// area = (x2-x1)*(y2-y1), compared as (double)iou > iou_threshold; FMA
// contraction is off so the kept set is bit-identical to the CPU kernel.
// Every loop is bounded (work-queue loops exit when the queue is empty).
#pragma clang fp contract(off)
#include <string.h>
#include <math.h>
#include "ycx_internal.h"

namespace {

constexpr int kThreads = 1024;
constexpr int kMaxNc = 1024;      // classes handled in LDS
constexpr int kRegMax = 512;      // largest class finished in registers (R = 8 slots per lane)
constexpr int kLdsKeys = 8192;    // largest class sorted in LDS
constexpr int kMaxRows = 131072;  // rows (candidates) per image
constexpr int kMaskThreads = 256;
constexpr int kMaskBlocks = 2048;

struct Seg {  // one large class = one task range of nms_mask
  int img, off, S, nbw;
  long long mask_off;  // u64 words from the image's mask base
  int task_start, pad;
};

struct Layout {
  size_t hdr, segs, per_image_base;  // header + segment table (batch), then per image:
  size_t keys, box, area, bucket, kept, cnt, offs, kc, big, mask, per_image;
  int max_segs;
};

__host__ __device__ inline int next_pow2(int v) {
  int p = 1;
  while (p < v) p <<= 1;
  return p;
}

__host__ __device__ inline size_t al(size_t v) { return (v + 255) & ~(size_t)255; }

__host__ __device__ inline Layout layout(int n, int rows) {
  Layout L;
  L.max_segs = rows / (kRegMax + 1) + 1;
  L.hdr = 0;
  L.segs = 256;
  L.per_image_base = al(L.segs + (size_t)n * L.max_segs * sizeof(Seg));
  size_t o = 0;
  L.keys = o; o = al(o + (size_t)next_pow2(rows) * 8);
  L.box = o; o = al(o + (size_t)rows * 16);
  L.area = o; o = al(o + (size_t)rows * 4);
  L.bucket = o; o = al(o + (size_t)rows * 4);
  L.kept = o; o = al(o + (size_t)rows * 4);
  L.cnt = o; o = al(o + kMaxNc * 4);
  L.offs = o; o = al(o + kMaxNc * 4);
  L.kc = o; o = al(o + kMaxNc * 4);
  L.big = o; o = al(o + (size_t)(L.max_segs + 1) * 4);
  L.mask = o; o = al(o + (size_t)rows * ((rows + 63) / 64) * 8);
  L.per_image = o;
  return L;
}

struct Hdr {
  int nseg, ntasks;
};

// Sort key within a class: score descending (inverted fp32 bits; scores are
// products of sigmoids, never negative), then row ascending (stable sort).
__device__ __forceinline__ unsigned long long make_key(const ycx_cand& c) {
  const float score = c.obj * c.cls_conf;
  return ((unsigned long long)(0xFFFFFFFFu - __float_as_uint(score)) << 32) | (unsigned)c.row;
}

// The IoU threshold in division-free form. With T the smallest float above
// thr and Tm its predecessor, fl(x/y) > thr  <=>  fl(x/y) >= T  <=>  x/y >= m
// (x/y > m when the tie at m rounds down to Tm, i.e. T's mantissa is odd),
// m = (Tm + T)/2. For finite x >= 0 and finite y > 0, m*y is exact in double
// (25 + 24 significant bits), so the test below is exact; anything else takes
// the literal division.
struct Thr {
  double thr, m;
  int incl, fast;
};

__device__ __forceinline__ bool suppress(float ax1, float ay1, float ax2, float ay2, float aa, float bx1, float by1,
                                         float bx2, float by2, float ba, const Thr& t) {
  const float xx1 = fmaxf(ax1, bx1), yy1 = fmaxf(ay1, by1);
  const float xx2 = fminf(ax2, bx2), yy2 = fminf(ay2, by2);
  const float w = fmaxf(0.0f, xx2 - xx1), h = fmaxf(0.0f, yy2 - yy1);
  const float inter = w * h;
  const float den = aa + ba - inter;
  if (t.fast && den > 0.0f && den < INFINITY && inter < INFINITY) {
    const double lhs = (double)inter, rhs = t.m * (double)den;
    return t.incl ? lhs >= rhs : lhs > rhs;
  }
  return (double)(inter / den) > t.thr;
}

__device__ __forceinline__ float bcast(float v, int lane) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), lane));
}

template <int R>
__device__ __forceinline__ float pick(const float (&a)[R], int r) {
  float v = a[0];
#pragma unroll
  for (int k = 1; k < R; ++k) v = (r == k) ? a[k] : v;
  return v;
}

// A whole class in registers: position e = r*64 + lane, r < R.
template <int R>
__device__ void class_in_registers(const ycx_cand* __restrict__ ci, const int* __restrict__ bucket,
                                   int* __restrict__ kept, int S, Thr thr, int* kc_out) {
  constexpr int N = 64 * R;
  const int lane = threadIdx.x & 63;
  unsigned long long key[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int e = r * 64 + lane;
    key[r] = e < S ? make_key(ci[bucket[e]]) : ~0ull;
  }
#pragma unroll
  for (int k = 2; k <= N; k <<= 1) {  // bitonic sort, ascending over e
#pragma unroll
    for (int j = k >> 1; j > 0; j >>= 1) {
      if (j >= 64) {
        const int js = j >> 6;
#pragma unroll
        for (int r = 0; r < R; ++r) {
          if ((r & js) == 0) {
            const int r2 = r | js;
            const bool up = ((r * 64) & k) == 0;
            const unsigned long long a = key[r], b = key[r2];
            if ((a > b) == up) { key[r] = b; key[r2] = a; }
          }
        }
      } else {
#pragma unroll
        for (int r = 0; r < R; ++r) {
          const unsigned long long o = __shfl_xor(key[r], j);
          const int e = r * 64 + lane;
          const bool up = (e & k) == 0, lower = (lane & j) == 0;
          const unsigned long long mn = key[r] < o ? key[r] : o, mx = key[r] < o ? o : key[r];
          key[r] = (lower == up) ? mn : mx;
        }
      }
    }
  }
  float x1[R], y1[R], x2[R], y2[R], ar[R];
  int row[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int e = r * 64 + lane;
    row[r] = (int)(unsigned)key[r];
    if (e < S) {
      const ycx_cand c = ci[row[r]];
      x1[r] = c.x1; y1[r] = c.y1; x2[r] = c.x2; y2[r] = c.y2;
      ar[r] = (c.x2 - c.x1) * (c.y2 - c.y1);
    } else {
      x1[r] = y1[r] = x2[r] = y2[r] = ar[r] = 0.0f;
    }
  }
  unsigned rm = 0u, km = 0u;  // bit r: position r*64+lane removed / kept
  for (int i = 0; i < S; ++i) {
    const int ri = i >> 6, li = i & 63;
    if ((__builtin_amdgcn_readlane(rm, li) >> ri) & 1u) continue;
    if (lane == li) km |= 1u << ri;
    const float bx1 = bcast(pick<R>(x1, ri), li), by1 = bcast(pick<R>(y1, ri), li);
    const float bx2 = bcast(pick<R>(x2, ri), li), by2 = bcast(pick<R>(y2, ri), li);
    const float ba = bcast(pick<R>(ar, ri), li);
#pragma unroll
    for (int r = 0; r < R; ++r) {
      if (r < ri) continue;  // uniform: every position of an earlier slot precedes i
      const int e = r * 64 + lane;
      if (e > i && e < S && !((rm >> r) & 1u) &&
          suppress(bx1, by1, bx2, by2, ba, x1[r], y1[r], x2[r], y2[r], ar[r], thr))
        rm |= 1u << r;
    }
  }
  int base = 0;  // kept rows, compacted in sorted (score-descending) order
  const unsigned long long lt = (1ull << lane) - 1ull;
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const bool b = (km >> r) & 1u;
    const unsigned long long m = __ballot(b);
    if (b) kept[base + __popcll(m & lt)] = row[r];
    base += __popcll(m);
  }
  if (lane == 0) *kc_out = base;
}

// Exclusive scan of in[0..n) into out[0..n) by ONE wave; returns the total.
__device__ int wave_exclusive_scan(const int* in, int* out, int n) {
  const int lane = threadIdx.x & 63;
  const int per = (n + 63) / 64;
  const int b = lane * per, e = min(n, b + per);
  int s = 0;
  for (int i = b; i < e; ++i) s += in[i];
  int incl = s;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int t = __shfl_up(incl, d);
    if (lane >= d) incl += t;
  }
  int run = incl - s;
  for (int i = b; i < e; ++i) {
    const int v = in[i];
    out[i] = run;
    run += v;
  }
  return __shfl(incl, 63);
}

__device__ void block_bitonic(unsigned long long* keys, int P) {
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

struct Ptrs {
  unsigned long long* keysg;
  f32x4* box;
  float* area;
  int *bucket, *kept, *cnt, *offs, *kc, *big;
  unsigned long long* mask;
};

__device__ __forceinline__ Ptrs image_ptrs(char* ws, const Layout& L, int img) {
  char* b = ws + L.per_image_base + (size_t)img * L.per_image;
  Ptrs p;
  p.keysg = reinterpret_cast<unsigned long long*>(b + L.keys);
  p.box = reinterpret_cast<f32x4*>(b + L.box);
  p.area = reinterpret_cast<float*>(b + L.area);
  p.bucket = reinterpret_cast<int*>(b + L.bucket);
  p.kept = reinterpret_cast<int*>(b + L.kept);
  p.cnt = reinterpret_cast<int*>(b + L.cnt);
  p.offs = reinterpret_cast<int*>(b + L.offs);
  p.kc = reinterpret_cast<int*>(b + L.kc);
  p.big = reinterpret_cast<int*>(b + L.big);
  p.mask = reinterpret_cast<unsigned long long*>(b + L.mask);
  return p;
}

// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(kThreads) nms_prep(ycx_nms_desc d, const ycx_cand* __restrict__ cand,
                                                     const int* __restrict__ cand_rows,
                                                     const int* __restrict__ cand_counts, char* ws, Thr thr) {
  __shared__ unsigned long long s_keys[kLdsKeys];
  __shared__ int s_cnt[kMaxNc], s_off[kMaxNc], s_fill[kMaxNc], s_kc[kMaxNc], s_big[kMaxNc];
  __shared__ int s_next, s_nbig;
  const int img = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int nc = d.nc, rows = d.rows_total;
  const Layout L = layout(d.n, rows);
  const Ptrs P = image_ptrs(ws, L, img);
  Hdr* hdr = reinterpret_cast<Hdr*>(ws + L.hdr);
  Seg* segs = reinterpret_cast<Seg*>(ws + L.segs);
  const ycx_cand* ci = cand + (size_t)img * rows;
  const int* cr = cand_rows + (size_t)img * rows;
  const int cnt = min(cand_counts[img], rows);

  for (int c = tid; c < nc; c += kThreads) { s_cnt[c] = 0; s_fill[c] = 0; s_kc[c] = 0; }
  if (tid == 0) { s_next = 0; s_nbig = 0; }
  __syncthreads();
  for (int i = tid; i < cnt; i += kThreads) atomicAdd(&s_cnt[ci[cr[i]].cls], 1);
  __syncthreads();
  if (wid == 0) wave_exclusive_scan(s_cnt, s_off, nc);
  __syncthreads();
  for (int i = tid; i < cnt; i += kThreads) {
    const int r = cr[i];
    const int c = ci[r].cls;
    P.bucket[s_off[c] + atomicAdd(&s_fill[c], 1)] = r;
  }
  __syncthreads();

  // Classes of <= kRegMax candidates: one wave each, in registers.
  for (int it = 0; it <= nc + 64; ++it) {  // bounded work-queue loop
    int c = 0;
    if (lane == 0) c = atomicAdd(&s_next, 1);
    c = __builtin_amdgcn_readfirstlane(__shfl(c, 0));
    if (c >= nc) break;
    const int S = __builtin_amdgcn_readfirstlane(s_cnt[c]);
    if (S == 0) continue;
    if (S > kRegMax) {
      if (lane == 0) s_big[atomicAdd(&s_nbig, 1)] = c;
      continue;
    }
    const int* bk = P.bucket + s_off[c];
    int* kp = P.kept + s_off[c];
    if (S <= 64) class_in_registers<1>(ci, bk, kp, S, thr, &s_kc[c]);
    else if (S <= 128) class_in_registers<2>(ci, bk, kp, S, thr, &s_kc[c]);
    else if (S <= 256) class_in_registers<4>(ci, bk, kp, S, thr, &s_kc[c]);
    else class_in_registers<8>(ci, bk, kp, S, thr, &s_kc[c]);
  }
  __syncthreads();

  // Large classes: workgroup sort (LDS keys when they fit), sorted rows back
  // into the bucket, sorted boxes/areas for nms_mask, one task range queued.
  const int nbig = s_nbig;
  long long mask_off = 0;
  for (int q = 0; q < nbig; ++q) {
    const int c = s_big[q];
    const int S = s_cnt[c], off = s_off[c];
    const int Pn = next_pow2(S);
    unsigned long long* keys = Pn <= kLdsKeys ? s_keys : P.keysg;
    for (int i = tid; i < Pn; i += kThreads) keys[i] = i < S ? make_key(ci[P.bucket[off + i]]) : ~0ull;
    __syncthreads();
    block_bitonic(keys, Pn);
    for (int i = tid; i < S; i += kThreads) {
      const int r = (int)(unsigned)keys[i];
      const ycx_cand b = ci[r];
      P.bucket[off + i] = r;
      P.box[off + i] = f32x4{b.x1, b.y1, b.x2, b.y2};
      P.area[off + i] = (b.x2 - b.x1) * (b.y2 - b.y1);
    }
    const int nbw = (S + 63) / 64;
    if (tid == 0) {
      const int sid = atomicAdd(&hdr->nseg, 1);
      const int t0 = atomicAdd(&hdr->ntasks, nbw);
      segs[sid] = Seg{img, off, S, nbw, mask_off, t0, 0};
    }
    mask_off += (long long)S * nbw;
    __syncthreads();
  }
  // Per-image class tables for nms_finish.
  for (int c = tid; c < nc; c += kThreads) {
    P.cnt[c] = s_cnt[c];
    P.offs[c] = s_off[c];
    P.kc[c] = s_kc[c];
  }
  for (int q = tid; q < nbig; q += kThreads) P.big[1 + q] = s_big[q];
  if (tid == 0) P.big[0] = nbig;
}

// ---------------------------------------------------------------------------
// One wave per (large class, 64-row strip): rows i = 64*bi + lane against every
// column block bj >= bi; column boxes are broadcast from registers by readlane.
__global__ void __launch_bounds__(kMaskThreads) nms_mask(ycx_nms_desc d, char* ws, Thr thr) {
  const Layout L = layout(d.n, d.rows_total);
  const Hdr* hdr = reinterpret_cast<const Hdr*>(ws + L.hdr);
  const Seg* segs = reinterpret_cast<const Seg*>(ws + L.segs);
  // Per-wave LDS slice holding one 64-box column block (boxes + areas); every
  // lane reads column c by a broadcast ds_read (same address in all lanes).
  __shared__ f32x4 s_box[kMaskThreads / 64][64];
  __shared__ float s_area[kMaskThreads / 64][64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int nseg = hdr->nseg, ntasks = hdr->ntasks;
  const int gw = (blockIdx.x * kMaskThreads + threadIdx.x) >> 6;
  const int nw = gridDim.x * (kMaskThreads >> 6);
  f32x4* cb = s_box[wv];
  float* ca = s_area[wv];
  for (int t = gw; t < ntasks; t += nw) {
    int s = 0;
    while (s + 1 < nseg && !(segs[s].task_start <= t && t < segs[s].task_start + segs[s].nbw)) ++s;
    const Seg sg = segs[s];
    const Ptrs P = image_ptrs(ws, L, sg.img);
    const int bi = t - sg.task_start;
    const int i = bi * 64 + lane;
    const bool rv = i < sg.S;
    const f32x4 a = rv ? P.box[sg.off + i] : f32x4{0.f, 0.f, 0.f, 0.f};
    const float aa = rv ? P.area[sg.off + i] : 0.0f;
    unsigned long long* mrow = P.mask + sg.mask_off + (long long)i * sg.nbw;
    // column block bi first (its own rows), then prefetch one block ahead
    f32x4 nb = a;
    float na = aa;
    for (int bj = bi; bj < sg.nbw; ++bj) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // previous block's LDS reads done
      cb[lane] = nb;
      ca[lane] = na;
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      const int jn = (bj + 1) * 64 + lane;
      const bool nv = bj + 1 < sg.nbw && jn < sg.S;
      nb = nv ? P.box[sg.off + jn] : f32x4{0.f, 0.f, 0.f, 0.f};
      na = nv ? P.area[sg.off + jn] : 0.0f;
      const int cmax = min(64, sg.S - bj * 64);  // uniform
      unsigned lo = 0u, hi = 0u;
#pragma unroll
      for (int c = 0; c < 64; ++c) {
        const f32x4 b = cb[c];
        const float ba = ca[c];
        const bool sup = c < cmax && (bj > bi || c > lane) &&
                         suppress(a[0], a[1], a[2], a[3], aa, b[0], b[1], b[2], b[3], ba, thr);
        if (c < 32) lo |= sup ? (1u << c) : 0u;
        else hi |= sup ? (1u << (c - 32)) : 0u;
      }
      if (rv) mrow[bj] = ((unsigned long long)hi << 32) | lo;
    }
  }
}

// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(kThreads) nms_finish(ycx_nms_desc d, const ycx_cand* __restrict__ cand, char* ws,
                                                       float* __restrict__ dets, int* __restrict__ keep_rows,
                                                       int* __restrict__ keep_counts) {
  __shared__ unsigned long long s_rem[kMaxRows / 64 + 64 * 4];
  __shared__ int s_kc[kMaxNc], s_koff[kMaxNc], s_off[kMaxNc], s_big[kMaxNc];
  __shared__ long long s_moff[kMaxNc];
  __shared__ int s_woff[kMaxNc];
  __shared__ int s_next, s_total, s_nbig;
  const int img = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int nc = d.nc, rows = d.rows_total;
  const Layout L = layout(d.n, rows);
  const Ptrs P = image_ptrs(ws, L, img);
  const ycx_cand* ci = cand + (size_t)img * rows;
  for (int c = tid; c < nc; c += kThreads) { s_kc[c] = P.kc[c]; s_off[c] = P.offs[c]; }
  if (tid == 0) {
    const int nbig = P.big[0];
    s_nbig = nbig;
    s_next = 0;
    long long mo = 0;
    int wo = 0;
    for (int q = 0; q < nbig; ++q) {  // same order as nms_prep: mask offsets, LDS word offsets
      const int c = P.big[1 + q];
      const int S = P.cnt[c];
      s_big[q] = c;
      s_moff[q] = mo;
      s_woff[q] = wo;
      mo += (long long)S * ((S + 63) / 64);
      wo += (S + 63) / 64;
    }
  }
  __syncthreads();
  const int nbig = s_nbig;
  for (int it = 0; it <= nbig + 16; ++it) {  // bounded work-queue loop: one wave per large class
    int q = 0;
    if (lane == 0) q = atomicAdd(&s_next, 1);
    q = __builtin_amdgcn_readfirstlane(__shfl(q, 0));
    if (q >= nbig) break;
    const int c = s_big[q];
    const int S = __builtin_amdgcn_readfirstlane(P.cnt[c]);
    const int off = s_off[c], nbw = (S + 63) / 64;
    unsigned long long* rem = s_rem + s_woff[q];
    const unsigned long long* mask = P.mask + s_moff[q];
    for (int w = lane; w < nbw; w += 64) rem[w] = 0ull;
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    int nk = 0;
    const unsigned long long lt = (1ull << lane) - 1ull;
    for (int b = 0; b < nbw; ++b) {
      // (a) resolve the 64 rows of block b serially: only the diagonal words
      //     mask[64b + r][b] matter inside the block; lane r holds row r's word.
      const int i = b * 64 + lane;
      const unsigned long long diag = i < S ? mask[(long long)i * nbw + b] : 0ull;
      unsigned long long wb = rem[b];
      unsigned long long kb = 0ull;
      const int rmax = min(64, S - b * 64);
      for (int r = 0; r < rmax; ++r) {
        if ((wb >> r) & 1ull) continue;
        kb |= 1ull << r;
        const unsigned lo = __builtin_amdgcn_readlane((unsigned)diag, r);
        const unsigned hi = __builtin_amdgcn_readlane((unsigned)(diag >> 32), r);
        wb |= ((unsigned long long)hi << 32) | lo;
      }
      if ((kb >> lane) & 1ull) P.kept[off + nk + __popcll(kb & lt)] = P.bucket[off + i];
      nk += __popcll(kb);
      // (b) propagate the kept rows of block b to every later word, 8 independent
      //     row loads in flight per lane.
      for (int w = b + 1 + lane; w < nbw; w += 64) {
        unsigned long long acc = 0ull, m = kb;
        for (int g = 0; g < 64 && m; g += 8) {
          int rr[8];
#pragma unroll
          for (int u = 0; u < 8; ++u) {
            rr[u] = m ? __builtin_ctzll(m) : -1;
            m = m ? (m & (m - 1ull)) : 0ull;
          }
          unsigned long long v[8];
#pragma unroll
          for (int u = 0; u < 8; ++u) v[u] = rr[u] >= 0 ? mask[(long long)(b * 64 + rr[u]) * nbw + w] : 0ull;
#pragma unroll
          for (int u = 0; u < 8; ++u) acc |= v[u];
        }
        rem[w] |= acc;
      }
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    }
    if (lane == 0) s_kc[c] = nk;
  }
  __syncthreads();
  if (wid == 0) {
    const int total = wave_exclusive_scan(s_kc, s_koff, nc);
    if (lane == 0) s_total = total;
  }
  __syncthreads();
  const int total = s_total;
  if (tid == 0) keep_counts[img] = total;
  const int nout = min(total, d.max_det);
  for (int pos = tid; pos < d.max_det; pos += kThreads) {
    float* o = dets + ((size_t)img * d.max_det + pos) * 7;
    if (pos < nout) {
      int lo = 0, hi = nc - 1;  // the last class whose output range starts at or before pos
      while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (s_koff[mid] <= pos) lo = mid; else hi = mid - 1;
      }
      while (lo > 0 && (s_kc[lo] == 0 || s_koff[lo] + s_kc[lo] <= pos)) --lo;
      const int row = P.kept[s_off[lo] + (pos - s_koff[lo])];
      const ycx_cand c = ci[row];
      o[0] = c.x1; o[1] = c.y1; o[2] = c.x2; o[3] = c.y2;
      o[4] = c.obj; o[5] = c.cls_conf; o[6] = (float)c.cls;
      keep_rows[(size_t)img * d.max_det + pos] = row;
    } else {
      for (int t = 0; t < 7; ++t) o[t] = 0.0f;
      keep_rows[(size_t)img * d.max_det + pos] = -1;
    }
  }
}

Thr make_thr(double thr) {
  Thr t{thr, 0.0, 0, 0};
  if (!(thr >= 0.0) || !(thr < 3.0e38)) return t;  // negative / NaN / huge: literal division
  float T = (float)thr;
  if (!((double)T > thr)) T = nextafterf(T, INFINITY);
  for (float Tm = nextafterf(T, -INFINITY); (double)Tm > thr; Tm = nextafterf(T, -INFINITY)) T = Tm;
  const float Tm = nextafterf(T, -INFINITY);
  uint32_t bits;
  memcpy(&bits, &T, 4);
  t.m = ((double)Tm + (double)T) * 0.5;
  t.incl = (bits & 1u) == 0;  // round-half-even sends the midpoint to T iff T is even
  t.fast = 1;
  return t;
}

}  // namespace

extern "C" size_t ycx_nms_workspace_size(const ycx_nms_desc* d) {
  if (!d || d->n <= 0 || d->rows_total <= 0) return 0;
  const Layout L = layout(d->n, d->rows_total);
  return L.per_image_base + L.per_image * (size_t)d->n;
}

extern "C" ycx_status ycx_sort_nms(const ycx_nms_desc* d, const ycx_cand* cand, const int32_t* cand_rows,
                                   const int32_t* cand_counts, void* workspace, size_t workspace_bytes, float* dets,
                                   int32_t* keep_rows, int32_t* keep_counts, void* stream) {
  YCX_CHECK_ARG(d && cand && cand_rows && cand_counts && workspace && dets && keep_rows && keep_counts);
  YCX_CHECK_ARG(d->n > 0 && d->rows_total > 0 && d->nc > 0 && d->max_det > 0);
  if (workspace_bytes < ycx_nms_workspace_size(d)) return YCX_ERR_CAPACITY;
  YCX_CHECK_SUPPORTED(d->nc <= kMaxNc && d->rows_total <= kMaxRows);
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (hipMemsetAsync(workspace, 0, 256, st) != hipSuccess) return YCX_ERR_LAUNCH;  // task-queue header
  char* ws = reinterpret_cast<char*>(workspace);
  const Thr t = make_thr(d->iou_thres);
  hipLaunchKernelGGL(nms_prep, dim3(d->n), dim3(kThreads), 0, st, *d, cand, cand_rows, cand_counts, ws, t);
  hipLaunchKernelGGL(nms_mask, dim3(kMaskBlocks), dim3(kMaskThreads), 0, st, *d, ws, t);
  hipLaunchKernelGGL(nms_finish, dim3(d->n), dim3(kThreads), 0, st, *d, cand, ws, dets, keep_rows, keep_counts);
  return ycx_launch_status();
}
