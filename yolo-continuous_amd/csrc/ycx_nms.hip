// Per-image, per-class greedy NMS with torchvision.ops.nms semantics -- the
// loop of detect.py:124-137 (unique classes ascending, nms per class, results
// concatenated class by class) for the whole batch in seven launches.
//
//  nms_mark / nms_bucket / nms_prep   16 workgroups per image: a flag byte per
//              candidate row and class histograms of row slices, exclusive scan ->
//              one bucket per class listing its rows in ascending order; every
//              wave pulls whole classes from an LDS counter and a class of S <= 512
//              candidates is finished entirely in registers (64*R keys
//              bitonic-sorted across lanes and register slots, greedy scan with
//              removed/kept bit masks, box i broadcast by readlane). Larger
//              classes are listed: the fast list (the class fits the LDS) and the
//              wide list (the others).
//  A big class, one 1024-thread workgroup per phase (grid-strided task loops):
//              (1) score sort (score desc, row asc = torchvision's stable descending
//              order) -> rank. (2) spatial counting sort: level = size octave of
//              max(w, h) relative to the class extent, cell = centre cell in that
//              level's grid. (3) per box, the higher-ranked boxes with IoU > thr
//              ("suppressors") are searched only where they can exist: IoU > t
//              forces w_j/w_i and h_j/h_i into (t, 1/t) (so only a few levels
//              qualify) and the centres within a window the sizes bound. (4) greedy
//              resolution as a parallel fixed point: a box is kept once all its
//              suppressors are removed, removed once any is kept; every round
//              decides at least the highest-ranked undecided box, and each decision
//              equals the greedy one by induction on rank. (5) kept rows compacted
//              in rank order.
//  nms_fast    (1)-(2) of every class; a fast class also (3)-(5) in LDS, unless the
//              batch has few big classes (kSplitTasks), when it is split like the
//              wide ones.
//  nms_search  (3) of the wide and split classes, their positions spread evenly
//              over the grid.
//  nms_resolve (4)-(5) of the wide and split classes.
//  nms_finish  one workgroup per image: exclusive scan of the per-class kept
//              counts places every kept row in class order; padded outputs.
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
// the big-class kernels' workgroup, LDS budget and grid (build-time knobs, DESIGN.md §6 tried-and-rejected)
#ifndef YCX_NMS_BIG_THREADS
#define YCX_NMS_BIG_THREADS 1024
#endif
#ifndef YCX_NMS_BIG_LDS
#define YCX_NMS_BIG_LDS 159744
#endif
constexpr int kBigThreads = YCX_NMS_BIG_THREADS;
constexpr int kBigLds = YCX_NMS_BIG_LDS;
constexpr int kMaxNc = 1024;      // classes handled in LDS
constexpr int kRegMax = 512;      // largest class finished in registers (R = 8 slots per lane)
constexpr int kMaxRows = 131072;  // rows (candidates) per image
#ifndef YCX_NMS_BIG_BLOCKS
#define YCX_NMS_BIG_BLOCKS 256
#endif
constexpr int kBigBlocks = YCX_NMS_BIG_BLOCKS;   // nms_fast / nms_wide grid (task-strided)
#ifndef YCX_NMS_SEARCH_BLOCKS
#define YCX_NMS_SEARCH_BLOCKS YCX_NMS_BIG_BLOCKS
#endif
constexpr int kSearchBlocks = YCX_NMS_SEARCH_BLOCKS;  // nms_search grid (equal position ranges)
constexpr int kSlots = 16;        // int suppressor ranks cached per box (64 bytes; 32 when u16)

#ifdef YCX_NMS_PROFILE
// Development counters: shader cycles per big-class phase, summed over tasks.
__device__ unsigned long long g_nms_prof[16];
__device__ unsigned long long g_nms_wprof[16];  // wide: phases 0-4, [5] rounds, [6] round visits, [7] tasks,
                                               // [8] sort key build, [9] sort passes, [10] pass count
#define YCX_PROF_MARK(i)                                               \
  if (tid == 0) {                                                      \
    const unsigned long long now_ = __builtin_amdgcn_s_memtime();      \
    atomicAdd(&g_nms_prof[i], now_ - t_prev_);                         \
    t_prev_ = now_;                                                    \
  }
#define YCX_WPROF_MARK(i)                                              \
  if (tid == 0) {                                                      \
    const unsigned long long now_ = __builtin_amdgcn_s_memtime();      \
    atomicAdd(&g_nms_wprof[i], now_ - t_prev_);                        \
    t_prev_ = now_;                                                    \
  }
#else
#define YCX_PROF_MARK(i)
#define YCX_WPROF_MARK(i)
#endif

struct Task {  // one large class
  int img, cls, off, S;
};

constexpr int kPrepB = 16;  // workgroups per image in the class bucketing (nms_mark / nms_bucket)
#ifndef YCX_PREP_CLS_B
#define YCX_PREP_CLS_B 4
#endif
// workgroups per image over the classes (nms_prep): 4 measured best of 1 / 4 / 16 (dense
// G3 load 24.0k -> 58.9k img/s decode + NMS; C2 neutral; C4 +1.3 %; 16: C2 post 0.51 -> 0.57 ms)
constexpr int kPrepClsB = YCX_PREP_CLS_B;

// Big classes per batch (fast + wide lists) up to which the fast classes are split too: their
// sort + spatial index stay in nms_fast, their suppressor search joins the wide classes' in
// nms_search (positions spread evenly over the grid) and their fixed point runs in nms_resolve.
// Past it (C2: ~160 fast classes per batch) every fast class already has a CU of its own for
// its whole life and runs unsplit (a split at that load cost 7 %).
#ifndef YCX_NMS_SPLIT_TASKS
#define YCX_NMS_SPLIT_TASKS 64
#endif
constexpr int kSplitTasks = YCX_NMS_SPLIT_TASKS;

struct Layout {
  size_t hdr, tasks, wframes, wcells, fframes, fcells, bcnt, bits, per_image_base;  // header + task tables +
                                  // wide / split-fast class indexes + slice class counts (batch), then per image:
  size_t keys, bucket, kept, sbox, srank, nsup, slots, state, cnt, offs, kc, per_image;
  int max_tasks, max_wide;  // big classes per image; wide classes per image
};

__host__ __device__ inline int wide_min_s();  // the smallest class the wide path can get
__host__ __device__ inline size_t wide_cells_bytes();
__host__ __device__ inline size_t fast_cells_bytes();
struct WFrame;  // per wide class: extent normalisation, level stats (nms_wide_a -> _s, _b)
__host__ __device__ inline size_t wframe_bytes();

__host__ __device__ inline int next_pow2(int v) {
  int p = 1;
  while (p < v) p <<= 1;
  return p;
}

__host__ __device__ inline size_t al(size_t v) { return (v + 255) & ~(size_t)255; }

__host__ __device__ inline Layout layout(int n, int rows, int nc) {
  Layout L;
  L.max_tasks = rows / (kRegMax + 1) + 1;
  L.hdr = 0;
  L.tasks = 256;
  L.max_wide = rows / wide_min_s() + 1;
  L.wframes = al(L.tasks + 2 * (size_t)n * L.max_tasks * sizeof(Task));  // fast list, then wide list
  L.wcells = al(L.wframes + (size_t)n * L.max_wide * wframe_bytes());
  L.fframes = al(L.wcells + (size_t)n * L.max_wide * wide_cells_bytes());
  L.fcells = al(L.fframes + (size_t)kSplitTasks * wframe_bytes());
  L.bcnt = al(L.fcells + (size_t)kSplitTasks * fast_cells_bytes());
  L.bits = al(L.bcnt + (size_t)n * kPrepB * nc * 4);  // row-slice class counts [n][kPrepB][nc]; then per
                                                      // image a candidate flag byte per row
  L.per_image_base = al(L.bits + (size_t)n * rows);
  size_t o = 0;
  // keys: a class at bucket offset `off` with S rows sorts at keys + 2*off; its
  // power-of-two span is < 2S and off + S <= rows, so 2*rows keys suffice.
  L.keys = o; o = al(o + (size_t)2 * rows * 8);
  L.bucket = o; o = al(o + (size_t)rows * 4);
  L.kept = o; o = al(o + (size_t)rows * 4);
  L.sbox = o; o = al(o + (size_t)rows * 16);
  L.srank = o; o = al(o + (size_t)rows * 4);
  L.nsup = o; o = al(o + (size_t)rows * 4);
  L.slots = o; o = al(o + (size_t)rows * kSlots * 4);
  L.state = o; o = al(o + (size_t)rows);
  L.cnt = o; o = al(o + kMaxNc * 4);
  L.offs = o; o = al(o + kMaxNc * 4);
  L.kc = o; o = al(o + kMaxNc * 4);
  L.per_image = o;
  return L;
}

// Whether a class of S > kRegMax candidates takes the LDS-resident fast path (nms_fast):
// S <= 8192 (13-bit element ids, E <= 8 registers) and cells + 19 B per box fit the LDS.
__host__ __device__ inline bool fast_task(int S);

struct Hdr {
  int ntasks;  // the fast list: classes the LDS-resident path takes (nms_fast)
  int nwide;   // the wide list (nms_wide_a's work in nms_fast, then nms_search / nms_resolve)
};

// Whether the fast classes of this batch are split (kSplitTasks); every kernel decides alike.
__device__ __forceinline__ bool split_fast(const Hdr* h) { return h->ntasks + h->nwide <= kSplitTasks; }

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
  // greedy scan in rank order i = ri * 64 + li; the slot ri is a compile-time constant of the
  // unrolled outer loop, so box i's registers are read by index, never through a dynamically
  // indexed array (a select chain over the slots was folded into one, which lives in scratch)
#pragma unroll
  for (int ri = 0; ri < R; ++ri) {
    if (ri * 64 >= S) break;  // uniform
    const int lim = min(64, S - ri * 64);
    for (int li = 0; li < lim; ++li) {
      const int i = ri * 64 + li;
      if ((__builtin_amdgcn_readlane(rm, li) >> ri) & 1u) continue;
      if (lane == li) km |= 1u << ri;
      const float bx1 = bcast(x1[ri], li), by1 = bcast(y1[ri], li);
      const float bx2 = bcast(x2[ri], li), by2 = bcast(y2[ri], li);
      const float ba = bcast(ar[ri], li);
#pragma unroll
      for (int r = ri; r < R; ++r) {  // every position of an earlier slot precedes i
        const int e = r * 64 + lane;
        if (e > i && e < S && !((rm >> r) & 1u) &&
            suppress(bx1, by1, bx2, by2, ba, x1[r], y1[r], x2[r], y2[r], ar[r], thr))
          rm |= 1u << r;
      }
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

struct Ptrs {
  unsigned long long* keys;
  int *bucket, *kept;
  f32x4* sbox;
  int *srank, *nsup, *slots;
  unsigned char* state;
  int *cnt, *offs, *kc;
};

__device__ __forceinline__ Ptrs image_ptrs(char* ws, const Layout& L, int img) {
  char* b = ws + L.per_image_base + (size_t)img * L.per_image;
  Ptrs p;
  p.keys = reinterpret_cast<unsigned long long*>(b + L.keys);
  p.bucket = reinterpret_cast<int*>(b + L.bucket);
  p.kept = reinterpret_cast<int*>(b + L.kept);
  p.sbox = reinterpret_cast<f32x4*>(b + L.sbox);
  p.srank = reinterpret_cast<int*>(b + L.srank);
  p.nsup = reinterpret_cast<int*>(b + L.nsup);
  p.slots = reinterpret_cast<int*>(b + L.slots);
  p.state = reinterpret_cast<unsigned char*>(b + L.state);
  p.cnt = reinterpret_cast<int*>(b + L.cnt);
  p.offs = reinterpret_cast<int*>(b + L.offs);
  p.kc = reinterpret_cast<int*>(b + L.kc);
  return p;
}

// ---------------------------------------------------------------------------
// Class bucketing of each image's candidates, on kPrepB workgroups per image (one per
// image took 0.19 ms per batch at C2 and 0.36 ms at C4, 8 workgroups on the whole chip):
// nms_mark flags the candidate rows and histograms the row slices per class (workgroup b
// takes slice b of the candidate list); nms_bucket places row slice b's rows at class offset
// + the earlier slices' counts in row order (below); nms_prep then finishes the small classes
// and lists the big ones, classes c = b mod kPrepB on workgroup b.
__device__ __forceinline__ void prep_slice(int cnt, int b, int& i0, int& i1) {
  i0 = (int)((long long)cnt * b / kPrepB);
  i1 = (int)((long long)cnt * (b + 1) / kPrepB);
}

// nms_mark sets the flag byte of every listed candidate's row (the list is in append order; plain
// byte stores: 32 candidates per u32 word made atomicOr on a bitmap 42 us at C2) and adds the
// class histogram of each row slice b = rows [r0, r1) (LDS counts of its list slice, then one
// global atomic per nonzero (slice, class)); nms_bucket then walks its row slice in ascending
// order, so every class bucket lists its rows in ascending order (a stable counting sort by
// class). The score sorts downstream are stable LSD passes over the score digits only: equal
// scores keep that row order, which is the reference's (score desc, row asc).
__device__ __forceinline__ void row_slice(int rows, int b, int& r0, int& r1) {
  r0 = (int)((long long)rows * b / kPrepB);
  r1 = (int)((long long)rows * (b + 1) / kPrepB);
}
__device__ __forceinline__ int slice_of_row(int rows, int r) { return (int)((kPrepB * ((long long)r + 1) - 1) / rows); }

__global__ void __launch_bounds__(kThreads) nms_mark(ycx_nms_desc d, const ycx_cand* __restrict__ cand,
                                                     const int* __restrict__ cand_rows,
                                                     const int* __restrict__ cand_counts, char* ws) {
  extern __shared__ unsigned s_cnt[];  // [row slice][class]: kPrepB * nc counters (dynamic LDS)
  const int b = blockIdx.x, img = blockIdx.y, tid = threadIdx.x;
  const int nc = d.nc, rows = d.rows_total;
  const Layout L = layout(d.n, rows, d.nc);
  unsigned char* flag = reinterpret_cast<unsigned char*>(ws + L.bits) + (size_t)img * rows;
  const ycx_cand* ci = cand + (size_t)img * rows;
  const int* cr = cand_rows + (size_t)img * rows;
  for (int k = tid; k < kPrepB * nc; k += kThreads) s_cnt[k] = 0;
  if (b == 0 && img == 0 && tid < 64) reinterpret_cast<int*>(ws + L.hdr)[tid] = 0;  // the task-queue header (256 B)
  __syncthreads();
  int i0, i1;
  prep_slice(min(cand_counts[img], rows), b, i0, i1);
  for (int i = i0 + tid; i < i1; i += kThreads) {
    const int r = cr[i];
    flag[r] = 1;
    atomicAdd(&s_cnt[slice_of_row(rows, r) * nc + ci[r].cls], 1u);
  }
  __syncthreads();
  int* bc = reinterpret_cast<int*>(ws + L.bcnt) + (size_t)img * kPrepB * nc;  // zeroed by ycx_sort_nms
  for (int k = tid; k < kPrepB * nc; k += kThreads) {
    const unsigned v = s_cnt[k];
    if (v) atomicAdd(&bc[k], (int)v);
  }
}

__global__ void __launch_bounds__(kThreads) nms_bucket(ycx_nms_desc d, const ycx_cand* __restrict__ cand,
                                                       const int* __restrict__ cand_rows,
                                                       const int* __restrict__ cand_counts, char* ws) {
  constexpr int NW = kThreads / 64;
  __shared__ int s_cnt[kMaxNc], s_off[kMaxNc], s_base[kMaxNc];
  __shared__ unsigned short s_wc[NW][kMaxNc];  // per (wave, class) rows of the current chunk
  const int b = blockIdx.x, img = blockIdx.y, tid = threadIdx.x, wid = tid >> 6, lane = tid & 63;
  const int nc = d.nc, rows = d.rows_total;
  const Layout L = layout(d.n, rows, d.nc);
  const Ptrs P = image_ptrs(ws, L, img);
  const ycx_cand* ci = cand + (size_t)img * rows;
  const unsigned char* flag = reinterpret_cast<const unsigned char*>(ws + L.bits) + (size_t)img * rows;
  const int* bc = reinterpret_cast<const int*>(ws + L.bcnt) + (size_t)img * kPrepB * nc;
  for (int c = tid; c < nc; c += kThreads) {
    int tot = 0, before = 0;
    for (int q = 0; q < kPrepB; ++q) {
      const int v = bc[(size_t)q * nc + c];
      before += q < b ? v : 0;
      tot += v;
    }
    s_cnt[c] = tot;
    s_base[c] = before;
  }
  for (int k = tid; k < NW * kMaxNc; k += kThreads) (&s_wc[0][0])[k] = 0;
  __syncthreads();
  if (wid == 0) wave_exclusive_scan(s_cnt, s_off, nc);
  __syncthreads();
  if (b == 0)
    for (int c = tid; c < nc; c += kThreads) {
      P.cnt[c] = s_cnt[c];
      P.offs[c] = s_off[c];
    }
  // rows of the slice in chunks of kThreads, thread t <-> row r0 + t: a class's rows go to its
  // bucket in row order (rank among the chunk's earlier rows of the class: earlier waves' counts
  // plus the lanes below in this wave; s_base carries the earlier chunks)
  int nbits = 0;
  while ((1 << nbits) <= nc) ++nbits;  // class + 1 in [0, nc]: 0 = no candidate
  const unsigned long long lt = (1ull << lane) - 1ull;
  int rb, r_end;
  row_slice(rows, b, rb, r_end);
  for (int r0 = rb; r0 < r_end; r0 += kThreads) {  // uniform trip count
    const int r = r0 + tid;
    const bool valid = r < r_end && flag[r];
    const int c1 = valid ? ci[r].cls + 1 : 0;
    unsigned long long m = ~0ull;
    for (int bit = 0; bit < nbits; ++bit) {
      const unsigned long long bl = __ballot((c1 >> bit) & 1);
      m &= ((c1 >> bit) & 1) ? bl : ~bl;
    }
    if (valid && (m & lt) == 0) s_wc[wid][c1 - 1] = (unsigned short)__popcll(m);
    __syncthreads();
    if (valid) {
      const int c = c1 - 1;
      int q = s_off[c] + s_base[c] + __popcll(m & lt);
      for (int w = 0; w < wid; ++w) q += s_wc[w][c];
      P.bucket[q] = r;
    }
    __syncthreads();
    for (int c = tid; c < nc; c += kThreads) {
      int add = 0;
      for (int w = 0; w < NW; ++w) {
        add += s_wc[w][c];
        s_wc[w][c] = 0;
      }
      s_base[c] += add;
    }
    __syncthreads();
  }

}

__global__ void __launch_bounds__(kThreads) nms_prep(ycx_nms_desc d, const ycx_cand* __restrict__ cand, char* ws,
                                                     Thr thr) {
  __shared__ int s_kc[kMaxNc];
  __shared__ int s_next;
  const int b = blockIdx.x, img = blockIdx.y, tid = threadIdx.x, lane = tid & 63;
  const int nc = d.nc, rows = d.rows_total;
  const Layout L = layout(d.n, rows, d.nc);
  const Ptrs P = image_ptrs(ws, L, img);
  Hdr* hdr = reinterpret_cast<Hdr*>(ws + L.hdr);
  Task* tasks = reinterpret_cast<Task*>(ws + L.tasks);
  const ycx_cand* ci = cand + (size_t)img * rows;
  const int nown = (nc - b + kPrepClsB - 1) / kPrepClsB;  // classes b, b + kPrepClsB, ...

  for (int k = tid; k < nown; k += kThreads) s_kc[k] = 0;
  if (tid == 0) s_next = 0;
  __syncthreads();
  // Classes of <= kRegMax candidates: one wave each, in registers; larger
  // classes become nms_fast / nms_wide tasks.
  for (int it = 0; it <= nown + 64; ++it) {  // bounded work-queue loop
    int k = 0;
    if (lane == 0) k = atomicAdd(&s_next, 1);
    k = __builtin_amdgcn_readfirstlane(__shfl(k, 0));
    if (k >= nown) break;
    const int c = b + k * kPrepClsB;
    const int S = __builtin_amdgcn_readfirstlane(P.cnt[c]), off = __builtin_amdgcn_readfirstlane(P.offs[c]);
    if (S == 0) continue;
    if (S > kRegMax) {
      if (lane == 0) {
        if (fast_task(S)) tasks[atomicAdd(&hdr->ntasks, 1)] = Task{img, c, off, S};
        else tasks[(size_t)d.n * L.max_tasks + atomicAdd(&hdr->nwide, 1)] = Task{img, c, off, S};
      }
      continue;
    }
    const int* bk = P.bucket + off;
    int* kp = P.kept + off;
    if (S <= 64) class_in_registers<1>(ci, bk, kp, S, thr, &s_kc[k]);
    else if (S <= 128) class_in_registers<2>(ci, bk, kp, S, thr, &s_kc[k]);
    else if (S <= 256) class_in_registers<4>(ci, bk, kp, S, thr, &s_kc[k]);
    else class_in_registers<8>(ci, bk, kp, S, thr, &s_kc[k]);
  }
  __syncthreads();
  // this workgroup's classes' kept counts (nms_fast / nms_wide overwrite kc of theirs)
  for (int k = tid; k < nown; k += kThreads) P.kc[b + k * kPrepClsB] = s_kc[k];
}

// ---------------------------------------------------------------------------
// big-class helpers

// Order-preserving int image of a float (LDS atomicMin/Max on floats).
__device__ __forceinline__ int f2o(float f) {
  const int i = __float_as_int(f);
  return i >= 0 ? i : i ^ 0x7FFFFFFF;
}
__device__ __forceinline__ float o2f(int i) { return __int_as_float(i >= 0 ? i : i ^ 0x7FFFFFFF); }

__device__ __forceinline__ int clamp_cell(float v, int G) {
  return (int)fminf(fmaxf(floorf(v), 0.0f), (float)(G - 1));
}

// (x2 - x1) * (y2 - y1): the reference's area expression, bit-identical to the
// one the candidates were filtered with (contraction is off in this file).
__device__ __forceinline__ float box_area(const f32x4 b) { return (b[2] - b[0]) * (b[3] - b[1]); }

// Block-wide exclusive scan helper: returns this thread's exclusive prefix of
// `v` over the workgroup and writes the block total to *total.
__device__ __forceinline__ int block_exclusive(int v, int* s_w, int* total) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  int incl = v;
#pragma unroll
  for (int dd = 1; dd < 64; dd <<= 1) {
    const int t = __shfl_up(incl, dd);
    if (lane >= dd) incl += t;
  }
  if (lane == 63) s_w[wid] = incl;
  __syncthreads();
  int pre = 0, tot = 0;
  for (int w = 0; w < (int)(blockDim.x >> 6); ++w) {
    const int x = s_w[w];
    pre += w < wid ? x : 0;
    tot += x;
  }
  __syncthreads();
  *total = tot;
  return pre + incl - v;
}

// ---------------------------------------------------------------------------
// The fast path: a class of S <= kFastMax boxes held entirely in LDS.
// Same greedy semantics and the same suppressor / fixed-point logic as the
// general path (resolve), with three changes that cut the per-class cost:
//  * every candidate is gathered from global memory ONCE (into registers), and
//    the rank sort, extent, histogram and scatter work from those registers
//    (the general path re-gathers ci[bucket[r]] in each of four passes);
//  * a finer grid per size level (4 << L cells a side, capped at 64: cells of
//    1/4 - 1/2 of the level's box size instead of 1 - 2) and a tighter window:
//    IoU > t forces the overlap width above t * max(w_i, w_j) (inter <= ox *
//    min(h_i, h_j), union >= max(a_i, a_j)), so |cx_i - cx_j| < (w_i + w_j) / 2 -
//    t * max(w_i, w_j), maximised over the partner level's width range [nw, mw]
//    (the bound is piecewise linear in w_j with its kink at w_i); likewise in y.
//    On the bench load this visits 3-4x fewer candidates (tools/nms_study.py);
//  * after the search the suppressor lists move into LDS (CSR over the dead
//    box region) so the fixed-point rounds never touch global memory.
// Keys carry (row << 13 | e): e < 8192 is the element's load slot, so after the
// sort every rank finds its box in the loading thread's registers.
// ---------------------------------------------------------------------------
constexpr int kFastMax = 8192;
constexpr int kFLevels = 7;
__host__ __device__ constexpr int fgrid(int L) { return (4 << L) < 64 ? (4 << L) : 64; }
__host__ __device__ constexpr int fbase(int L) { return L == 0 ? 0 : fbase(L - 1) + fgrid(L - 1) * fgrid(L - 1); }
constexpr int kFWild = fbase(kFLevels);  // boxes without a finite positive extent
constexpr int kFCells = kFWild + 1;
constexpr int kFCellBytes = ((kFCells + 1) / 2 * 4 + 255) & ~255;  // u16 end positions, packed in u32 words

// Stable LSD radix sort of the S real keys held blocked in registers (element e = tid * E + i;
// e >= S holds no key) by bits [lo, 64), 4-bit digits, digits that no two keys differ in
// skipped. One pass: each thread's per-digit counts (nibbles of one u64, E <= 8 < 16) go to
// a digit-major table T[16][kBigThreads] (u16), an exclusive scan of T in that order gives
// every (digit, thread) its first output slot, the keys are scattered to dst in LDS and read
// back blocked. Stable because a thread's elements keep their order inside a digit and
// threads are ordered inside each digit, i.e. the (tid, i) order of the input is preserved.
// The whole order is the 64-bit key order restricted to bits [lo, 64). The fast path passes
// lo = 32: it sorts the score bits [32, 64) only, and the (score desc, row asc) order on equal
// scores comes from the stability of the passes over the input order, which nms_bucket makes
// ascending by row within every class (the low bits only name the element).
template <int E>
__device__ void radix_sort_regs(unsigned long long (&key)[E], int S, int lo, unsigned long long* dst,
                                unsigned short* T, int* s_w, unsigned long long* s_msk) {
  static_assert(E <= 8, "nibble counters");
  const int tid = threadIdx.x, lane = tid & 63;
  unsigned long long a = ~0ull, o = 0ull;
#pragma unroll
  for (int i = 0; i < E; ++i)
    if (tid * E + i < S) { a &= key[i]; o |= key[i]; }
#pragma unroll
  for (int sh = 32; sh > 0; sh >>= 1) {
    a &= __shfl_xor(a, sh);
    o |= __shfl_xor(o, sh);
  }
  if (tid == 0) { s_msk[0] = ~0ull; s_msk[1] = 0ull; }
  __syncthreads();
  if (lane == 0) {
    atomicAnd(&s_msk[0], a);
    atomicOr(&s_msk[1], o);
  }
  __syncthreads();
  const unsigned long long diff = s_msk[0] ^ s_msk[1];
  for (int sh = lo; sh < 64; sh += 4) {
    if (((diff >> sh) & 0xF) == 0) continue;  // uniform: every key has the same digit here
    unsigned long long cnt = 0;
#pragma unroll
    for (int i = 0; i < E; ++i)
      if (tid * E + i < S) cnt += 1ull << (4 * ((key[i] >> sh) & 0xF));
#pragma unroll
    for (int d = 0; d < 16; ++d) T[d * kBigThreads + tid] = (unsigned short)((cnt >> (4 * d)) & 0xF);
    __syncthreads();
    {  // exclusive scan of T in (digit, thread) order: thread t owns entries 16 t .. 16 t + 15
      int v[16], sum = 0;
#pragma unroll
      for (int q = 0; q < 16; ++q) { v[q] = T[16 * tid + q]; sum += v[q]; }
      int total;
      int run = block_exclusive(sum, s_w, &total);
#pragma unroll
      for (int q = 0; q < 16; ++q) { T[16 * tid + q] = (unsigned short)run; run += v[q]; }
    }
    __syncthreads();
    unsigned long long seen = 0;  // this thread's elements placed so far, per digit (nibbles)
#pragma unroll
    for (int i = 0; i < E; ++i) {
      if (tid * E + i >= S) continue;
      const int d = (int)((key[i] >> sh) & 0xF);
      dst[T[d * kBigThreads + tid] + (int)((seen >> (4 * d)) & 0xF)] = key[i];
      seen += 1ull << (4 * d);
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < E; ++i)
      if (tid * E + i < S) key[i] = dst[tid * E + i];
    __syncthreads();  // every read of dst and T done before the next pass rewrites them
  }
}

// LDS bytes of the fast path for a class of S boxes (cells, boxes, u16 ranks, state)
__host__ __device__ inline int fast_lds_bytes(int S) { return kFCellBytes + 16 * S + ((2 * S + 15) & ~15) + S; }
__host__ __device__ inline int wide_min_s() {
#ifdef YCX_NMS_NO_FAST
  return kRegMax + 1;
#else
  return min(kFastMax + 1, (kBigLds - kFCellBytes - 32) / 19 + 1);  // fast_task() fails from here on
#endif
}
__host__ __device__ inline size_t wide_cells_bytes() { return ((size_t)kFCells * 4 + 255) & ~(size_t)255; }
__host__ __device__ inline size_t fast_cells_bytes() { return (size_t)kFCellBytes; }  // u16 cell ends
struct WFrame {
  float X0, Y0, inv;
  int img, cls, off, S, slot;
  int lv[kFLevels][5];
};
__host__ __device__ inline size_t wframe_bytes() { return (sizeof(WFrame) + 15) & ~(size_t)15; }
__host__ __device__ inline bool fast_task(int S) {
#ifdef YCX_NMS_NO_FAST
  return false;
#else
  return S <= kFastMax && fast_lds_bytes(S) <= kBigLds;
#endif
}

struct FGeo {
  float cx, cy, w, h;
  int level, cell;
};

__device__ __forceinline__ FGeo fgeometry(const f32x4 b, float X0, float Y0, float inv, bool all_pairs) {
  FGeo g;
  const float nx1 = (b[0] - X0) * inv, ny1 = (b[1] - Y0) * inv;
  const float nx2 = (b[2] - X0) * inv, ny2 = (b[3] - Y0) * inv;
  g.w = nx2 - nx1;
  g.h = ny2 - ny1;
  g.cx = (nx1 + nx2) * 0.5f;
  g.cy = (ny1 + ny2) * 0.5f;
  const float s = fmaxf(g.w, g.h);
  const bool reg = !all_pairs && g.w > 0.0f && g.h > 0.0f && s < INFINITY && b[0] > -INFINITY && b[1] > -INFINITY;
  if (!reg) {
    g.level = -1;
    g.cell = kFWild;
    return g;
  }
  const int e = (int)(__float_as_uint(s) >> 23) - 126;  // s < 2^e
  const int L = min(max(-e, 0), kFLevels - 1);
  const int G = fgrid(L);
  g.level = L;
  g.cell = fbase(L) + clamp_cell(g.cy * (float)G, G) * G + clamp_cell(g.cx * (float)G, G);
  return g;
}

// Per-level box count and extreme sizes (float bits: the sizes are non-negative), summed per
// thread in registers over all its boxes, then wave-reduced into s_lv with one set of LDS
// atomics per wave and level (instead of a ballot and four reductions per box and level).
struct LevelStats {
  int n[kFLevels], mxw[kFLevels], mxh[kFLevels], mnw[kFLevels], mnh[kFLevels];
  __device__ __forceinline__ LevelStats() {
#pragma unroll
    for (int L = 0; L < kFLevels; ++L) {
      n[L] = 0;
      mxw[L] = mxh[L] = 0;
      mnw[L] = mnh[L] = 0x7F800000;
    }
  }
  __device__ __forceinline__ void add(const FGeo& g) {
#pragma unroll
    for (int L = 0; L < kFLevels; ++L) {
      if (g.level == L) {
        ++n[L];
        mxw[L] = max(mxw[L], __float_as_int(g.w));
        mxh[L] = max(mxh[L], __float_as_int(g.h));
        mnw[L] = min(mnw[L], __float_as_int(g.w));
        mnh[L] = min(mnh[L], __float_as_int(g.h));
      }
    }
  }
  __device__ __forceinline__ void flush(int (*s_lv)[5]) {
#pragma unroll
    for (int L = 0; L < kFLevels; ++L) {
      int c = n[L], a = mxw[L], b = mxh[L], e = mnw[L], f = mnh[L];
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        c += __shfl_xor(c, o);
        a = max(a, __shfl_xor(a, o));
        b = max(b, __shfl_xor(b, o));
        e = min(e, __shfl_xor(e, o));
        f = min(f, __shfl_xor(f, o));
      }
      if ((threadIdx.x & 63) == 0 && c > 0) {
        atomicAdd(&s_lv[L][0], c);
        atomicMax(&s_lv[L][1], a);
        atomicMax(&s_lv[L][2], b);
        atomicMin(&s_lv[L][3], e);
        atomicMin(&s_lv[L][4], f);
      }
    }
  }
};

// max over w_j in [nw, mw] of (w_i + w_j) / 2 - t max(w_i, w_j): the largest centre
// distance at which a partner of that width range can still pass IoU > t
__device__ __forceinline__ float reach(float wi, float nw, float mw, float t) {
  auto f = [&](float wj) { return 0.5f * (wi + wj) - t * fmaxf(wi, wj); };
  return fmaxf(fmaxf(f(nw), f(mw)), f(fminf(fmaxf(wi, nw), mw)));
}

__device__ __forceinline__ int u16_at(const unsigned* w, int k) { return (int)((w[k >> 1] >> ((k & 1) * 16)) & 0xFFFFu); }

// Position ranges [q0, q1) of the spatial order that can hold a suppressor of the
// box of geometry g (as for_ranges, with the fine grid and the tight window);
// cend(k) = end position of cell k (u16 words in the fast path, u32 in the wide one).
template <class CE, class F>
__device__ __forceinline__ void f_ranges(CE&& cend, const int (*lv)[5], const FGeo& g, int S, float t_lo,
                                         float inv_t, F&& run) {
  if (g.level < 0) {
    run(0, S);
    return;
  }
  run(cend(kFWild - 1), cend(kFWild));
  constexpr float kSlack = 1e-6f, kEps = 1e-5f;
  for (int L = 0; L < kFLevels; ++L) {
    if (lv[L][0] == 0) continue;
    const float mw = __int_as_float(lv[L][1]), mh = __int_as_float(lv[L][2]);
    const float nw = __int_as_float(lv[L][3]), nh = __int_as_float(lv[L][4]);
    if (mw + kSlack < t_lo * g.w || mh + kSlack < t_lo * g.h) continue;  // all too narrow / too flat
    if (nw - kSlack > (g.w + kSlack) * inv_t || nh - kSlack > (g.h + kSlack) * inv_t) continue;  // too big
    const int G = fgrid(L), base = fbase(L);
    const float Gf = (float)G;
    const float rx = reach(g.w, nw, mw, t_lo) + kEps, ry = reach(g.h, nh, mh, t_lo) + kEps;
    const int ix0 = clamp_cell((g.cx - rx) * Gf, G), ix1 = clamp_cell((g.cx + rx) * Gf, G);
    const int iy0 = clamp_cell((g.cy - ry) * Gf, G), iy1 = clamp_cell((g.cy + ry) * Gf, G);
    for (int iy = iy0; iy <= iy1; ++iy) {  // cells ix0..ix1 of a grid row are contiguous positions
      const int k0 = base + iy * G + ix0, k1 = base + iy * G + ix1;
      run(k0 ? cend(k0 - 1) : 0, cend(k1));
    }
  }
}

// The fast path caches 32 suppressor ranks per box as u16 (the same 64 bytes per row
// as the general path's 16 ints): past 32 it keeps the 32 highest-ranked, found with
// one 64-byte read, so a box rarely needs a rescan and the search never walks a
// dependent chain of global loads.
constexpr int kFSlots = 32;
// classes up to this size keep u16 slots (wide ones too) and stage their u16 ranks in LDS beside
// the u32 cell ends for the search (nms_search); larger ones keep 16 int slots
constexpr int kSlot16Max = (kBigLds - (((kFCells * 4) + 15) & ~15)) / 2;
static_assert(kSlot16Max <= 65535, "u16 ranks");

// f(k, v) for the first c of a box's u16 slots, read as 16-byte chunks (4 registers live)
template <class F>
__device__ __forceinline__ void for_slots16(const unsigned short* sl, int c, F&& f) {
  const int4* s4 = reinterpret_cast<const int4*>(sl);
  for (int q = 0; q < (c + 7) / 8; ++q) {
    const int4 x = s4[q];
    const int w[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
    for (int h = 0; h < 8; ++h)
      if (8 * q + h < c) f(8 * q + h, (int)(((unsigned)w[h >> 1] >> (16 * (h & 1))) & 0xFFFFu));
  }
}

// The combined state of a box's cached suppressors csr[b0 .. b0 + c): 2 if one is kept, else
// 1 if one is undecided, else 0 (all removed). Four ranks, then their four states, are read
// together (no read waits on the previous state); the scan stops once one is kept.
__device__ __forceinline__ int csr_state(const unsigned short* csr, int b0, int c, const unsigned char* st) {
  int res = 0;
  for (int k = 0; k < c && res != 2; k += 4) {
    int v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = k + u < c ? (int)csr[b0 + k + u] : -1;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (v[u] >= 0) {
        const unsigned char sj = st[v[u]];
        res = max(res, sj == 1 ? 2 : (sj == 0 ? 1 : 0));
      }
    }
  }
  return res;
}

// the rare replacement past kFSlots: keep the kFSlots highest-ranked (smallest ranks)
__device__ __forceinline__ void replace_slot16(unsigned short* sl, int rj) {
  int km = 0, vm = -1;
  for_slots16(sl, kFSlots, [&](int k, int v) {
    km = v > vm ? k : km;
    vm = v > vm ? v : vm;
  });
  if (rj < vm) sl[km] = (unsigned short)rj;
}

template <int E>
__device__ __forceinline__ void big_fast(const Task& tk, const ycx_cand* __restrict__ ci, const Ptrs& P, char* smem, int (*s_lv)[5],
                         int* s_ext, int* s_w, int* s_flag, const Thr& thr, float t_lo, float inv_t, int all_pairs,
                         unsigned long long* s_prof, unsigned long long* s_msk, WFrame* pub, char* pub_cells) {
  const int tid = threadIdx.x, lane = tid & 63;
  const int S = tk.S, off = tk.off;
  const int* bucket = P.bucket + off;
#ifdef YCX_NMS_PROFILE
  unsigned long long t_prev_ = __builtin_amdgcn_s_memtime();
#endif
  __syncthreads();  // s_ext / s_lv initialised
  // (1) sort keys of elements e = tid * E + i (score desc, row asc; e in the low bits)
  unsigned long long key[E];
#pragma unroll
  for (int i = 0; i < E; ++i) {
    const int e = tid * E + i;
    const int row = e < S ? bucket[e] : -1;
    if (row >= 0) {
      const ycx_cand& c = ci[row];
      const float score = c.obj * c.cls_conf;
      key[i] = ((unsigned long long)(0xFFFFFFFFu - __float_as_uint(score)) << 32) | ((unsigned)row << 13) | (unsigned)e;
    } else {
      key[i] = ~0ull;
    }
  }
  // (2) rank sort in registers (exchange through LDS), then every element learns its rank
  unsigned long long* xch = reinterpret_cast<unsigned long long*>(smem);
  unsigned short* rank_of = reinterpret_cast<unsigned short*>(smem + 8 * kFastMax);
  // bits [32, 64) only: the bucket lists the class's rows in ascending order and the passes are
  // stable, so equal scores keep row order (the row digits were 4 of a C2 class's ~11 passes)
  radix_sort_regs<E>(key, S, 32, xch, reinterpret_cast<unsigned short*>(smem + 10 * kFastMax), s_w, s_msk);
  __syncthreads();
#pragma unroll
  for (int i = 0; i < E; ++i)
    if (tid * E + i < S) rank_of[key[i] & 0x1FFF] = (unsigned short)(tid * E + i);
  __syncthreads();
  int myrank[E];
  f32x4 box[E];  // the elements' boxes, gathered again now that the keys are dead
#pragma unroll
  for (int i = 0; i < E; ++i) {
    const int e = tid * E + i;
    myrank[i] = e < S ? rank_of[e] : 0;
    if (e < S) {
      const ycx_cand& c = ci[bucket[e]];
      box[i] = f32x4{c.x1, c.y1, c.x2, c.y2};
    } else {
      box[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
  }
  __syncthreads();  // every element's bucket entry read
  int* rank_row = P.bucket + off;  // bucket in rank order from here
#pragma unroll
  for (int i = 0; i < E; ++i)
    if (tid * E + i < S) rank_row[tid * E + i] = (int)((key[i] >> 13) & 0x7FFFF);

  // class extent of the regular boxes (wave reduce, four LDS atomics per wave)
  {
    int mn0 = 0x7FFFFFFF, mn1 = 0x7FFFFFFF, mx2 = (int)0x80000000, mx3 = (int)0x80000000;
#pragma unroll
    for (int i = 0; i < E; ++i) {
      const f32x4 b = box[i];
      if (tid * E + i < S && b[2] > b[0] && b[3] > b[1] && b[0] > -INFINITY && b[1] > -INFINITY && b[2] < INFINITY &&
          b[3] < INFINITY) {
        mn0 = min(mn0, f2o(b[0]));
        mn1 = min(mn1, f2o(b[1]));
        mx2 = max(mx2, f2o(b[2]));
        mx3 = max(mx3, f2o(b[3]));
      }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      mn0 = min(mn0, __shfl_xor(mn0, o));
      mn1 = min(mn1, __shfl_xor(mn1, o));
      mx2 = max(mx2, __shfl_xor(mx2, o));
      mx3 = max(mx3, __shfl_xor(mx3, o));
    }
    if (lane == 0) {
      atomicMin(&s_ext[0], mn0);
      atomicMin(&s_ext[1], mn1);
      atomicMax(&s_ext[2], mx2);
      atomicMax(&s_ext[3], mx3);
    }
  }
  __syncthreads();  // rank_of dead: LDS becomes the cell table + boxes; extent complete
  YCX_PROF_MARK(0)
  // (3) spatial counting sort on the fine grid
  unsigned* cells = reinterpret_cast<unsigned*>(smem);
  for (int k = tid; k < kFCellBytes / 4; k += kBigThreads) cells[k] = 0;
  __syncthreads();
  const float X0 = o2f(s_ext[0]), Y0 = o2f(s_ext[1]);
  const float Ex = fmaxf(o2f(s_ext[2]) - X0, o2f(s_ext[3]) - Y0);
  const float inv = (Ex > 0.0f && Ex < INFINITY) ? 1.0f / Ex : 0.0f;  // 0: every box irregular
#pragma unroll
  for (int i = 0; i < E; ++i) {
    if (tid * E + i < S) {
      const int k = fgeometry(box[i], X0, Y0, inv, all_pairs).cell;
      atomicAdd(&cells[k >> 1], 1u << ((k & 1) * 16));
    }
  }
  {  // per-level count / extreme sizes
    LevelStats ls;
#pragma unroll
    for (int i = 0; i < E; ++i)
      if (tid * E + i < S) ls.add(fgeometry(box[i], X0, Y0, inv, all_pairs));
    ls.flush(s_lv);
  }
  __syncthreads();
  {  // exclusive scan of the u16 counts, in place: each thread a contiguous run of cells
    constexpr int kPer = (kFCells + kBigThreads - 1) / kBigThreads;
    const int c0 = tid * kPer, c1 = min(kFCells, c0 + kPer);
    int s = 0;
    for (int k = c0; k < c1; ++k) s += u16_at(cells, k);
    int total;
    int run = block_exclusive(s, s_w, &total);
    __syncthreads();  // every count read before any is overwritten
    unsigned short* c16 = reinterpret_cast<unsigned short*>(cells);
    for (int k = c0; k < c1; ++k) {
      const int v = c16[k];
      c16[k] = (unsigned short)run;
      run += v;
    }
  }
  __syncthreads();
  f32x4* lbox = reinterpret_cast<f32x4*>(smem + kFCellBytes);
  unsigned short* lr = reinterpret_cast<unsigned short*>(smem + kFCellBytes + 16 * S);
  unsigned char* st = reinterpret_cast<unsigned char*>(smem + kFCellBytes + 16 * S + ((2 * S + 15) & ~15));
#pragma unroll
  for (int i = 0; i < E; ++i) {
    if (tid * E + i >= S) continue;
    const int k = fgeometry(box[i], X0, Y0, inv, all_pairs).cell;
    const unsigned old = atomicAdd(&cells[k >> 1], 1u << ((k & 1) * 16));  // ends as the end of cell k
    const int q = (int)((old >> ((k & 1) * 16)) & 0xFFFFu);
    lbox[q] = box[i];
    lr[q] = (unsigned short)myrank[i];
    P.sbox[off + q] = box[i];  // global copies for the rare rescan after the boxes' LDS is reused
    P.srank[off + q] = myrank[i];
  }
  __syncthreads();
  YCX_PROF_MARK(1)
  if (pub) {  // split: the search and the fixed point run in nms_search / nms_resolve
    unsigned* gc = reinterpret_cast<unsigned*>(pub_cells);
    for (int k = tid; k < kFCellBytes / 4; k += kBigThreads) gc[k] = cells[k];
    if (tid == 0) {
      pub->X0 = X0;
      pub->Y0 = Y0;
      pub->inv = inv;
      pub->img = tk.img;
      pub->cls = tk.cls;
      pub->off = off;
      pub->S = S;
    }
    if (tid < kFLevels * 5) pub->lv[tid / 5][tid % 5] = s_lv[tid / 5][tid % 5];
    __syncthreads();  // every read of the LDS done before the next task reuses it
    return;
  }
  // (4) suppressors of every box (spatial order), kSlots highest-ranked kept (global slots)
#ifdef YCX_NMS_PROFILE
  const unsigned long long w_t0 = __builtin_amdgcn_s_memtime();
  unsigned long long w_vis = 0, w_mx = 0, w_ns = 0, w_over = 0;  // summed in registers: one atomic per wave
  if (tid == 0) { s_prof[0] = 0; s_prof[1] = 0; }
  __syncthreads();
#endif
  for (int p = tid; p < S; p += kBigThreads) {
    const int r = lr[p];
    const f32x4 b = lbox[p];
    const float a = box_area(b);
    const FGeo g = fgeometry(b, X0, Y0, inv, all_pairs);
    unsigned short* sl = reinterpret_cast<unsigned short*>(P.slots + (size_t)(off + p) * kSlots);
    int ns = 0;
#ifdef YCX_NMS_PROFILE
    int visits = 0;
#endif
    auto test = [&](int rj, const f32x4& o) {
      const bool cand = rj < r && (all_pairs || (o[0] < b[2] && o[2] > b[0] && o[1] < b[3] && o[3] > b[1]));
      if (cand && suppress(o[0], o[1], o[2], o[3], box_area(o), b[0], b[1], b[2], b[3], a, thr)) {
        if (ns < kFSlots) {
          sl[ns] = (unsigned short)rj;
        } else {  // rare: keep the kFSlots highest-ranked (smallest ranks)
          replace_slot16(sl, rj);
        }
        ++ns;
      }
    };
    f_ranges([&](int k) { return u16_at(cells, k); }, s_lv, g, S, t_lo, inv_t, [&](int q0, int q1) {
#ifdef YCX_NMS_PROFILE
      visits += q1 - q0;
#endif
      int q = q0;
      for (; q + 4 <= q1; q += 4) {
        int rj[4];
        f32x4 o[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          rj[u] = lr[q + u];
          o[u] = lbox[q + u];
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) test(rj[u], o[u]);
      }
      for (; q < q1; ++q) test(lr[q], lbox[q]);
    });
    P.nsup[off + p] = ns;
#ifdef YCX_NMS_PROFILE
    w_over += ns > kFSlots ? 1 : 0;
    w_ns += ns;
    int mx = visits;
    for (int o = 32; o > 0; o >>= 1) mx = max(mx, __shfl_xor(mx, o));
    w_mx += mx;
    w_vis += (unsigned long long)visits;
#endif
  }
#ifdef YCX_NMS_PROFILE
  {  // per-wave search time and visits: the slowest wave bounds the phase
    const unsigned long long d = __builtin_amdgcn_s_memtime() - w_t0;
    unsigned long long v = w_vis, ns_ = w_ns, ov = w_over;
    for (int o = 32; o > 0; o >>= 1) {
      v += __shfl_xor(v, o);
      ns_ += __shfl_xor(ns_, o);
      ov += __shfl_xor(ov, o);
    }
    if (lane == 0) {
      atomicAdd(&g_nms_prof[6], ov);
      atomicAdd(&g_nms_prof[8], v);
      atomicAdd(&g_nms_prof[9], w_mx);
      atomicAdd(&g_nms_prof[10], ns_);
      atomicAdd(&g_nms_prof[11], d);
      atomicMax(&s_prof[0], d);
      atomicMax(&s_prof[1], v);
    }
    __syncthreads();
    if (tid == 0) {
      atomicAdd(&g_nms_prof[12], s_prof[0]);
      atomicAdd(&g_nms_prof[13], s_prof[1]);
    }
  }
#endif
  for (int r = tid; r < S; r += kBigThreads) st[r] = 0;
  // (5) suppressor lists into LDS (CSR over the dead box region), if they fit
  __syncthreads();  // every search read of lbox done: its region becomes the CSR
  unsigned* csr_off = reinterpret_cast<unsigned*>(lbox);                     // [S]
  unsigned short* csr_ns = reinterpret_cast<unsigned short*>(csr_off + S);  // [S] min(ns, 0xFFFF)
  unsigned short* csr = csr_ns + ((S + 1) & ~1);                             // [total]
  int my_total = 0;  // positions p = tid + k * kBigThreads (the search's own: its nsup writes are this thread's)
  for (int p = tid; p < S; p += kBigThreads) my_total += min(P.nsup[off + p], kFSlots);
  int total;
  int base = block_exclusive(my_total, s_w, &total);
  const bool lds_csr = 4 * S + 2 * ((S + 1) & ~1) + 2 * total <= 16 * S;
  if (lds_csr) {
    for (int p = tid; p < S; p += kBigThreads) {
      const int ns = P.nsup[off + p], c = min(ns, kFSlots);
      for_slots16(reinterpret_cast<const unsigned short*>(P.slots + (size_t)(off + p) * kSlots), c,
                  [&](int k, int v) { csr[base + k] = (unsigned short)v; });
      csr_off[p] = base;
      csr_ns[p] = (unsigned short)min(ns, 0xFFFF);
      base += c;
    }
  }
  __syncthreads();
  YCX_PROF_MARK(2)
  // (6) greedy as a fixed point over ranks: 0 undecided, 1 kept, 2 removed
  for (int it = 0; it <= S; ++it) {  // every round decides at least one box
    if (tid == 0) *s_flag = 0;
    __syncthreads();
    int undecided = 0;
    for (int p = tid; p < S; p += kBigThreads) {
      const int r = lr[p];
      if (st[r] != 0) continue;
      int ns, res = 0;  // 0: every suppressor removed, 1: some undecided, 2: one kept
      if (lds_csr) {
        ns = csr_ns[p];
        res = csr_state(csr, (int)csr_off[p], min(ns, kFSlots), st);
      } else {
        ns = P.nsup[off + p];
        for_slots16(reinterpret_cast<const unsigned short*>(P.slots + (size_t)(off + p) * kSlots), min(ns, kFSlots),
                    [&](int, int v) {
                      const unsigned char sj = st[v];
                      res = res == 2 ? 2 : (sj == 1 ? 2 : (sj == 0 ? 1 : res));
                    });
      }
      if (ns > kFSlots && res == 0) {  // the cached ones are all removed: rescan (global copies)
        const f32x4 b = P.sbox[off + p];
        const float a = box_area(b);
        const FGeo g = fgeometry(b, X0, Y0, inv, all_pairs);
        bool stop = false;
        f_ranges([&](int k) { return u16_at(cells, k); }, s_lv, g, S, t_lo, inv_t, [&](int q0, int q1) {
          for (int q = q0; q < q1 && !stop; ++q) {
            const int rj = P.srank[off + q];
            if (rj >= r) continue;
            const unsigned char sj = st[rj];
            if (sj == 2) continue;
            const f32x4 o = P.sbox[off + q];
            if (suppress(o[0], o[1], o[2], o[3], box_area(o), b[0], b[1], b[2], b[3], a, thr)) {
              if (sj == 1) { res = 2; stop = true; }
              else res = 1;
            }
          }
        });
      }
      if (res == 2) st[r] = 2;
      else if (res == 0) st[r] = 1;
      else undecided = 1;
    }
    if (undecided) *s_flag = 1;
    __syncthreads();
    const int more = *s_flag;
    __syncthreads();
#ifdef YCX_NMS_PROFILE
    if (tid == 0) atomicAdd(&g_nms_prof[5], 1ull);
#endif
    if (!more) break;
  }
  YCX_PROF_MARK(3)
  // (7) kept rows in rank order: thread tid takes ranks tid * E .. + E - 1
  int nk = 0;
#pragma unroll
  for (int i = 0; i < E; ++i) nk += (tid * E + i < S && st[tid * E + i] == 1) ? 1 : 0;
  int kt;
  int pos = block_exclusive(nk, s_w, &kt);
#pragma unroll
  for (int i = 0; i < E; ++i) {
    const int r = tid * E + i;
    if (r < S && st[r] == 1) P.kept[off + pos++] = rank_row[r];
  }
  if (tid == 0) P.kc[tk.cls] = kt;
  __syncthreads();
  YCX_PROF_MARK(4)
}

// ---------------------------------------------------------------------------
// The LDS-resident classes (S <= kFastMax and fast_lds_bytes(S) fits): big_fast, one
// 1024-thread workgroup per class (grid-strided task loop), beside the wide classes' sort and index.
__device__ __forceinline__ void wide_a_task(const ycx_nms_desc& d, const ycx_cand* __restrict__ cand, char* ws,
                                            const Layout& L, int t, const Task& tk, char* smem, int (*s_lv)[5],
                                            int* s_ext, int* s_w, unsigned long long* s_msk, int all_pairs);

template <int E>  // one launch per register-array width: each instance allocates its own registers
__global__ void __launch_bounds__(kBigThreads) __attribute__((amdgpu_waves_per_eu(4))) nms_fast(
    ycx_nms_desc d, const ycx_cand* __restrict__ cand, char* ws, Thr thr, float t_lo, float inv_t, int all_pairs,
    int with_wide) {
  __shared__ __attribute__((aligned(16))) char smem[kBigLds];
  __shared__ int s_lv[kFLevels][5];
  __shared__ int s_ext[4];
  __shared__ int s_w[kBigThreads / 64];
  __shared__ int s_flag;
  __shared__ unsigned long long s_prof[2];  // profile build: per-task wave maxima
  __shared__ unsigned long long s_msk[2];   // radix sort: AND / OR of the keys
  const int tid = threadIdx.x;
  const int rows = d.rows_total;
  const Layout L = layout(d.n, rows, d.nc);
  const Hdr* hdr = reinterpret_cast<const Hdr*>(ws + L.hdr);
  const Task* tasks = reinterpret_cast<const Task*>(ws + L.tasks);
  const int ntasks = hdr->ntasks, nwide = with_wide ? hdr->nwide : 0;
  // the wide classes' sort + spatial index first (the longest items), then the fast classes
  for (int w = blockIdx.x; w < nwide + ntasks; w += gridDim.x) {
    if (w < nwide) {
      constexpr int kCellB = ((kFCells * 4) + 255) & ~255;  // u32 cell ends
      static_assert(kBigLds >= 16 * (kMaxRows / kBigThreads) * (kBigThreads / 64) * 4 &&
                        kBigLds >= 64 * 32 * (kBigThreads / 64) * 4 && kBigLds >= kCellB + 1024,
                    "wide path LDS: radix counts, cells");
      const Task* wt = tasks + (size_t)d.n * L.max_tasks;  // the wide list
      wide_a_task(d, cand, ws, L, w, wt[w], smem, s_lv, s_ext, s_w, s_msk, all_pairs);
      continue;
    }
    const int t = w - nwide;
    const Task tk = tasks[t];

    const Ptrs P = image_ptrs(ws, L, tk.img);
    const ycx_cand* ci = cand + (size_t)tk.img * rows;
#ifdef YCX_NMS_PROFILE
    if (tid == 0) atomicAdd(&g_nms_prof[7], 1ull);
#endif
    if (tid == 0) {
      s_ext[0] = s_ext[1] = 0x7FFFFFFF;  // min x1, min y1
      s_ext[2] = s_ext[3] = (int)0x80000000;  // max x2, max y2
    }
    if (tid < kFLevels) {
      s_lv[tid][0] = 0;
      s_lv[tid][1] = s_lv[tid][2] = 0;  // +0.0f
      s_lv[tid][3] = s_lv[tid][4] = 0x7F800000;  // +inf
    }
    const bool split = with_wide && split_fast(hdr);
    WFrame* pub = split ? reinterpret_cast<WFrame*>(ws + L.fframes + (size_t)t * wframe_bytes()) : nullptr;
    char* pub_cells = ws + L.fcells + (size_t)t * fast_cells_bytes();
    big_fast<E>(tk, ci, P, smem, s_lv, s_ext, s_w, &s_flag, thr, t_lo, inv_t, all_pairs, s_prof, s_msk, pub, pub_cells);
  }
}

// ---------------------------------------------------------------------------
// nms_wide: classes past the LDS-resident fast path (S > kFastMax or too big for LDS:
// the 1280^2 C4 load has ~18k-box classes). The fast path's algorithm with global
// arrays where LDS runs out: a stable LSD radix rank sort of the workspace keys
// (replacing the general path's global bitonic, O(S log^2 S) passes over global
// memory), one gather per box into a rank-ordered copy, the fine grid (u32 cells in
// LDS) and the tight window, int suppressor slots with one-read replacement, and the
// fixed point over an LDS state array when S fits.
// ---------------------------------------------------------------------------
template <class F>
__device__ __forceinline__ void for_slots32(const int* sl, int c, F&& f) {
  const int4* s4 = reinterpret_cast<const int4*>(sl);
  for (int q = 0; q < (c + 3) / 4; ++q) {
    const int4 x = s4[q];
    const int w[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
    for (int h = 0; h < 4; ++h)
      if (4 * q + h < c) f(4 * q + h, w[h]);
  }
}

__device__ __forceinline__ void replace_slot32(int* sl, int rj) {  // keep the kSlots smallest ranks
  int km = 0, vm = -1;
  for_slots32(sl, kSlots, [&](int k, int v) {
    km = v > vm ? k : km;
    vm = v > vm ? v : vm;
  });
  if (rj < vm) sl[km] = rj;
}

// Stable LSD rank sort (B-bit digits, digits every key shares skipped) of a wide class's S
// keys (score desc, row asc) in global scratch. Striped layout (coalesced): element p = i *
// kBigThreads + tid, i < E = ceil(S / kBigThreads) <= 128. A pass counts, per (digit, i, wave),
// the wave's elements of slot i with that digit (the lanes with equal digits found by B
// ballots), scans the counts in (digit, i, wave) order -- the input order within each digit --
// and scatters every key to its count's offset plus its rank among the equal-digit lanes below
// it: stable, and the lanes of a group write consecutive addresses. Keys move in batches of 8
// slots per thread with the batch's loads issued together (one memory round trip per 8 keys,
// not per key); the last pass scatters the rows themselves into bucket (rank order).
// a / b: 8 S bytes each; C: LDS u32 [2^B][E][16] (<= 128 KiB: B = 6 up to E = 32, else 4).
template <int B>
__device__ __forceinline__ unsigned long long same_digit_lanes(int dg) {
  unsigned long long m = ~0ull;
#pragma unroll
  for (int bit = 0; bit < B; ++bit) {
    const unsigned long long bl = __ballot((dg >> bit) & 1);
    m &= ((dg >> bit) & 1) ? bl : ~bl;
  }
  return m;
}

template <int B>  // digit bits
__device__ void radix_rank(const ycx_cand* __restrict__ ci, int* bucket, int S, unsigned long long* a,
                           unsigned long long* b, unsigned* C, int* s_w, unsigned long long* s_msk) {
  constexpr int D = 1 << B;
  constexpr unsigned long long DM = D - 1;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  constexpr int NW = kBigThreads / 64;
  const int E = (S + kBigThreads - 1) / kBigThreads;
  const int nch = (E + 7) / 8;  // uniform
  const unsigned long long lt = (1ull << lane) - 1ull;  // lanes below this one
  auto at = [&](int c, int j) { return (8 * c + j) * kBigThreads + tid; };
#ifdef YCX_NMS_PROFILE
  const unsigned long long t_sort0 = __builtin_amdgcn_s_memtime();
#endif
  unsigned long long an = ~0ull, orr = 0ull;
  for (int c = 0; c < nch; ++c) {  // keys built from the candidates into a
    int row[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) row[j] = at(c, j) < S ? bucket[at(c, j)] : -1;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if (row[j] >= 0) {
        const unsigned long long key = make_key(ci[row[j]]);
        a[at(c, j)] = key;
        an &= key;
        orr |= key;
      }
    }
  }
#pragma unroll
  for (int sh = 32; sh > 0; sh >>= 1) {
    an &= __shfl_xor(an, sh);
    orr |= __shfl_xor(orr, sh);
  }
  if (tid == 0) { s_msk[0] = ~0ull; s_msk[1] = 0ull; }
  __syncthreads();  // every bucket read done (the last pass rewrites bucket)
  if (lane == 0) {
    atomicAnd(&s_msk[0], an);
    atomicOr(&s_msk[1], orr);
  }
  __syncthreads();
  const unsigned long long diff = s_msk[0] ^ s_msk[1];
  // digits of the high word (the score) only: the bucket lists the class's rows in ascending
  // order and the passes are stable, so equal scores keep row order (nms_bucket)
  int last = -1;  // the last digit any two keys differ in (none: every score equal, bucket already in order)
  for (int sh = 32; sh < 64; sh += B)
    if ((diff >> sh) & DM) last = sh;
  const int nC = D * E * NW;
#ifdef YCX_NMS_PROFILE
  unsigned long long t_prev_ = __builtin_amdgcn_s_memtime();
  if (tid == 0) atomicAdd(&g_nms_wprof[8], t_prev_ - t_sort0);
#endif
  for (int sh = 32; sh <= last; sh += B) {
    if (((diff >> sh) & DM) == 0) continue;  // uniform
    for (int c = tid; c < nC; c += kBigThreads) C[c] = 0;
    __syncthreads();
    for (int c = 0; c < nch; ++c) {
      unsigned long long k[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) k[j] = at(c, j) < S ? a[at(c, j)] : 0ull;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int i = 8 * c + j;
        if (i >= E) break;  // uniform: the ballots need every lane
        const bool ok = at(c, j) < S;
        const int dg = ok ? (int)((k[j] >> sh) & DM) : D;  // D: past the end (matches no digit)
        const unsigned long long m = same_digit_lanes<B>(dg & (D - 1)) & __ballot(ok);
        if (ok && (m & lt) == 0) C[(dg * E + i) * NW + wid] = (unsigned)__popcll(m);  // the group's first lane
      }
    }
    __syncthreads();
    {  // exclusive scan of C in (digit, i, wave) order: thread t owns a contiguous run
      const int per = (nC + kBigThreads - 1) / kBigThreads, c0 = min(nC, tid * per), c1 = min(nC, c0 + per);
      int sum = 0;
      for (int c = c0; c < c1; ++c) sum += (int)C[c];
      int total;
      unsigned run = (unsigned)block_exclusive(sum, s_w, &total);
      for (int c = c0; c < c1; ++c) {
        const unsigned v = C[c];
        C[c] = run;
        run += v;
      }
    }
    __syncthreads();
    const bool fin = sh == last;
    for (int c = 0; c < nch; ++c) {
      unsigned long long k[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) k[j] = at(c, j) < S ? a[at(c, j)] : 0ull;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int i = 8 * c + j;
        if (i >= E) break;
        const bool ok = at(c, j) < S;
        const int dg = ok ? (int)((k[j] >> sh) & DM) : D;
        const unsigned long long m = same_digit_lanes<B>(dg & (D - 1)) & __ballot(ok);
        if (ok) {
          const unsigned q = C[(dg * E + i) * NW + wid] + (unsigned)__popcll(m & lt);
          if (fin) bucket[q] = (int)(unsigned)k[j];
          else b[q] = k[j];
        }
      }
    }
    __syncthreads();  // the pass's output complete (and every read of a and C done) before the next pass
    unsigned long long* t = a;
    a = b;
    b = t;
#ifdef YCX_NMS_PROFILE
    if (tid == 0) atomicAdd(&g_nms_wprof[10], 1ull);
#endif
  }
#ifdef YCX_NMS_PROFILE
  if (tid == 0) atomicAdd(&g_nms_wprof[9], __builtin_amdgcn_s_memtime() - t_prev_);
#endif
}

// nms_wide_a's work for wide task t: the class's keys sorted, boxes in rank order, the
// spatial index published for nms_wide_s / nms_wide_b (run inside nms_fast's launch, beside
// the fast classes: both are one workgroup per class and neither waits on the other)
__device__ __forceinline__ void wide_a_task(const ycx_nms_desc& d, const ycx_cand* __restrict__ cand, char* ws,
                                            const Layout& L, int t, const Task& tk, char* smem, int (*s_lv)[5],
                                            int* s_ext, int* s_w, unsigned long long* s_msk, int all_pairs) {
  const int tid = threadIdx.x, lane = tid & 63;
  const int rows = d.rows_total;
  unsigned* cells = reinterpret_cast<unsigned*>(smem);
    const int S = tk.S, off = tk.off;
    const Ptrs P = image_ptrs(ws, L, tk.img);
    const ycx_cand* ci = cand + (size_t)tk.img * rows;
    int* bucket = P.bucket + off;
#ifdef YCX_NMS_PROFILE
    unsigned long long t_prev_ = __builtin_amdgcn_s_memtime();
    if (tid == 0) atomicAdd(&g_nms_wprof[7], 1ull);
#endif
    if (tid == 0) {
      s_ext[0] = s_ext[1] = 0x7FFFFFFF;
      s_ext[2] = s_ext[3] = (int)0x80000000;
    }
    if (tid < kFLevels) {
      s_lv[tid][0] = 0;
      s_lv[tid][1] = s_lv[tid][2] = 0;
      s_lv[tid][3] = s_lv[tid][4] = 0x7F800000;
    }
    // (1) keys (score desc, row asc), radix-sorted: rank r = position; bucket in rank order
    unsigned long long* ka = P.keys + 2 * (size_t)off;
    if (S <= 32 * kBigThreads)  // 6-bit digits while the count table (64 x E x 16 u32) fits the LDS
      radix_rank<6>(ci, bucket, S, ka, ka + S, reinterpret_cast<unsigned*>(smem), s_w, s_msk);
    else
      radix_rank<4>(ci, bucket, S, ka, ka + S, reinterpret_cast<unsigned*>(smem), s_w, s_msk);
    __syncthreads();
    YCX_WPROF_MARK(0)
    // (2) boxes in rank order (the dead keys' region, 16 B per rank) and the class extent
    f32x4* rbox = reinterpret_cast<f32x4*>(ka);
    {
      int mn0 = 0x7FFFFFFF, mn1 = 0x7FFFFFFF, mx2 = (int)0x80000000, mx3 = (int)0x80000000;
      for (int r0 = tid; r0 < S; r0 += 8 * kBigThreads) {  // batches of 8 ranks: the loads issued together
        int row[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) row[j] = r0 + j * kBigThreads < S ? bucket[r0 + j * kBigThreads] : -1;
        f32x4 bx[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          if (row[j] >= 0) {
            const ycx_cand& c = ci[row[j]];
            bx[j] = f32x4{c.x1, c.y1, c.x2, c.y2};
          }
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          if (row[j] < 0) continue;
          const f32x4 c = bx[j];
          rbox[r0 + j * kBigThreads] = c;
          if (c[2] > c[0] && c[3] > c[1] && c[0] > -INFINITY && c[1] > -INFINITY && c[2] < INFINITY && c[3] < INFINITY) {
            mn0 = min(mn0, f2o(c[0]));
            mn1 = min(mn1, f2o(c[1]));
            mx2 = max(mx2, f2o(c[2]));
            mx3 = max(mx3, f2o(c[3]));
          }
        }
      }
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        mn0 = min(mn0, __shfl_xor(mn0, o));
        mn1 = min(mn1, __shfl_xor(mn1, o));
        mx2 = max(mx2, __shfl_xor(mx2, o));
        mx3 = max(mx3, __shfl_xor(mx3, o));
      }
      if (lane == 0) {
        atomicMin(&s_ext[0], mn0);
        atomicMin(&s_ext[1], mn1);
        atomicMax(&s_ext[2], mx2);
        atomicMax(&s_ext[3], mx3);
      }
    }
    for (int k = tid; k < kFCells; k += kBigThreads) cells[k] = 0;
    __syncthreads();
    const float X0 = o2f(s_ext[0]), Y0 = o2f(s_ext[1]);
    const float Ex = fmaxf(o2f(s_ext[2]) - X0, o2f(s_ext[3]) - Y0);
    const float inv = (Ex > 0.0f && Ex < INFINITY) ? 1.0f / Ex : 0.0f;
    // (3) spatial counting sort on the fine grid
    {
      LevelStats ls;
      for (int rb = 0; rb < S; rb += 8 * kBigThreads) {  // batches of 8 ranks per thread
        f32x4 bx[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int r = rb + j * kBigThreads + tid;
          if (r < S) bx[j] = rbox[r];
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          if (rb + j * kBigThreads + tid < S) {
            const FGeo g = fgeometry(bx[j], X0, Y0, inv, all_pairs);
            atomicAdd(&cells[g.cell], 1u);
            ls.add(g);
          }
        }
      }
      ls.flush(s_lv);
    }
    __syncthreads();
    {  // exclusive scan of the cell counts in place
      constexpr int kPer = (kFCells + kBigThreads - 1) / kBigThreads;
      const int c0 = tid * kPer, c1 = min(kFCells, c0 + kPer);
      int sum = 0;
      for (int k = c0; k < c1; ++k) sum += (int)cells[k];
      int total;
      int run = block_exclusive(sum, s_w, &total);
      __syncthreads();
      for (int k = c0; k < c1; ++k) {
        const int v = (int)cells[k];
        cells[k] = (unsigned)run;
        run += v;
      }
    }
    __syncthreads();
    f32x4* sbox = P.sbox + off;
    int* srank = P.srank + off;
    for (int r0 = tid; r0 < S; r0 += 8 * kBigThreads) {  // batches of 8 ranks per thread
      f32x4 bx[8];
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (r0 + j * kBigThreads < S) bx[j] = rbox[r0 + j * kBigThreads];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int r = r0 + j * kBigThreads;
        if (r >= S) continue;
        const int q = (int)atomicAdd(&cells[fgeometry(bx[j], X0, Y0, inv, all_pairs).cell], 1u);  // -> cell ends
        sbox[q] = bx[j];
        srank[q] = r;
      }
    }
    __syncthreads();
    // publish the class's spatial index for the search and resolve launches
    WFrame* fr = reinterpret_cast<WFrame*>(ws + L.wframes + (size_t)t * wframe_bytes());
    unsigned* gcells = reinterpret_cast<unsigned*>(ws + L.wcells + (size_t)t * wide_cells_bytes());
    for (int k = tid; k < kFCells; k += kBigThreads) gcells[k] = cells[k];
    if (tid == 0) {
      fr->X0 = X0;
      fr->Y0 = Y0;
      fr->inv = inv;
      fr->img = tk.img;
      fr->cls = tk.cls;
      fr->off = off;
      fr->S = S;
    }
    if (tid < kFLevels * 5) fr->lv[tid / 5][tid % 5] = s_lv[tid / 5][tid % 5];
    YCX_WPROF_MARK(1)
    __syncthreads();
}

// load a wide class's frame (level stats to LDS) and cell table (to LDS); returns the frame
__device__ __forceinline__ WFrame load_wide(const char* ws, const Layout& L, int t, unsigned* cells, int (*s_lv)[5]) {
  const WFrame* fr = reinterpret_cast<const WFrame*>(ws + L.wframes + (size_t)t * wframe_bytes());
  const unsigned* gcells = reinterpret_cast<const unsigned*>(ws + L.wcells + (size_t)t * wide_cells_bytes());
  for (int k = threadIdx.x; k < kFCells; k += kBigThreads) cells[k] = gcells[k];
  if (threadIdx.x < kFLevels * 5) s_lv[threadIdx.x / 5][threadIdx.x % 5] = fr->lv[threadIdx.x / 5][threadIdx.x % 5];
  const WFrame f = *fr;
  __syncthreads();
  return f;
}

// the same for a split fast class (u16 cell ends, copied as packed words)
__device__ __forceinline__ WFrame load_fast(const char* ws, const Layout& L, int t, unsigned* cells, int (*s_lv)[5]) {
  const WFrame* fr = reinterpret_cast<const WFrame*>(ws + L.fframes + (size_t)t * wframe_bytes());
  const unsigned* gcells = reinterpret_cast<const unsigned*>(ws + L.fcells + (size_t)t * fast_cells_bytes());
  for (int k = threadIdx.x; k < kFCellBytes / 4; k += kBigThreads) cells[k] = gcells[k];
  if (threadIdx.x < kFLevels * 5) s_lv[threadIdx.x / 5][threadIdx.x % 5] = fr->lv[threadIdx.x / 5][threadIdx.x % 5];
  const WFrame f = *fr;
  __syncthreads();
  return f;
}

// The classes nms_search and nms_resolve take: the wide list, then (split) the fast list.
struct BigList {
  const Task* wide;
  const Task* fast;
  int nwide, nfast;
  __device__ __forceinline__ int size() const { return nwide + nfast; }
  __device__ __forceinline__ int S(int t) const { return t < nwide ? wide[t].S : fast[t - nwide].S; }
};

__device__ __forceinline__ BigList big_list(const char* ws, const Layout& L, int n) {
  const Hdr* h = reinterpret_cast<const Hdr*>(ws + L.hdr);
  const Task* tasks = reinterpret_cast<const Task*>(ws + L.tasks);
  BigList b;
  b.wide = tasks + (size_t)n * L.max_tasks;
  b.fast = tasks;
  b.nwide = h->nwide;
  b.nfast = split_fast(h) ? h->ntasks : 0;
  return b;
}

// Suppressor search of positions [p0, p1) of one class (spatial order): every box's
// higher-ranked boxes with IoU > thr, the highest-ranked kept in its 64-byte slot row
// (kSlot16: 32 u16 ranks, the fast path's format, for any class of S <= 65535; else 16 int
// ranks) and their count. kFast: u16 cell ends (else u32).
template <bool kFast, bool kSlot16, class RankT>
__device__ __forceinline__ void search_range(const WFrame& f, const unsigned* cells, const int (*s_lv)[5],
                                             const f32x4* sbox, const RankT* srank, const Ptrs& P, int p0,
                                             int p1, const Thr& thr, float t_lo, float inv_t, int all_pairs) {
  const int S = f.S, off = f.off;
  auto cend = [&](int k) -> int {
    if constexpr (kFast) return u16_at(cells, k);
    else return (int)cells[k];
  };
  for (int p = p0 + (int)threadIdx.x; p < p1; p += kBigThreads) {
    const int r = (int)srank[p];
    const f32x4 b = sbox[p];
    const float a = box_area(b);
    const FGeo g = fgeometry(b, f.X0, f.Y0, f.inv, all_pairs);
    int* sl = P.slots + (size_t)(off + p) * kSlots;
    int ns = 0;
    auto test = [&](int rj, const f32x4& o) {
      const bool cnd = rj < r && (all_pairs || (o[0] < b[2] && o[2] > b[0] && o[1] < b[3] && o[3] > b[1]));
      if (cnd && suppress(o[0], o[1], o[2], o[3], box_area(o), b[0], b[1], b[2], b[3], a, thr)) {
        if constexpr (kSlot16) {
          unsigned short* s16 = reinterpret_cast<unsigned short*>(sl);
          if (ns < kFSlots) s16[ns] = (unsigned short)rj;
          else replace_slot16(s16, rj);
        } else {
          if (ns < kSlots) sl[ns] = rj;
          else replace_slot32(sl, rj);
        }
        ++ns;
      }
    };
    f_ranges(cend, s_lv, g, S, t_lo, inv_t, [&](int q0, int q1) {
      int q = q0;
      for (; q + 4 <= q1; q += 4) {  // four candidates in flight; a box is loaded only when it outranks
        int rj[4];
        f32x4 o[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) rj[u] = (int)srank[q + u];
#pragma unroll
        for (int u = 0; u < 4; ++u) o[u] = rj[u] < r ? sbox[q + u] : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int u = 0; u < 4; ++u) test(rj[u], o[u]);
      }
      for (; q < q1; ++q) {
        const int rq = (int)srank[q];
        if (rq < r) test(rq, sbox[q]);
      }
    });
    P.nsup[off + p] = ns;
  }
}

// classes past u16 ranks (S > kSlot16Max)
__device__ __forceinline__ void search_wide_int(const WFrame& f, const unsigned* cells, const int (*s_lv)[5],
                                                          const Ptrs& P, int p0, int p1, const Thr& thr, float t_lo,
                                                          float inv_t, int all_pairs) {
  search_range<false, false>(f, cells, s_lv, P.sbox + f.off, P.srank + f.off, P, p0, p1, thr, t_lo, inv_t, all_pairs);
}

// Suppressor search of every split class: the concatenated positions of the list are cut into
// gridDim.x equal ranges, one per workgroup (a range may span classes: each class's index is
// staged in LDS once per workgroup), so the whole grid shares the search however few and
// however unequal the classes are.
__global__ void __launch_bounds__(kBigThreads) __attribute__((amdgpu_waves_per_eu(4))) nms_search(
    ycx_nms_desc d, char* ws, Thr thr, float t_lo, float inv_t, int all_pairs) {
  // a wide class: its u32 cell ends; a fast class: u16 cell ends, then its boxes and u16 ranks
  // in spatial order (what its own search read from LDS in nms_fast): fast_lds_bytes(S) fits
  __shared__ __attribute__((aligned(16))) char smem[kBigLds];
  __shared__ int s_lv[kFLevels][5];
  unsigned* cells = reinterpret_cast<unsigned*>(smem);
  const Layout L = layout(d.n, d.rows_total, d.nc);
  const BigList bl = big_list(ws, L, d.n);
  const int nt = bl.size();
  long long tot = 0;
  for (int t = 0; t < nt; ++t) tot += bl.S(t);
  const long long lo = tot * blockIdx.x / gridDim.x, hi = tot * (blockIdx.x + 1) / gridDim.x;
  long long s0 = 0;
  for (int t = 0; t < nt && s0 < hi; ++t) {  // bounded: the list is finite
    const int S = bl.S(t);
    const long long a = lo > s0 ? lo : s0, b = hi < s0 + S ? hi : s0 + S;
    if (a < b) {
      if (t >= bl.nwide) {
        const WFrame f = load_fast(ws, L, t - bl.nwide, cells, s_lv);
        const Ptrs P = image_ptrs(ws, L, f.img);
        f32x4* lbox = reinterpret_cast<f32x4*>(smem + kFCellBytes);
        unsigned short* lr = reinterpret_cast<unsigned short*>(smem + kFCellBytes + 16 * S);
        for (int p = threadIdx.x; p < S; p += kBigThreads) {
          lbox[p] = P.sbox[f.off + p];
          lr[p] = (unsigned short)P.srank[f.off + p];
        }
        __syncthreads();
        search_range<true, true>(f, cells, s_lv, lbox, lr, P, (int)(a - s0), (int)(b - s0), thr, t_lo, inv_t,
                                 all_pairs);
      } else {
        const WFrame f = load_wide(ws, L, t, cells, s_lv);
        const Ptrs P = image_ptrs(ws, L, f.img);
        constexpr int kCellB = ((kFCells * 4) + 15) & ~15;
        if (S <= kSlot16Max) {  // the ranks (u16) staged beside the cells; boxes read from L2
          unsigned short* lr = reinterpret_cast<unsigned short*>(smem + kCellB);
          for (int p = threadIdx.x; p < S; p += kBigThreads) lr[p] = (unsigned short)P.srank[f.off + p];
          __syncthreads();
          search_range<false, true>(f, cells, s_lv, P.sbox + f.off, lr, P, (int)(a - s0), (int)(b - s0), thr, t_lo,
                                    inv_t, all_pairs);
        } else {
          search_wide_int(f, cells, s_lv, P, (int)(a - s0), (int)(b - s0), thr, t_lo, inv_t, all_pairs);
        }
      }
      __syncthreads();  // every read of this class's LDS done before the next one is staged
    }
    s0 += S;
  }
}

// Greedy fixed point of a wide class (one workgroup): positions p = tid + k * kBigThreads,
// k < E; each thread tracks its undecided positions in a bit mask (only the owner of a position
// ever decides its rank), so a round touches only those, two at a time with their rank, count
// and 64-byte slot row loaded together. Then the kept rows in rank order (each thread a
// contiguous run of ranks, one scan).
template <bool k16>
__device__ __forceinline__ void resolve_wide(const Layout& L, char* ws, int t, const Task tk, char* smem,
                                                       int (*s_lv)[5], int* s_w, int* s_flag, const Thr thr,
                                                       float t_lo, float inv_t, int all_pairs) {
  constexpr int kCellB = ((kFCells * 4) + 255) & ~255;  // u32 cell ends
  const int tid = threadIdx.x;
  unsigned* cells = reinterpret_cast<unsigned*>(smem);
#ifdef YCX_NMS_PROFILE
  unsigned long long t_prev_ = __builtin_amdgcn_s_memtime();
#endif
  const WFrame f = load_wide(ws, L, t, cells, s_lv);
  const Ptrs P = image_ptrs(ws, L, tk.img);
  const int S = tk.S, off = tk.off;
  const int* bucket = P.bucket + off;
  const f32x4* sbox = P.sbox + off;
  const int* srank = P.srank + off;
  const int* nsup = P.nsup + off;
  const int4* slots = reinterpret_cast<const int4*>(P.slots + (size_t)off * kSlots);
  auto cend = [&](int k) { return (int)cells[k]; };
  unsigned char* st = S <= kBigLds - kCellB ? reinterpret_cast<unsigned char*>(smem + kCellB) : P.state + off;
  for (int r = tid; r < S; r += kBigThreads) st[r] = 0;
  const int E = (S + kBigThreads - 1) / kBigThreads;  // <= kMaxRows / kBigThreads = 128
  unsigned und[4];
#pragma unroll
  for (int w = 0; w < 4; ++w) {
    const int kn = min(32, max(0, E - 32 * w));  // slots k of this word below E
    unsigned m = kn == 32 ? ~0u : ((1u << kn) - 1u);
    if (kn > 0 && tid + (32 * w + kn - 1) * kBigThreads >= S) m &= ~(1u << (kn - 1));  // the last slot may be past S
    und[w] = m;
  }
  __syncthreads();
  YCX_WPROF_MARK(2)
  // k16: 32 u16 slots per row (8 per 16-byte chunk); else 16 ints (4 per chunk)
  constexpr int kCap = k16 ? kFSlots : kSlots, kPer = k16 ? 8 : 4;
  // res: 0 every suppressor removed (keep), 1 some undecided, 2 one kept (remove)
  auto decide = [&](int p, int r, int ns, const int4 (&s)[4]) -> int {
    int res = 0;
    const int c = min(ns, kCap);
#pragma unroll
    for (int h = 0; h < kCap; ++h) {
      const int4 x = s[h / kPer];
      int v;
      if constexpr (k16) {
        const int wv = ((h >> 1) & 3) == 0 ? x.x : ((h >> 1) & 3) == 1 ? x.y : ((h >> 1) & 3) == 2 ? x.z : x.w;
        v = (int)(((unsigned)wv >> (16 * (h & 1))) & 0xFFFFu);
      } else {
        v = (h & 3) == 0 ? x.x : (h & 3) == 1 ? x.y : (h & 3) == 2 ? x.z : x.w;
      }
      if (h < c) {  // independent reads: no state read waits on the previous one
        const unsigned char sj = st[v];
        res = max(res, sj == 1 ? 2 : (sj == 0 ? 1 : 0));
      }
    }
    if (ns > kCap && res == 0) {  // the cached ones are all removed: rescan
      const f32x4 b = sbox[p];
      const float a = box_area(b);
      const FGeo g = fgeometry(b, f.X0, f.Y0, f.inv, all_pairs);
      bool stop = false;
      f_ranges(cend, s_lv, g, S, t_lo, inv_t, [&](int q0, int q1) {
        for (int q = q0; q < q1 && !stop; ++q) {
          const int rj = srank[q];
          if (rj >= r) continue;
          const unsigned char sj = st[rj];
          if (sj == 2) continue;
          const f32x4 o = sbox[q];
          if (suppress(o[0], o[1], o[2], o[3], box_area(o), b[0], b[1], b[2], b[3], a, thr)) {
            if (sj == 1) { res = 2; stop = true; }
            else res = 1;
          }
        }
      });
    }
    return res;
  };
  for (int it = 0; it <= S; ++it) {  // every round decides at least one box
    if (tid == 0) *s_flag = 0;
    __syncthreads();
    int undecided = 0;
#ifdef YCX_NMS_PROFILE
    unsigned und0[4] = {und[0], und[1], und[2], und[3]};
#endif
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      unsigned m = und[w];
      while (m) {
        const int k0 = 32 * w + __builtin_ctz(m);
        m &= m - 1u;
        const int k1 = m ? 32 * w + __builtin_ctz(m) : -1;
        if (m) m &= m - 1u;
        const int pa = tid + k0 * kBigThreads, pb = k1 >= 0 ? tid + k1 * kBigThreads : pa;
        const int ra = srank[pa], rb = srank[pb];
        const int na = nsup[pa], nb = nsup[pb];
        int4 sa[4], sb[4];
        sa[0] = slots[(size_t)pa * 4];
        sb[0] = slots[(size_t)pb * 4];
#pragma unroll
        for (int q = 1; q < 4; ++q) {  // the further chunks only when they hold cached ranks
          sa[q] = q * kPer < na ? slots[(size_t)pa * 4 + q] : int4{0, 0, 0, 0};
          sb[q] = q * kPer < nb ? slots[(size_t)pb * 4 + q] : int4{0, 0, 0, 0};
        }
        const int resa = decide(pa, ra, na, sa);
        if (resa == 1) {
          undecided = 1;
        } else {
          st[ra] = resa == 2 ? 2 : 1;
          und[w] &= ~(1u << (k0 & 31));
        }
        if (k1 >= 0) {
          const int resb = decide(pb, rb, nb, sb);
          if (resb == 1) {
            undecided = 1;
          } else {
            st[rb] = resb == 2 ? 2 : 1;
            und[w] &= ~(1u << (k1 & 31));
          }
        }
      }
    }
    if (undecided) *s_flag = 1;
#ifdef YCX_NMS_PROFILE
    {  // positions this round looked at (undecided at its start), summed over the waves
      int v = 0;
#pragma unroll
      for (int w = 0; w < 4; ++w) v += __popc(und0[w]);
      for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
      if ((tid & 63) == 0) atomicAdd(&g_nms_wprof[6], (unsigned long long)v);
    }
#endif
    __syncthreads();
    const int more = *s_flag;
    __syncthreads();
#ifdef YCX_NMS_PROFILE
    if (tid == 0) atomicAdd(&g_nms_wprof[5], 1ull);
#endif
    if (!more) break;
  }
  YCX_WPROF_MARK(3)
  const int r0 = min(S, tid * E), r1 = min(S, r0 + E);
  int nk = 0;
  for (int r = r0; r < r1; ++r) nk += st[r] == 1 ? 1 : 0;
  int kt;
  int pos = block_exclusive(nk, s_w, &kt);
  for (int r = r0; r < r1; ++r)
    if (st[r] == 1) P.kept[off + pos++] = bucket[r];
  if (tid == 0) P.kc[tk.cls] = kt;
  __syncthreads();
  YCX_WPROF_MARK(4)
}

// Greedy fixed point of a split fast class (one workgroup): the fast path's phases (5)-(7)
// with the ranks by position (u16) and the suppressor lists (CSR) staged in LDS from the
// search's global output, undecided positions tracked per thread as in resolve_wide.
__device__ __forceinline__ void resolve_fast(const Layout& L, char* ws, int t, char* smem,
                                                       int (*s_lv)[5], int* s_w, int* s_flag, const Thr thr,
                                                       float t_lo, float inv_t, int all_pairs) {
  const int tid = threadIdx.x;
  const WFrame* fr = reinterpret_cast<const WFrame*>(ws + L.fframes + (size_t)t * wframe_bytes());
  const unsigned* gcells = reinterpret_cast<const unsigned*>(ws + L.fcells + (size_t)t * fast_cells_bytes());
  if (tid < kFLevels * 5) s_lv[tid / 5][tid % 5] = fr->lv[tid / 5][tid % 5];
  const WFrame f = *fr;
  const Ptrs P = image_ptrs(ws, L, f.img);
  const int S = f.S, off = f.off;
  const f32x4* sbox = P.sbox + off;
  const int* srank = P.srank + off;
  const int* nsup = P.nsup + off;
  const unsigned short* gsl = reinterpret_cast<const unsigned short*>(P.slots + (size_t)off * kSlots);
  unsigned short* lr = reinterpret_cast<unsigned short*>(smem);                              // [S]
  unsigned char* st = reinterpret_cast<unsigned char*>(smem + ((2 * S + 15) & ~15));          // [S]
  unsigned* csr_off = reinterpret_cast<unsigned*>(smem + ((2 * S + 15) & ~15) + ((S + 15) & ~15));  // [S]
  unsigned short* csr_ns = reinterpret_cast<unsigned short*>(csr_off + S);                    // [S]
  unsigned short* csr = csr_ns + ((S + 1) & ~1);                                              // [total]
  const int E = (S + kBigThreads - 1) / kBigThreads;  // <= kFastMax / kBigThreads = 8
  int my_total = 0;
  for (int k = 0; k < E; ++k) {
    const int p = tid + k * kBigThreads;
    if (p < S) {
      lr[p] = (unsigned short)srank[p];
      st[p] = 0;
      my_total += min(nsup[p], kFSlots);
    }
  }
  int total;
  int base = block_exclusive(my_total, s_w, &total);
  const size_t csr_end = (size_t)(((2 * S + 15) & ~15) + ((S + 15) & ~15)) + 4 * (size_t)S + 2 * (size_t)((S + 1) & ~1) +
                         2 * (size_t)total;
  const bool lds_csr = csr_end <= (size_t)kBigLds;
  if (lds_csr) {
    for (int k = 0; k < E; ++k) {
      const int p = tid + k * kBigThreads;
      if (p >= S) break;
      const int ns = nsup[p], c = min(ns, kFSlots);
      for_slots16(gsl + (size_t)p * (2 * kSlots), c, [&](int j, int v) { csr[base + j] = (unsigned short)v; });
      csr_off[p] = base;
      csr_ns[p] = (unsigned short)min(ns, 0xFFFF);
      base += c;
    }
  }
  unsigned und = 0;
  for (int k = 0; k < E; ++k)
    if (tid + k * kBigThreads < S) und |= 1u << k;
  __syncthreads();
  auto cend = [&](int k) { return u16_at(gcells, k); };
  for (int it = 0; it <= S; ++it) {  // every round decides at least one box
    if (tid == 0) *s_flag = 0;
    __syncthreads();
    int undecided = 0;
    unsigned m = und;
    while (m) {
      const int k = __builtin_ctz(m);
      m &= m - 1u;
      const int p = tid + k * kBigThreads;
      const int r = lr[p];
      int ns, res = 0;
      if (lds_csr) {
        ns = csr_ns[p];
        res = csr_state(csr, (int)csr_off[p], min(ns, kFSlots), st);
      } else {
        ns = nsup[p];
        for_slots16(gsl + (size_t)p * (2 * kSlots), min(ns, kFSlots), [&](int, int v) {
          const unsigned char sj = st[v];
          res = res == 2 ? 2 : (sj == 1 ? 2 : (sj == 0 ? 1 : res));
        });
      }
      if (ns > kFSlots && res == 0) {  // the cached ones are all removed: rescan (global copies)
        const f32x4 b = sbox[p];
        const float a = box_area(b);
        const FGeo g = fgeometry(b, f.X0, f.Y0, f.inv, all_pairs);
        bool stop = false;
        f_ranges(cend, s_lv, g, S, t_lo, inv_t, [&](int q0, int q1) {
          for (int q = q0; q < q1 && !stop; ++q) {
            const int rj = srank[q];
            if (rj >= r) continue;
            const unsigned char sj = st[rj];
            if (sj == 2) continue;
            const f32x4 o = sbox[q];
            if (suppress(o[0], o[1], o[2], o[3], box_area(o), b[0], b[1], b[2], b[3], a, thr)) {
              if (sj == 1) { res = 2; stop = true; }
              else res = 1;
            }
          }
        });
      }
      if (res == 1) {
        undecided = 1;
      } else {
        st[r] = res == 2 ? 2 : 1;
        und &= ~(1u << k);
      }
    }
    if (undecided) *s_flag = 1;
    __syncthreads();
    const int more = *s_flag;
    __syncthreads();
    if (!more) break;
  }
  const int r0 = min(S, tid * E), r1 = min(S, r0 + E);
  int nk = 0;
  for (int r = r0; r < r1; ++r) nk += st[r] == 1 ? 1 : 0;
  int kt;
  int pos = block_exclusive(nk, s_w, &kt);
  const int* rank_row = P.bucket + off;
  for (int r = r0; r < r1; ++r)
    if (st[r] == 1) P.kept[off + pos++] = rank_row[r];
  if (tid == 0) P.kc[f.cls] = kt;
  __syncthreads();
}

// Fixed point and compaction of every split class, one workgroup per class (wide classes
// first: the longest items).
__global__ void __launch_bounds__(kBigThreads) __attribute__((amdgpu_waves_per_eu(4))) nms_resolve(
    ycx_nms_desc d, char* ws, Thr thr, float t_lo, float inv_t, int all_pairs) {
  __shared__ __attribute__((aligned(16))) char smem[kBigLds];
  __shared__ int s_lv[kFLevels][5];
  __shared__ int s_w[kBigThreads / 64];
  __shared__ int s_flag;
  const Layout L = layout(d.n, d.rows_total, d.nc);
  const BigList bl = big_list(ws, L, d.n);
  for (int t = blockIdx.x; t < bl.size(); t += gridDim.x) {
    if (t < bl.nwide) {
      const Task tk = bl.wide[t];
      if (tk.S <= kSlot16Max) resolve_wide<true>(L, ws, t, tk, smem, s_lv, s_w, &s_flag, thr, t_lo, inv_t, all_pairs);
      else resolve_wide<false>(L, ws, t, tk, smem, s_lv, s_w, &s_flag, thr, t_lo, inv_t, all_pairs);
    }
    else resolve_fast(L, ws, t - bl.nwide, smem, s_lv, s_w, &s_flag, thr, t_lo, inv_t, all_pairs);
  }
}

// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(kThreads) nms_finish(ycx_nms_desc d, const ycx_cand* __restrict__ cand, char* ws,
                                                       float* __restrict__ dets, int* __restrict__ keep_rows,
                                                       int* __restrict__ keep_counts) {
  __shared__ int s_kc[kMaxNc], s_koff[kMaxNc], s_off[kMaxNc];
  __shared__ int s_total;
  const int img = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int nc = d.nc, rows = d.rows_total;
  const Layout L = layout(d.n, rows, d.nc);
  const Ptrs P = image_ptrs(ws, L, img);
  const ycx_cand* ci = cand + (size_t)img * rows;
  for (int c = tid; c < nc; c += kThreads) { s_kc[c] = P.kc[c]; s_off[c] = P.offs[c]; }
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

#ifdef YCX_NMS_PROFILE
extern "C" int ycx_nms_prof_read(unsigned long long* out, int reset) {  // out[0..15] fast, [16..31] wide
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_nms_prof), sizeof(g_nms_prof)) != hipSuccess) return 1;
  if (hipMemcpyFromSymbol(out + 16, HIP_SYMBOL(g_nms_wprof), sizeof(g_nms_wprof)) != hipSuccess) return 1;  // out[16..31]
  if (reset) {
    unsigned long long z[16] = {};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_nms_prof), z, sizeof(z)) != hipSuccess) return 1;
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_nms_wprof), z, sizeof(z)) != hipSuccess) return 1;
  }
  return 0;
}
#endif

extern "C" size_t ycx_nms_workspace_size(const ycx_nms_desc* d) {
  if (!d || d->n <= 0 || d->rows_total <= 0) return 0;
  const Layout L = layout(d->n, d->rows_total, d->nc);
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
  char* ws = reinterpret_cast<char*>(workspace);
  const Thr t = make_thr(d->iou_thres);
  // Spatial pruning needs IoU > thr to imply overlap and bounded size ratios,
  // i.e. thr >= 0; a negative or NaN threshold compares every pair.
  const int all_pairs = !(d->iou_thres >= 0.0);
  const float t_lo = all_pairs ? 0.0f : (float)(fmin(d->iou_thres, 1.0) * (1.0 - 1e-3));
  const float inv_t = t_lo > 0.0f ? 1.0f / t_lo : INFINITY;
  {  // the row-slice class counts and the candidate flags (adjacent in the layout)
    const Layout L = layout(d->n, d->rows_total, d->nc);
    if (hipMemsetAsync(ws + L.bcnt, 0, L.bits + (size_t)d->n * d->rows_total - L.bcnt, st) != hipSuccess)
      return YCX_ERR_LAUNCH;
  }
  hipLaunchKernelGGL(nms_mark, dim3(kPrepB, d->n), dim3(kThreads), (size_t)kPrepB * d->nc * sizeof(unsigned), st, *d,
                     cand, cand_rows, cand_counts, ws);
  hipLaunchKernelGGL(nms_bucket, dim3(kPrepB, d->n), dim3(kThreads), 0, st, *d, cand, cand_rows, cand_counts, ws);
  hipLaunchKernelGGL(nms_prep, dim3(kPrepClsB, d->n), dim3(kThreads), 0, st, *d, cand, ws, t);
  // one width for every fast class: the radix sort and the per-element loops skip the
  // elements past S, so E = 8 costs a small class little, and one launch replaces four;
  // with the wide classes' sort + spatial index (nms_wide_a's work) in the same launch: at C4
  // the 24 wide and 24 fast classes of a batch then run side by side instead of in turn
  // (YCX_NMS_NO_FAST: every class on the wide path, the fast list empty)
  hipLaunchKernelGGL(nms_fast<8>, dim3(kBigBlocks), dim3(kBigThreads), 0, st, *d, cand, ws, t, t_lo, inv_t, all_pairs, 1);
  hipLaunchKernelGGL(nms_search, dim3(kSearchBlocks), dim3(kBigThreads), 0, st, *d, ws, t, t_lo, inv_t, all_pairs);
  hipLaunchKernelGGL(nms_resolve, dim3(kBigBlocks), dim3(kBigThreads), 0, st, *d, ws, t, t_lo, inv_t, all_pairs);
  hipLaunchKernelGGL(nms_finish, dim3(d->n), dim3(kThreads), 0, st, *d, cand, ws, dets, keep_rows, keep_counts);
  return ycx_launch_status();
}
