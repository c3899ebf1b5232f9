/* ORACLE (test infrastructure only): greedy NMS restated in C for speed.
 *
 * The same algorithm as oracle/ref_post.py:nms, which restates
 * torchvision.ops.nms as called at detect.py:133 (torchvision's published CPU
 * kernel, torchvision/csrc/ops/cpu/nms_kernel.cpp; torchvision is absent here
 * and unpinned, so this primitive is PARITY UNPINNED):
 *   areas = (x2 - x1) * (y2 - y1)                      fp32
 *   order = stable descending sort of the scores       ties keep input order, NaN last
 *   for i in order, unless suppressed: keep i; suppress every later j with
 *     (float)(w*h) / (float)(area_i + area_j - w*h) > iou_threshold   (fp32 ratio,
 *     compared in double), w = max(0, min(x2) - max(x1)), h likewise.
 * Every float operation is the one numpy performs on float32 arrays in
 * ref_post.nms; build with -ffp-contract=off (no FMA contraction) so the
 * roundings are identical. Used by the tests and bench.py's cpu_baseline leg
 * only, never by the product path. */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

static const float* g_scores;

/* numpy's float32 maximum / minimum: a NaN operand propagates */
static inline float np_max(float a, float b) { return (isnan(a) || a > b) ? a : b; }
static inline float np_min(float a, float b) { return (isnan(a) || a < b) ? a : b; }

/* argsort(-scores, kind='stable') order: key = -score ascending, NaN last */
static inline int before(float sj, float si) {
  const float kj = -sj, ki = -si;
  if (isnan(kj)) return 0;
  if (isnan(ki)) return 1;
  return kj < ki;
}

static void merge_sort(int64_t* a, int64_t* tmp, int64_t n) {
  if (n < 2) return;
  int64_t h = n / 2;
  merge_sort(a, tmp, h);
  merge_sort(a + h, tmp, n - h);
  int64_t i = 0, j = h, k = 0;
  while (i < h && j < n) {
    /* descending; on equal scores the earlier index first (stable) */
    if (before(g_scores[a[j]], g_scores[a[i]])) tmp[k++] = a[j++];
    else tmp[k++] = a[i++];
  }
  while (i < h) tmp[k++] = a[i++];
  while (j < n) tmp[k++] = a[j++];
  memcpy(a, tmp, (size_t)n * sizeof(int64_t));
}

/* boxes [n][4] xyxy fp32, scores [n] fp32; writes the kept indices (score
 * order) to keep[] and returns their count, or -1 on allocation failure. */
int64_t ycx_oracle_nms(const float* boxes, const float* scores, int64_t n, double iou_threshold, int64_t* keep) {
  if (n <= 0) return 0;
  int64_t* order = (int64_t*)malloc((size_t)n * sizeof(int64_t));
  int64_t* tmp = (int64_t*)malloc((size_t)n * sizeof(int64_t));
  float* areas = (float*)malloc((size_t)n * sizeof(float));
  unsigned char* sup = (unsigned char*)calloc((size_t)n, 1);
  if (!order || !tmp || !areas || !sup) {
    free(order); free(tmp); free(areas); free(sup);
    return -1;
  }
  for (int64_t i = 0; i < n; ++i) {
    order[i] = i;
    const float* b = boxes + 4 * i;
    areas[i] = (b[2] - b[0]) * (b[3] - b[1]);
  }
  g_scores = scores;
  merge_sort(order, tmp, n);
  int64_t nk = 0;
  for (int64_t a = 0; a < n; ++a) {
    const int64_t i = order[a];
    if (sup[i]) continue;
    keep[nk++] = i;
    const float* bi = boxes + 4 * i;
    for (int64_t c = a + 1; c < n; ++c) {
      const int64_t j = order[c];
      if (sup[j]) continue;
      const float* bj = boxes + 4 * j;
      const float xx1 = np_max(bi[0], bj[0]);
      const float yy1 = np_max(bi[1], bj[1]);
      const float xx2 = np_min(bi[2], bj[2]);
      const float yy2 = np_min(bi[3], bj[3]);
      const float w = np_max(0.0f, xx2 - xx1), h = np_max(0.0f, yy2 - yy1);
      const float inter = w * h;
      const float den = (areas[i] + areas[j]) - inter;
      const float ovr = inter / den;
      if ((double)ovr > iou_threshold) sup[j] = 1;
    }
  }
  free(order); free(tmp); free(areas); free(sup);
  return nk;
}
