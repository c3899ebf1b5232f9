/* Host-side AddressSanitizer/UBSan driver for libycx_hip's host code.
 * Built by `make -C yolo-continuous_amd/csrc asan` from --offload-host-only objects
 * (no device code) and run on the CPU by tests/test_native_asan.py. It walks every
 * host path that runs before a launch: struct sizes, status strings, the tile
 * heuristic on the yolov7 640 conv list, the XCD tile-map
 * bijection, NMS workspace sizing, and descriptor validation that must reject bad
 * arguments without launching. Prints "abi_check ok" and exits 0 when every check
 * holds; ASan/UBSan abort the process on a memory or UB error. */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "ycx.h"

static int fails = 0;
#define EXPECT(c)                                            \
  do {                                                       \
    if (!(c)) {                                              \
      fprintf(stderr, "FAIL %s:%d %s\n", __FILE__, __LINE__, #c); \
      ++fails;                                               \
    }                                                        \
  } while (0)

static ycx_conv_desc conv(int n, int h, int w, int cin, int cout, int k, int s) {
  ycx_conv_desc d;
  memset(&d, 0, sizeof d);
  d.n = n; d.h = h; d.w = w; d.cin = cin; d.in_c_stride = cin;
  d.kh = d.kw = k; d.stride = s; d.pad = k / 2;
  d.ho = (h + 2 * d.pad - k) / s + 1; d.wo = (w + 2 * d.pad - k) / s + 1;
  d.cout = cout; d.cout_pad = (cout + 127) / 128 * 128; d.out_c_stride = cout;
  d.act = YCX_ACT_SILU; d.dtype = YCX_DT_BF16; d.out_layout = YCX_OUT_NHWC;
  d.out_scale = 1.0f; d.res_scale = 1.0f;
  return d;
}

int main(void) {
  EXPECT(ycx_abi_version() == YCX_ABI_VERSION);
  const size_t want[12] = {sizeof(ycx_conv_desc), sizeof(ycx_pool_desc), sizeof(ycx_copy_desc),
                           sizeof(ycx_decode_desc), sizeof(ycx_cand), sizeof(ycx_filter_desc),
                           sizeof(ycx_decode_filter_desc), sizeof(ycx_nms_desc), sizeof(ycx_op),
                           sizeof(ycx_letterbox_desc), sizeof(ycx_correct_desc), sizeof(ycx_head_desc)};
  for (int i = 0; i < 12; ++i) EXPECT(ycx_struct_size(i) == want[i]);
  EXPECT(ycx_struct_size(12) == 0 && ycx_struct_size(-1) == 0);
  for (int s = -1; s <= 5; ++s) EXPECT(ycx_strerror(s) != NULL && strlen(ycx_strerror(s)) > 0);
  for (int t = -2; t < 64; ++t) EXPECT(ycx_conv_tile_name(t) != NULL);

  /* the tile heuristic over yolov7's conv shapes at 640, bs 1 and 32 */
  static const int shapes[][6] = {
      {640, 640, 3, 32, 3, 1},    {640, 640, 32, 64, 3, 2},  {320, 320, 64, 64, 3, 1},
      {320, 320, 64, 128, 3, 2},  {160, 160, 128, 64, 1, 1}, {160, 160, 64, 64, 3, 1},
      {160, 160, 256, 256, 1, 1}, {80, 80, 128, 128, 3, 1},  {80, 80, 512, 512, 1, 1},
      {40, 40, 256, 256, 3, 1},   {40, 40, 1024, 1024, 1, 1}, {20, 20, 512, 512, 3, 1},
      {20, 20, 2048, 512, 1, 1},  {20, 20, 1024, 255, 1, 1}, {80, 80, 256, 255, 1, 1}};
  for (int b = 0; b < 2; ++b)
    for (size_t i = 0; i < sizeof shapes / sizeof shapes[0]; ++i) {
      ycx_conv_desc d = conv(b ? 32 : 1, shapes[i][0], shapes[i][1], shapes[i][2], shapes[i][3], shapes[i][4],
                             shapes[i][5]);
      const int t = ycx_conv_pick_tile(&d);
      EXPECT(t >= 0 && t < 64);
      d.res_c_stride = d.cout;
      EXPECT(ycx_conv_pick_tile(&d) >= 0);
      d.dtype = YCX_DT_F32;
      EXPECT(ycx_conv_pick_tile(&d) >= 0);
    }

  /* the XCD region map is a bijection of [0, nwg) onto the tile grid */
  static const int grids[][2] = {{8, 800}, {4, 100}, {16, 50}, {2, 13}, {8, 7}, {1, 1}};
  for (size_t g = 0; g < sizeof grids / sizeof grids[0]; ++g)
    for (int gc = 0; gc <= 8; gc = gc ? gc * 2 : 1) {
      const int n_ct = grids[g][0], nwg = n_ct * grids[g][1];
      char* seen = (char*)calloc((size_t)nwg, 1);
      for (int b = 0; b < nwg; ++b) {
        const int v = ycx_conv_tile_of(b, nwg, n_ct, gc); /* ct * 65536 + pt */
        const int ct = v >> 16, pt = v & 0xFFFF, id = ct * (nwg / n_ct) + pt;
        EXPECT(v >= 0 && ct < n_ct && pt < nwg / n_ct);
        if (v >= 0 && id < nwg) seen[id]++;
      }
      for (int i = 0; i < nwg; ++i) EXPECT(seen[i] == 1);
      free(seen);
    }

  /* NMS workspace sizing: grows with the problem, zero/overflow-safe */
  ycx_nms_desc nd;
  memset(&nd, 0, sizeof nd);
  nd.n = 32; nd.rows_total = 25200; nd.nc = 80; nd.max_det = 300;
  const size_t w1 = ycx_nms_workspace_size(&nd);
  nd.rows_total = 100800;
  const size_t w2 = ycx_nms_workspace_size(&nd);
  EXPECT(w1 > 0 && w2 > w1);
  EXPECT(ycx_conv_tile_of(0, 10, 3, 2) == -1); /* nwg not a multiple of n_ct */

  /* validation rejects bad arguments before any launch */
  ycx_conv_desc d = conv(1, 40, 40, 256, 256, 3, 1);
  char dummy[64];
  EXPECT(ycx_conv2d(NULL, dummy, dummy, (const float*)dummy, dummy, NULL, NULL) != YCX_OK);
  EXPECT(ycx_conv2d(&d, NULL, dummy, (const float*)dummy, dummy, NULL, NULL) != YCX_OK);
  ycx_conv_desc bad = d;
  bad.ho = 7; /* inconsistent with h, k, s, pad */
  EXPECT(ycx_conv2d(&bad, dummy, dummy, (const float*)dummy, dummy, NULL, NULL) != YCX_OK);
  bad = d;
  bad.in_c_off = 8; /* slice past the stride */
  EXPECT(ycx_conv2d(&bad, dummy, dummy, (const float*)dummy, dummy, NULL, NULL) != YCX_OK);
  bad = d;
  bad.cout_pad = 100;
  EXPECT(ycx_conv2d(&bad, dummy, dummy, (const float*)dummy, dummy, NULL, NULL) != YCX_OK);
  ycx_pool_desc pd;
  memset(&pd, 0, sizeof pd);
  EXPECT(ycx_maxpool(&pd, dummy, dummy, NULL) != YCX_OK);
  EXPECT(ycx_maxpool(NULL, dummy, dummy, NULL) != YCX_OK);
  ycx_copy_desc cd;
  memset(&cd, 0, sizeof cd);
  EXPECT(ycx_copy_channels(&cd, dummy, dummy, NULL) != YCX_OK);
  EXPECT(ycx_run_ops(NULL, 1, NULL, NULL) != YCX_OK);
  EXPECT(ycx_run_ops((const ycx_op*)dummy, 0, NULL, NULL) == YCX_OK); /* empty plan: nothing to launch */
  uint32_t oob[2] = {7, 7};
  EXPECT(ycx_debug_bounds(oob, 0) == YCX_ERR_UNSUPPORTED && oob[0] == 0); /* release build */
  EXPECT(ycx_debug_bounds(NULL, 0) == YCX_ERR_BAD_ARG);
  EXPECT(ycx_set_trace(0) == YCX_OK);
  {
    /* roctx is resolved at run time (dlopen), not at link time: a build host without the
       profiler SDK gets YCX_ERR_UNSUPPORTED and tracing stays off */
    ycx_status st = ycx_set_trace(1);
    EXPECT(st == YCX_OK || st == YCX_ERR_UNSUPPORTED);
    EXPECT(ycx_set_trace(0) == YCX_OK);
  }

  if (fails) {
    fprintf(stderr, "abi_check: %d failures\n", fails);
    return 1;
  }
  printf("abi_check ok\n");
  return 0;
}
