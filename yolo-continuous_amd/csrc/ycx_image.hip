// Image-side pre/post steps of detect.py around the network:
//   ycx_letterbox      detect.py:16-26 + image_enhance/letter_box.py:27-60
//                      (uint8 HWC -> bilinear resize -> 114 border -> fp32 CHW / 255)
//   ycx_correct_boxes  detect.py:139-165 (yolo_correct_boxes on the NMS output)
// Both reproduce the host arithmetic exactly: double where numpy promotes to
// float64, fp32 where it stays fp32, no FMA contraction.
#pragma clang fp contract(off)
#include <math.h>
#include "ycx_internal.h"

namespace {

// blockIdx.y: image of a batch (src advanced by src_image_stride bytes, dst by one
// c x out_h x out_w image)
__global__ void __launch_bounds__(256) letterbox_kernel(ycx_letterbox_desc d, const uint8_t* __restrict__ src,
                                                        float* __restrict__ dst, long long src_image_stride) {
  const int idx = blockIdx.x * 256 + threadIdx.x;
  const int plane = d.out_h * d.out_w;
  if (idx >= plane) return;
  src += (size_t)blockIdx.y * src_image_stride;
  dst += (size_t)blockIdx.y * d.c * plane;
  const int oy = idx / d.out_w, ox = idx - oy * d.out_w;
  const int cy = oy - d.top, cx = ox - d.left;
  const bool inside = (unsigned)cy < (unsigned)d.new_h && (unsigned)cx < (unsigned)d.new_w;
  for (int c = 0; c < d.c; ++c) {
    int v = d.pad;
    if (inside) {
      if (d.new_w == d.w0 && d.new_h == d.h0) {
        v = src[(size_t)cy * d.src_row_stride + (size_t)cx * d.c + c];
      } else {
        // resize_bilinear: half-pixel centres, edge clamp, float64 weights
        const double sx = (double)d.w0 / (double)d.new_w, sy = (double)d.h0 / (double)d.new_h;
        const double xs = ((double)cx + 0.5) * sx - 0.5, ys = ((double)cy + 0.5) * sy - 0.5;
        const double fxs = floor(xs), fys = floor(ys);
        const int x0 = (int)fmin(fmax(fxs, 0.0), (double)(d.w0 - 1));
        const int y0 = (int)fmin(fmax(fys, 0.0), (double)(d.h0 - 1));
        const int x1 = min(x0 + 1, d.w0 - 1), y1 = min(y0 + 1, d.h0 - 1);
        const double fx = fmin(fmax(xs - fxs, 0.0), 1.0), fy = fmin(fmax(ys - fys, 0.0), 1.0);
        const uint8_t* r0 = src + (size_t)y0 * d.src_row_stride;
        const uint8_t* r1 = src + (size_t)y1 * d.src_row_stride;
        const double p00 = (double)(float)r0[(size_t)x0 * d.c + c], p01 = (double)(float)r0[(size_t)x1 * d.c + c];
        const double p10 = (double)(float)r1[(size_t)x0 * d.c + c], p11 = (double)(float)r1[(size_t)x1 * d.c + c];
        const double top = p00 * (1.0 - fx) + p01 * fx;
        const double bot = p10 * (1.0 - fx) + p11 * fx;
        const double val = rint(top * (1.0 - fy) + bot * fy);
        v = (int)fmin(fmax(val, 0.0), 255.0);
      }
    }
    dst[(size_t)c * plane + idx] = (float)v / 255.0f;  // astype(float32) / 255.
  }
}

__global__ void __launch_bounds__(256) correct_boxes_kernel(ycx_correct_desc d, float* __restrict__ dets,
                                                            const int32_t* __restrict__ counts,
                                                            const int32_t* __restrict__ image_hw) {
  const int idx = blockIdx.x * 256 + threadIdx.x;
  if (idx >= d.n * d.max_det) return;
  const int img = idx / d.max_det, k = idx - img * d.max_det;
  if (k >= min(counts[img], d.max_det)) return;
  float* o = dets + (size_t)idx * 7;
  // box_xy, box_wh = (o[:, 0:2] + o[:, 2:4]) / 2, o[:, 2:4] - o[:, 0:2]   (fp32)
  const float bx = (o[0] + o[2]) / 2.0f, by = (o[1] + o[3]) / 2.0f;
  const float bw = o[2] - o[0], bh = o[3] - o[1];
  // yolo_correct_boxes: yx / hw order. numpy promotes the centres to float64
  // ((box_yx - offset) * scale is a new array), but `box_hw *= scale` is in
  // place on the float32 array and `box_hw / 2.` stays float32.
  double yx0 = by, yx1 = bx;
  float hw0 = bh, hw1 = bw;
  const double ih = image_hw[2 * img], iw = image_hw[2 * img + 1];
  if (d.letterbox) {
    const double in_h = d.input_h, in_w = d.input_w;
    const double m = fmin(in_h / ih, in_w / iw);                    // np.min(input_shape / image_shape)
    const double nh = rint(ih * m), nw = rint(iw * m);               // np.round(image_shape * ...)
    const double off0 = (in_h - nh) / 2.0 / in_h, off1 = (in_w - nw) / 2.0 / in_w;
    const double s0 = in_h / nh, s1 = in_w / nw;
    yx0 = (yx0 - off0) * s0;
    yx1 = (yx1 - off1) * s1;
    hw0 = (float)((double)hw0 * s0);
    hw1 = (float)((double)hw1 * s1);
  }
  const float h2 = hw0 / 2.0f, w2 = hw1 / 2.0f;
  double mn0, mn1, mx0, mx1;
  if (d.letterbox) {  // float64 centres
    mn0 = yx0 - h2; mn1 = yx1 - w2;
    mx0 = yx0 + h2; mx1 = yx1 + w2;
  } else {            // everything still float32 until `boxes *= image_shape`
    mn0 = (float)yx0 - h2; mn1 = (float)yx1 - w2;
    mx0 = (float)yx0 + h2; mx1 = (float)yx1 + w2;
  }
  o[0] = (float)(mn0 * ih);
  o[1] = (float)(mn1 * iw);
  o[2] = (float)(mx0 * ih);
  o[3] = (float)(mx1 * iw);
}

}  // namespace

extern "C" ycx_status ycx_letterbox_batch(const ycx_letterbox_desc* d, int32_t n, int64_t src_image_stride,
                                          const uint8_t* src, float* dst, void* stream) {
  YCX_CHECK_ARG(d && src && dst && n > 0 && n <= 65535);
  YCX_CHECK_ARG(d->h0 > 0 && d->w0 > 0 && d->c > 0 && d->c <= 4 && d->src_row_stride >= d->w0 * d->c);
  YCX_CHECK_ARG(d->new_h > 0 && d->new_w > 0 && d->top >= 0 && d->left >= 0);
  YCX_CHECK_ARG(d->top + d->new_h <= d->out_h && d->left + d->new_w <= d->out_w);
  YCX_CHECK_ARG(d->pad >= 0 && d->pad <= 255);
  YCX_CHECK_ARG(n == 1 || src_image_stride >= (int64_t)d->h0 * d->src_row_stride);
  const long long plane = (long long)d->out_h * d->out_w;
  YCX_CHECK_SUPPORTED(plane * d->c < (1LL << 31));
  hipLaunchKernelGGL(letterbox_kernel, dim3(ycx_cdiv(plane, 256), (unsigned)n), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), *d, src, dst, (long long)src_image_stride);
  return ycx_launch_status();
}

extern "C" ycx_status ycx_letterbox(const ycx_letterbox_desc* d, const uint8_t* src, float* dst, void* stream) {
  return ycx_letterbox_batch(d, 1, 0, src, dst, stream);
}

extern "C" ycx_status ycx_correct_boxes(const ycx_correct_desc* d, float* dets, const int32_t* counts,
                                        const int32_t* image_hw, void* stream) {
  YCX_CHECK_ARG(d && dets && counts && image_hw);
  YCX_CHECK_ARG(d->n > 0 && d->max_det > 0 && d->input_h > 0 && d->input_w > 0);
  hipLaunchKernelGGL(correct_boxes_kernel, dim3(ycx_cdiv((long long)d->n * d->max_det, 256)), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), *d, dets, counts, image_hw);
  return ycx_launch_status();
}
