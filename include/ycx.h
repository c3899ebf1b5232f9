/*
 * ycx.h — C ABI of libycx_hip.so, the MI355X (gfx950) YOLO inference hot path.
 *
 * Every entry point is `extern "C"`, takes plain pointers/sizes, returns an
 * int32 status (0 = OK) and launches asynchronously on the caller's HIP
 * stream (passed as `void*`, i.e. a hipStream_t). The library never allocates
 * device memory on the hot path: activations, packed weights, workspaces and
 * outputs are owned by the caller (PyTorch's caching allocator in the Python
 * host package).
 *
 * Reference interfaces each entry point replaces (xin-pu/yolo-continuous):
 *   ycx_conv2d          Conv.forward = act(bn(conv2d(x)))      nets/common.py:97-109
 *                       RepConv.forward (re-parameterised)      nets/common.py:477-495
 *                       Detect head 1x1 convs (bias, no act)    nets/detect.py:27-38
 *                       IDetect conv + ImplicitA/M (folded)     nets/idetect.py:26-31
 *   ycx_stem_conv       first Conv on the fp32 NCHW image       nets/common.py:105-106 (Cin=3)
 *   ycx_stem_conv2      first two Convs fused (3->32, then 3x3   cfg/net/yolov7.yaml:7-8,
 *                       stride 2 -> 64); the stem output stays   nets/common.py:97-109
 *                       in LDS
 *   ycx_maxpool         MP / SP / SPPCSPC max-pools             nets/common.py:25-40, 257
 *   ycx_copy_channels   nn.Upsample(None, 2, 'nearest')         cfg/net/yolov7.yaml:71,85
 *                       Concat (only when a slice cannot alias)  nets/common.py:54-60
 *   ycx_decode          decode_box (one head level)             detect.py:29-87
 *   ycx_filter_decoded  non_max_suppression lines 98-121        detect.py:98-121
 *   ycx_decode_filter   decode_box + the same filter, fused     detect.py:29-121
 *   ycx_conv2d_head     Detect head conv (one level) fused with  nets/detect.py:27-38 +
 *                       decode_box + the candidate filter        detect.py:29-121
 *   ycx_idetect_decode  IDetect eval branch (strides supplied)  nets/idetect.py:33-45
 *   ycx_sort_nms        per-class torchvision.ops.nms loop      detect.py:124-137
 *   ycx_run_ops         Model.forward layer loop                nets/yolo.py:143-153
 *   ycx_letterbox       image -> network input                   detect.py:16-26,
 *                                                                image_enhance/letter_box.py:27-60
 *   ycx_correct_boxes   yolo_correct_boxes on the NMS output     detect.py:139-165
 */
#ifndef YCX_H_
#define YCX_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define YCX_ABI_VERSION 9

typedef int32_t ycx_status;
enum {
  YCX_OK = 0,
  YCX_ERR_BAD_ARG = 1,      /* null pointer, negative size, inconsistent shape  */
  YCX_ERR_UNSUPPORTED = 2,  /* shape/dtype the kernels do not implement          */
  YCX_ERR_LAUNCH = 3,       /* hipGetLastError() after a launch was not success   */
  YCX_ERR_CAPACITY = 4      /* workspace / output capacity too small              */
};

/* YCX_DT_FP8: OCP e4m3fn activations and weights (CDNA4 block-scaled MFMA with
 * unit block scales, fp32 accumulate). Each activation buffer carries one
 * power-of-two scale s (stored byte = e4m3(clamp(v * s, +-448))); weights
 * carry one per output channel (see ycx_conv_desc).
 * YCX_DT_F16: IEEE half activations and weights, fp32 accumulate: the bf16
 * kernels on the f16 MFMA (same rate, 11-bit significand): the precision mode
 * that holds north_star's 1e-3 at bf16 speed. Activations must stay below
 * 65504 in magnitude (fp16 range). */
enum { YCX_DT_BF16 = 0, YCX_DT_F32 = 1, YCX_DT_FP8 = 2, YCX_DT_F16 = 3 };
/* YCX_ACT_SILU_PS: SiLU of a conv whose packed weights and bias were pre-multiplied by
 * k = -log2(e) (fp8: the fp32 bias and dequantisation rows instead), so the epilogue holds
 * c' = k c and computes silu(c) = c' / (k (1 + 2^c')) = c' * rcp(fma(2^c', k, k)) -- one
 * exp, one fma, one rcp and one multiply per value instead of a multiply more (r06). The
 * 16-bit and fp8 kernels; not the fp32 parity path. */
enum { YCX_ACT_NONE = 0, YCX_ACT_SILU = 1, YCX_ACT_LEAKY = 2, YCX_ACT_SILU_PS = 3 };
enum {
  YCX_OUT_NHWC = 0,       /* activation dtype, [N][Ho][Wo][out_c_stride] at out_c_off         */
  YCX_OUT_NCHW_F32 = 1,   /* fp32 [N][out_c_stride][Ho][Wo] at out_c_off (Detect raw logits)   */
  YCX_OUT_NHWC_UP2 = 2    /* activation dtype, each pixel written to its 2x2 block of a
                             [N][2Ho][2Wo][out_c_stride] buffer (conv fused with nearest x2)   */
};

/* Convolution: NHWC activations, weights packed [cout_pad][kh][kw][cin] in the
 * activation dtype, fp32 bias[cout_pad] (BN folded in). groups = 1.
 * YCX_DT_FP8: weight rows are zero-padded to a multiple of 128 bytes
 * ([cout_pad][ceil(kh*kw*cin / 128) * 128] e4m3 of w * s_w[co]); bias points
 * to fp32 [2 * cout_pad]: the bias, then dq[co] = 1 / (s_w[co] * s_x); the
 * epilogue computes act(acc * dq + bias) (+ residual * res_scale) and stores
 * e4m3(clamp(v * out_scale)) (fp32 NCHW head outputs: unscaled). The stem
 * (ycx_stem_conv) reads the fp32 image with fp32 weights and only its output
 * is e4m3 (out_scale). cout_pad % 64 == 0 and cin in {32, 64, 128k}. */
typedef struct ycx_conv_desc {
  int32_t n, h, w, cin, in_c_off, in_c_stride;
  int32_t ho, wo, cout, cout_pad, out_c_off, out_c_stride;
  int32_t kh, kw, stride, pad;
  int32_t act;              /* YCX_ACT_*                                           */
  float leaky_slope;        /* for YCX_ACT_LEAKY (0.1 in yolov7-tiny.yaml)          */
  int32_t dtype;            /* YCX_DT_*: activations & weights                     */
  int32_t out_layout;       /* YCX_OUT_*                                            */
  int32_t res_c_off, res_c_stride; /* residual (same dtype/shape as the output)   */
  int32_t tile;             /* 0 = auto, else a tile id (see ycx_conv_tile_name)    */
  float out_scale;          /* YCX_DT_FP8 only: output quantisation scale          */
  float res_scale;          /* YCX_DT_FP8 only: residual dequantisation (1 / s_res) */
  int32_t in_pool;          /* 1: x is the (2h, 2w) map that MP's k2 s2 max-pool reduces to the
                             * (h, w) input (nets/common.py:25-31), pooled in the conv's operand
                             * staging (1x1/s1/p0: 16-bit with cin % 64 == 0, or YCX_DT_FP8
                             * with cin % 128 == 0, r04); 0: x is the input */
  int32_t k_split;          /* > 1: the K loop (kh*kw*cin) is cut into k_split contiguous ranges run by
                             * separate workgroups, whose fp32 partial sums go to a caller-owned
                             * workspace (ycx_conv2d_ws, ycx_conv_workspace_size) and are summed in a
                             * fixed order by a second launch (bias, act, residual, store): deterministic.
                             * 16-bit LDS-DMA tiles only (16, 18, 56), r06. 0 or 1: no split */
} ycx_conv_desc;

/* Max-pool, NHWC, pad value -inf (torch.nn.MaxPool2d semantics, floor mode).
 * YCX_DT_FP8: input and output share one scale (max commutes with it). */
typedef struct ycx_pool_desc {
  int32_t n, h, w, c, in_c_off, in_c_stride;
  int32_t ho, wo, out_c_off, out_c_stride;
  int32_t k, stride, pad;
  int32_t dtype;
  /* levels > 1: a cascade of `levels` identical 'same' pools (stride 1, pad k/2) in one
   * launch, pool i of pool i-1 (SPPCSPC's 5/9/13 as 5, 5o5, 5o5o5: nets/common.py:257),
   * level i written to channels out_c_off + i*c of y. 0 or 1: one pool. */
  int32_t levels;
} ycx_pool_desc;

/* Channel-slice copy with optional nearest x2 upsample (scale = 1 or 2).
 * out_layout YCX_OUT_NHWC keeps the dtype; YCX_OUT_NCHW_F32 writes fp32
 * [N][out_c_stride][Ho][Wo] (a model output that is not a Detect head). */
typedef struct ycx_copy_desc {
  int32_t n, h, w, c, in_c_off, in_c_stride;
  int32_t out_c_off, out_c_stride;
  int32_t scale;
  int32_t dtype;
  int32_t out_layout;
  float dequant;            /* YCX_DT_FP8 with YCX_OUT_NCHW_F32: 1 / s_in (else unused) */
} ycx_copy_desc;

/* Decode of one head level (detect.py:29-87 semantics). head is fp32 NCHW
 * [n][na*no][h][w]; out is fp32 [n][rows_total][no], written at row_off.
 * anchors_scaled[2a], [2a+1] = anchor_w/stride_w, anchor_h/stride_h computed in
 * double and rounded to fp32 exactly as detect.py:43-44 does. */
typedef struct ycx_decode_desc {
  int32_t n, h, w, na, no;
  int32_t rows_total, row_off;
  float anchors_scaled[16];
} ycx_decode_desc;

/* One NMS candidate (32 bytes): normalised xyxy box, objectness, best class
 * confidence, best class id, row index into the concatenated [rows_total]. */
typedef struct ycx_cand {
  float x1, y1, x2, y2;
  float obj, cls_conf;
  int32_t cls, row;
} ycx_cand;

/* Filter of a decoded [n][rows][no] tensor (detect.py:98-121): xywh -> xyxy in
 * place, class max (first index on ties), score = obj*cls_conf >= conf_thres. */
typedef struct ycx_filter_desc {
  int32_t n, rows, no, nc;
  float conf_thres;         /* compared in fp32, as torch does for a float32 tensor */
  int32_t write_xyxy;       /* 1: mutate pred[..., :4] to xyxy like detect.py:103  */
} ycx_filter_desc;

/* Fused decode + filter straight from the three fp32 NCHW head tensors. */
typedef struct ycx_decode_filter_desc {
  int32_t n, nl, na, no, nc;
  int32_t h[4], w[4];       /* per level, in head order (P5, P4, P3 for Detect)    */
  int32_t row_off[4];       /* first row of each level in the concatenated rows    */
  int32_t rows_total;
  float anchors_scaled[4][16];
  float conf_thres;
} ycx_decode_filter_desc;

/* Per-image, per-class greedy NMS with torchvision.ops.nms semantics. */
typedef struct ycx_nms_desc {
  int32_t n, rows_total, nc;
  int32_t max_det;          /* output rows per image (padded); counts are not capped */
  double iou_thres;         /* compared as (double)iou > iou_thres, like torchvision */
} ycx_nms_desc;

/* Letterbox of one uint8 HWC image (BGR kept, as detect.py feeds it) into an
 * fp32 CHW network input: bilinear resize to new_h x new_w (half-pixel
 * centres, edge clamp, float64 weights, round-half-even to uint8), content at
 * (top, left) of out_h x out_w, border value `pad`, then value / 255 in fp32.
 * The host computes the geometry (round(w r) etc.) like letter_box.py. */
typedef struct ycx_letterbox_desc {
  int32_t h0, w0, c;          /* source image (c <= 4)                     */
  int32_t src_row_stride;     /* bytes between source rows (>= w0 * c)     */
  int32_t out_h, out_w;       /* letterboxed size                          */
  int32_t new_h, new_w;       /* resized content size                      */
  int32_t top, left;          /* content offset                            */
  int32_t pad;                /* border value, 114 in the reference        */
} ycx_letterbox_desc;

/* yolo_correct_boxes (detect.py:139-165) applied in place to the padded NMS
 * output dets[n][max_det][7]: rows 0..min(counts[i], max_det) become
 * [y1, x1, y2, x2] in original-image pixels (float64 math, stored fp32, as
 * numpy does). image_hw: [n][2] int32 original (h, w) per image. */
typedef struct ycx_correct_desc {
  int32_t n, max_det;
  int32_t input_h, input_w;   /* network input size                        */
  int32_t letterbox;          /* letterbox_image flag                      */
} ycx_correct_desc;

/* Decode + candidate filter of one Detect head level, fused into the head's
 * 1x1 conv (ycx_conv2d_head): the fp32 logits of a tile never leave the CU.
 * Candidates are the same as ycx_decode_filter's for this level (same float
 * operations in the same order): rows row_off + a * h * w + cell. */
typedef struct ycx_head_desc {
  int32_t na, no, nc;           /* anchors, outputs per anchor (nc + 5), classes      */
  int32_t rows_total, row_off;  /* candidate rows per image (all levels), this level's */
  float conf_thres;             /* obj * cls_conf >= conf_thres, compared in fp32     */
  float anchors_scaled[16];     /* as ycx_decode_desc                                 */
} ycx_head_desc;

/* A pre-built op for ycx_run_ops (the static execution plan of Model.forward). */
enum { YCX_OP_CONV = 1, YCX_OP_STEM = 2, YCX_OP_POOL = 3, YCX_OP_COPY = 4, YCX_OP_STEM2 = 5, YCX_OP_HEAD = 6,
       YCX_OP_CONV_PAIR = 7 };
typedef struct ycx_op {
  int32_t kind;
  int32_t pad_;
  union {
    ycx_conv_desc conv;
    ycx_pool_desc pool;
    ycx_copy_desc copy;
    ycx_conv_desc pair[2];  /* STEM2: [0] the stem, [1] the stride-2 conv it feeds;
                               CONV_PAIR: [0] the first 1x1 conv, [1] the 1x1 conv reading it */
    struct {
      ycx_conv_desc conv;
      ycx_head_desc head;
    } head;                 /* HEAD: the head conv and its level's decode           */
  } d;
  const void* in;           /* x                                                    */
  const void* weight;       /* packed weights (conv/stem; STEM2: the stem's)        */
  const float* bias;        /* bias (conv/stem; STEM2: the stem's)                  */
  void* out;                /* y                                                    */
  const void* residual;     /* optional residual (conv)                             */
  const void* weight2;      /* STEM2 / CONV_PAIR: the second conv's packed weights  */
  const float* bias2;       /* STEM2 / CONV_PAIR: the second conv's bias            */
  void* cand;               /* HEAD: ycx_cand [n][rows_total]                      */
  int32_t* cand_rows;       /* HEAD: [n][rows_total]                                */
  int32_t* cand_counts;     /* HEAD: [n], zeroed before the first level's op        */
  int32_t* status;          /* HEAD (nullable): the range guard flag, below         */
  void* out2;               /* CONV_PAIR: the second conv's output (out: the first's, nullable) */
  void* workspace;          /* CONV with d.conv.k_split > 1: fp32 partials, >= ycx_conv_workspace_size */
} ycx_op;

int ycx_abi_version(void);
/* sizeof() of the ABI structs, so FFI mirrors can verify their layout:
 * 0 conv_desc, 1 pool_desc, 2 copy_desc, 3 decode_desc, 4 cand, 5 filter_desc,
 * 6 decode_filter_desc, 7 nms_desc, 8 op, 9 letterbox_desc, 10 correct_desc,
 * 11 head_desc.
 * Returns 0 for an unknown id. */
size_t ycx_struct_size(int32_t which);
const char* ycx_strerror(ycx_status s);
const char* ycx_conv_tile_name(int32_t tile);
/* The tile ycx_conv2d uses for d->tile == 0. d->res_c_stride > 0 means the
 * call will pass a residual (tile 22, the weight-resident 1x1, takes none). */
int32_t ycx_conv_pick_tile(const ycx_conv_desc* d);
/* Introspection (host only, no device call): the (output-channel tile, pixel
 * tile) that workgroup `bid` of an LDS-DMA conv launch of nwg = n_ct * n_pt
 * workgroups computes under channel-group count gc (the XCD region map), as
 * ct * 65536 + pt; -1 on bad arguments. Lets tests prove the map bijective. */
int32_t ycx_conv_tile_of(int32_t bid, int32_t nwg, int32_t n_ct, int32_t gc);

ycx_status ycx_conv2d(const ycx_conv_desc* d, const void* x, const void* w,
                      const float* bias, void* y, const void* residual, void* stream);
/* ycx_conv2d with a caller-owned workspace for d->k_split > 1 (split-K: fp32 partials of
 * every K range, then one reduce launch; ycx_conv2d itself returns YCX_ERR_CAPACITY for
 * k_split > 1). ycx_conv_workspace_size: the bytes it needs (0 without a split). */
size_t ycx_conv_workspace_size(const ycx_conv_desc* d);
ycx_status ycx_conv2d_ws(const ycx_conv_desc* d, const void* x, const void* w, const float* bias, void* y,
                         const void* residual, void* workspace, size_t workspace_bytes, void* stream);
/* The K split the library recommends for this conv on the tile it picks (1: none). */
int32_t ycx_conv_pick_ksplit(const ycx_conv_desc* d);
/* Detect head 1x1 conv of one level (bf16, act none, cout = na * no <= 256,
 * out_layout YCX_OUT_NCHW_F32) fused with that level's decode + filter: appends
 * the passing rows to cand / cand_rows / cand_counts exactly as
 * ycx_decode_filter does. `heads` (nullable) also receives the raw fp32 NCHW
 * logits [n][cout][ho][wo] (the compat Model.forward output).
 * `status` (nullable, one int32 the caller zeroes): set to YCX_HEAD_NONFINITE when
 * any logit of the launch is inf or NaN -- the fp16 plan's range guard (an
 * activation past 65504 becomes inf at its producer's store and reaches the heads
 * as inf / NaN). Never cleared by the library. No reference counterpart: the
 * reference computes in fp32 (nets/yolo.py:143-153). */
enum { YCX_HEAD_NONFINITE = 1 };
ycx_status ycx_conv2d_head(const ycx_conv_desc* d, const ycx_head_desc* h, const void* x, const void* w,
                           const float* bias, float* heads, ycx_cand* cand, int32_t* cand_rows,
                           int32_t* cand_counts, int32_t* status, void* stream);
/* Two chained 1x1 / stride-1 convs in one launch (Conv, nets/common.py:97-109, twice):
 * ya = act_a(W_a x + b_a) (cin 64 / 128 / 256 -> cout 256, `ya` nullable: then it is
 * not stored) and yb = act_b(W_b ya + b_b) (256 -> cout_pad 128 or 256), where `b` reads
 * nothing but `a`'s output: the yolov7 160^2 ELAN exit (layer 11 -> layer 14,
 * cfg/net/yolov7.yaml). The intermediate stays on chip (one HBM read of it saved);
 * outputs bit-identical to two ycx_conv2d calls with the weight-resident 1x1 (tile 22).
 * NHWC 16-bit (d->dtype bf16 / fp16), channel slices as ycx_conv2d. */
ycx_status ycx_conv2d_pair(const ycx_conv_desc* a, const ycx_conv_desc* b, const void* x, const void* w_a,
                           const float* bias_a, void* ya, const void* w_b, const float* bias_b, void* yb,
                           void* stream);
/* Stem conv: fp32 NCHW input (the model input, cin <= 4), weights fp32
 * [kh][kw][cin][cout_pad], output NHWC in d->dtype. in_c_* describe the NCHW
 * channel count (in_c_stride = channels of the input tensor). */
ycx_status ycx_stem_conv(const ycx_conv_desc* d, const float* x, const float* w,
                         const float* bias, void* y, void* stream);
/* The stem (3x3, stride 1 or 2, pad 1, 3 -> 32, bf16 NHWC result kept in LDS)
 * followed by a 3x3 / stride-2 / pad-1 conv 32 -> cout (cout_pad 64) that
 * consumes only it: one kernel, the 32-channel stem map never reaches HBM.
 * `stem` and `conv` are the two layers' own descriptors (conv->h/w = the stem
 * output size); conv output as for ycx_conv2d (NHWC bf16, channel slice).
 * Requires conv->ho % 4 == 0, conv->wo % 32 == 0 and stem->act == conv->act.
 * dtype YCX_DT_FP8 (both descriptors): the pair still computes in bf16 with
 * bf16 w_conv and plain bias; only the output is e4m3 (conv->out_scale). */
ycx_status ycx_stem_conv2(const ycx_conv_desc* stem, const ycx_conv_desc* conv, const float* x,
                          const float* w_stem, const float* b_stem, const void* w_conv,
                          const float* b_conv, void* y, void* stream);
ycx_status ycx_maxpool(const ycx_pool_desc* d, const void* x, void* y, void* stream);
ycx_status ycx_copy_channels(const ycx_copy_desc* d, const void* x, void* y, void* stream);
/* fp32 -> OCP e4m3fn bytes: y[i] = e4m3(clamp(x[i] * scale, +-448)), round to
 * nearest even: the exact cast of the YCX_DT_FP8 epilogues (calibration checks). */
ycx_status ycx_quantize_fp8(const float* x, void* y, int64_t n, float scale, void* stream);

ycx_status ycx_decode(const ycx_decode_desc* d, const float* head, float* out, void* stream);
/* IDetect's eval outputs for one level (nets/idetect.py:33-45): xview gets the
 * raw map as (n, na, h, w, no); z [n][rows_total][no] gets, at row_off, the
 * decoded rows xy = (sigmoid*2 - 0.5 + grid) * stride, wh = (sigmoid*2)^2 *
 * anchor (pixels; d->anchors_scaled holds the level's anchor_grid in pixels).
 * The reference leaves IDetect.stride unset (its eval raises); the caller
 * supplies it. */
ycx_status ycx_idetect_decode(const ycx_decode_desc* d, float stride, const float* head, float* z, float* xview,
                              void* stream);
/* Candidate outputs of both filters:
 *   cand        [n][rows] ycx_cand, written only at the rows that pass (dense by row)
 *   cand_rows   [n][rows] int32, the passing row indices, compacted (any order)
 *   cand_counts [n] int32, number of passing rows; MUST be zeroed before the call
 *               (the filters append with wave-aggregated atomics). */
ycx_status ycx_filter_decoded(const ycx_filter_desc* d, float* pred, ycx_cand* cand,
                              int32_t* cand_rows, int32_t* cand_counts, void* stream);
ycx_status ycx_decode_filter(const ycx_decode_filter_desc* d, const float* const* heads,
                             ycx_cand* cand, int32_t* cand_rows, int32_t* cand_counts, void* stream);
/* Device self-check behind the class scan of the decode filters (no reference
 * counterpart): adds to *violations (device uint64, caller-zeroed) the number of
 * adjacent finite-float pairs x < y with sigmoid(x) > sigmoid(y) for the
 * decoders' sigmoid, over every float, plus (r06) the floats m in [-80, 6] at
 * which sigmoid(m - max(|m|, 1) 2^-12) is not below sigmoid(m). The filters'
 * exact class argmax relies on it being 0 (ycx_internal.h, ycx_class_argmax and
 * the fast path of ycx_class_finish). */
ycx_status ycx_check_sigmoid_monotone(unsigned long long* violations, void* stream);
size_t ycx_nms_workspace_size(const ycx_nms_desc* d);
/* Sorts each image's candidates by (class asc, score desc, row asc) — the order
 * of detect.py:124-137 with a stable torchvision sort — and runs greedy NMS per
 * class. cand_rows must list each row at most once per image (both filters and the
 * fused head decode append every passing row exactly once): the class buckets are
 * counted per list entry and filled per distinct row. Outputs: dets [n][max_det][7] = x1,y1,x2,y2,obj,cls_conf,cls (fp32),
 * keep_rows [n][max_det] (row index, -1 padded), keep_counts [n] (not capped
 * by max_det; rows beyond max_det are dropped from dets/keep_rows). */
ycx_status ycx_sort_nms(const ycx_nms_desc* d, const ycx_cand* cand, const int32_t* cand_rows,
                        const int32_t* cand_counts, void* workspace, size_t workspace_bytes,
                        float* dets, int32_t* keep_rows, int32_t* keep_counts, void* stream);

ycx_status ycx_letterbox(const ycx_letterbox_desc* d, const uint8_t* src, float* dst, void* stream);
/* n same-sized images in one launch: image i is read at src + i * src_image_stride
 * bytes and written to dst + i * c * out_h * out_w (one NCHW fp32 batch): the
 * preprocessing of detect.py:16-26 for a whole batch (bench.py --image-in). */
ycx_status ycx_letterbox_batch(const ycx_letterbox_desc* d, int32_t n, int64_t src_image_stride,
                               const uint8_t* src, float* dst, void* stream);
ycx_status ycx_correct_boxes(const ycx_correct_desc* d, float* dets, const int32_t* counts,
                             const int32_t* image_hw, void* stream);

/* Run a static op list in order on one stream. If `events` is non-null it must
 * hold n_ops+1 hipEvent_t; event i is recorded before op i and event n_ops
 * after the last (per-op kernel timing for the roofline report). */
ycx_status ycx_run_ops(const ycx_op* ops, int32_t n_ops, void* stream, void* const* events);

/* 1: ycx_run_ops wraps every op in a roctx range "op<i> <kind> <tile> n HxW cin->cout k s"
 * (rocprofv3 --marker-trace); 0 (default): no tracing. The roctx library is dlopen'ed
 * on the first ycx_set_trace(1); YCX_ERR_UNSUPPORTED (tracing stays off) if it is
 * absent. No reference counterpart (its only instrument is the @timer decorator,
 * utils/helper_torch.py:10-20). */
ycx_status ycx_set_trace(int32_t on);
/* Kernel-side bounds checks (`make -C yolo-continuous_amd/csrc debug` builds
 * libycx_hip_dbg.so with -DYCX_DEBUG_BOUNDS; select it with YCX_LIB=<path>): every
 * conv epilogue store is tested against the output extent its descriptor implies and
 * skipped if outside. out[0] = violations since the last reset, out[1] = the first
 * offending source line. YCX_ERR_UNSUPPORTED from a release build. */
ycx_status ycx_debug_bounds(uint32_t* out, int32_t reset);
/* Capture ycx_run_ops into a HIP graph and instantiate it (graph_exec out). */
ycx_status ycx_graph_capture(const ycx_op* ops, int32_t n_ops, void* stream, void** graph_exec);
ycx_status ycx_graph_launch(void* graph_exec, void* stream);
ycx_status ycx_graph_destroy(void* graph_exec);

#ifdef __cplusplus
}
#endif
#endif /* YCX_H_ */
