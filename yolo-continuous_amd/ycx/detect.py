"""Inference entry points (drop-in for the reference detect.py) on the HIP kernels.

Reference API kept (same names, argument meaning, return types):
  decode_box(inputs, anchors, anchors_mask, num_labels, image_size)      detect.py:29-87
  non_max_suppression(prediction, num_classes, input_shape, image_shape,
                      letterbox_image, conf_thres=0.5, nms_thres=0.4)    detect.py:90-144
  yolo_correct_boxes(box_xy, box_wh, input_shape, image_shape, letterbox) detect.py:147-165
  prepare_model(plan)                                                     detect.py:168-180
  predict(cfg_file, image_path, conf_threshold=0.3, nms_threshold=0.3)   detect.py:208-265

Device tensors in, device kernels doing the work: decode_box runs ycx_decode
per level; non_max_suppression runs ycx_filter_decoded (which also mutates
``prediction[..., :4]`` to xyxy in place, like detect.py:98-103),
ycx_sort_nms and ycx_correct_boxes (the reference's numpy
``yolo_correct_boxes`` step, reproduced bit for bit on the device); only the
final per-image (K, 7) arrays are copied to the host.

``Detector`` is the fused fast path used by bench.py: forward -> fused
decode+filter -> sort+NMS, all on device, static buffers, optional HIP graph.
"""
from __future__ import annotations

import ctypes
import os
import weakref

import numpy as np
import torch

from . import _lib as L


def _scaled_anchors(anchors, mask, image_size0, h, w):
    """anchor / stride with stride = image_size[0] / grid (detect.py:38-44): float64
    division, then rounded to fp32 like FloatTensor(scaled_anchors)."""
    a = np.asarray(anchors).reshape(-1, 2)
    sw, sh = image_size0 / w, image_size0 / h
    return [np.float32(aw / sw) for aw, _ in a[mask]], [np.float32(ah / sh) for _, ah in a[mask]]


def _require_device(t, what):
    if not isinstance(t, torch.Tensor) or t.device.type != 'cuda':
        raise RuntimeError(f"ycx: {what} must be a tensor on a ROCm device (there is no CPU path)")


def decode_box(inputs, anchors, anchors_mask, num_labels, image_size=(640, 640)):
    """list of fp32 NCHW heads [bs, na*(5+nc), H, W] -> list of [bs, na*H*W, 5+nc].
    The per-level outputs are views of one [bs, sum(rows), 5+nc] tensor, so
    ``torch.cat(outputs, 1)`` (detect.py:230) is a copy the caller may skip via
    ``decode_box.last_concat``."""
    no = num_labels + 5
    bs = inputs[0].shape[0]
    rows = [len(anchors_mask[i]) * p.shape[2] * p.shape[3] for i, p in enumerate(inputs)]
    out = torch.empty((bs, sum(rows), no), dtype=torch.float32, device=inputs[0].device)
    stream = L.stream_handle(out.device)
    off, views = 0, []
    for i, pred in enumerate(inputs):
        _require_device(pred, "decode_box input")
        pred = pred.float().contiguous()
        na = len(anchors_mask[i])
        if pred.shape[1] != na * no:
            raise ValueError(f"ycx: head {i} has {pred.shape[1]} channels, expected {na}*{no}")
        h, w = pred.shape[2], pred.shape[3]
        aw, ah = _scaled_anchors(anchors, anchors_mask[i], image_size[0], h, w)
        d = L.DecodeDesc()
        d.n, d.h, d.w, d.na, d.no, d.rows_total, d.row_off = bs, h, w, na, no, sum(rows), off
        for a in range(na):
            d.anchors_scaled[2 * a], d.anchors_scaled[2 * a + 1] = aw[a], ah[a]
        L.check(L.lib.ycx_decode(ctypes.byref(d), pred.data_ptr(), out.data_ptr(), stream), "ycx_decode")
        views.append(out[:, off:off + rows[i]])
        off += rows[i]
    decode_box.last_concat = out
    return views


def _nms_buffers(n, rows, device):
    cand = torch.empty((n, rows, 8), dtype=torch.float32, device=device)  # ycx_cand, 32 B
    cand_rows = torch.empty((n, rows), dtype=torch.int32, device=device)
    counts = torch.zeros((n,), dtype=torch.int32, device=device)
    return cand, cand_rows, counts


def device_nms(cand, cand_rows, counts, nc, iou_thres, max_det):
    """ycx_sort_nms -> (dets [n, max_det, 7], keep_rows [n, max_det], keep_counts [n]) on device."""
    n, rows = cand.shape[0], cand.shape[1]
    d = L.NmsDesc()
    d.n, d.rows_total, d.nc, d.max_det, d.iou_thres = n, rows, nc, max_det, float(iou_thres)
    ws_bytes = int(L.lib.ycx_nms_workspace_size(ctypes.byref(d)))
    ws = torch.empty((max(ws_bytes, 1),), dtype=torch.uint8, device=cand.device)
    dets = torch.empty((n, max_det, 7), dtype=torch.float32, device=cand.device)
    keep = torch.empty((n, max_det), dtype=torch.int32, device=cand.device)
    kc = torch.empty((n,), dtype=torch.int32, device=cand.device)
    L.check(L.lib.ycx_sort_nms(ctypes.byref(d), cand.data_ptr(), cand_rows.data_ptr(), counts.data_ptr(),
                               ws.data_ptr(), ws_bytes, dets.data_ptr(), keep.data_ptr(), kc.data_ptr(),
                               L.stream_handle(cand.device)), "ycx_sort_nms")
    return dets, keep, kc


def nms_device(prediction, num_classes, conf_thres=0.5, nms_thres=0.4, max_det=None, write_xyxy=True):
    """Device part of non_max_suppression: returns (dets, keep_rows, keep_counts)."""
    _require_device(prediction, "prediction")
    if prediction.dtype != torch.float32 or not prediction.is_contiguous():
        raise ValueError("ycx: prediction must be a contiguous fp32 tensor")
    n, rows, no = prediction.shape
    cand, cand_rows, counts = _nms_buffers(n, rows, prediction.device)
    f = L.FilterDesc()
    f.n, f.rows, f.no, f.nc, f.conf_thres, f.write_xyxy = n, rows, no, num_classes, float(conf_thres), int(write_xyxy)
    L.check(L.lib.ycx_filter_decoded(ctypes.byref(f), prediction.data_ptr(), cand.data_ptr(), cand_rows.data_ptr(),
                                     counts.data_ptr(), L.stream_handle(prediction.device)), "ycx_filter_decoded")
    return device_nms(cand, cand_rows, counts, num_classes, nms_thres, max_det or rows)


def correct_boxes_device(dets, counts, input_shape, image_hw, letterbox_image=True):
    """yolo_correct_boxes (detect.py:139-165) on the device, in place on the
    padded NMS output dets [n, max_det, 7]: the kept rows become [y1, x1, y2, x2]
    in original-image pixels (the numpy float64/float32 arithmetic reproduced
    exactly). image_hw: one (h, w) for every image, or an [n, 2] array."""
    _require_device(dets, "dets")
    n, max_det = dets.shape[0], dets.shape[1]
    hw = torch.as_tensor(np.asarray(image_hw, dtype=np.int32).reshape(-1, 2))
    if hw.shape[0] == 1:
        hw = hw.expand(n, 2)
    hw = hw.contiguous().to(dets.device)
    d = L.CorrectDesc()
    d.n, d.max_det, d.input_h, d.input_w, d.letterbox = n, max_det, int(input_shape[0]), int(input_shape[1]), \
        int(bool(letterbox_image))
    L.check(L.lib.ycx_correct_boxes(ctypes.byref(d), dets.data_ptr(), counts.data_ptr(), hw.data_ptr(),
                                    L.stream_handle(dets.device)), "ycx_correct_boxes")
    return dets


def non_max_suppression(prediction, num_classes, input_shape, image_shape, letterbox_image, conf_thres=0.5,
                        nms_thres=0.4):
    """detect.py:90-144 semantics: list (per image) of np.float32 [K, 7] rows
    (y1, x1, y2, x2 in original-image pixels, obj, cls_conf, cls) or None.
    Everything up to the per-image host lists runs on the device (filter,
    sort, NMS, yolo_correct_boxes)."""
    dets, _, kc = nms_device(prediction, num_classes, conf_thres, nms_thres)
    correct_boxes_device(dets, kc, input_shape, image_shape, letterbox_image)
    counts = kc.cpu().numpy()
    dets = dets.cpu().numpy()
    output = [None] * prediction.shape[0]
    for i in range(prediction.shape[0]):
        k = int(counts[i])
        if k > 0:
            output[i] = dets[i, :k].copy()
    return output


def yolo_correct_boxes(box_xy, box_wh, input_shape, image_shape, letterbox_image):
    """Host form of the letterbox undo (detect.py:147-165), kept for the
    reference's callers; non_max_suppression itself runs the device kernel
    (correct_boxes_device). Returns [y1, x1, y2, x2] in original-image pixels.

    Numerics follow the reference exactly: centres are corrected in float64,
    sizes are scaled IN PLACE on the caller's float32 ``box_wh`` view (so they
    stay float32 and the caller's array is modified, as in the reference), and
    the final pixel scaling is an in-place multiply of the stacked corners."""
    yx = box_xy[..., ::-1]
    hw = box_wh[..., ::-1]
    ins = np.array(input_shape)
    img = np.array(image_shape)
    if letterbox_image:
        fitted = np.round(img * np.min(ins / img))
        yx = (yx - (ins - fitted) / 2. / ins) * (ins / fitted)
        hw *= ins / fitted
    half = hw / 2.
    corners = np.concatenate([yx - half, yx + half], axis=-1)
    corners *= np.concatenate([img, img], axis=-1)
    return corners


def idetect_outputs(head, outs, input_hw):
    """IDetect's eval return value (nets/idetect.py:33-45) from the engine's raw
    head maps (NCHW fp32, one per level, P3..P5 order): (z [n, sum na*ny*nx, no]
    decoded in pixels, [x_i (n, na, ny, nx, no)]), one ycx_idetect_decode per
    level. The reference leaves IDetect.stride unset (its eval raises
    TypeError); unless head.stride is given, stride_i = input height / ny_i
    (documented deviation)."""
    n, na, no = outs[0].shape[0], head.na, head.no
    dev = outs[0].device
    rows = sum(na * o.shape[2] * o.shape[3] for o in outs)
    z = torch.empty((n, rows, no), dtype=torch.float32, device=dev)
    xs, off = [], 0
    grid_anchors = head.anchor_grid.detach().to('cpu', torch.float32).reshape(len(outs), na, 2)
    st = L.stream_handle(dev)
    for i, o in enumerate(outs):
        ny, nx = int(o.shape[2]), int(o.shape[3])
        stride = float(head.stride[i]) if head.stride is not None else float(np.float32(input_hw[0]) / np.float32(ny))
        d = L.DecodeDesc()
        d.n, d.h, d.w, d.na, d.no, d.rows_total, d.row_off = n, ny, nx, na, no, rows, off
        for a in range(na):
            d.anchors_scaled[2 * a], d.anchors_scaled[2 * a + 1] = float(grid_anchors[i, a, 0]), float(grid_anchors[i, a, 1])
        xv = torch.empty((n, na, ny, nx, no), dtype=torch.float32, device=dev)
        L.check(L.lib.ycx_idetect_decode(ctypes.byref(d), ctypes.c_float(stride), o.contiguous().data_ptr(),
                                         z.data_ptr(), xv.data_ptr(), st), "ycx_idetect_decode")
        xs.append(xv)
        off += na * ny * nx
    return z, xs


class DevicePost:
    """decode_box + non_max_suppression on device for fixed head shapes
    (``detect.py:29-144``): ycx_decode_filter -> ycx_sort_nms on the current
    stream. ``heads`` are fp32 NCHW [n, na*(5+nc), h, w] in Detect order
    (P5, P4, P3); their storage is read at every call.

    Outputs stay on device: dets [n, max_det, 7] (normalised xyxy, obj,
    cls_conf, cls), keep_rows [n, max_det] (row into the concatenated
    [sum na*H*W] candidates, -1 padded), keep_counts [n] (uncapped).

    ``fused`` (set by a Detector whose plan decodes in the head convs): the
    candidates are already written by the forward, a call runs the NMS only."""

    def __init__(self, heads, nc, anchors, anchors_mask, image_size, device, conf_thres=0.3, nms_thres=0.3,
                 max_det=300):
        self.device = torch.device(device)
        for hd in heads:
            _require_device(hd, "DevicePost heads")
            if hd.dtype != torch.float32 or not hd.is_contiguous():
                raise ValueError("ycx: DevicePost needs contiguous fp32 heads")
        self.heads = heads
        self.fused = False
        n = heads[0].shape[0]
        d = L.DecodeFilterDesc()
        d.n, d.nl, d.na, d.no, d.nc = n, len(heads), len(anchors_mask[0]), nc + 5, nc
        off = 0
        self.level_descs = []
        for l, hd in enumerate(heads):
            h, w = hd.shape[2], hd.shape[3]
            if hd.shape[0] != n or hd.shape[1] != d.na * d.no:
                raise ValueError(f"ycx: head {l} has shape {tuple(hd.shape)}, expected [{n}, {d.na * d.no}, h, w]")
            d.h[l], d.w[l], d.row_off[l] = h, w, off
            aw, ah = _scaled_anchors(anchors, anchors_mask[l], image_size[0], h, w)
            for a in range(len(aw)):
                d.anchors_scaled[l][2 * a], d.anchors_scaled[l][2 * a + 1] = aw[a], ah[a]
            off += len(anchors_mask[l]) * h * w
        d.rows_total, d.conf_thres = off, float(conf_thres)
        for l in range(len(heads)):  # the same level parameters for the fused head convs
            hdsc = L.HeadDesc()
            hdsc.na, hdsc.no, hdsc.nc, hdsc.rows_total, hdsc.row_off = d.na, d.no, nc, off, d.row_off[l]
            hdsc.conf_thres = d.conf_thres
            for k in range(2 * d.na):
                hdsc.anchors_scaled[k] = d.anchors_scaled[l][k]
            self.level_descs.append(hdsc)
        self.rows = off
        self.df_desc = d
        self.heads_arr = (ctypes.c_void_p * 4)(*[h.data_ptr() for h in heads], *([None] * (4 - len(heads))))
        self.cand, self.cand_rows, self.counts = _nms_buffers(n, off, device)
        nd = L.NmsDesc()
        nd.n, nd.rows_total, nd.nc, nd.max_det, nd.iou_thres = n, off, nc, max_det, float(nms_thres)
        self.nms_desc = nd
        self.ws_bytes = int(L.lib.ycx_nms_workspace_size(ctypes.byref(nd)))
        self.ws = torch.empty((self.ws_bytes,), dtype=torch.uint8, device=device)
        self.dets = torch.empty((n, max_det, 7), dtype=torch.float32, device=device)
        self.keep = torch.empty((n, max_det), dtype=torch.int32, device=device)
        self.kc = torch.empty((n,), dtype=torch.int32, device=device)

    def __call__(self):
        st = L.stream_handle(self.device)
        if not self.fused:
            self.counts.zero_()
            L.check(L.lib.ycx_decode_filter(ctypes.byref(self.df_desc), self.heads_arr, self.cand.data_ptr(),
                                            self.cand_rows.data_ptr(), self.counts.data_ptr(), st),
                    "ycx_decode_filter")
        L.check(L.lib.ycx_sort_nms(ctypes.byref(self.nms_desc), self.cand.data_ptr(), self.cand_rows.data_ptr(),
                                   self.counts.data_ptr(), self.ws.data_ptr(), self.ws_bytes, self.dets.data_ptr(),
                                   self.keep.data_ptr(), self.kc.data_ptr(), st), "ycx_sort_nms")
        return self.dets, self.keep, self.kc


def _release_engine(model_ref, shape, device, slot):
    """Drop a private engine (activations, packed weights, HIP graph). Its
    kernels may still run on a slot stream that the caching allocator does not
    know about (the engine's buffers carry no record_stream), and the graph may
    still be executing: wait for the whole device first, so neither the memory
    nor the graph is reused or destroyed under work in flight."""
    model = model_ref()
    if model is None:
        return
    try:
        torch.cuda.synchronize(torch.device(device))
    except RuntimeError:  # interpreter shutdown: the runtime is already gone, nothing can still run
        pass
    model.release_slot(shape, device, slot)


class Detector:
    """Fused device pipeline for a fixed batch shape: Model forward (static plan,
    optionally one HIP graph) -> candidates -> ycx_sort_nms (DevicePost).

    bf16 and fp8 Detect models decode in the head convs (``fuse_heads``, default): each
    head level's ycx_conv2d_head appends that level's candidates straight from
    the fp32 logits held on chip (detect.py:29-121), so the forward ends with
    the candidate list and the post is the NMS alone. ``keep_heads`` also
    stores the raw fp32 NCHW logits in ``self.heads`` (the parity tests read
    them; bench.py turns it off). Other plans run ycx_decode_filter in post().

    Outputs stay on device: dets [n, max_det, 7] (normalised xyxy, obj,
    cls_conf, cls), keep_rows [n, max_det] (row into the concatenated
    [sum na*H*W] candidates, -1 padded), keep_counts [n] (uncapped)."""

    def __init__(self, model, shape, device, anchors, anchors_mask, image_size=None, conf_thres=0.3,
                 nms_thres=0.3, max_det=300, use_graph=True, slot=None, fuse_heads=True, keep_heads=True):
        self.model = model
        # a private engine unless the caller names a slot: the static buffers of one
        # Detector must never alias model(x)'s or another Detector's (in flight on
        # another stream). A private engine lives as long as this Detector: close()
        # (or the finaliser, when the Detector is collected) drops it from the model.
        own = slot is None
        slot = model.new_slot() if own else slot
        self.engine = model.engine_for(shape, device, slot)
        self._release = (weakref.finalize(self, _release_engine, weakref.ref(model), tuple(shape), str(device), slot)
                         if own else None)
        self.device = torch.device(device)
        n, _, H, W = shape
        image_size = image_size or (H, W)
        self.x, heads = self.engine.bind_static(torch.zeros(shape, dtype=torch.float32, device=device))
        if not isinstance(heads, list):
            raise ValueError("ycx: Detector needs a model whose last layer is a Detect head")
        self.heads = heads
        self._post = DevicePost(heads, model.num_classes, anchors, anchors_mask, image_size, device, conf_thres,
                                nms_thres, max_det)
        for k in ("rows", "df_desc", "cand", "cand_rows", "counts", "nms_desc", "ws_bytes", "ws", "dets", "keep",
                  "kc"):
            setattr(self, k, getattr(self._post, k))
        # the range guard: the fused head kernels set it on any inf / NaN logit (sticky)
        self.status = torch.zeros((1,), dtype=torch.int32, device=device)
        self.fused = bool(fuse_heads) and self.engine.enable_head_decode(
            self._post.level_descs, self.cand, self.cand_rows, self.counts, keep_heads=keep_heads,
            status=self.status)
        self._post.fused = self.fused
        self.keep_heads = keep_heads or not self.fused
        self.use_graph = use_graph and not L.TRACE
        if self.use_graph:
            self.engine.capture()

    def post(self):
        if not self.fused and self.engine.dt in (L.DT_F16, L.DT_BF16):  # unfused 16-bit plans (diagnostic path)
            for h in self.heads:
                self.status.bitwise_or_(torch.isfinite(h).all().logical_not().to(torch.int32))
        return self._post()

    def overflowed(self):
        """True when a forward of this Detector produced an inf / NaN head logit
        (reads the device flag: waits for the work queued on it)."""
        return bool(self.status.item())

    def check(self):
        """Raise YcxRangeError if any forward so far left the plan's range (the
        fp16 plan: an activation past 65504). The fast path never raises by
        itself (that would need a host sync per batch): callers check at their
        own sync points -- ConcurrentDetector / PipelinedDetector.check() does it
        for every slot, bench.py after its timed region, predict() per call."""
        if self.overflowed():
            raise L.YcxRangeError(
                f"ycx: the {self.model.precision} plan produced non-finite head logits (an activation "
                f"left the {self.model.precision} range, |a| > 65504 for fp16); rebuild the Model with "
                f"precision='bf16' or 'f32'")

    def reset_status(self):
        self.status.zero_()

    def close(self):
        """Release this Detector's private engine (activations, packed weights,
        HIP graph) once the device has finished the work queued on it; the
        Detector is unusable afterwards."""
        if self._release is not None:
            self._release()
        self.engine = None

    def forward(self, events=None):
        """The model forward on the static input buffer (current stream); with
        fused heads it also produces this batch's candidates."""
        if self.fused:
            self.counts.zero_()
        if self.use_graph and events is None:
            self.engine.replay()
        else:
            self.engine.run_static(events)
        return self.heads

    def __call__(self, images=None, events=None):
        if images is not None:
            self.x.copy_(images)
        self.forward(events)
        return self.post()


class PipelinedDetector:
    """Batches in flight on two HIP streams: while batch i's decode + NMS runs
    on the post stream, batch i+1's forward already runs on the forward stream.
    ``depth`` Detector slots (own activation buffers, heads and NMS workspace)
    rotate; a slot's forward waits for the previous post that read its heads.

    submit(images) enqueues one batch and returns (dets, keep_rows,
    keep_counts, done_event); the tensors are valid once done_event completes
    (``synchronize()`` or ``torch.cuda.current_stream().wait_event(done)``)."""

    def __init__(self, model, shape, device, anchors, anchors_mask, depth=2, **kw):
        self.device = torch.device(device)
        self.slots = [Detector(model, shape, device, anchors, anchors_mask, **kw) for _ in range(depth)]
        # different priorities come from different stream pools and so land on
        # different hardware queues (two same-pool streams may share one)
        self.s_fwd = torch.cuda.Stream(self.device, priority=0)
        self.s_post = torch.cuda.Stream(self.device, priority=-1)
        self.fwd_done = [torch.cuda.Event() for _ in self.slots]
        self.post_done = [torch.cuda.Event() for _ in self.slots]
        self.i = 0

    def submit(self, images=None, timing=None, pre=None, then=None):
        """``timing`` = (start, end) timing events: recorded when the batch's
        forward starts and when its detections are complete. ``pre`` / ``then``
        as in ConcurrentDetector.submit (forward stream / post stream)."""
        k = self.i % len(self.slots)
        self.i += 1
        det = self.slots[k]
        self.s_fwd.wait_stream(torch.cuda.current_stream(self.device))  # caller's inputs are ready
        with torch.cuda.stream(self.s_fwd):
            self.s_fwd.wait_event(self.post_done[k])  # the slot's heads were consumed
            if timing is not None:
                timing[0].record(self.s_fwd)
            if images is not None:
                det.x.copy_(images)
                images.record_stream(self.s_fwd)  # the caller may free it before this copy runs
            if pre is not None:
                pre(k, det)
            det.forward()
            self.fwd_done[k].record(self.s_fwd)
        with torch.cuda.stream(self.s_post):
            self.s_post.wait_event(self.fwd_done[k])
            dets, keep, kc = det.post()
            if then is not None:
                dets, keep, kc = then(dets, keep, kc)
            self.post_done[k].record(self.s_post)
            if timing is not None:
                timing[1].record(self.s_post)
        return dets, keep, kc, self.post_done[k]

    def synchronize(self):
        cur = torch.cuda.current_stream(self.device)
        cur.wait_stream(self.s_fwd)
        cur.wait_stream(self.s_post)

    def check(self):
        """Wait for the batches in flight; raise YcxRangeError if any slot's
        forward produced non-finite head logits (Detector.check)."""
        self.synchronize()
        for d in self.slots:
            d.check()

    def close(self):
        """Wait for the batches in flight, then release every slot's engine."""
        self.synchronize()
        torch.cuda.synchronize(self.device)
        for d in self.slots:
            d.close()


class ConcurrentDetector:
    """``depth`` batches in flight, each on its own slot and HIP stream: batch i
    runs forward + decode + NMS on stream i % depth, so consecutive batches'
    kernels interleave on the GPU and fill each other's tails (the last, partly
    empty wave of blocks of every conv, the small 20^2/40^2 layers, the
    one-block-per-class NMS). Same interface as PipelinedDetector; a slot's
    outputs stay valid until the slot is submitted again (``depth`` batches
    later). Throughput-oriented: the per-batch latency grows with depth.

    depth 3: HIP spreads streams over GPU_MAX_HW_QUEUES (4) hardware queues and
    two same-priority streams may share one; with three, at least two batches
    always run concurrently (tests/probes/step_split.py concurrent)."""

    def __init__(self, model, shape, device, anchors, anchors_mask, depth=3, **kw):
        self.device = torch.device(device)
        self.slots = [Detector(model, shape, device, anchors, anchors_mask, **kw) for _ in range(depth)]
        # streams of our own, not torch pool streams: the pool is handed out
        # round-robin to every component (the RCCL communicator included), and a
        # slot stream that shares its hardware queue with the communicator's
        # serialises every batch behind the previous batch's all-gather
        # (tests/probes/dist_probe.py: 7.8 vs 6.0 ms per step)
        self.streams = [L.dedicated_stream(self.device, 0, slot=i) for i in range(len(self.slots))]
        self.done = [torch.cuda.Event() for _ in self.slots]
        self.i = 0

    @property
    def s_post(self):  # the stream of the most recent batch (where its collective goes)
        return self.streams[(self.i - 1) % len(self.slots)]

    def submit(self, images=None, timing=None, then=None, post=True, pre=None):
        """Enqueue one batch on the next slot's stream. ``pre(slot_index, detector)``,
        if given, runs on that stream first and fills ``detector.x`` (the image-in
        path: H2D copy + ycx_letterbox_batch). ``then(dets, keep, kc)``, if given,
        runs on that stream right after the NMS (the multi-GPU path issues its
        all-gather there) and its return value replaces the outputs.
        ``post=False`` (diagnostics only) enqueues the forward alone."""
        k = self.i % len(self.slots)
        self.i += 1
        det, s = self.slots[k], self.streams[k]
        s.wait_stream(torch.cuda.current_stream(self.device))  # caller's inputs are ready
        with torch.cuda.stream(s):
            if timing is not None:
                timing[0].record(s)
            if images is not None:
                det.x.copy_(images)
                images.record_stream(s)  # the caller may free it before this copy runs
            if pre is not None:
                pre(k, det)
            det.forward()
            dets, keep, kc = det.post() if post else (det.dets, det.keep, det.kc)
            if then is not None:
                dets, keep, kc = then(dets, keep, kc)
            self.done[k].record(s)
            if timing is not None and timing[1] is not None:
                timing[1].record(s)
        return dets, keep, kc, self.done[k]

    def synchronize(self):
        cur = torch.cuda.current_stream(self.device)
        for s in self.streams:
            cur.wait_stream(s)

    def check(self):
        """Wait for the batches in flight; raise YcxRangeError if any slot's
        forward produced non-finite head logits (Detector.check)."""
        self.synchronize()
        for d in self.slots:
            d.check()

    def close(self):
        """Wait for the batches in flight, then release every slot's engine."""
        self.synchronize()
        torch.cuda.synchronize(self.device)
        for d in self.slots:
            d.close()


def prepare_model(plan, weights=None, device=None, precision='fp16'):
    """detect.py:168-180: build the Model from the plan and load its weights.
    ``weights`` overrides plan.save_path (a state_dict or a path, loaded with
    weights_only=True); 'synthetic' loads the seeded recipe of ycx.utils.synth."""
    from .nets.yolo import Model, WeightInitial
    from .utils.helper_io import cvt_cfg
    net = Model(cvt_cfg(plan.model_cfg), plan.anchors, plan.num_labels, image_chan=plan.image_chan,
                weight_initial=WeightInitial.Random, precision=precision)
    src = weights if weights is not None else plan.save_path
    if isinstance(src, str) and src == 'synthetic':
        from .utils.synth import synthetic_state_dict
        sd = synthetic_state_dict(net, seed=0)
    elif isinstance(src, dict):
        sd = src
    else:
        sd = torch.load(src, map_location='cpu', weights_only=True)
    net.load_state_dict(sd)
    net = net.eval()
    if device is not None:
        net = net.to(device)
    return net


def predict(cfg_file, image_path=None, conf_threshold=0.3, nms_threshold=0.3, *, image=None, device=None,
            weights=None, show=False, precision='fp16'):
    """detect.py:208-265, headless by default. ``image`` may be an HWC uint8 BGR
    array instead of a path. Returns (and prints) the reference's TargetBox
    records (utils/target_box.py): corners floored and clamped to the image as
    detect.py:236-244 does, score obj * cls_conf, the plan's label name and its
    palette colour (utils/helper_cv.py:60-64)."""
    from .cfg.train_plan import TrainPlan
    from .utils.helper_io import check_file
    from .utils.helper_torch import select_device
    from .utils.letterbox import letterbox_gpu, read_image
    from .utils.target_box import TargetBox, colors_for
    plan = TrainPlan(check_file(cfg_file))
    dev = select_device(device if device is not None else plan.device)
    target = (plan.image_size, plan.image_size)
    anchors = np.asarray(plan.anchors).reshape(-1, 2)
    colors = colors_for(plan.num_labels)
    original = image if image is not None else read_image(image_path)
    net = prepare_model(plan, weights=weights, device=dev, precision=precision)
    images = letterbox_gpu(original, target, device=dev).unsqueeze(0)  # detect.py:23-26 on the GPU
    with torch.no_grad():
        pred = net(images)
    outputs = decode_box(pred, anchors, plan.anchors_mask, plan.num_labels, image_size=target)
    all_outputs = torch.cat(outputs, 1)
    results = non_max_suppression(all_outputs, plan.num_labels, target, np.array(original.shape[0:2]), True,
                                  conf_thres=conf_threshold, nms_thres=nms_threshold)
    boxes = []
    if results[0] is not None:
        for row in results[0]:  # rows are (y1, x1, y2, x2, obj, cls_conf, cls) after yolo_correct_boxes
            y1, x1, y2, x2 = row[0], row[1], row[2], row[3]
            box = [max(0, int(np.floor(x1))), max(0, int(np.floor(y1))),
                   min(original.shape[1], int(np.floor(x2))), min(original.shape[0], int(np.floor(y2)))]
            label = int(row[6])
            tb = TargetBox(box, row[4] * row[5], plan.labels[label], colors[label])
            print(tb)
            boxes.append(tb)
    return boxes
