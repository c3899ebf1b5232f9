"""ORACLE (test infrastructure only): CPU restatement of the post-processing.

decode_box              detect.py:29-87   (same torch ops, same order -> bit-exact on CPU)
non_max_suppression     detect.py:90-144  (xyxy in place, class max, >= conf, per-class nms)
yolo_correct_boxes      detect.py:147-165 (numpy)
nms                     torchvision.ops.nms as called at detect.py:133 — torchvision is
                        absent and unpinned, so this restates its CPU kernel
                        (torchvision/csrc/ops/cpu/nms_kernel.cpp, published algorithm):
                        areas = (x2-x1)*(y2-y1) in fp32; order = stable descending sort
                        of scores; greedy: keep i, suppress j when
                        inter / (area_i + area_j - inter) > iou_threshold, with the fp32
                        ratio compared against the double threshold.  PARITY UNPINNED.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np
import torch

_C_LIB = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_c", "libycx_oracle.so")
_c = None


def _clib():
    """oracle/nms_ref.c (built by __graft_entry__.build() / oracle/Makefile), or None."""
    global _c
    if _c is None:
        _c = False
        if os.path.exists(_C_LIB):
            lib = ctypes.CDLL(_C_LIB)
            lib.ycx_oracle_nms.restype = ctypes.c_int64
            lib.ycx_oracle_nms.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_double,
                                           ctypes.c_void_p]
            _c = lib
    return _c or None


def nms(boxes, scores, iou_threshold):
    """torchvision.ops.nms restated (CPU algorithm): int64 keep indices,
    score-descending. Runs the C restatement (oracle/nms_ref.c, the same float32
    operations; tests/test_oracle_golden.py checks the two agree) when it is
    built, else the numpy one below."""
    lib = _clib()
    if lib is None:
        return nms_numpy(boxes, scores, iou_threshold)
    b = np.ascontiguousarray(boxes.detach().cpu().numpy(), dtype=np.float32)
    s = np.ascontiguousarray(scores.detach().cpu().numpy(), dtype=np.float32)
    n = b.shape[0]
    keep = np.empty((max(n, 1),), dtype=np.int64)
    k = lib.ycx_oracle_nms(b.ctypes.data, s.ctypes.data, n, float(iou_threshold), keep.ctypes.data)
    if k < 0:
        raise MemoryError("oracle nms")
    return torch.from_numpy(keep[:k].copy())


def nms_numpy(boxes, scores, iou_threshold):
    """torchvision.ops.nms restated in numpy (the reference form of the oracle)."""
    b = boxes.detach().cpu().numpy().astype(np.float32, copy=False)
    s = scores.detach().cpu().numpy().astype(np.float32, copy=False)
    n = b.shape[0]
    if n == 0:
        return torch.empty((0,), dtype=torch.int64)
    x1, y1, x2, y2 = b[:, 0], b[:, 1], b[:, 2], b[:, 3]
    areas = (x2 - x1) * (y2 - y1)
    order = np.argsort(-s, kind='stable')  # stable descending (ties keep input order)
    suppressed = np.zeros(n, dtype=bool)
    keep = []
    thr = float(iou_threshold)
    for _i in range(n):
        i = order[_i]
        if suppressed[i]:
            continue
        keep.append(i)
        rest = order[_i + 1:]
        rest = rest[~suppressed[rest]]
        if rest.size == 0:
            continue
        xx1 = np.maximum(x1[i], x1[rest])
        yy1 = np.maximum(y1[i], y1[rest])
        xx2 = np.minimum(x2[i], x2[rest])
        yy2 = np.minimum(y2[i], y2[rest])
        w = np.maximum(np.float32(0), xx2 - xx1)
        h = np.maximum(np.float32(0), yy2 - yy1)
        inter = w * h
        ovr = inter / (areas[i] + areas[rest] - inter)
        suppressed[rest[ovr.astype(np.float64) > thr]] = True
    return torch.as_tensor(np.asarray(keep, dtype=np.int64))


def decode_box(inputs, anchors, anchors_mask, num_labels, image_size=(640, 640)):
    outputs = []
    for i, pred in enumerate(inputs):
        bs, h, w = pred.size(0), pred.size(2), pred.size(3)
        stride_h = image_size[0] / h
        stride_w = image_size[0] / w
        sa = [(aw / stride_w, ah / stride_h) for aw, ah in anchors[anchors_mask[i]]]
        na = len(anchors_mask[i])
        p = torch.sigmoid(pred.view(bs, na, num_labels + 5, h, w).permute(0, 1, 3, 4, 2).contiguous())
        x, y, ww, hh = p[..., 0], p[..., 1], p[..., 2], p[..., 3]
        conf, cls = p[..., 4], p[..., 5:]
        grid_x = torch.linspace(0, w - 1, w).repeat(h, 1).repeat(bs * na, 1, 1).view(x.shape).float()
        grid_y = torch.linspace(0, h - 1, h).repeat(w, 1).t().repeat(bs * na, 1, 1).view(y.shape).float()
        t = torch.tensor(sa, dtype=torch.float32)
        anchor_w = t.index_select(1, torch.tensor([0])).repeat(bs, 1).repeat(1, 1, h * w).view(ww.shape)
        anchor_h = t.index_select(1, torch.tensor([1])).repeat(bs, 1).repeat(1, 1, h * w).view(hh.shape)
        boxes = torch.empty(p[..., :4].shape, dtype=torch.float32)
        boxes[..., 0] = x * 2. - 0.5 + grid_x
        boxes[..., 1] = y * 2. - 0.5 + grid_y
        boxes[..., 2] = (ww * 2) ** 2 * anchor_w
        boxes[..., 3] = (hh * 2) ** 2 * anchor_h
        scale = torch.tensor([w, h, w, h], dtype=torch.float32)
        outputs.append(torch.cat((boxes.view(bs, -1, 4) / scale, conf.view(bs, -1, 1),
                                  cls.view(bs, -1, num_labels)), -1))
    return outputs


def nms_keep_rows(prediction, num_classes, conf_thres, nms_thres):
    """The device-comparable part of non_max_suppression: per image, the kept
    candidate rows (indices into the concatenated rows) and their (K, 7)
    detections, in output order (class asc, score desc). Mutates prediction
    to xyxy like the reference."""
    bc = prediction.new(prediction.shape)
    bc[:, :, 0] = prediction[:, :, 0] - prediction[:, :, 2] / 2
    bc[:, :, 1] = prediction[:, :, 1] - prediction[:, :, 3] / 2
    bc[:, :, 2] = prediction[:, :, 0] + prediction[:, :, 2] / 2
    bc[:, :, 3] = prediction[:, :, 1] + prediction[:, :, 3] / 2
    prediction[:, :, :4] = bc[:, :, :4]
    rows_out, dets_out = [], []
    for image_pred in prediction:
        class_conf, class_pred = torch.max(image_pred[:, 5:5 + num_classes], 1, keepdim=True)
        mask = (image_pred[:, 4] * class_conf[:, 0] >= conf_thres).squeeze()
        idx = torch.nonzero(mask).reshape(-1)
        det = torch.cat((image_pred[idx, :5], class_conf[idx].float(), class_pred[idx].float()), 1)
        rows, dets = [], []
        for c in det[:, -1].unique():
            sel = det[:, -1] == c
            dc, ic = det[sel], idx[sel]
            keep = nms(dc[:, :4], dc[:, 4] * dc[:, 5], nms_thres)
            rows.append(ic[keep])
            dets.append(dc[keep])
        rows_out.append(torch.cat(rows) if rows else torch.empty((0,), dtype=torch.int64))
        dets_out.append(torch.cat(dets) if dets else torch.empty((0, 7)))
    return rows_out, dets_out


def yolo_correct_boxes(box_xy, box_wh, input_shape, image_shape, letterbox_image):
    box_yx = box_xy[..., ::-1]
    box_hw = box_wh[..., ::-1]
    input_shape = np.array(input_shape)
    image_shape = np.array(image_shape)
    if letterbox_image:
        new_shape = np.round(image_shape * np.min(input_shape / image_shape))
        offset = (input_shape - new_shape) / 2. / input_shape
        scale = input_shape / new_shape
        box_yx = (box_yx - offset) * scale
        box_hw *= scale
    box_mins = box_yx - (box_hw / 2.)
    box_maxes = box_yx + (box_hw / 2.)
    boxes = np.concatenate([box_mins[..., 0:1], box_mins[..., 1:2], box_maxes[..., 0:1], box_maxes[..., 1:2]], -1)
    boxes *= np.concatenate([image_shape, image_shape], axis=-1)
    return boxes


def non_max_suppression(prediction, num_classes, input_shape, image_shape, letterbox_image, conf_thres=0.5,
                        nms_thres=0.4):
    _, dets = nms_keep_rows(prediction, num_classes, conf_thres, nms_thres)
    output = []
    for d in dets:
        if d.shape[0] == 0:
            output.append(None)
            continue
        o = d.numpy()
        box_xy, box_wh = (o[:, 0:2] + o[:, 2:4]) / 2, o[:, 2:4] - o[:, 0:2]
        o[:, :4] = yolo_correct_boxes(box_xy, box_wh, input_shape, image_shape, letterbox_image)
        output.append(o)
    return output


def idetect_eval(outs, anchors, na, no, strides):
    """IDetect's eval branch restated (nets/idetect.py:33-45) on its raw maps
    (NCHW per level, P3..P5): returns (cat(z, 1), [x_i (bs, na, ny, nx, no)]).
    The reference never reaches this code (IDetect.stride is None, :8), so the
    strides are supplied; everything else is its op sequence."""
    anchor_grid = torch.tensor(anchors).float().view(len(outs), 1, -1, 1, 1, 2)
    z, xs = [], []
    for i, xi in enumerate(outs):
        bs, _, ny, nx = xi.shape
        xi = xi.view(bs, na, no, ny, nx).permute(0, 1, 3, 4, 2).contiguous()
        yv, xv = torch.meshgrid([torch.arange(ny), torch.arange(nx)], indexing='ij')
        grid = torch.stack((xv, yv), 2).view((1, 1, ny, nx, 2)).float()
        y = xi.sigmoid()
        y[..., 0:2] = (y[..., 0:2] * 2. - 0.5 + grid) * torch.tensor(strides[i], dtype=torch.float32)
        y[..., 2:4] = (y[..., 2:4] * 2) ** 2 * anchor_grid[i]
        z.append(y.view(bs, -1, no))
        xs.append(xi)
    return torch.cat(z, 1), xs
