"""Test infrastructure (oracle): CPU restatement of the reference letterbox and
box correction, the checkers for ycx_letterbox / ycx_correct_boxes.

letterbox: image_enhance/letter_box.py:27-60 with scale_fill_prob = 0, as used
by detect.py:16-26 — aspect-preserving resize to round(w r) x round(h r), then a
constant 114 border split as round(d -/+ 0.1). The reference resizes with
cv2.resize(INTER_LINEAR); OpenCV is not installed here and no fixture holds its
output, so the bilinear kernel below (half-pixel centres, edge clamp, float64
weights, round-half-even to uint8 — the documented INTER_LINEAR convention) is
PARITY UNPINNED against cv2; the GPU kernel is held to it
bit-exactly.
"""
from __future__ import annotations

import numpy as np


def letterbox_geometry(h0, w0, new_shape=(640, 640)):
    """(rw, rh, top, left, out_h, out_w) exactly as letter_box.py:27-60 computes them."""
    r = min(new_shape[0] / w0, new_shape[1] / h0)
    rw, rh = int(round(w0 * r)), int(round(h0 * r))
    dw, dh = (new_shape[0] - rw) / 2, (new_shape[1] - rh) / 2
    top, bottom = int(round(dh - 0.1)), int(round(dh + 0.1))
    left, right = int(round(dw - 0.1)), int(round(dw + 0.1))
    return rw, rh, top, left, rh + top + bottom, rw + left + right


def resize_bilinear(img, new_w, new_h):
    h, w = img.shape[:2]
    sx, sy = w / new_w, h / new_h
    xs = (np.arange(new_w) + 0.5) * sx - 0.5
    ys = (np.arange(new_h) + 0.5) * sy - 0.5
    x0 = np.clip(np.floor(xs).astype(np.int64), 0, w - 1)
    y0 = np.clip(np.floor(ys).astype(np.int64), 0, h - 1)
    x1 = np.clip(x0 + 1, 0, w - 1)
    y1 = np.clip(y0 + 1, 0, h - 1)
    fx = np.clip(xs - np.floor(xs), 0, 1)[None, :, None]
    fy = np.clip(ys - np.floor(ys), 0, 1)[:, None, None]
    f = img.astype(np.float32)
    top = f[y0][:, x0] * (1 - fx) + f[y0][:, x1] * fx
    bot = f[y1][:, x0] * (1 - fx) + f[y1][:, x1] * fx
    return np.clip(np.rint(top * (1 - fy) + bot * fy), 0, 255).astype(np.uint8)


def letterbox(img, new_shape=(640, 640), color=(114, 114, 114)):
    h0, w0 = img.shape[:2]
    rw, rh, top, left, oh, ow = letterbox_geometry(h0, w0, new_shape)
    if (rw, rh) != (w0, h0):
        img = resize_bilinear(img, rw, rh)
    out = np.empty((oh, ow, img.shape[2]), dtype=np.uint8)
    out[...] = np.asarray(color, dtype=np.uint8)
    out[top:top + rh, left:left + rw] = img
    return out


def letterbox_tensor(img, new_shape=(640, 640)):
    """detect.py:25-26: HWC uint8 -> CHW float32 / 255 (BGR kept, as the reference feeds it)."""
    return np.transpose(letterbox(img, new_shape).astype(np.float32) / 255., (2, 0, 1))
