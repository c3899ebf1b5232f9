"""Host letterbox for predict() (image_enhance/letter_box.py:27-60, scale_fill_prob=0).

Aspect-preserving resize to round(w*r) x round(h*r) with bilinear sampling
(cv2.INTER_LINEAR convention: half-pixel centres, edge clamp), then a constant
114 border split as round(d -/+ 0.1). OpenCV is not installed here, so
bit-parity with cv2.resize is unpinned; the on-device letterbox
is the §8(f) "next" row.
"""
from __future__ import annotations

import numpy as np


def read_image(path):
    """HWC uint8 BGR, like cv2.imread (detect.py:23)."""
    try:
        import cv2  # noqa: F401
        img = cv2.imread(path)
        if img is None:
            raise FileNotFoundError(path)
        return img
    except ImportError:
        from PIL import Image
        rgb = np.asarray(Image.open(path).convert('RGB'))
        return np.ascontiguousarray(rgb[..., ::-1])


def _resize_bilinear(img, new_w, new_h):
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
    r = min(new_shape[0] / w0, new_shape[1] / h0)
    rw, rh = int(round(w0 * r)), int(round(h0 * r))
    dw, dh = (new_shape[0] - rw) / 2, (new_shape[1] - rh) / 2
    if (rw, rh) != (w0, h0):
        img = _resize_bilinear(img, rw, rh)
    top, bottom = int(round(dh - 0.1)), int(round(dh + 0.1))
    left, right = int(round(dw - 0.1)), int(round(dw + 0.1))
    out = np.empty((rh + top + bottom, rw + left + right, img.shape[2]), dtype=np.uint8)
    out[...] = np.asarray(color, dtype=np.uint8)
    out[top:top + rh, left:left + rw] = img
    return out
