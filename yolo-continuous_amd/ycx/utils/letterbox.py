"""Letterbox for predict() (detect.py:16-26, image_enhance/letter_box.py:27-60,
scale_fill_prob = 0): the geometry on the host, the pixels on the GPU
(ycx_letterbox: bilinear resize, 114 border, fp32 CHW / 255 in one kernel).

The reference resizes with cv2.resize(INTER_LINEAR); OpenCV is not installed
here, so the kernel follows the documented INTER_LINEAR convention (half-pixel
centres, edge clamp) and its bit-parity with cv2 is unpinned;
tests hold it to the CPU restatement in oracle/ref_letterbox.py.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from .. import _lib as L


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


def letterbox_geometry(h0, w0, new_shape=(640, 640)):
    """(rw, rh, top, left, out_h, out_w) as letter_box.py:27-60 computes them."""
    r = min(new_shape[0] / w0, new_shape[1] / h0)
    rw, rh = int(round(w0 * r)), int(round(h0 * r))
    dw, dh = (new_shape[0] - rw) / 2, (new_shape[1] - rh) / 2
    top, bottom = int(round(dh - 0.1)), int(round(dh + 0.1))
    left, right = int(round(dw - 0.1)), int(round(dw + 0.1))
    return rw, rh, top, left, rh + top + bottom, rw + left + right


def letterbox_gpu(image, new_shape=(640, 640), device=None, out=None, pad=114):
    """HWC uint8 image (numpy or torch) -> letterboxed fp32 CHW tensor on the
    GPU (BGR kept, values / 255). ``out`` may be a preallocated [C, H, W] fp32
    device tensor (e.g. one slot of a batch)."""
    dev = torch.device(device) if device is not None else (out.device if out is not None else torch.device('cuda'))
    if dev.type != 'cuda':
        raise RuntimeError("ycx: letterbox_gpu needs a ROCm device; there is no CPU path")
    src = torch.as_tensor(image)
    if src.dtype != torch.uint8 or src.dim() != 3:
        raise ValueError("ycx: letterbox expects an HWC uint8 image")
    src = src.to(dev).contiguous()
    h0, w0, c = src.shape
    rw, rh, top, left, oh, ow = letterbox_geometry(h0, w0, new_shape)
    if out is None:
        out = torch.empty((c, oh, ow), dtype=torch.float32, device=dev)
    if tuple(out.shape) != (c, oh, ow) or out.dtype != torch.float32 or not out.is_contiguous():
        raise ValueError(f"ycx: letterbox output must be a contiguous fp32 [{c}, {oh}, {ow}] tensor")
    d = L.LetterboxDesc()
    d.h0, d.w0, d.c, d.src_row_stride = h0, w0, c, w0 * c
    d.out_h, d.out_w, d.new_h, d.new_w, d.top, d.left, d.pad = oh, ow, rh, rw, top, left, pad
    L.check(L.lib.ycx_letterbox(ctypes.byref(d), src.data_ptr(), out.data_ptr(), L.stream_handle(dev)),
            "ycx_letterbox")
    return out


def letterbox_batch_gpu(images, out, pad=114):
    """A device batch of same-sized HWC uint8 images [n, h0, w0, c] -> letterboxed
    fp32 NCHW ``out`` [n, c, H, W] in one ycx_letterbox_batch launch on the
    current stream (detect.py:16-26 for every image of the batch)."""
    if images.device.type != 'cuda' or out.device != images.device:
        raise RuntimeError("ycx: letterbox_batch_gpu needs device tensors on one ROCm device")
    if images.dtype != torch.uint8 or images.dim() != 4 or not images.is_contiguous():
        raise ValueError("ycx: letterbox_batch_gpu expects a contiguous [n, h, w, c] uint8 tensor")
    n, h0, w0, c = images.shape
    rw, rh, top, left, oh, ow = letterbox_geometry(h0, w0, (out.shape[3], out.shape[2]))
    if tuple(out.shape) != (n, c, oh, ow) or out.dtype != torch.float32 or not out.is_contiguous():
        raise ValueError(f"ycx: letterbox output must be a contiguous fp32 [{n}, {c}, {oh}, {ow}] tensor")
    d = L.LetterboxDesc()
    d.h0, d.w0, d.c, d.src_row_stride = h0, w0, c, w0 * c
    d.out_h, d.out_w, d.new_h, d.new_w, d.top, d.left, d.pad = oh, ow, rh, rw, top, left, pad
    L.check(L.lib.ycx_letterbox_batch(ctypes.byref(d), n, h0 * w0 * c, images.data_ptr(), out.data_ptr(),
                                      L.stream_handle(images.device)), "ycx_letterbox_batch")
    return out
