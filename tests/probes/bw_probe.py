"""HBM read+write rate of ycx_copy_channels on a layer-sized NHWC tensor (development probe)."""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "yolo-continuous_amd"))
from ycx import _lib as L  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    for shape in [(32, 160, 160, 256), (32, 80, 80, 512), (32, 128, 128, 512)]:
        n, h, w, c = shape
        x = torch.ones(shape, dtype=torch.bfloat16, device=dev)
        y = torch.empty_like(x)
        d = L.CopyDesc()
        d.n, d.h, d.w, d.c, d.in_c_off, d.in_c_stride = n, h, w, c, 0, c
        d.out_c_off, d.out_c_stride, d.scale, d.dtype, d.out_layout = 0, c, 1, L.DT_BF16, L.OUT_NHWC
        st = L.stream_handle(dev)
        for _ in range(3):
            L.check(L.lib.ycx_copy_channels(ctypes.byref(d), x.data_ptr(), y.data_ptr(), st))
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            L.lib.ycx_copy_channels(ctypes.byref(d), x.data_ptr(), y.data_ptr(), st)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 20
        nb = 2 * x.numel() * 2
        t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0.record()
        for _ in range(20):
            y.copy_(x)
        t1.record()
        torch.cuda.synchronize()
        ms2 = t0.elapsed_time(t1) / 20
        t0.record()
        for _ in range(20):
            y.fill_(1.0)
        t1.record()
        torch.cuda.synchronize()
        ms3 = t0.elapsed_time(t1) / 20
        print(f"{shape}: ycx_copy {ms:.4f} ms {nb / ms / 1e6:.0f} GB/s   torch copy_ {ms2:.4f} ms {nb / ms2 / 1e6:.0f} GB/s"
              f"   torch fill_ (write only) {ms3:.4f} ms {nb / 2 / ms3 / 1e6:.0f} GB/s", flush=True)


if __name__ == "__main__":
    main()
