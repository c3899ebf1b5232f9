"""Time ycx_stem_conv2 (fused) against ycx_stem_conv + ycx_conv2d at yolov7's bs=32 640^2 shapes (probe)."""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "yolo-continuous_amd"))
from ycx import _lib as L  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    n, h, w = 32, 640, 640
    x = torch.rand(n, 3, h, w, device=dev)
    ws = torch.randn(3, 3, 3, 32, device=dev) * 0.3
    bs = torch.zeros(32, device=dev)
    wc = (torch.randn(64, 3, 3, 32, device=dev) * 0.05).to(torch.bfloat16)
    bc = torch.zeros(64, device=dev)
    mid = torch.empty(n, h, w, 32, device=dev, dtype=torch.bfloat16)
    y = torch.empty(n, 320, 320, 64, device=dev, dtype=torch.bfloat16)
    ds, dc = L.ConvDesc(), L.ConvDesc()
    ds.n, ds.h, ds.w, ds.cin, ds.in_c_off, ds.in_c_stride = n, h, w, 3, 0, 3
    ds.ho, ds.wo, ds.cout, ds.cout_pad, ds.out_c_off, ds.out_c_stride = h, w, 32, 32, 0, 32
    ds.kh = ds.kw = 3
    act = int(os.environ.get("STEM2_ACT", L.ACT_SILU_PS))  # the plans run SILU_PS (pre-scaled weights)
    ds.stride, ds.pad, ds.act, ds.dtype, ds.out_layout = 1, 1, act, L.DT_BF16, L.OUT_NHWC
    dc.n, dc.h, dc.w, dc.cin, dc.in_c_off, dc.in_c_stride = n, h, w, 32, 0, 32
    dc.ho, dc.wo, dc.cout, dc.cout_pad, dc.out_c_off, dc.out_c_stride = 320, 320, 64, 64, 0, 64
    dc.kh = dc.kw = 3
    dc.stride, dc.pad, dc.act, dc.dtype, dc.out_layout = 2, 1, act, L.DT_BF16, L.OUT_NHWC
    st = L.stream_handle(dev)

    def fused():
        L.check(L.lib.ycx_stem_conv2(ctypes.byref(ds), ctypes.byref(dc), x.data_ptr(), ws.data_ptr(), bs.data_ptr(),
                                     wc.data_ptr(), bc.data_ptr(), y.data_ptr(), st))

    def split():
        L.check(L.lib.ycx_stem_conv(ctypes.byref(ds), x.data_ptr(), ws.data_ptr(), bs.data_ptr(), mid.data_ptr(), st))
        L.check(L.lib.ycx_conv2d(ctypes.byref(dc), mid.data_ptr(), wc.data_ptr(), bc.data_ptr(), y.data_ptr(), None, st))

    which = sys.argv[1:] or ["fused", "split"]
    for name, f in (("fused", fused), ("split", split)):
        if name not in which:
            continue
        for _ in range(3):
            f()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            f()
        e1.record()
        torch.cuda.synchronize()
        print(f"{name}: {e0.elapsed_time(e1) / 10:.4f} ms", flush=True)


if __name__ == "__main__":
    main()
