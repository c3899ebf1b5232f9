"""fp8 conv microbenchmark through the C ABI (development probe).

    YCX_F8_PERSIST=2 python tests/probes/conv_bench_f8.py [tile ...]
Times the fp8 conv tiles on the yolov7 bs=64 layer shapes of the fp8 plan.
"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "yolo-continuous_amd"))
from ycx import _lib as L  # noqa: E402

SHAPES = [  # n, h, w, cin, cout, k, s
    (64, 320, 320, 64, 64, 3, 1),
    (64, 160, 160, 256, 256, 1, 1),
    (64, 320, 320, 64, 128, 3, 2),
    (64, 80, 80, 512, 512, 1, 1),
    (64, 160, 160, 256, 128, 1, 1),
    (64, 160, 160, 128, 128, 1, 1),
    (64, 80, 80, 128, 256, 3, 1),
    (64, 40, 40, 1024, 1024, 1, 1),
    (64, 160, 160, 64, 64, 3, 1),
    (64, 40, 40, 256, 512, 3, 1),
    (64, 20, 20, 512, 1024, 3, 1),
    (64, 80, 80, 512, 256, 1, 1),
    (64, 80, 80, 256, 256, 1, 1),
    (64, 80, 80, 128, 128, 3, 1),
    (64, 40, 40, 256, 256, 3, 1),
    (64, 20, 20, 512, 512, 3, 1),
]


def run(shape, tile, iters=20):
    n, h, w, cin, cout, k, s = shape
    dev = torch.device("cuda:0")
    p = k // 2
    ho, wo = (h + 2 * p - k) // s + 1, (w + 2 * p - k) // s + 1
    cpad = -(-cout // 64) * 64
    if tile == 34 and cpad % 128:
        return None
    ktp = -(-k * k * cin // 128) * 128
    x = torch.randint(0, 0x70, (n, h, w, cin), device=dev, dtype=torch.uint8)
    wt = torch.randint(0, 0x50, (cpad, ktp), device=dev, dtype=torch.uint8)
    b = torch.ones(2 * cpad, device=dev) * 1e-3
    y = torch.empty(n, ho, wo, cout, device=dev, dtype=torch.uint8)
    d = L.ConvDesc()
    d.n, d.h, d.w, d.cin, d.in_c_off, d.in_c_stride = n, h, w, cin, 0, cin
    d.ho, d.wo, d.cout, d.cout_pad, d.out_c_off, d.out_c_stride = ho, wo, cout, cpad, 0, cout
    d.kh = d.kw = k
    d.stride, d.pad, d.act, d.dtype, d.out_layout, d.tile = s, p, int(os.environ.get("CONV_ACT", L.ACT_SILU)), L.DT_FP8, L.OUT_NHWC, tile
    d.out_scale, d.res_scale = 1.0, 1.0
    st = L.stream_handle(dev)
    args = (ctypes.byref(d), x.data_ptr(), wt.data_ptr(), b.data_ptr(), y.data_ptr(), None, st)
    if L.lib.ycx_conv2d(*args) != 0:
        return None
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(3):
        L.lib.ycx_conv2d(*args)
    e0.record()
    for _ in range(iters):
        L.lib.ycx_conv2d(*args)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / iters
    flops = 2.0 * n * ho * wo * cout * cin * k * k
    nbytes = 1.0 * (n * h * w * cin + n * ho * wo * cout + cpad * ktp)
    return ms, flops / ms / 1e9, nbytes / ms / 1e6


if __name__ == "__main__":
    tiles = [int(t) for t in sys.argv[1:]] or [0]
    tag = os.environ.get("YCX_F8_PERSIST", "default")
    for sh in SHAPES:
        row = [f"P={tag}", str(sh)]
        for t in tiles:
            r = run(sh, t)
            row.append(f"t{t}: " + ("n/a" if r is None else f"{r[0]:.4f} ms {r[1]:.0f} TF {r[2]:.0f} GB/s"))
        print("  ".join(row), flush=True)
