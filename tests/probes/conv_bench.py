"""Microbenchmark of one conv layer shape through the C ABI (development probe).

    python tests/probes/conv_bench.py [tile ...]
Times every listed tile id on a set of representative yolov7 bs=32 shapes.
"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "yolo-continuous_amd"))
from ycx import _lib as L  # noqa: E402

SHAPES = [  # n, h, w, cin, cout, k, s
    (32, 40, 40, 256, 256, 3, 1),
    (32, 80, 80, 128, 128, 3, 1),
    (32, 80, 80, 512, 512, 1, 1),
    (32, 320, 320, 64, 64, 3, 1),
    (32, 160, 160, 64, 64, 3, 1),
    (32, 20, 20, 512, 512, 3, 1),
    (32, 640, 640, 32, 64, 3, 2),
    (32, 160, 160, 128, 64, 1, 1),
    (32, 160, 160, 256, 256, 1, 1),
    (32, 160, 160, 256, 128, 1, 1),
    (32, 320, 320, 64, 128, 3, 2),
    (32, 80, 80, 256, 255, 1, 1),
    (32, 80, 80, 128, 256, 3, 1),
    (32, 80, 80, 64, 64, 3, 1),
    (32, 40, 40, 1024, 1024, 1, 1),
    (32, 80, 80, 256, 256, 1, 1),
    (32, 40, 40, 256, 512, 3, 1),
    (32, 160, 160, 128, 128, 1, 1),
    (32, 80, 80, 512, 256, 1, 1),
    (32, 80, 80, 512, 128, 1, 1),
    (32, 40, 40, 512, 512, 1, 1),
    (32, 20, 20, 256, 256, 3, 1),
    (32, 20, 20, 512, 256, 3, 1),
    (32, 40, 40, 256, 256, 3, 2),
    (32, 20, 20, 512, 256, 1, 1),
    (32, 40, 40, 256, 128, 1, 1),
    (32, 20, 20, 512, 1024, 3, 1),
    (32, 40, 40, 256, 512, 3, 1),
]
# CONV_ACT=0|1|2: the activation (default SiLU). CONV_DT=fp16: IEEE half elements (default bf16). CONV_EXTRA="64,32,32,4096,4096,1,1;32,40,40,1024,1024,1,1": extra shapes appended (indices continue)
for _s in filter(None, os.environ.get("CONV_EXTRA", "").split(";")):
    SHAPES.append(tuple(int(v) for v in _s.split(",")))


def run(shape, tile, iters=20):
    n, h, w, cin, cout, k, s = shape
    dev = torch.device("cuda:0")
    p = k // 2
    ho, wo = (h + 2 * p - k) // s + 1, (w + 2 * p - k) // s + 1
    cpad = 64 if cout <= 64 else -(-cout // 128) * 128
    if tile in (11, 24, 25, 27, 29, 30, 40, 41, 44, 45, 46, 47):
        cpad = -(-cout // 256) * 256
    if tile in (1, 4, 7, 9, 12, 14, 16, 20, 21, 26, 28, 31, 32, 42, 43, 49) and cpad % 128:
        return None
    tdt, ldt = (torch.float16, L.DT_F16) if os.environ.get("CONV_DT") == "fp16" else (torch.bfloat16, L.DT_BF16)
    x = torch.randn(n, h, w, cin, device=dev).to(tdt)
    wt = (torch.randn(cpad, k * k * cin, device=dev) * 0.05).to(tdt)
    b = torch.zeros(cpad, device=dev)
    y = torch.empty(n, ho, wo, cout, device=dev, dtype=tdt)
    d = L.ConvDesc()
    d.n, d.h, d.w, d.cin, d.in_c_off, d.in_c_stride = n, h, w, cin, 0, cin
    d.ho, d.wo, d.cout, d.cout_pad, d.out_c_off, d.out_c_stride = ho, wo, cout, cpad, 0, cout
    d.kh = d.kw = k
    d.stride, d.pad, d.act, d.dtype, d.out_layout, d.tile = s, p, int(os.environ.get("CONV_ACT", L.ACT_SILU)), ldt, L.OUT_NHWC, tile
    st = L.stream_handle(dev)
    args = (ctypes.byref(d), x.data_ptr(), wt.data_ptr(), b.data_ptr(), y.data_ptr(), None, st)
    rc = L.lib.ycx_conv2d(*args)
    if rc != 0:
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
    nbytes = 2.0 * (n * h * w * cin + n * ho * wo * cout + cpad * k * k * cin)
    return ms, flops / ms / 1e9, nbytes / ms / 1e6


if __name__ == "__main__":
    tiles = [int(t) for t in sys.argv[1:]] or [0]
    only = os.environ.get("CONV_SHAPES")  # e.g. "3,4": indices into SHAPES
    shapes = [SHAPES[int(i)] for i in only.split(",")] if only else SHAPES
    for sh in shapes:
        row = [str(sh)]
        for t in tiles:
            r = run(sh, t)
            row.append(f"t{t}: " + ("n/a" if r is None else f"{r[0]:.4f} ms {r[1]:.0f} TF {r[2]:.0f} GB/s"))
        print("  ".join(row), flush=True)
