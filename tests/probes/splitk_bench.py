"""Split-K / ring-depth sweep of the 20^2 (and 40^2) yolov7 conv shapes at bs 32 (development probe, r06).

    python tests/probes/splitk_bench.py [iters]
For every shape: tiles 16 / 18 / 56 / 12 at k_split 1..4, isolated (back-to-back launches of one
op on one stream), plus the largest |difference| of each output from the tile-16 unsplit one.
Times include the split-K reduce launch.
"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "yolo-continuous_amd"))
from ycx import _lib as L  # noqa: E402

SHAPES = [  # n, h, w, cin, cout, k, s  (yolov7 bs 32 at 640^2: the 20^2 layers, two 40^2 ones)
    (32, 20, 20, 256, 256, 3, 1),
    (32, 20, 20, 512, 256, 3, 1),
    (32, 20, 20, 512, 512, 3, 1),
    (32, 20, 20, 1024, 512, 1, 1),
    (32, 20, 20, 2048, 512, 1, 1),
    (32, 20, 20, 1024, 1024, 1, 1),
    (32, 20, 20, 512, 1024, 3, 1),
    (32, 40, 40, 512, 512, 3, 2),
    (32, 40, 40, 256, 256, 3, 2),
    (32, 40, 40, 256, 128, 3, 1),
]


def run(shape, tile, ks, iters, ref=None):
    n, h, w, cin, cout, k, s = shape
    dev = torch.device("cuda:0")
    p = k // 2
    ho, wo = (h + 2 * p - k) // s + 1, (w + 2 * p - k) // s + 1
    cpad = 64 if cout <= 64 else -(-cout // 128) * 128
    if tile in (16, 12) and cpad % 128:
        return None, None
    g = torch.Generator(device="cpu").manual_seed(0)
    x = torch.randn(n, h, w, cin, generator=g).to(torch.bfloat16).to(dev)
    wt = (torch.randn(cpad, k * k * cin, generator=g) * (k * k * cin) ** -0.5).to(torch.bfloat16).to(dev)
    b = torch.zeros(cpad, device=dev)
    y = torch.empty(n, ho, wo, cout, device=dev, dtype=torch.bfloat16)
    d = L.ConvDesc()
    d.n, d.h, d.w, d.cin, d.in_c_off, d.in_c_stride = n, h, w, cin, 0, cin
    d.ho, d.wo, d.cout, d.cout_pad, d.out_c_off, d.out_c_stride = ho, wo, cout, cpad, 0, cout
    d.kh = d.kw = k
    d.stride, d.pad, d.act, d.dtype, d.out_layout, d.tile = s, p, L.ACT_SILU, L.DT_BF16, L.OUT_NHWC, tile
    d.k_split = ks
    nws = int(L.lib.ycx_conv_workspace_size(ctypes.byref(d)))
    ws = torch.empty(max(nws, 4) // 4, device=dev)
    st = L.stream_handle(dev)
    args = (ctypes.byref(d), x.data_ptr(), wt.data_ptr(), b.data_ptr(), y.data_ptr(), None, ws.data_ptr(), nws, st)
    if L.lib.ycx_conv2d_ws(*args) != 0:
        return None, None
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(3):
        L.lib.ycx_conv2d_ws(*args)
    e0.record()
    for _ in range(iters):
        L.lib.ycx_conv2d_ws(*args)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1000 / iters
    diff = None if ref is None else float((y.float() - ref.float()).abs().max())
    return us, (y if ref is None else diff)


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    for sh in SHAPES:
        base_us, ref = run(sh, 16, 0, iters)
        if ref is None:
            base_us, ref = run(sh, 18, 0, iters)
        flop = 2 * sh[0] * (sh[1] // sh[6]) * (sh[2] // sh[6]) * sh[3] * sh[4] * sh[5] ** 2
        row = []
        for tile in (16, 18, 56, 12):
            for ks in (0, 2, 3, 4):
                us, diff = run(sh, tile, ks, iters, ref)
                if us is None:
                    continue
                row.append(f"t{tile}k{max(ks, 1)}:{us:.1f}({flop / us / 1e6:.0f}TF,d{diff:.3g})")
        print(sh, " ".join(row), flush=True)


if __name__ == "__main__":
    main()
