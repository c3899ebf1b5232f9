"""Interleaved A/B of conv kernel builds (development probe, guide §5.4 rule 24).

    python tests/probes/conv_ab.py LIB_A.so LIB_B.so ... [--tile T] [--shapes 0,5,14] [--rounds 5]

Every library is loaded side by side (ctypes); per shape the builds run in
rotating order for ``rounds`` rounds of ``iters`` launches each, on the same
operands (random bf16). Prints the median and min time per build and shape,
and checks each build's output against the first build's (max |diff|).
"""
import argparse
import ctypes
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "yolo-continuous_amd"))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from ycx import _lib as L  # noqa: E402
from conv_bench import SHAPES  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--tile", type=int, default=0)
    ap.add_argument("--tiles", default=None, help="compare these tile ids of the FIRST library instead")
    ap.add_argument("--shapes", default=None)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    args = ap.parse_args()
    libs = []
    for p in args.libs:
        lib = ctypes.CDLL(os.path.abspath(p))
        lib.ycx_conv2d.restype = ctypes.c_int32
        lib.ycx_conv2d.argtypes = [ctypes.c_void_p] * 7
        libs.append(lib)
    tiles = [args.tile] * len(libs)
    if args.tiles:
        tiles = [int(t) for t in args.tiles.split(",")]
        libs = [libs[0]] * len(tiles)
    dev = torch.device("cuda:0")
    shapes = [SHAPES[int(i)] for i in args.shapes.split(",")] if args.shapes else SHAPES
    st = L.stream_handle(dev)
    for sh in shapes:
        n, h, w, cin, cout, k, s = sh
        p = k // 2
        ho, wo = (h + 2 * p - k) // s + 1, (w + 2 * p - k) // s + 1
        cpad = 64 if cout <= 64 else -(-cout // 128) * 128
        g = torch.Generator(device=dev).manual_seed(0)
        x = torch.randn(n, h, w, cin, device=dev, generator=g).to(torch.bfloat16)
        wt = (torch.randn(cpad, k * k * cin, device=dev, generator=g) * (1.0 / (k * k * cin) ** 0.5)).to(torch.bfloat16)
        b = torch.randn(cpad, device=dev, generator=g) * 0.1
        ys = [torch.empty(n, ho, wo, cout, device=dev, dtype=torch.bfloat16) for _ in libs]
        d = L.ConvDesc()
        d.n, d.h, d.w, d.cin, d.in_c_off, d.in_c_stride = n, h, w, cin, 0, cin
        d.ho, d.wo, d.cout, d.cout_pad, d.out_c_off, d.out_c_stride = ho, wo, cout, cpad, 0, cout
        d.kh = d.kw = k
        d.stride, d.pad, d.act, d.dtype, d.out_layout = s, p, L.ACT_SILU, L.DT_BF16, L.OUT_NHWC
        descs = []
        for t in tiles:
            dd = L.ConvDesc()
            ctypes.pointer(dd)[0] = d
            dd.tile = t
            descs.append(dd)
        calls = [(lib, (ctypes.byref(dd), x.data_ptr(), wt.data_ptr(), b.data_ptr(), y.data_ptr(), None, st))
                 for lib, y, dd in zip(libs, ys, descs)]
        ok = [lib.ycx_conv2d(*a) == 0 for lib, a in calls]
        torch.cuda.synchronize()
        times = [[] for _ in libs]
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for r in range(args.rounds):
            for j in range(len(libs)):
                i = (j + r) % len(libs)
                if not ok[i]:
                    continue
                lib, a = calls[i]
                lib.ycx_conv2d(*a)
                e0.record()
                for _ in range(args.iters):
                    lib.ycx_conv2d(*a)
                e1.record()
                torch.cuda.synchronize()
                times[i].append(e0.elapsed_time(e1) / args.iters)
        flops = 2.0 * n * ho * wo * cout * cin * k * k
        row = [str(sh)]
        for i in range(len(libs)):
            if not ok[i]:
                row.append(f"[{i}] n/a")
                continue
            md, mn = statistics.median(times[i]), min(times[i])
            diff = float((ys[i].float() - ys[0].float()).abs().max()) if ok[0] else float('nan')
            row.append(f"[{i}] {md * 1e3:.1f}us ({mn * 1e3:.1f}) {flops / md / 1e9:.0f}TF d={diff:.3g}")
        print("  ".join(row), flush=True)


if __name__ == "__main__":
    main()
