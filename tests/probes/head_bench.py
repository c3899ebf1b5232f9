"""Time ycx_conv2d_head (Detect-head conv + decode + filter) per level in
isolation, interleaving several builds of the library (development probe).

    python tests/probes/head_bench.py LIB_A.so [LIB_B.so ...] [--rounds 5]
"""
import argparse
import ctypes
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "yolo-continuous_amd"))
from ycx import _lib as L  # noqa: E402

LEVELS = [(32, 20, 20, 1024), (32, 40, 40, 512), (32, 80, 80, 256)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    args = ap.parse_args()
    libs = []
    for p in args.libs:
        lib = ctypes.CDLL(os.path.abspath(p))
        lib.ycx_conv2d_head.restype = ctypes.c_int32
        lib.ycx_conv2d_head.argtypes = [ctypes.c_void_p] * 11
        libs.append(lib)
    dev = torch.device("cuda:0")
    st = L.stream_handle(dev)
    na, nc = 3, 80
    no = nc + 5
    rows_total = sum(na * h * w for _, h, w, _ in LEVELS)
    off = 0
    for n, h, w, cin in LEVELS:
        g = torch.Generator(device=dev).manual_seed(0)
        x = torch.randn(n, h, w, cin, device=dev, generator=g).to(torch.bfloat16)
        wt = (torch.randn(256, cin, device=dev, generator=g) / cin ** 0.5).to(torch.bfloat16)
        wt[na * no:] = 0
        b = torch.zeros(256, device=dev)
        d = L.ConvDesc()
        d.n, d.h, d.w, d.cin, d.in_c_off, d.in_c_stride = n, h, w, cin, 0, cin
        d.ho, d.wo, d.cout, d.cout_pad, d.out_c_off, d.out_c_stride = h, w, na * no, 256, 0, na * no
        d.kh = d.kw = 1
        d.stride, d.pad, d.act, d.dtype, d.out_layout = 1, 0, L.ACT_NONE, L.DT_BF16, L.OUT_NCHW_F32
        hd = L.HeadDesc()
        hd.na, hd.no, hd.nc, hd.rows_total, hd.row_off, hd.conf_thres = na, no, nc, rows_total, off, 0.3
        for k in range(2 * na):
            hd.anchors_scaled[k] = 10.0 + k
        off += na * h * w
        outs = []
        for _ in libs:
            cand = torch.empty((n, rows_total, 8), dtype=torch.float32, device=dev)
            rows = torch.empty((n, rows_total), dtype=torch.int32, device=dev)
            cnt = torch.zeros((n,), dtype=torch.int32, device=dev)
            outs.append((cand, rows, cnt))
        calls = [(lib, (ctypes.byref(d), ctypes.byref(hd), x.data_ptr(), wt.data_ptr(), b.data_ptr(), None,
                        o[0].data_ptr(), o[1].data_ptr(), o[2].data_ptr(), None, st)) for lib, o in zip(libs, outs)]
        times = [[] for _ in libs]
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for r in range(args.rounds):
            for j in range(len(libs)):
                i = (j + r) % len(libs)
                lib, a = calls[i]
                assert lib.ycx_conv2d_head(*a) == 0
                e0.record()
                for _ in range(args.iters):
                    lib.ycx_conv2d_head(*a)
                e1.record()
                torch.cuda.synchronize()
                times[i].append(e0.elapsed_time(e1) / args.iters)
        for o in outs:
            o[2].zero_()
        for lib, a in calls:
            lib.ycx_conv2d_head(*a)
        torch.cuda.synchronize()
        row = [f"({n},{h},{w},{cin})"]
        for i, o in enumerate(outs):
            same = torch.equal(o[2], outs[0][2])
            row.append(f"[{i}] {statistics.median(times[i]) * 1e3:.1f}us cands/img {int(o[2].float().mean())} "
                       f"{'=' if same else '!='}")
        print("  ".join(row), flush=True)


if __name__ == "__main__":
    main()
