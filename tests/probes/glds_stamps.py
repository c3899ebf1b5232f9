"""Per-phase cycle breakdown of the glds main loop (development probe).

    YCX_LIB=.../libycx_stamp.so python tests/probes/glds_stamps.py [tile] [shape idx ...]
Needs a -DYCX_GLDS_STAMP build (tools/build_variant.sh stamp -DYCX_GLDS_STAMP).
Buckets per wave (summed over workgroups, averaged per workgroup):
prologue | vmcnt wait | barrier | DMA issue | ds_read issue | MFMA issue | epilogue | total
"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "yolo-continuous_amd"))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from ycx import _lib as L  # noqa: E402
from conv_bench import SHAPES  # noqa: E402

NAMES = ["prolog", "vmwait", "barrier", "dma", "ds_read", "mfma", "epilog", "total"]


def main():
    tile = int(sys.argv[1]) if len(sys.argv) > 1 else 16
    idx = [int(i) for i in sys.argv[2:]] or [0, 14, 26]
    lib = L.lib
    lib.ycx_debug_glds_stamps.restype = ctypes.c_int
    lib.ycx_debug_glds_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
    dev = torch.device("cuda:0")
    buf = (ctypes.c_ulonglong * 129)()
    for i in idx:
        n, h, w, cin, cout, k, s = SHAPES[i]
        p = k // 2
        ho, wo = (h + 2 * p - k) // s + 1, (w + 2 * p - k) // s + 1
        cpad = 64 if cout <= 64 else -(-cout // 128) * 128
        if tile in (11, 24, 25, 40, 41, 44, 45, 46, 47):
            cpad = -(-cout // 256) * 256
        x = torch.randn(n, h, w, cin, device=dev).to(torch.bfloat16)
        wt = (torch.randn(cpad, k * k * cin, device=dev) * 0.05).to(torch.bfloat16)
        b = torch.zeros(cpad, device=dev)
        y = torch.empty(n, ho, wo, cout, device=dev, dtype=torch.bfloat16)
        d = L.ConvDesc()
        d.n, d.h, d.w, d.cin, d.in_c_off, d.in_c_stride = n, h, w, cin, 0, cin
        d.ho, d.wo, d.cout, d.cout_pad, d.out_c_off, d.out_c_stride = ho, wo, cout, cpad, 0, cout
        d.kh = d.kw = k
        d.stride, d.pad, d.act, d.dtype, d.out_layout, d.tile = s, p, L.ACT_SILU, L.DT_BF16, L.OUT_NHWC, tile
        args = (ctypes.byref(d), x.data_ptr(), wt.data_ptr(), b.data_ptr(), y.data_ptr(), None, L.stream_handle(dev))
        for _ in range(3):
            L.check(lib.ycx_conv2d(*args))
        torch.cuda.synchronize()
        lib.ycx_debug_glds_stamps(buf, 1)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            lib.ycx_conv2d(*args)
        e1.record()
        torch.cuda.synchronize()
        lib.ycx_debug_glds_stamps(buf, 1)
        wgs = buf[128]
        print(f"{SHAPES[i]} tile {tile}: {e0.elapsed_time(e1) / 10 * 1e3:.1f} us/launch, {wgs // 10} WGs/launch")
        for wv in (0, 4):
            row = [buf[wv * 8 + b] / wgs for b in range(8)]
            print(f"  wave {wv}: " + "  ".join(f"{n} {v:8.0f}" for n, v in zip(NAMES, row)))
        print(flush=True)


if __name__ == "__main__":
    main()
