"""Workload for the rocprofv3 PMC passes (HBM traffic per kernel launch).

Run under `rocprofv3 --pmc FETCH_SIZE ...` and again under `--pmc WRITE_SIZE`
(separate passes: the TCC slots cannot hold both, MI355X_MICROARCH.md). It
runs, in this dispatch order:

1. one calibration copy through ycx_copy_channels with a known byte count,
   larger than the 256 MiB Infinity Cache (read 512 MiB, write 512 MiB);
2. ONE eager forward of the bench plan (ycx_run_ops, no HIP graph, so each
   op is one dispatch in op order) followed by the post-processing;
and writes the op list (name, flops, shape) to gpurun_out/pmc_ops.json so
tools/pmc_traffic.py can attribute dispatches to plan ops.

    rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o run --output-format csv -- \
        python3 tools/pmc_workload.py
"""
from __future__ import annotations

import ctypes
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "yolo-continuous_amd")]

import torch  # noqa: E402

import bench  # noqa: E402
from ycx import _lib as L  # noqa: E402

CAL_SHAPE = (32, 128, 128, 512)  # bf16 NHWC: 512 MiB


def calibration_copy(dev):
    n, h, w, c = CAL_SHAPE
    x = torch.ones(CAL_SHAPE, dtype=torch.bfloat16, device=dev)
    y = torch.empty_like(x)
    d = L.CopyDesc()
    d.n, d.h, d.w, d.c, d.in_c_off, d.in_c_stride = n, h, w, c, 0, c
    d.out_c_off, d.out_c_stride, d.scale, d.dtype, d.out_layout = 0, c, 1, L.DT_BF16, L.OUT_NHWC
    torch.cuda.synchronize()
    L.check(L.lib.ycx_copy_channels(ctypes.byref(d), x.data_ptr(), y.data_ptr(), L.stream_handle(dev)))
    torch.cuda.synchronize()
    return x.numel() * 2


def main():
    args = bench.parse(sys.argv[1:])
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    _, det, _, _, shape = bench.setup(args, dev, use_graph=False)
    torch.cuda.synchronize()
    cal_bytes = calibration_copy(dev)
    det()  # eager: ycx_run_ops (one dispatch per op) + decode_filter + sort_nms
    torch.cuda.synchronize()
    os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
    with open(os.path.join(REPO, "gpurun_out", "pmc_ops.json"), "w") as f:
        json.dump(dict(shape=list(shape), calibration=dict(kernel="copy_kernel", read_bytes=cal_bytes,
                                                          write_bytes=cal_bytes),
                       ops=det.engine.op_info), f, indent=1)


if __name__ == "__main__":
    main()
