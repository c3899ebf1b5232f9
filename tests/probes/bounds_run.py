"""Runs the G1 nets and yolov7 / yolov7-tiny (f32, bf16, fp16, fp8, with the fused
Detector path) on the kernel-side bounds-check library (YCX_LIB=libycx_hip_dbg.so,
built with -DYCX_DEBUG_BOUNDS) and prints one JSON line with the store-violation
count. Launched as a subprocess by tests/test_gpu_debug_bounds.py."""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.dirname(HERE), os.path.join(os.path.dirname(os.path.dirname(HERE)), "yolo-continuous_amd"),
                os.path.dirname(os.path.dirname(HERE))]

import ctypes  # noqa: E402

import torch  # noqa: E402

from helpers import ANCHORS, MASK, g1_case, make_model  # noqa: E402
from ycx import _lib as L  # noqa: E402
from ycx.detect import Detector  # noqa: E402
from ycx.utils.synth import synthetic_images  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    out = (ctypes.c_uint32 * 2)()
    assert L.lib.ycx_debug_bounds(out, 1) == 0, "not the YCX_DEBUG_BOUNDS library"
    manifest = json.load(open(os.path.join(os.path.dirname(HERE), "golden", "manifest.json")))
    runs = 0
    for precision in ("f32", "bf16", "fp16"):
        for name in manifest["g1"]:
            m, _, x, _ = g1_case(manifest, name, precision)
            m.to(dev)
            m(x.to(dev))
            runs += 1
    for net, size, precision in (("yolov7", 160, "bf16"), ("yolov7", 160, "fp16"), ("yolov7", 160, "f32"),
                                 ("yolov7-tiny", 160, "bf16"), ("yolov7", 160, "fp8")):
        m, _ = make_model(net, 80, 0, precision)
        m.to(dev)
        x = synthetic_images(2, 3, size, size, seed=1).to(dev)
        if precision == "fp8":
            m.calibrate_fp8(device=dev, hw=(size, size), n=2)
        m(x)
        det = Detector(m, tuple(x.shape), dev, ANCHORS, MASK, conf_thres=0.3, nms_thres=0.45)
        det(x)
        runs += 2
    torch.cuda.synchronize()
    assert L.lib.ycx_debug_bounds(out, 0) == 0
    print(json.dumps({"runs": runs, "violations": int(out[0]), "first_line": int(out[1])}))


if __name__ == "__main__":
    main()
