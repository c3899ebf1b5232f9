"""ORACLE — test infrastructure only. NOT part of the product path.

A CPU fp32 restatement of the reference's inference path
(xin-pu/yolo-continuous: nets/yolo.py Model.forward, nets/common.py blocks,
nets/detect.py head, detect.py decode_box / non_max_suppression /
yolo_correct_boxes, and torchvision.ops.nms as called at detect.py:133).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this package, and only as the checker (or the timed CPU baseline) — never as a
compute path of the HIP product (yolo-continuous_amd/ycx), which has no CPU
fallback.

Pinning: ref_forward and ref_post are checked bit-exact
against golden vectors produced by importing the reference itself in the build
container (tests/golden/make_golden.py -> tests/golden/*.npz). torchvision is
not installed and unpinned (no requirements file), so the NMS primitive is a
restatement of torchvision's CPU nms kernel: "parity unpinned" at that one
boundary.
"""
