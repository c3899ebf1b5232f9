"""Forward vs post split of the bench step (development probe):
    python tests/probes/step_split.py
Times (1) graph forward alone, (2) post alone, (3) forward+post serial,
(4) the two-stream pipeline with the post stream at priority -1 and at 0."""
import os
import sys
import time

import torch

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..")
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "yolo-continuous_amd"))
import bench  # noqa: E402


def timed(fn, n=20, warm=5):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n * 1e3


def main():
    args = bench.parse([])
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    _, det, _, _, _ = bench.setup(args, dev)
    if len(sys.argv) > 1 and sys.argv[1] == "post":  # under rocprofv3: post kernels only
        det.forward()
        print(f"post {timed(det.post):.3f} ms", flush=True)
        return
    print(f"forward {timed(det.forward):.3f} ms  post {timed(det.post):.3f} ms  serial {timed(det):.3f} ms", flush=True)
    from ycx.detect import PipelinedDetector
    for prio in (-1, 0):
        pd = PipelinedDetector(det.model, (args.batch, 3, args.size, args.size), dev, bench.ANCHORS, bench.MASK,
                               depth=2, conf_thres=args.conf, nms_thres=args.iou, max_det=args.max_det)
        pd.s_post = torch.cuda.Stream(dev, priority=prio)
        print(f"pipelined post-priority {prio}: {timed(pd.submit, n=30):.3f} ms/step", flush=True)


if __name__ == "__main__":
    main()
