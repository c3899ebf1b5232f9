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


if __name__ == "__main__" and sys.argv[1:2] != ["concurrent"]:
    main()


class Concurrent:
    """Each slot has its own stream; a batch's forward + post run on its slot's stream,
    so consecutive batches' forwards overlap (fills each other's kernel tails)."""

    def __init__(self, model, shape, dev, depth, prio=(0,), **kw):
        from ycx.detect import Detector
        self.slots = [Detector(model, shape, dev, bench.ANCHORS, bench.MASK, slot=k, **kw) for k in range(depth)]
        self.streams = [torch.cuda.Stream(dev, priority=prio[k % len(prio)]) for k in range(depth)]
        self.i = 0

    def submit(self):
        k = self.i % len(self.slots)
        self.i += 1
        with torch.cuda.stream(self.streams[k]):
            self.slots[k].forward()
            return self.slots[k].post()


def concurrent_main():
    args = bench.parse([])
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    model, det, _, _, _ = bench.setup(args, dev)
    shape = (args.batch, 3, args.size, args.size)
    kw = dict(conf_thres=args.conf, nms_thres=args.iou, max_det=args.max_det)
    for depth, prio in ((2, (0,)), (2, (0, -1)), (3, (0,)), (3, (0, -1)), (4, (0,)), (4, (0, -1))):
        c = Concurrent(model, shape, dev, depth, prio, **kw)
        print(f"concurrent depth {depth} prio {prio}: {timed(c.submit, n=30):.3f} ms/step", flush=True)
        del c
        torch.cuda.empty_cache()


if __name__ == "__main__" and sys.argv[1:2] == ["concurrent"]:
    concurrent_main()
