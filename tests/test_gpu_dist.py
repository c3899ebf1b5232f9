"""The N > 1 code path on one GPU: a one-rank RCCL process group and the
ConcurrentDetector issuing the detections all-gather on each batch's own stream
(``submit(then=...)``, what bench.py runs at N > 1). The gathered result of a
one-rank group is the rank's own result, which must equal the single-stream
Detector's."""
import os
import socket

import pytest
import torch
import torch.distributed as dist

from helpers import ANCHORS, MASK, make_model
from ycx.detect import ConcurrentDetector, Detector
from ycx.dist import gather_detections
from ycx.utils.synth import synthetic_images

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_concurrent_detector_with_rccl_gather(device):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    dist.init_process_group("nccl", device_id=device, rank=0, world_size=1)
    try:
        m, _ = make_model('yolov7-tiny', 1, 0, 'bf16')
        m.to(device)
        shape = (2, 3, 320, 320)
        ref = Detector(m, shape, device, ANCHORS, MASK, use_graph=True)
        cd = ConcurrentDetector(m, shape, device, ANCHORS, MASK, depth=3, use_graph=True)

        def gather(dets, keep, kc):
            g_dets, g_kc, g_keep = gather_detections(dets, kc, keep)
            return g_dets, g_keep, g_kc

        imgs = [synthetic_images(*shape, seed=40 + i).to(device) for i in range(5)]
        outs = [cd.submit(x, then=gather)[:3] for x in imgs]
        cd.synchronize()
        torch.cuda.synchronize()
        for x, (dets, keep, kc) in zip(imgs, outs):
            rd, rk, rc = ref(x)
            torch.cuda.synchronize()
            assert torch.equal(kc, rc) and torch.equal(keep, rk) and torch.equal(dets, rd)
    finally:
        dist.destroy_process_group()
