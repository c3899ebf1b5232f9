"""Development probe: predict (f32, 640, 773x512 image) against the oracle chain, printing
the rows where the two disagree (tests/test_gpu_image.py::test_predict_vs_oracle_chain)."""
import os
import sys
import tempfile

import numpy as np
import torch
import yaml

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(HERE, '..'), os.path.join(HERE, '..', '..'), os.path.join(HERE, '..', '..', 'yolo-continuous_amd')]
from helpers import ANCHORS, MASK  # noqa: E402
from oracle import ref_forward, ref_letterbox, ref_post  # noqa: E402
from ycx.detect import predict  # noqa: E402
from ycx.nets.yolo import Model  # noqa: E402
from ycx.utils.helper_io import cvt_cfg  # noqa: E402
from ycx.utils.synth import synthetic_state_dict  # noqa: E402

size, hw, prec = 640, (512, 773), os.environ.get('PREC', 'f32')
plan = dict(device=0, image_size=size, image_chan=3, labels=['raccoon'], model_cfg='yolov7-tiny', anchors=ANCHORS,
            anchors_mask=MASK)
d = tempfile.mkdtemp()
cfg = os.path.join(d, 'plan.yaml')
open(cfg, 'w').write(yaml.safe_dump(plan))
img = np.random.default_rng(4).integers(0, 256, size=hw + (3,), dtype=np.uint8)
got = predict(cfg, image=img, weights='synthetic', device='cuda:0', conf_threshold=0.3, nms_threshold=0.3,
              precision=prec)
net_cfg = cvt_cfg('yolov7-tiny')
sd = synthetic_state_dict(Model(net_cfg, ANCHORS, 1), seed=0)
x = torch.from_numpy(ref_letterbox.letterbox_tensor(img, (size, size))).unsqueeze(0)
heads = ref_forward.build(net_cfg, ANCHORS, 1, sd)(x)
A = np.asarray(ANCHORS).reshape(-1, 2)
dec = torch.cat(ref_post.decode_box(heads, A, MASK, 1, (size, size)), 1)
res = ref_post.non_max_suppression(dec, 1, (size, size), np.array(img.shape[0:2]), True, 0.3, 0.3)[0]


def want(row):
    y1, x1, y2, x2 = row[0], row[1], row[2], row[3]
    return (max(0, int(np.floor(x1))), max(0, int(np.floor(y1))), min(img.shape[1], int(np.floor(x2))),
            min(img.shape[0], int(np.floor(y2))), float(row[4] * row[5]))


G = [(tb.left, tb.top, tb.right, tb.bottom, float(tb.score)) for tb in got]
W = [want(r) for r in res]
print('n got', len(G), 'n want', len(W))
for i, (g, w) in enumerate(zip(G, W)):
    ok = max(abs(a - b) for a, b in zip(g[:4], w[:4])) <= 1 and abs(g[4] - w[4]) <= 1e-3
    if not ok:
        print(i, 'got', g, 'want', w, 'raw', [float(v) for v in res[i][:7]])
for i in range(490, min(505, len(G))):
    print(i, G[i], W[i])
