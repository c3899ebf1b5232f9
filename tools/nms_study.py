"""NMS workload study (development tool, CPU only): the bench's seeded yolov7 on one
640x640 image through the oracle forward + decode + conf filter, then per large
class: size, kept count, suppressor-edge count (higher-ranked box with IoU > thr),
and the greedy dependency depth. Writes the per-class boxes to an npz so kernel
designs can be simulated offline.

    python tools/nms_study.py [--iou 0.3] [--conf 0.3] [--out /tmp/nms/classes.npz]
"""
import argparse
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "yolo-continuous_amd"), os.path.join(REPO, "tests")]

from oracle import ref_forward, ref_post  # noqa: E402
from helpers import ANCHORS, MASK, make_model  # noqa: E402
from ycx.utils.helper_io import cvt_cfg  # noqa: E402
from ycx.utils.synth import synthetic_images  # noqa: E402


def iou_matrix(b):
    x1, y1, x2, y2 = b[:, 0], b[:, 1], b[:, 2], b[:, 3]
    area = (x2 - x1) * (y2 - y1)
    ix = np.clip(np.minimum(x2[:, None], x2[None]) - np.maximum(x1[:, None], x1[None]), 0, None)
    iy = np.clip(np.minimum(y2[:, None], y2[None]) - np.maximum(y1[:, None], y1[None]), 0, None)
    inter = ix * iy
    return inter / (area[:, None] + area[None] - inter)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iou", type=float, default=0.3)
    ap.add_argument("--conf", type=float, default=0.3)
    ap.add_argument("--size", type=int, default=640)
    ap.add_argument("--out", default="/tmp/nms/classes.npz")
    args = ap.parse_args()
    torch.set_num_threads(os.cpu_count())
    m, sd = make_model('yolov7', 80, 0, 'f32')
    x = synthetic_images(1, 3, args.size, args.size, seed=1000)
    heads = ref_forward.build(cvt_cfg('yolov7'), ANCHORS, 80, sd)(x)
    A = np.asarray(ANCHORS).reshape(-1, 2)
    dec = torch.cat(ref_post.decode_box(heads, A, MASK, 80, (args.size, args.size)), 1)[0]
    cls_conf, cls = dec[:, 5:].max(1)
    score = dec[:, 4] * cls_conf
    keep = score >= args.conf
    xy, wh = dec[:, :2], dec[:, 2:4]
    boxes = torch.cat([xy - wh / 2, xy + wh / 2], 1)[keep].numpy()
    score, cls = score[keep].numpy(), cls[keep].numpy()
    print(f"rows {dec.shape[0]}, candidates {keep.sum().item()}")
    save = {}
    for c in np.unique(cls):
        idx = np.nonzero(cls == c)[0]
        if len(idx) <= 512:
            continue
        order = idx[np.argsort(-score[idx], kind='stable')]
        b = boxes[order]
        S = len(b)
        M = iou_matrix(b.astype(np.float64)) > args.iou
        sup = np.triu(M, 1).T  # sup[i, j]: j < i suppresses-candidate of i
        nsup = sup.sum(1)
        kept = np.zeros(S, bool)
        removed = np.zeros(S, bool)
        depth = np.zeros(S, int)
        for i in range(S):
            if removed[i]:
                continue
            kept[i] = True
            removed |= M[i] & (np.arange(S) > i)
        # fixed-point rounds: a box decides once all its suppressors are decided
        st = np.zeros(S, int)  # 0 undecided 1 kept 2 removed
        rounds = 0
        while (st == 0).any():
            rounds += 1
            new = st.copy()
            for i in np.nonzero(st == 0)[0]:
                js = np.nonzero(sup[i])[0]
                if (st[js] == 1).any():
                    new[i] = 2
                elif (st[js] == 2).all():
                    new[i] = 1
            st = new
        w, h = b[:, 2] - b[:, 0], b[:, 3] - b[:, 1]
        print(f"class {c}: S {S} kept {kept.sum()} edges {nsup.sum()} max nsup {nsup.max()} rounds {rounds} "
              f"w {w.min():.1f}-{np.median(w):.1f}-{w.max():.1f} h {h.min():.1f}-{np.median(h):.1f}-{h.max():.1f}")
        save[f"c{c}"] = b
        save[f"k{c}"] = kept
    np.savez(args.out, **save)


if __name__ == "__main__":
    main()
