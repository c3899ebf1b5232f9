"""Shared test helpers: build models/state_dicts exactly as the fixtures were made."""
import hashlib

import numpy as np
import torch

from ycx.nets.yolo import Model
from ycx.utils.helper_io import cvt_cfg
from ycx.utils.synth import synthetic_head_logits, synthetic_images, synthetic_state_dict

ANCHORS = [[12, 16, 19, 36, 40, 28], [36, 75, 76, 55, 72, 146], [142, 110, 192, 243, 459, 401]]
MASK = [[6, 7, 8], [3, 4, 5], [0, 1, 2]]


def sd_hash(sd):
    h = hashlib.sha256()
    for k in sorted(sd):
        h.update(k.encode())
        h.update(sd[k].detach().cpu().contiguous().numpy().tobytes())
    return h.hexdigest()


def arr_hash(arrs):
    h = hashlib.sha256()
    for a in arrs:
        h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()


def make_model(cfg, nc, w_seed, precision='bf16'):
    """ycx Model with the fixture's synthetic weights; returns (model, state_dict)."""
    m = Model(cvt_cfg(cfg), ANCHORS, nc, precision=precision).eval()
    sd = synthetic_state_dict(m, seed=w_seed)
    m.load_state_dict(sd)
    return m, sd


def make_model_cfg(cfg, nc, w_seed, precision='bf16'):
    """make_model for a config dict (e.g. a built-in network with its head swapped)."""
    m = Model(cfg, ANCHORS, nc, precision=precision).eval()
    sd = synthetic_state_dict(m, seed=w_seed)
    m.load_state_dict(sd)
    return m, sd


def g1_case(manifest, name, precision='bf16'):
    e = manifest['g1'][name]
    m, sd = make_model(e['cfg'], e['nc'], e['w_seed'], precision)
    x = synthetic_images(*e['shape'], seed=e['img_seed'])
    return m, sd, x, e


def g3_heads(e):
    size, bs = e['size'], e['bs']
    shapes = [(bs, size // 32, size // 32), (bs, size // 16, size // 16), (bs, size // 8, size // 8)]
    return synthetic_head_logits(shapes, e['nc'], seed=e['seed'], obj_shift=e['obj_shift'])


def rel_err(a, b):
    """max |a-b| / max |b| (the tolerance measure used for the 1e-3 parity bound)."""
    a = torch.as_tensor(a, dtype=torch.float64)
    b = torch.as_tensor(b, dtype=torch.float64)
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))


def fused_keep_report(cand, cand_rows, counts, keep, kc, b, heads_b, nc, conf, iou, size, max_det, mask=None):
    """Decompose the fused device path's result for image ``b`` against the
    oracle chain run on the SAME head logits (``heads_b``: CPU fp32 NCHW maps of
    that image, Detect order), so every difference is attributed:

      1. decode: the device's candidate rows and values vs the oracle's
         decode_box + filter (detect.py:29-121) -> ``member_flips`` (rows on one
         side of conf_thres only; each must sit at the threshold) and
         ``box_maxdiff`` (max |xyxy difference| over the common rows);
      2. NMS: the oracle's greedy NMS (torchvision semantics) run on the
         DEVICE's own candidates must give exactly the device's keep rows
         (``nms_exact``; this is the bit-exact-keep-indices claim);
      3. end to end: ``keep_flips`` = |device keep rows ^ oracle keep rows|,
         which can only come from 1. (sigmoid/exp ulps on the device).
    Returns a dict; tests print it and assert on each part."""
    from oracle import ref_post
    A = np.asarray(ANCHORS).reshape(-1, 2)
    dec = torch.cat(ref_post.decode_box([h.unsqueeze(0) if h.dim() == 3 else h for h in heads_b], A, mask or MASK, nc,
                                        (size, size)), 1)
    ref_rows, _ = ref_post.nms_keep_rows(dec.clone(), nc, conf, iou)
    ref_rows = ref_rows[0].numpy()
    # oracle filter on its own decode (xyxy from xywh, score = obj * max cls >= conf)
    d0 = dec[0]
    cls_conf, cls_id = torch.max(d0[:, 5:5 + nc], 1)
    score = d0[:, 4] * cls_conf
    ref_pass = set(torch.nonzero(score >= conf).reshape(-1).tolist())
    # device candidates
    n = int(counts[b])
    rows = np.sort(cand_rows[b, :n].numpy().astype(np.int64))
    c = cand[b, torch.as_tensor(rows)] if n else cand[b, :0]
    cls = c[:, 6].contiguous().view(torch.int32).long()
    row_f = c[:, 7].contiguous().view(torch.int32).long()
    assert torch.equal(row_f, torch.as_tensor(rows)), "ycx_cand.row disagrees with cand_rows"
    dev_pass = set(rows.tolist())
    member = sorted(dev_pass ^ ref_pass)
    # each membership flip must sit at the threshold (|score - conf| a few ulps of conf)
    boundary = [abs(float(score[r]) - conf) for r in member]
    common = sorted(dev_pass & ref_pass)
    box_maxdiff = 0.0
    if common:
        idx = torch.as_tensor(common)
        xywh = d0[idx, :4]
        ref_xyxy = torch.stack([xywh[:, 0] - xywh[:, 2] / 2, xywh[:, 1] - xywh[:, 3] / 2,
                                xywh[:, 0] + xywh[:, 2] / 2, xywh[:, 1] + xywh[:, 3] / 2], 1)
        pos = np.searchsorted(rows, np.asarray(common))
        box_maxdiff = float((c[torch.as_tensor(pos), :4] - ref_xyxy).abs().max())
        cls_same = bool(torch.equal(cls[torch.as_tensor(pos)], cls_id[idx]))
    else:
        cls_same = True
    # oracle NMS on the device's own candidates (class asc, row order within a class)
    own = []
    scores = c[:, 4] * c[:, 5]
    for k in torch.unique(cls).tolist():
        sel = torch.nonzero(cls == k).reshape(-1)
        kept = ref_post.nms(c[sel, :4], scores[sel], iou)
        own.append(torch.as_tensor(rows)[sel[kept]])
    own = torch.cat(own).numpy() if own else np.zeros((0,), np.int64)
    k = int(kc[b])
    got = keep[b, :min(k, max_det)].numpy().astype(np.int64)
    nms_exact = k == len(own) and np.array_equal(got, own[:max_det])
    flipped = set(own.tolist()) ^ set(ref_rows.tolist())
    # explain the flips: in every class that has one, the flip that comes first in
    # the greedy order must be a direct threshold crossing -- some higher-ranked
    # KEPT candidate of that class whose fp32 IoU with it lies on different sides of
    # nms_thres under the device's and the oracle's boxes, or a score-order swap;
    # later flips in the class can cascade from it
    unexplained = 0
    if flipped and common:
        ref_box = {}
        for r, bx in zip(common, ref_xyxy.numpy()):
            ref_box[r] = bx
        dev_box = {int(r): c[i, :4].numpy() for i, r in enumerate(rows)}
        ref_score = {r: float(np.float32(d0[r, 4]) * np.float32(cls_conf[r])) for r in common}
        dev_score = {int(r): float(scores[i]) for i, r in enumerate(rows)}
        cls_of = {int(r): int(cls[i]) for i, r in enumerate(rows)}
        for kcls in sorted({cls_of[r] for r in flipped if r in cls_of}):
            members = [r for r in common if cls_of.get(r) == kcls]
            order = sorted(members, key=lambda r: (-ref_score[r], r))
            rank = {r: i for i, r in enumerate(order)}
            first = min((r for r in flipped if cls_of.get(r) == kcls and r in rank), key=lambda r: rank[r])
            ref_kept = set(ref_rows.tolist())
            higher = [r for r in order[:rank[first]] if r in ref_kept]  # kept by both (all above `first` agree)
            dev_order = sorted(members, key=lambda r: (-dev_score[r], r))
            swapped = dev_order.index(first) != rank[first]

            def ious(boxes_of):
                a = np.asarray([boxes_of[r] for r in higher], np.float32).reshape(-1, 4)
                f = np.asarray(boxes_of[first], np.float32)
                with np.errstate(invalid='ignore', divide='ignore'):
                    w = np.maximum(np.float32(0), np.minimum(a[:, 2], f[2]) - np.maximum(a[:, 0], f[0]))
                    h = np.maximum(np.float32(0), np.minimum(a[:, 3], f[3]) - np.maximum(a[:, 1], f[1]))
                    inter = w * h
                    area_a = (a[:, 2] - a[:, 0]) * (a[:, 3] - a[:, 1])
                    area_f = (f[2] - f[0]) * (f[3] - f[1])
                    return (inter / (area_a + area_f - inter)).astype(np.float64) > iou
            crossing = bool(np.any(ious(dev_box) != ious(ref_box))) if higher else False
            if not (crossing or swapped):
                unexplained += 1
    keep_flips = len(set(got.tolist()) ^ set(ref_rows[:max_det].tolist())) if k <= max_det else len(flipped)
    return dict(n_cand=len(dev_pass), n_cand_ref=len(ref_pass), member_flips=len(member),
                member_max_dist=max(boundary) if boundary else 0.0, box_maxdiff=box_maxdiff, cls_same=cls_same,
                nms_exact=bool(nms_exact), n_keep=k, n_keep_ref=len(ref_rows), keep_flips=keep_flips,
                unexplained_flips=unexplained)


def decoded_flip_report(dec_dev, dec_ref, nc, conf, iou):
    """Attribute every difference between the oracle's greedy chain (filter +
    per-class NMS, detect.py:98-137) run on two decoded tensors of ONE image --
    ``dec_dev`` from the device's forward, ``dec_ref`` from the oracle's -- to
    the forward's perturbation of scores and boxes:

      - ``member_flips``: rows that pass conf_thres on one side only; each must
        lie within ``max_score_delta`` of the threshold (``member_far`` counts
        those that do not);
      - keep flips: in every class with a differing keep decision, the flip
        that comes first in the oracle's greedy order must be caused directly:
        a membership flip at or above it, a score-order swap at or above it, or
        a kept higher-ranked box whose fp32 IoU with it lies on different sides
        of nms_thres under the two box sets (``unexplained_flips`` counts the
        classes where none holds; later flips of a class cascade from the
        first).
    Rows are compared by index, so both tensors must be (rows, 5 + nc) xywh."""
    from oracle import ref_post

    def prep(d):
        d = d.detach().to('cpu', torch.float32).clone()
        xyxy = torch.stack([d[:, 0] - d[:, 2] / 2, d[:, 1] - d[:, 3] / 2,
                            d[:, 0] + d[:, 2] / 2, d[:, 1] + d[:, 3] / 2], 1)
        cc, ci = torch.max(d[:, 5:5 + nc], 1)
        return xyxy.numpy(), (d[:, 4] * cc).numpy(), ci.numpy()

    bd, sd_, cd = prep(dec_dev)
    br, sr, cr = prep(dec_ref)
    kd = ref_post.nms_keep_rows(dec_dev.detach().to('cpu', torch.float32).clone().unsqueeze(0), nc, conf, iou)[0][0]
    kr = ref_post.nms_keep_rows(dec_ref.detach().to('cpu', torch.float32).clone().unsqueeze(0), nc, conf, iou)[0][0]
    kd, kr = set(kd.tolist()), set(kr.tolist())
    pd_, pr = set(np.flatnonzero(sd_ >= conf).tolist()), set(np.flatnonzero(sr >= conf).tolist())
    member = pd_ ^ pr
    union = sorted(pd_ | pr)
    delta = float(np.abs(sd_[union] - sr[union]).max()) if union else 0.0
    member_far = sum(1 for r in member if abs(float(sr[r]) - conf) > delta)
    cls_flips = sum(1 for r in union if cd[r] != cr[r])
    flipped = kd ^ kr

    def iou_gt(b, i, js):
        a = b[js].astype(np.float32).reshape(-1, 4)
        f = b[i].astype(np.float32)
        with np.errstate(invalid='ignore', divide='ignore'):
            w = np.maximum(np.float32(0), np.minimum(a[:, 2], f[2]) - np.maximum(a[:, 0], f[0]))
            h = np.maximum(np.float32(0), np.minimum(a[:, 3], f[3]) - np.maximum(a[:, 1], f[1]))
            inter = w * h
            den = (a[:, 2] - a[:, 0]) * (a[:, 3] - a[:, 1]) + (f[2] - f[0]) * (f[3] - f[1]) - inter
            return (inter / den).astype(np.float64) > iou

    unexplained, classes = 0, 0
    for k in sorted({int(cr[r]) for r in flipped} | {int(cd[r]) for r in flipped}):
        members = [r for r in union if int(cr[r]) == k or int(cd[r]) == k]
        cand_f = [r for r in flipped if r in members]
        if not cand_f:
            continue
        classes += 1
        order_r = sorted(members, key=lambda r: (-float(sr[r]), r))
        order_d = sorted(members, key=lambda r: (-float(sd_[r]), r))
        rank = {r: i for i, r in enumerate(order_r)}
        first = min(cand_f, key=lambda r: rank[r])
        pos = rank[first]
        above = order_r[:pos]
        if any(r in member or cd[r] != cr[r] for r in above + [first]):
            continue  # a membership / class flip at or above it changes the greedy input
        if order_d[:pos + 1] != order_r[:pos + 1]:
            continue  # a score-order swap at or above it
        higher = [r for r in above if r in kr]  # kept by both chains (all decisions above agree)
        if higher and bool(np.any(iou_gt(bd, first, higher) != iou_gt(br, first, higher))):
            continue  # an IoU threshold crossing against a kept higher-ranked box
        unexplained += 1
    return dict(n_pass_dev=len(pd_), n_pass_ref=len(pr), member_flips=len(member), member_far=member_far,
                max_score_delta=delta, cls_flips=cls_flips, n_keep_dev=len(kd), n_keep_ref=len(kr),
                keep_flips=len(flipped), flip_classes=classes, unexplained_flips=unexplained)
