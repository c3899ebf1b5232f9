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
