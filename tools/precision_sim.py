"""Where does the bf16 plan's error come from? (development tool, CPU only)

Runs the oracle forward (oracle/ref_forward.py) with the bf16 engine's rounding
simulated per layer class -- BN folded into the weights in float64, weights
rounded to bf16, activations rounded to bf16 at every conv output (heads stay
fp32), fp32 accumulation -- with parts of that rounding switched off, and prints
the decoded box / obj / cls error (max |sim - fp32| / max |fp32|) of each mode.

    python tools/precision_sim.py [--size 640] [--bs 2]
"""
import argparse
import os
import sys

import numpy as np
import torch
import torch.nn.functional as F

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "yolo-continuous_amd"), os.path.join(REPO, "tests")]

from oracle import ref_forward, ref_post  # noqa: E402
from helpers import ANCHORS, MASK, make_model  # noqa: E402
from ycx.utils.helper_io import cvt_cfg  # noqa: E402
from ycx.utils.synth import synthetic_images  # noqa: E402

MODE = dict(w=True, a=True, skip_last=0, head_w=True, head_a=True)
COUNT = [0]
TOTAL = [0]


def bf(t):
    return t.to(torch.bfloat16).to(torch.float32)


def fold(p):
    w = p('conv.weight').double()
    std = (p('bn.running_var').double() + 1e-5).sqrt()
    t = p('bn.weight').double() / std
    b = p('bn.bias').double() - p('bn.running_mean').double() * t
    return (w * t.reshape(-1, 1, 1, 1)), b


def sim_conv(p, x, k, s, act, pad=None):
    pad = k // 2 if pad is None else pad
    COUNT[0] += 1
    late = COUNT[0] > TOTAL[0] - MODE['skip_last']
    w, b = fold(p)
    w = w.float()
    if MODE['w'] and not late:
        w = bf(w)
    xin = x
    y = F.conv2d(xin, w, b.float(), s, pad)
    y = ref_forward._apply_act(y, act)
    if MODE['a'] and not late:
        y = bf(y)
    return y


def run(fwd, x):
    COUNT[0] = 0
    return fwd(x)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=640)
    ap.add_argument("--bs", type=int, default=2)
    args = ap.parse_args()
    torch.set_num_threads(os.cpu_count())
    m, sd = make_model('yolov7', 80, 0, 'bf16')
    cfg = cvt_cfg('yolov7')
    x = synthetic_images(args.bs, 3, args.size, args.size, seed=3)
    ref = ref_forward.build(cfg, ANCHORS, 80, sd)(x)
    A = np.asarray(ANCHORS).reshape(-1, 2)
    dref = torch.cat(ref_post.decode_box(ref, A, MASK, 80, (args.size, args.size)), 1)
    orig_conv = ref_forward._conv
    ref_forward._conv = sim_conv
    # count convs once
    MODE.update(w=False, a=False, skip_last=0)
    TOTAL[0] = 10 ** 9
    run(ref_forward.build(cfg, ANCHORS, 80, sd), x[:1, :, :64, :64])
    TOTAL[0] = COUNT[0]
    print("convs through _conv:", TOTAL[0])
    # Detect heads: inputs are bf16 activations already; head weights in bf16 unless head_w False
    orig_run = ref_forward.run_module

    def run_module(mm, a, p, xx):
        if mm == 'Detect' and MODE['head_w']:
            outs = []
            for name, xi in (('P5', xx[2]), ('P4', xx[1]), ('P3', xx[0])):
                outs.append(F.conv2d(xi, bf(p(f'yolo_head_{name}.weight')), p(f'yolo_head_{name}.bias')))
            return outs
        return orig_run(mm, a, p, xx)
    ref_forward.run_module = run_module
    modes = [
        ("bf16 everywhere (the engine)", dict(w=True, a=True, skip_last=0, head_w=True)),
        ("fp32 weights, bf16 activations", dict(w=False, a=True, skip_last=0, head_w=False)),
        ("bf16 weights, fp32 activations", dict(w=True, a=False, skip_last=0, head_w=True)),
        ("bf16, head 1x1 weights fp32", dict(w=True, a=True, skip_last=0, head_w=False)),
        ("bf16, last 3 convs fp32 (RepConvs)", dict(w=True, a=True, skip_last=3, head_w=False)),
        ("bf16, last 12 convs fp32", dict(w=True, a=True, skip_last=12, head_w=False)),
        ("bf16, last 30 convs fp32", dict(w=True, a=True, skip_last=30, head_w=False)),
    ]
    for name, md in modes:
        MODE.update(md)
        out = run(ref_forward.build(cfg, ANCHORS, 80, sd), x)
        dec = torch.cat(ref_post.decode_box(out, A, MASK, 80, (args.size, args.size)), 1)
        errs = {}
        for k, sl in (('box', slice(0, 4)), ('obj', slice(4, 5)), ('cls', slice(5, 85))):
            errs[k] = float((dec[..., sl].double() - dref[..., sl].double()).abs().max() /
                            dref[..., sl].double().abs().max())
        hd = max(float((o.double() - r.double()).abs().max() / r.double().abs().max()) for o, r in zip(out, ref))
        print(f"{name:40s} heads {hd:.5f}  decoded " + "  ".join(f"{k} {v:.2e}" for k, v in errs.items()), flush=True)
    ref_forward._conv = orig_conv
    ref_forward.run_module = orig_run


if __name__ == "__main__":
    main()
