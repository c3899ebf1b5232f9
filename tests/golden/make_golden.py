"""Generate the golden fixtures by running the REFERENCE itself (build container only).

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

Imports xin-pu/yolo-continuous read-only from /root/reference:
nets.yolo.Model for the forward, and detect.py for decode_box /
non_max_suppression with ``cv2`` stubbed (unused by those functions) and
``torchvision.ops.nms`` replaced by oracle.ref_post.nms (torchvision is not
installed and not pinned: parity unpinned at that primitive). Weights follow
ycx.utils.synth (seeded, platform independent); a hash of every state_dict is
stored so tests can prove they regenerate the same tensors.

Outputs (data only, no reference source):
  tests/golden/manifest.json             configs, seeds, shapes, hashes
  tests/golden/g1_ops.npz                per-op mini networks (G1)
  tests/golden/g2_nets.npz               yolov7 @160 bs1 nc80, yolov7-tiny @640 bs1 nc1 (G2)
  tests/golden/g3_post.npz               decode + NMS (G3)
  yolo-continuous_amd/ycx/cfg/net/*.json the reference network YAMLs as JSON
"""
from __future__ import annotations

import hashlib
import json
import os
import sys
import types

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
REF = os.environ.get("YCX_REFERENCE", "/root/reference")
GOLD = os.path.join(REPO, "tests", "golden")
NETDIR = os.path.join(REPO, "yolo-continuous_amd", "ycx", "cfg", "net")
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "yolo-continuous_amd"))

from ycx.utils.synth import synthetic_head_logits, synthetic_images, synthetic_state_dict  # noqa: E402
from oracle import ref_post  # noqa: E402

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


def import_reference():
    sys.path.insert(0, REF)
    sys.modules.setdefault('cv2', types.ModuleType('cv2'))
    tv = types.ModuleType('torchvision')
    tv.ops = types.ModuleType('torchvision.ops')
    tv.ops.nms = ref_post.nms
    sys.modules['torchvision'] = tv
    sys.modules['torchvision.ops'] = tv.ops
    from nets.yolo import Model  # noqa
    import detect  # noqa
    from utils.helper_io import cvt_cfg  # noqa
    return Model, detect, cvt_cfg


def stem(cin_out=32, act=None):
    a = [cin_out, 3, 1] if act is None else [cin_out, 3, 1, 'None', 1, act]
    return [-1, 1, 'Conv', a]


def mini_nets():
    leaky = 'nn.LeakyReLU(0.1)'
    d = lambda bb, hd=None: {'depth_multiple': 1.0, 'width_multiple': 1.0, 'backbone': bb, 'head': hd or []}
    return {
        'conv_k3s1_cin32': (d([stem(), [-1, 1, 'Conv', [64, 3, 1]]]), 3),
        'conv_k3s2_cin32': (d([stem(), [-1, 1, 'Conv', [64, 3, 2]]]), 3),
        'conv_k1_cin64': (d([stem(), [-1, 1, 'Conv', [64, 3, 1]], [-1, 1, 'Conv', [128, 1, 1]],
                             [-1, 1, 'Conv', [256, 3, 2]], [-1, 1, 'Conv', [128, 1, 1]]]), 3),
        'conv_leaky': (d([stem(act=leaky), [-1, 1, 'Conv', [64, 3, 2, 'None', 1, leaky]],
                          [-1, 1, 'Conv', [32, 1, 1, 'None', 1, leaky]]]), 3),
        'stem_s2_leaky': (d([[-1, 1, 'Conv', [32, 3, 2, 'None', 1, leaky]], [-1, 1, 'Conv', [64, 1, 1]]]), 3),
        'pools': (d([stem(), [-1, 1, 'Conv', [64, 3, 1]], [-1, 1, 'MP', []], [-1, 1, 'SP', [5]], [-2, 1, 'SP', [9]],
                     [-3, 1, 'SP', [13]], [[-1, -2, -3, -4], 1, 'Concat', [1]], [-1, 1, 'Conv', [64, 1, 1]]]), 3),
        'upsample_concat': (d([stem(), [-1, 1, 'Conv', [64, 3, 2]], [-1, 1, 'Conv', [64, 1, 1]],
                               [-1, 1, 'nn.Upsample', ['None', 2, 'nearest']], [[-1, 0], 1, 'Concat', [1]],
                               [-1, 1, 'Conv', [64, 3, 1]]]), 3),
        'upsample_shared': (d([stem(), [-1, 1, 'Conv', [64, 3, 2]], [-1, 1, 'nn.Upsample', ['None', 2, 'nearest']],
                               [[-1, 0], 1, 'Concat', [1]], [[2, 0], 1, 'Concat', [1]],
                               [[-1, -2], 1, 'Concat', [1]], [-1, 1, 'Conv', [64, 1, 1]]]), 3),
        'sppcspc': (d([stem(), [-1, 1, 'Conv', [64, 3, 1]], [-1, 1, 'SPPCSPC', [64]]]), 3),
        'repconv': (d([stem(), [-1, 1, 'Conv', [64, 3, 1]], [-1, 1, 'RepConv', [128, 3, 1]],
                       [-1, 1, 'RepConv', [128, 3, 1]], [-1, 1, 'RepConv', [128, 3, 2]]]), 3),
        'csp_blocks': (d([stem(), [-1, 1, 'Conv', [64, 3, 1]], [-1, 2, 'BottleneckCSPA', [64]],
                          [-1, 1, 'BottleneckCSPB', [64]], [-1, 2, 'BottleneckCSPC', [64]], [-1, 1, 'SPPF', [64, 5]],
                          [-1, 1, 'SPP', [64]], [-1, 2, 'Bottleneck', [64]]]), 3),
        'detect': (d([stem(), [-1, 1, 'Conv', [64, 3, 2]], [-1, 1, 'Conv', [128, 3, 2]], [-1, 1, 'Conv', [256, 3, 2]]],
                     [[[1, 2, 3], 1, 'Detect', ['nc', 'anchors']]]), 3),
        'idetect': (d([stem(), [-1, 1, 'Conv', [64, 3, 2]], [-1, 1, 'Conv', [128, 3, 2]], [-1, 1, 'Conv', [256, 3, 2]]],
                      [[[1, 2, 3], 1, 'IDetect', ['nc', 'anchors']]]), 3),
        # round 2 (appended: seeds follow the position): an upsample that cannot fuse into its
        # producer (a pool) lands in the middle of a concat buffer (channel offset 32)
        'upsample_offset': (d([stem(), [-1, 1, 'Conv', [64, 3, 2]], [-1, 1, 'MP', []],
                               [-1, 1, 'nn.Upsample', ['None', 2, 'nearest']], [0, 1, 'Conv', [32, 3, 2]],
                               [[-1, -2, 1], 1, 'Concat', [1]], [-1, 1, 'Conv', [64, 1, 1]]]), 3),
        # IAuxDetect (nets/iaux_detect.py): main heads on layers 1-3, aux heads on 4-6; eval output
        # with the strides set on the module (its stride is None, like IDetect's)
        'iauxdetect': (d([stem(), [-1, 1, 'Conv', [64, 3, 2]], [-1, 1, 'Conv', [128, 3, 2]],
                          [-1, 1, 'Conv', [256, 3, 2]], [1, 1, 'Conv', [64, 1, 1]], [2, 1, 'Conv', [128, 1, 1]],
                          [3, 1, 'Conv', [256, 1, 1]]],
                         [[[1, 2, 3, 4, 5, 6], 1, 'IAuxDetect', ['nc', 'anchors']]]), 3),
    }

AUX_STRIDES = [2.0, 4.0, 8.0]  # 24 / (12, 6, 3), as the build derives them


def run_ref(Model, cfg, nc, x, seed, idetect_raw=False, strides=None):
    m = Model(cfg, ANCHORS, nc).eval()
    sd = synthetic_state_dict(m, seed=seed)
    m.load_state_dict(sd)
    if idetect_raw:  # the reference's IDetect eval branch crashes (stride=None): take the raw maps
        m.model[-1].training = True
    if strides is not None:  # eval branch with the strides set on the head (nothing else touched)
        m.model[-1].stride = torch.tensor(strides)
    with torch.no_grad():
        y = m(x)
    if strides is not None:  # (cat(z, 1), x[:nl]) -> [z, x0, x1, ...]
        y = [y[0]] + list(y[1])
    ys = y if isinstance(y, (list, tuple)) else [y]
    return [t.detach().numpy().copy() for t in ys], sd_hash(sd), len(sd)


def make_idetect_eval(Model, manifest):
    """G4: IDetect's eval branch run by the reference itself. Its stride is
    None (nets/idetect.py:8) so eval raises; here the strides the build uses
    (input size / ny) are set on the module first, nothing else is touched."""
    cfg, nc = mini_nets()['idetect']
    x = synthetic_images(2, 3, 24, 24, seed=300)
    m = Model(cfg, ANCHORS, nc).eval()
    sd = synthetic_state_dict(m, seed=12)
    m.load_state_dict(sd)
    strides = [2.0, 4.0, 8.0]  # 24 / (12, 6, 3)
    m.model[-1].stride = torch.tensor(strides)
    with torch.no_grad():
        z, xs = m(x)
    g4 = {'idetect_eval/z': z.numpy().copy()}
    for j, t in enumerate(xs):
        g4[f'idetect_eval/x{j}'] = t.numpy().copy()
    manifest['g4'] = {'idetect_eval': dict(cfg=cfg, nc=nc, shape=[2, 3, 24, 24], img_seed=300, w_seed=12,
                                           strides=strides, sd_hash=sd_hash(sd), n_x=len(xs))}
    np.savez(os.path.join(GOLD, 'g4_idetect.npz'), **g4)
    print('G4 idetect_eval', z.shape, [t.shape for t in xs])


def add_g1(Model, names):
    """Append G1 cases (by name) to an existing g1_ops.npz / manifest; the seeds
    come from the case's position in mini_nets(), exactly as a full run sets them."""
    with open(os.path.join(GOLD, 'manifest.json')) as f:
        manifest = json.load(f)
    g1 = dict(np.load(os.path.join(GOLD, 'g1_ops.npz')))
    nets = list(mini_nets().items())
    for i, (name, (cfg, nc)) in enumerate(nets):
        if name not in names:
            continue
        x = synthetic_images(2, 3, 24, 24, seed=100 + i)
        strides = AUX_STRIDES if name == 'iauxdetect' else None
        outs, h, nkeys = run_ref(Model, cfg, nc, x, seed=i, idetect_raw=(name == 'idetect'), strides=strides)
        for k in [k for k in g1 if k.startswith(name + '/')]:
            del g1[k]
        for j, o in enumerate(outs):
            g1[f'{name}/{j}'] = o
        manifest['g1'][name] = dict(cfg=cfg, nc=nc, shape=[2, 3, 24, 24], img_seed=100 + i, w_seed=i,
                                    sd_hash=h, n_keys=nkeys, n_out=len(outs))
        if strides is not None:
            manifest['g1'][name]['strides'] = strides
        print('G1+', name, [o.shape for o in outs])
    np.savez(os.path.join(GOLD, 'g1_ops.npz'), **g1)
    with open(os.path.join(GOLD, 'manifest.json'), 'w') as f:
        json.dump(manifest, f, indent=1)


def main():
    Model, detect, cvt_cfg = import_reference()
    if len(sys.argv) > 2 and sys.argv[1] == 'g1add':  # append named G1 cases only
        add_g1(Model, sys.argv[2:])
        return
    if len(sys.argv) > 1 and sys.argv[1] == 'g4':  # add only the IDetect-eval fixture
        with open(os.path.join(GOLD, 'manifest.json')) as f:
            manifest = json.load(f)
        make_idetect_eval(Model, manifest)
        with open(os.path.join(GOLD, 'manifest.json'), 'w') as f:
            json.dump(manifest, f, indent=1)
        return
    torch.set_num_threads(8)
    os.makedirs(NETDIR, exist_ok=True)
    for name in ('yolov7', 'yolov7-tiny'):
        cfg = cvt_cfg(os.path.join(REF, 'cfg', 'net', f'{name}.yaml'))
        with open(os.path.join(NETDIR, f'{name}.json'), 'w') as f:
            json.dump(cfg, f, indent=1)
    manifest = {'anchors': ANCHORS, 'anchors_mask': MASK, 'g1': {}, 'g2': {}, 'g3': {}}

    # ---- G1: per-op mini networks, 2 x 3 x 24 x 24 (pixel counts off the tile grid) ----
    g1 = {}
    for i, (name, (cfg, nc)) in enumerate(mini_nets().items()):
        x = synthetic_images(2, 3, 24, 24, seed=100 + i)
        strides = AUX_STRIDES if name == 'iauxdetect' else None
        outs, h, nkeys = run_ref(Model, cfg, nc, x, seed=i, idetect_raw=(name == 'idetect'), strides=strides)
        for j, o in enumerate(outs):
            g1[f'{name}/{j}'] = o
        manifest['g1'][name] = dict(cfg=cfg, nc=nc, shape=[2, 3, 24, 24], img_seed=100 + i, w_seed=i,
                                    sd_hash=h, n_keys=nkeys, n_out=len(outs))
        if strides is not None:
            manifest['g1'][name]['strides'] = strides
        print('G1', name, [o.shape for o in outs])
    np.savez(os.path.join(GOLD, 'g1_ops.npz'), **g1)

    # ---- G2: full networks ----
    g2 = {}
    for name, net, nc, hw in (('yolov7_160', 'yolov7', 80, 160), ('tiny_640', 'yolov7-tiny', 1, 640)):
        cfg = cvt_cfg(os.path.join(REF, 'cfg', 'net', f'{net}.yaml'))
        x = synthetic_images(1, 3, hw, hw, seed=7)
        outs, h, nkeys = run_ref(Model, cfg, nc, x, seed=0)
        for j, o in enumerate(outs):
            g2[f'{name}/{j}'] = o
        manifest['g2'][name] = dict(net=net, nc=nc, shape=[1, 3, hw, hw], img_seed=7, w_seed=0, sd_hash=h,
                                    n_keys=nkeys, out_shapes=[list(o.shape) for o in outs])
        print('G2', name, nkeys, [o.shape for o in outs])
    np.savez(os.path.join(GOLD, 'g2_nets.npz'), **g2)

    # ---- G3: decode + NMS from synthetic head logits ----
    g3 = {}
    anchors = np.asarray(ANCHORS).reshape(-1, 2)
    cases = [('coco80_bs4', 80, 4, 640, -3.0, 0.3, 0.3), ('nc1_bs2', 1, 2, 640, -2.0, 0.3, 0.45),
             ('nc3_dense', 3, 2, 320, -1.0, 0.25, 0.5)]
    for name, nc, bs, size, shift, conf, iou in cases:
        shapes = [(bs, size // 32, size // 32), (bs, size // 16, size // 16), (bs, size // 8, size // 8)]
        heads = synthetic_head_logits(shapes, nc, seed=11, obj_shift=shift)
        dec = detect.decode_box(heads, anchors, MASK, nc, image_size=(size, size))
        allp = torch.cat(dec, 1)
        dec_np = allp.numpy().copy()
        passing = []
        for b in range(bs):
            cm = allp[b, :, 5:].max(1)[0]
            passing.append(np.nonzero((allp[b, :, 4] * cm >= conf).numpy())[0])
        rows, _ = ref_post.nms_keep_rows(allp.clone(), nc, conf, iou)
        img_shape = np.array([512, 773])
        res = detect.non_max_suppression(allp.clone(), nc, (size, size), img_shape, True, conf_thres=conf,
                                         nms_thres=iou)
        for b in range(bs):
            g3[f'{name}/pass_rows/{b}'] = passing[b].astype(np.int64)
            g3[f'{name}/pass_vals/{b}'] = dec_np[b, passing[b]]
            g3[f'{name}/keep_rows/{b}'] = rows[b].numpy().astype(np.int64)
            g3[f'{name}/final/{b}'] = res[b] if res[b] is not None else np.zeros((0, 7), np.float32)
        manifest['g3'][name] = dict(nc=nc, bs=bs, size=size, obj_shift=shift, seed=11, conf=conf, iou=iou,
                                    image_shape=img_shape.tolist(), heads_hash=arr_hash([h.numpy() for h in heads]),
                                    decoded_sum=float(dec_np.astype(np.float64).sum()),
                                    decoded_abs_sum=float(np.abs(dec_np.astype(np.float64)).sum()),
                                    decoded_hash=arr_hash([dec_np]),
                                    n_pass=[int(len(p)) for p in passing], n_keep=[int(len(r)) for r in rows])
        print('G3', name, 'pass', [len(p) for p in passing], 'keep', [len(r) for r in rows])
    np.savez(os.path.join(GOLD, 'g3_post.npz'), **g3)
    make_idetect_eval(Model, manifest)
    with open(os.path.join(GOLD, 'manifest.json'), 'w') as f:
        json.dump(manifest, f, indent=1)


if __name__ == '__main__':
    main()
