"""ORACLE (test infrastructure only): CPU fp32 restatement of Model.forward.

Builds the layer list from a network config + a reference-schema state_dict and
runs it with the same ATen op sequence as the reference modules in eval mode:

  Conv     conv2d(bias=None) -> batch_norm(eval, eps) -> silu | leaky_relu | id
                                                   nets/common.py:97-109
  RepConv  act(BN(conv3) + BN(conv1) [+ BN(x)])    nets/common.py:477-486
  MP / SP  max_pool2d                              nets/common.py:25-40
  Concat   cat(dim=1)                              nets/common.py:54-60
  Upsample interpolate(scale 2, nearest)           cfg/net/yolov7.yaml:71
  SPPCSPC  cv7(cat[cv6 cv5 cat[x1, mp5, mp9, mp13], cv2 x])  nets/common.py:262-266
  SPPF / SPP / Bottleneck / BottleneckCSPA,B,C    nets/common.py:185-341, 771-784
  Detect   [conv_P5(x2), conv_P4(x1), conv_P3(x0)] nets/detect.py:27-38
  IDetect  raw (bs, na, ny, nx, no) maps           nets/idetect.py:26-32 (training-mode view;
                                                   the reference's eval branch crashes)
  IAuxDetect main heads only (eval discards m2)    nets/iaux_detect.py:27-49

The channel bookkeeping restates parse_model (nets/yolo.py:15-87). Layer
execution restates the interpreter loop (nets/yolo.py:143-153).
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F

_CONV_LIKE = {'Conv', 'nn.Conv2d', 'RepConv', 'SPP', 'SPPF', 'SPPCSPC', 'Bottleneck', 'BottleneckCSPA',
              'BottleneckCSPB', 'BottleneckCSPC'}
_CSP_LIKE = {'SPPCSPC', 'BottleneckCSPA', 'BottleneckCSPB', 'BottleneckCSPC'}


def _arg(a, nc, anchors):
    if not isinstance(a, str):
        return a
    if a == 'None':
        return None
    if a in ('nc', 'num_classes'):
        return nc
    if a == 'anchors':
        return anchors
    if a.startswith('nn.LeakyReLU('):
        return ('leaky', float(a[len('nn.LeakyReLU('):-1]))
    try:
        return eval(a, {'__builtins__': {}}, {})  # literals only (test infrastructure)
    except Exception:
        return a


def _act_of(arg):
    """Conv's act argument -> ('silu'|'leaky'|'none', slope) (nets/common.py:103)."""
    if arg is True:
        return ('silu', 0.0)
    if isinstance(arg, tuple) and arg[0] == 'leaky':
        return arg
    return ('none', 0.0)


class _P:
    """Parameter accessor: state_dict entries below a key prefix."""

    def __init__(self, sd, prefix):
        self.sd, self.prefix = sd, prefix

    def __call__(self, name):
        return self.sd[self.prefix + name]

    def sub(self, name):
        return _P(self.sd, self.prefix + name + '.')

    def has(self, name):
        return (self.prefix + name) in self.sd


def _conv(p: _P, x, k, s, act, pad=None):
    """Conv.forward: act(bn(conv(x)))."""
    pad = k // 2 if pad is None else pad
    y = F.conv2d(x, p('conv.weight'), None, s, pad)
    y = F.batch_norm(y, p('bn.running_mean'), p('bn.running_var'), p('bn.weight'), p('bn.bias'), False, 0.0, 1e-5)
    return _apply_act(y, act)


def _apply_act(y, act):
    if act[0] == 'silu':
        return F.silu(y)
    if act[0] == 'leaky':
        return F.leaky_relu(y, act[1])
    return y


def _bn(p: _P, x):
    return F.batch_norm(x, p('running_mean'), p('running_var'), p('weight'), p('bias'), False, 0.0, 1e-5)


def build(cfg: dict, anchors, num_classes: int, state_dict: dict, image_chan: int = 3):
    """-> forward(x) closure running the network on CPU in fp32."""
    sd = {k: v.detach().to('cpu', torch.float32) if v.is_floating_point() else v for k, v in state_dict.items()}
    nc, gd, gw = num_classes, cfg['depth_multiple'], cfg['width_multiple']
    na = len(anchors[0]) // 2
    no = na * (nc + 5)
    ch = [image_chan]
    layers = []
    for i, (f, n, m, args) in enumerate(cfg['backbone'] + cfg['head']):
        args = [_arg(a, nc, anchors) for a in args]
        n = max(round(n * gd), 1) if n > 1 else n
        c2 = ch[f] if isinstance(f, int) else None
        if m in _CONV_LIKE:
            c1, c2 = ch[f], args[0]
            if c2 != no:
                c2 = math.ceil(c2 * gw / 8) * 8
            args = [c1, c2, *args[1:]]
            if m in _CSP_LIKE:
                args.insert(2, n)
                n = 1
        elif m == 'Concat':
            c2 = sum(ch[x] for x in f)
        layers.append(dict(i=i, f=f, n=n, m=m, args=args, p=_P(sd, f'model.{i}.')))
        if i == 0:
            ch = []
        ch.append(c2)

    def run_layer(L, x):
        if L['n'] > 1:  # nn.Sequential of repeats: keys model.i.j.*
            for j in range(L['n']):
                x = run_module(L['m'], L['args'], L['p'].sub(str(j)), x)
            return x
        return run_module(L['m'], L['args'], L['p'], x)

    # the save list (nets/yolo.py:82, 151): only outputs a later layer reads are kept
    save = {j % L['i'] for L in layers for j in ([L['f']] if isinstance(L['f'], int) else L['f']) if j != -1}

    def forward(x):
        y = []
        with torch.no_grad():
            for L in layers:
                f = L['f']
                if f != -1:
                    x = y[f] if isinstance(f, int) else [x if j == -1 else y[j] for j in f]
                x = run_layer(L, x)
                y.append(x if L['i'] in save else None)
        return x

    return forward


def _bottleneck(p, x, c1, c2, shortcut):
    y = _conv(p.sub('cv2'), _conv(p.sub('cv1'), x, 1, 1, ('silu', 0)), 3, 1, ('silu', 0))
    return x + y if (shortcut and c1 == c2) else y


def run_module(m, args, p: _P, x):
    if m == 'Conv':
        c1, c2, k = args[0], args[1], args[2] if len(args) > 2 else 1
        s = args[3] if len(args) > 3 else 1
        pad = args[4] if len(args) > 4 else None
        act = _act_of(args[6] if len(args) > 6 else True)
        return _conv(p, x, k, s, act, pad)
    if m == 'nn.Conv2d':
        k = args[2] if len(args) > 2 else 1
        s = args[3] if len(args) > 3 else 1
        pad = args[4] if len(args) > 4 else 0
        return F.conv2d(x, p('weight'), p('bias') if p.has('bias') else None, s, pad)
    if m == 'MP':
        k = args[0] if args else 2
        return F.max_pool2d(x, k, k)
    if m == 'SP':
        k = args[0] if args else 3
        s = args[1] if len(args) > 1 else 1
        return F.max_pool2d(x, k, s, k // 2)
    if m == 'Concat':
        return torch.cat(x, 1)
    if m == 'nn.Upsample':
        return F.interpolate(x, None, args[1], args[2])
    if m == 'RepConv':
        c1, c2 = args[0], args[1]
        s = args[3] if len(args) > 3 else 1
        act = _act_of(args[6] if len(args) > 6 else True)
        dense = _bn(p.sub('rbr_dense.1'), F.conv2d(x, p('rbr_dense.0.weight'), None, s, 1))
        one = _bn(p.sub('rbr_1x1.1'), F.conv2d(x, p('rbr_1x1.0.weight'), None, s, 0))
        idn = _bn(p.sub('rbr_identity'), x) if p.has('rbr_identity.weight') else 0
        return _apply_act(dense + one + idn, act)
    if m == 'SPPCSPC':
        k = args[6] if len(args) > 6 else (5, 9, 13)
        silu = ('silu', 0)
        x1 = _conv(p.sub('cv4'), _conv(p.sub('cv3'), _conv(p.sub('cv1'), x, 1, 1, silu), 3, 1, silu), 1, 1, silu)
        pools = [F.max_pool2d(x1, kk, 1, kk // 2) for kk in k]
        y1 = _conv(p.sub('cv6'), _conv(p.sub('cv5'), torch.cat([x1] + pools, 1), 1, 1, silu), 3, 1, silu)
        y2 = _conv(p.sub('cv2'), x, 1, 1, silu)
        return _conv(p.sub('cv7'), torch.cat((y1, y2), 1), 1, 1, silu)
    if m == 'SPPF':
        k = args[2] if len(args) > 2 else 5
        silu = ('silu', 0)
        x = _conv(p.sub('cv1'), x, 1, 1, silu)
        y1 = F.max_pool2d(x, k, 1, k // 2)
        y2 = F.max_pool2d(y1, k, 1, k // 2)
        return _conv(p.sub('cv2'), torch.cat([x, y1, y2, F.max_pool2d(y2, k, 1, k // 2)], 1), 1, 1, silu)
    if m == 'SPP':
        k = args[2] if len(args) > 2 else (5, 9, 13)
        silu = ('silu', 0)
        x = _conv(p.sub('cv1'), x, 1, 1, silu)
        return _conv(p.sub('cv2'), torch.cat([x] + [F.max_pool2d(x, kk, 1, kk // 2) for kk in k], 1), 1, 1, silu)
    if m == 'Bottleneck':
        c1, c2 = args[0], args[1]
        shortcut = args[2] if len(args) > 2 else True
        return _bottleneck(p, x, c1, c2, shortcut)
    if m in ('BottleneckCSPA', 'BottleneckCSPB', 'BottleneckCSPC'):
        c1, c2, n = args[0], args[1], args[2]
        shortcut = args[3] if len(args) > 3 else (m != 'BottleneckCSPB')
        silu = ('silu', 0)
        c_ = c2 if m == 'BottleneckCSPB' else int(c2 * 0.5)

        def stack(v):
            for j in range(n):
                v = _bottleneck(p.sub(f'm.{j}'), v, c_, c_, shortcut)
            return v
        if m == 'BottleneckCSPA':
            y1 = stack(_conv(p.sub('cv1'), x, 1, 1, silu))
            return _conv(p.sub('cv3'), torch.cat((y1, _conv(p.sub('cv2'), x, 1, 1, silu)), 1), 1, 1, silu)
        if m == 'BottleneckCSPB':
            x1 = _conv(p.sub('cv1'), x, 1, 1, silu)
            return _conv(p.sub('cv3'), torch.cat((stack(x1), _conv(p.sub('cv2'), x1, 1, 1, silu)), 1), 1, 1, silu)
        y1 = _conv(p.sub('cv3'), stack(_conv(p.sub('cv1'), x, 1, 1, silu)), 1, 1, silu)
        return _conv(p.sub('cv4'), torch.cat((y1, _conv(p.sub('cv2'), x, 1, 1, silu)), 1), 1, 1, silu)
    if m == 'Detect':
        out0 = F.conv2d(x[2], p('yolo_head_P5.weight'), p('yolo_head_P5.bias'))
        out1 = F.conv2d(x[1], p('yolo_head_P4.weight'), p('yolo_head_P4.bias'))
        out2 = F.conv2d(x[0], p('yolo_head_P3.weight'), p('yolo_head_P3.bias'))
        return [out0, out1, out2]
    if m in ('IDetect', 'IAuxDetect'):  # IAuxDetect eval: main heads on x[:nl] (nets/iaux_detect.py:28-31, 49)
        outs = []
        nl = len(x) if m == 'IDetect' else len(x) // 2
        for i in range(nl):
            xi = p(f'ia.{i}.implicit') + x[i]
            xi = F.conv2d(xi, p(f'm.{i}.weight'), p(f'm.{i}.bias'))
            outs.append(p(f'im.{i}.implicit') * xi)
        return outs
    raise NotImplementedError(f"oracle: module {m}")
