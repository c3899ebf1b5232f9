"""Static execution plan of ``Model.forward`` on the HIP kernels.

Lowering (once per input shape / device / precision):

1. Walk ``model.model`` exactly like the reference interpreter loop
   (nets/yolo.py:143-153: ``m.f`` indexing into the per-layer outputs) and lower
   each module into graph nodes — conv (BN folded, RepConv re-parameterised,
   Bottleneck residual fused into the epilogue), stem conv (first conv on the
   fp32 NCHW image), max-pool, upsample, concat, Detect/IDetect heads.
2. Passes: nearest-x2 upsample fused into its producing conv's store
   (YCX_OUT_NHWC_UP2); the SPPCSPC 5/9/13 pools run as a k5 cascade (exact for
   max with -inf padding); every concat input that a kernel produces is written
   straight into its channel slice of the concat buffer (Concat costs nothing;
   a copy kernel runs only for inputs that cannot alias).
3. Allocate one NHWC device buffer per remaining value (no reuse: a yolov7
   bs=32 640x640 plan is ~10 GB of bf16 activations, small next to 288 GB HBM),
   pack weights ([cout_pad][kh][kw][cin], bf16 or fp32) and build the ctypes
   op array consumed by the native loop ``ycx_run_ops`` (or a HIP graph).
"""
from __future__ import annotations

import ctypes
import math
import os

import numpy as np
import torch
from torch import nn

from . import _lib as L
from .nets.common import (SP, SPP, SPPCSPC, SPPF, MP, Bottleneck, BottleneckCSPA, BottleneckCSPB, BottleneckCSPC,
                          Concat, Conv, RepConv)
from .nets.detect import Detect, IAuxDetect, IDetect


class Buf:
    __slots__ = ('n', 'h', 'w', 'c', 'tensor')

    def __init__(self, n, h, w, c):
        self.n, self.h, self.w, self.c, self.tensor = n, h, w, c, None


class Val:
    """An activation: channels [coff, coff + c) of an NHWC buffer."""
    __slots__ = ('n', 'h', 'w', 'c', 'buf', 'coff', 'producer', 'consumers', 'role')

    def __init__(self, n, h, w, c, role='act'):
        self.n, self.h, self.w, self.c = n, h, w, c
        self.buf, self.coff, self.producer, self.consumers, self.role = None, 0, None, [], role


class Node:
    __slots__ = ('kind', 'inputs', 'out', 'p')

    def __init__(self, kind, inputs, out, **p):
        self.kind, self.inputs, self.out, self.p = kind, inputs, out, p


def _pair(v):
    return v if isinstance(v, (tuple, list)) else (v, v)


def _square(v, what):
    a, b = _pair(v)
    if a != b:
        raise NotImplementedError(f"ycx: non-square {what} {v}")
    return int(a)


def fold_bn(weight, bn):
    """conv weight (+BN) -> float64 (W, b): W*gamma/std, beta - mean*gamma/std
    (nets/common.py:14-17, 503-529)."""
    w = weight.detach().to('cpu', torch.float64)
    if bn is None:
        return w, torch.zeros(w.shape[0], dtype=torch.float64)
    std = (bn.running_var.detach().to('cpu', torch.float64) + bn.eps).sqrt()
    t = bn.weight.detach().to('cpu', torch.float64) / std
    b = bn.bias.detach().to('cpu', torch.float64) - bn.running_mean.detach().to('cpu', torch.float64) * t
    return w * t.reshape(-1, 1, 1, 1), b


def fold_repconv(m: RepConv):
    """RepConv -> one 3x3 conv (get_equivalent_kernel_bias, nets/common.py:488-529)."""
    if hasattr(m, 'rbr_reparam'):
        c = m.rbr_reparam
        b = c.bias.detach().to('cpu', torch.float64) if c.bias is not None else torch.zeros(c.out_channels,
                                                                                               dtype=torch.float64)
        return c.weight.detach().to('cpu', torch.float64), b
    k3, b3 = fold_bn(m.rbr_dense[0].weight, m.rbr_dense[1])
    k1, b1 = fold_bn(m.rbr_1x1[0].weight, m.rbr_1x1[1])
    k = k3 + torch.nn.functional.pad(k1, [1, 1, 1, 1])
    b = b3 + b1
    if m.rbr_identity is not None:
        idk = torch.zeros_like(k3)
        input_dim = m.in_channels // m.groups
        for i in range(m.in_channels):
            idk[i, i % input_dim, 1, 1] = 1.0
        kid, bid = fold_bn(idk, m.rbr_identity)
        k, b = k + kid, b + bid
    return k, b


def act_of(mod):
    if isinstance(mod, nn.SiLU):
        return L.ACT_SILU, 0.0
    if isinstance(mod, nn.LeakyReLU):
        return L.ACT_LEAKY, float(mod.negative_slope)
    if isinstance(mod, nn.Identity) or mod is None:
        return L.ACT_NONE, 0.0
    raise NotImplementedError(f"ycx: activation {type(mod).__name__} has no HIP epilogue")


class Graph:
    def __init__(self):
        self.nodes = []

    def add(self, kind, inputs, out, **p):
        node = Node(kind, list(inputs), out, **p)
        out.producer = node
        for v in inputs:
            v.consumers.append(node)
        self.nodes.append(node)
        return out

    # ---- primitive ops ----
    def conv(self, x: Val, w64, b64, k, s, p, act=(L.ACT_NONE, 0.0), residual=None, head=False):
        cout, cin = int(w64.shape[0]), int(w64.shape[1])
        if cin != x.c:
            raise NotImplementedError(f"ycx: grouped/mismatched conv (cin {cin} vs input {x.c})")
        ho, wo = (x.h + 2 * p - k) // s + 1, (x.w + 2 * p - k) // s + 1
        out = Val(x.n, ho, wo, cout, role='output' if head else 'act')
        ins = [x] + ([residual] if residual is not None else [])
        kind = 'stem' if x.role == 'input' else 'conv'
        if kind == 'stem' and residual is not None:
            raise NotImplementedError("ycx: residual on the input conv")
        return self.add(kind, ins, out, w=w64, b=b64, k=k, s=s, p=p, act=act[0], slope=act[1],
                        residual=residual, ho=ho, wo=wo, layout=L.OUT_NCHW_F32 if head else L.OUT_NHWC)

    def pool(self, x: Val, k, s, p):
        if x.role == 'input':
            raise NotImplementedError("ycx: pooling the raw input image")
        ho, wo = (x.h + 2 * p - k) // s + 1, (x.w + 2 * p - k) // s + 1
        return self.add('pool', [x], Val(x.n, ho, wo, x.c), k=k, s=s, p=p)

    def upsample(self, x: Val):
        return self.add('up', [x], Val(x.n, 2 * x.h, 2 * x.w, x.c))

    def concat(self, xs):
        n, h, w = xs[0].n, xs[0].h, xs[0].w
        if any((v.n, v.h, v.w) != (n, h, w) for v in xs):
            raise ValueError("ycx: Concat inputs differ in spatial size")
        return self.add('concat', xs, Val(n, h, w, sum(v.c for v in xs)))


def conv_module(g: Graph, m: Conv, x: Val, residual=None):
    c = m.conv
    if c.groups != 1 or _pair(c.dilation) != (1, 1):
        raise NotImplementedError("ycx: grouped/dilated conv")
    w, b = fold_bn(c.weight, m.bn)
    return g.conv(x, w, b, _square(c.kernel_size, 'kernel'), _square(c.stride, 'stride'),
                  _square(c.padding, 'padding'), act_of(m.act), residual=residual)


def pool_module(g: Graph, mp: nn.MaxPool2d, x: Val):
    if mp.ceil_mode or _pair(mp.dilation) != (1, 1):
        raise NotImplementedError("ycx: ceil_mode / dilated max-pool")
    k = _square(mp.kernel_size, 'pool kernel')
    s = _square(mp.stride if mp.stride is not None else k, 'pool stride')
    return g.pool(x, k, s, _square(mp.padding, 'pool padding'))


def pyramid(g: Graph, x: Val, pools):
    """SPP-style pools of x. s=1 'same' pools whose kernels step by 4 from 5
    (5, 9, 13) run as a cascade of k=5 pools: maxpool_{a+b-1} = maxpool_a o maxpool_b
    for stride 1 with -inf padding (exact, SPPF's own identity)."""
    ks = [(_square(m.kernel_size, 'k'), _square(m.stride, 's'), _square(m.padding, 'p')) for m in pools]
    cascade = all(s == 1 and p == k // 2 for k, s, p in ks) and [k for k, _, _ in ks] == [5 + 4 * i for i in range(len(ks))]
    outs, cur = [], x
    for (k, s, p), m in zip(ks, pools):
        if cascade:
            cur = g.pool(cur, 5, 1, 2)
            outs.append(cur)
        else:
            outs.append(pool_module(g, m, x))
    return outs


def lower_module(g: Graph, m, x):
    if isinstance(m, nn.Sequential):
        for mm in m:
            x = lower_module(g, mm, x)
        return x
    if isinstance(m, Conv):
        return conv_module(g, m, x)
    if isinstance(m, RepConv):
        w, b = fold_repconv(m)
        return g.conv(x, w, b, 3, m.stride, 1, act_of(m.act))
    if isinstance(m, nn.Conv2d):
        w = m.weight.detach().to('cpu', torch.float64)
        b = m.bias.detach().to('cpu', torch.float64) if m.bias is not None else torch.zeros(w.shape[0],
                                                                                            dtype=torch.float64)
        if m.groups != 1:
            raise NotImplementedError("ycx: grouped conv")
        return g.conv(x, w, b, _square(m.kernel_size, 'k'), _square(m.stride, 's'), _square(m.padding, 'p'))
    if isinstance(m, (MP, SP)):
        return pool_module(g, m.m, x)
    if isinstance(m, nn.MaxPool2d):
        return pool_module(g, m, x)
    if isinstance(m, Concat):
        if m.d != 1:
            raise NotImplementedError("ycx: Concat along a non-channel dim")
        return g.concat(x)
    if isinstance(m, nn.Upsample):
        sf = m.scale_factor
        sf = sf[0] if isinstance(sf, (tuple, list)) else sf
        if m.mode != 'nearest' or m.size is not None or float(sf) != 2.0:
            raise NotImplementedError("ycx: only nn.Upsample(None, 2, 'nearest') is supported")
        return g.upsample(x)
    if isinstance(m, nn.Identity):
        return x
    if isinstance(m, Bottleneck):
        y = conv_module(g, m.cv1, x)
        return conv_module(g, m.cv2, y, residual=x if m.add else None)
    if isinstance(m, SPPCSPC):
        x1 = conv_module(g, m.cv4, conv_module(g, m.cv3, conv_module(g, m.cv1, x)))
        y1 = conv_module(g, m.cv6, conv_module(g, m.cv5, g.concat([x1] + pyramid(g, x1, list(m.m)))))
        y2 = conv_module(g, m.cv2, x)
        return conv_module(g, m.cv7, g.concat([y1, y2]))
    if isinstance(m, SPPF):
        x1 = conv_module(g, m.cv1, x)
        y1 = pool_module(g, m.m, x1)
        y2 = pool_module(g, m.m, y1)
        y3 = pool_module(g, m.m, y2)
        return conv_module(g, m.cv2, g.concat([x1, y1, y2, y3]))
    if isinstance(m, SPP):
        x1 = conv_module(g, m.cv1, x)
        return conv_module(g, m.cv2, g.concat([x1] + pyramid(g, x1, list(m.m))))
    if isinstance(m, BottleneckCSPA):
        y1 = lower_module(g, m.m, conv_module(g, m.cv1, x))
        return conv_module(g, m.cv3, g.concat([y1, conv_module(g, m.cv2, x)]))
    if isinstance(m, BottleneckCSPB):
        x1 = conv_module(g, m.cv1, x)
        return conv_module(g, m.cv3, g.concat([lower_module(g, m.m, x1), conv_module(g, m.cv2, x1)]))
    if isinstance(m, BottleneckCSPC):
        y1 = conv_module(g, m.cv3, lower_module(g, m.m, conv_module(g, m.cv1, x)))
        return conv_module(g, m.cv4, g.concat([y1, conv_module(g, m.cv2, x)]))
    if isinstance(m, Detect):
        outs = []
        for conv, idx in m.heads_in_output_order():
            w = conv.weight.detach().to('cpu', torch.float64)
            b = conv.bias.detach().to('cpu', torch.float64)
            outs.append(g.conv(x[idx], w, b, 1, 1, 0, head=True))
        return outs
    if isinstance(m, IDetect):  # IAuxDetect too: its eval uses the main heads only (x[:nl])
        outs = []
        for i in range(m.nl):
            conv = m.m[i]
            # x_i = im * (conv(x_i + ia)) = (im*W) x + im*(b + W.ia)   (nets/idetect.py:30-31)
            w = conv.weight.detach().to('cpu', torch.float64)
            b = conv.bias.detach().to('cpu', torch.float64)
            ia = m.ia[i].implicit.detach().to('cpu', torch.float64).reshape(-1)
            im = m.im[i].implicit.detach().to('cpu', torch.float64).reshape(-1)
            b = (b + w[:, :, 0, 0] @ ia) * im
            w = w * im.reshape(-1, 1, 1, 1)
            outs.append(g.conv(x[i], w, b, 1, 1, 0, head=True))
        return outs
    raise NotImplementedError(f"ycx: no HIP lowering for {type(m).__name__}")


# Development A/B of tile choices: YCX_TILE_MAP="16:24/26,18:26" replaces the picked
# tile 16 by 24 where cout_pad allows, else 26; "16<600:25/26" only where the picked tile
# launches fewer than 600 workgroups (never set in the product path).
_TILE_MAP = {}
_TILE_SHAPE = {15: (64, 256), 16: (128, 128), 18: (64, 128), 24: (256, 256), 25: (256, 128), 26: (128, 256)}
for _kv in os.environ.get('YCX_TILE_MAP', '').split(','):
    if _kv:
        _a, _b = _kv.split(':')
        _t, _, _cap = _a.partition('<')
        _TILE_MAP[int(_t)] = (int(_cap) if _cap else 1 << 62, [int(t) for t in _b.split('/')])
# A/B switch: YCX_NO_KSPLIT=1 runs every conv unsplit even where ycx_conv_pick_ksplit splits its K loop
_NO_KSPLIT = bool(os.environ.get('YCX_NO_KSPLIT'))
# A/B switch: YCX_NO_SILU_PS=1 packs SiLU convs unscaled and runs the plain YCX_ACT_SILU epilogue
_NO_SILU_PS = bool(os.environ.get('YCX_NO_SILU_PS'))


def cascade_fits(h, w, c, esz):
    """Whether ycx_maxpool's one-launch cascade (levels > 1) takes an (h, w) map of c
    channels of esz bytes: it keeps two copies of the H x W plane of one channel
    slice (a 16-byte multiple dividing c, at most 128 channels) in 64 KB of LDS
    (ycx_misc.hip, ycx_maxpool). Mirrors the launcher's slice search exactly."""
    t = 128
    while t * esz >= 16:
        if c % t == 0 and 2 * h * w * t * esz <= 65536:
            return True
        t >>= 1
    return False


class Plan:
    """Device-independent lowering of a Model for one input shape: the graph
    after all passes, its outputs and its algorithmic FLOPs."""

    def __init__(self, model, shape):
        if len(shape) != 4:
            raise ValueError(f"ycx: expected an NCHW input, got shape {shape}")
        self.shape = tuple(int(s) for s in shape)
        n, c, h, w = self.shape
        g = Graph()
        self.input_val = Val(n, h, w, c, role='input')
        ys, x = [], self.input_val
        for m in model.model:  # nets/yolo.py:145-151
            if m.f != -1:
                x = ys[m.f] if isinstance(m.f, int) else [x if j == -1 else ys[j] for j in m.f]
            x = lower_module(g, m, x)
            ys.append(x)
        self.is_list = isinstance(x, list)
        self.out_vals = list(x) if self.is_list else [x]
        self.graph = g
        self._eliminate_dead()
        self._passes()

    @property
    def conv_flops(self):
        """Algorithmic FLOPs: sum of 2*N*Ho*Wo*Cout*Cin*k*k over the folded convs."""
        return sum(2 * nd.inputs[0].n * nd.p['ho'] * nd.p['wo'] * int(nd.p['w'].shape[0]) * int(nd.p['w'].shape[1])
                   * nd.p['k'] ** 2 for nd in self.graph.nodes if nd.kind in ('conv', 'stem'))

    def counts(self):
        """Node kinds after the passes; 'conv' counts the original convs (a merged
        sibling pair counts 2), 'merged' the merged nodes."""
        c = {}
        for nd in self.graph.nodes:
            kind = nd.kind
            if kind == 'conv' and nd.p.get('parts', 1) > 1:
                c['merged'] = c.get('merged', 0) + 1
                c['conv'] = c.get('conv', 0) + nd.p['parts'] - 1
            if kind == 'concat':
                c['copy'] = c.get('copy', 0) + len(nd.p['copies'])
            c[kind] = c.get(kind, 0) + 1
        return c

    def _eliminate_dead(self):
        """Drop nodes whose value nobody reads (IAuxDetect's aux branch in eval:
        nets/iaux_detect.py:32-33 computes it, :49 discards it)."""
        g = self.graph
        live = {id(v) for v in self.out_vals}
        keep = []
        for node in reversed(g.nodes):
            if id(node.out) in live:
                keep.append(node)
                live.update(id(v) for v in node.inputs)
            else:
                for v in node.inputs:
                    v.consumers = [c for c in v.consumers if c is not node]
        g.nodes = keep[::-1]

    def _passes(self):
        g = self.graph
        for v in self.out_vals:
            if v.role != 'output':  # not a head conv: convert NHWC -> fp32 NCHW at the end
                o = Val(v.n, v.h, v.w, v.c, role='output')
                g.add('tonchw', [v], o)
                self.out_vals[self.out_vals.index(v)] = o
        # Fuse nearest-x2 upsample into the producing conv's store.
        keep = []
        for node in g.nodes:
            if node.kind == 'up':
                v = node.inputs[0]
                prod = v.producer
                if prod is not None and prod.kind == 'conv' and len(v.consumers) == 1 and v.role == 'act':
                    prod.out = node.out
                    prod.p['layout'] = L.OUT_NHWC_UP2
                    node.out.producer = prod
                    continue
            keep.append(node)
        g.nodes = keep
        # Concat: producers write their channel slice directly when they can.
        for node in g.nodes:
            if node.kind != 'concat':
                continue
            out = node.out
            out.buf = Buf(out.n, out.h, out.w, out.c)
            copies, off = [], 0
            for v in node.inputs:
                if v.buf is None and v.role == 'act' and v.producer is not None and \
                        v.producer.kind in ('conv', 'stem', 'pool', 'up'):
                    v.buf, v.coff = out.buf, off
                else:
                    copies.append((v, off))
                off += v.c
            node.p['copies'] = copies
        for node in g.nodes:
            v = node.out
            if v.buf is None and v.role == 'act':
                v.buf = Buf(v.n, v.h, v.w, v.c)
        if not os.environ.get("YCX_NO_SIBLING_MERGE"):  # A/B switch for the bench
            self._merge_sibling_1x1()

    def _merge_sibling_1x1(self):
        """Two 1x1 convs that read the same activation and write adjacent channel
        slices of one buffer (ELAN's cv1/cv2 pair feeding its concat, e.g.
        cfg/net/yolov7.yaml:17-18) become one conv with the weights stacked: the
        input is read once and the GEMM is twice as wide. Every output channel
        is the same dot product over the same K as before."""
        g = self.graph

        def mergeable(nd):
            p = nd.p
            return (nd.kind == 'conv' and p['k'] == 1 and p['s'] == 1 and p['p'] == 0 and p['residual'] is None
                    and p['layout'] == L.OUT_NHWC and nd.out.role == 'act' and nd.out.buf is not None)

        changed = True
        while changed:
            changed = False
            cands = [nd for nd in g.nodes if mergeable(nd)]
            for a in cands:
                for b in cands:
                    if a is b or a.inputs[0] is not b.inputs[0]:
                        continue
                    if (a.p['act'], a.p['slope']) != (b.p['act'], b.p['slope']):
                        continue
                    va, vb = a.out, b.out
                    if va.buf is not vb.buf or va.coff + va.c != vb.coff:
                        continue
                    out = Val(va.n, va.h, va.w, va.c + vb.c)
                    out.buf, out.coff = va.buf, va.coff
                    w = torch.cat([a.p['w'], b.p['w']], 0)
                    bias = torch.cat([a.p['b'], b.p['b']], 0)
                    m = Node('conv', [a.inputs[0]], out, **dict(a.p, w=w, b=bias,
                                                               parts=a.p.get('parts', 1) + b.p.get('parts', 1)))
                    out.producer = m
                    va.producer = vb.producer = m  # the halves stay valid views for their consumers
                    x = a.inputs[0]
                    x.consumers = [c for c in x.consumers if c is not a and c is not b] + [m]
                    i = min(g.nodes.index(a), g.nodes.index(b))
                    g.nodes = [nd for nd in g.nodes if nd is not a and nd is not b]
                    g.nodes.insert(i, m)
                    changed = True
                    break
                if changed:
                    break


def pack_fp8_weights(wp):
    """float64 [cout_pad][cin][k][k] -> (e4m3 [cout_pad][ceil(k*k*cin / 128) * 128] as
    torch.float8_e4m3fn, float64 s_w[cout_pad]): per output channel the
    power-of-two scale that maps its max |w| into [224, 448], rows in
    [kh][kw][cin] order, zero-padded to whole 128-byte K steps (ycx.h)."""
    cpad = wp.shape[0]
    amax = wp.abs().amax(dim=(1, 2, 3))
    sw = torch.where(amax > 0, torch.exp2(torch.floor(torch.log2(448.0 / amax.clamp_min(1e-300)))),
                     torch.ones_like(amax))
    rows = (wp * sw.reshape(-1, 1, 1, 1)).permute(0, 2, 3, 1).reshape(cpad, -1)
    kt = rows.shape[1]
    ktp = -(-kt // 128) * 128
    out = torch.zeros((cpad, ktp), dtype=torch.float32)
    out[:, :kt] = rows.to(torch.float32)
    return out.clamp(-448.0, 448.0).to(torch.float8_e4m3fn), sw


class Engine:
    """A compiled plan bound to device memory for one (input shape, device, precision)."""

    def __init__(self, model, shape, device, precision='bf16', fuse_stem2=True, fp8_amax=None, prepacked=None,
                 fuse_pool=True, fuse_pair=True):
        if device.type != 'cuda':
            raise RuntimeError("ycx: the HIP path needs the model input on a ROCm device (tensor.to('cuda')); "
                               "there is no CPU path")
        self.plan = Plan(model, shape)
        self.shape, self.device, self.precision = self.plan.shape, device, precision
        self.dtype = {'bf16': torch.bfloat16, 'f32': torch.float32, 'fp8': torch.float8_e4m3fn,
                      'fp16': torch.float16}[precision]
        self.dt = {'bf16': L.DT_BF16, 'f32': L.DT_F32, 'fp8': L.DT_FP8, 'fp16': L.DT_F16}[precision]
        self.fuse_stem2 = fuse_stem2
        self.fuse_pool = fuse_pool  # False: every pool writes its map (fp8 calibration reads them all)
        self.fuse_pair = fuse_pair  # False: every 1x1 of a pair stores its map (fp8 calibration reads them all)
        self.prepacked = prepacked  # {'p<i>': packed tensor} from ycx.prepack (skips folding / packing)
        self.graph_exec = None
        self.graph, self.out_vals, self.is_list = self.plan.graph, self.plan.out_vals, self.plan.is_list
        self.scales = {}
        if self.dt == L.DT_FP8:
            if fp8_amax is None:
                raise ValueError("ycx: an fp8 engine needs calibration amax values (Model.calibrate_fp8)")
            self._assign_fp8_scales(fp8_amax)
        self._build()

    @property
    def h16(self):
        """The plan runs the 16-bit MFMA kernels (bf16 or IEEE half elements)."""
        return self.dt in (L.DT_BF16, L.DT_F16)

    def activation_bufs(self):
        """The plan's activation buffers in allocation order (the order of
        ``self.buffers``; fp8 calibration keys its amax list on it)."""
        skip_vals = {id(nd.out) for nd in self.graph.nodes if id(nd) in self._stem2_pairs()}
        bufs, seen = [], set()
        for node in self.graph.nodes:
            for v in [node.out] + node.inputs:
                b = v.buf
                if b is not None and id(b) not in seen and id(v) not in skip_vals:
                    seen.add(id(b))
                    bufs.append(b)
        return bufs

    def _assign_fp8_scales(self, amax):
        """One power-of-two scale per group of buffers tied by a pool or a copy
        (max-pool, nearest upsample and concat copies move bytes unchanged):
        s = 2^floor(log2(224 / amax)), i.e. the calibrated max lands in
        [224, 448) with 2x headroom below the e4m3 limit. Power-of-two scales
        make every rescale exact."""
        bufs = self.activation_bufs()
        if len(amax) != len(bufs) or any(a.get('c') != b.c for a, b in zip(amax, bufs)):
            raise ValueError("ycx: fp8 calibration was recorded on a different plan")
        parent = {id(b): id(b) for b in bufs}

        def find(i):
            while parent[i] != i:
                parent[i] = parent[parent[i]]
                i = parent[i]
            return i
        for nd in self.graph.nodes:
            if nd.kind in ('pool', 'up', 'concat'):
                ins = [v for v in nd.inputs if v.buf is not None]
                if nd.out.buf is None:
                    continue
                for v in ins:
                    parent[find(id(v.buf))] = find(id(nd.out.buf))
        gmax = {}
        for a, b in zip(amax, bufs):
            r = find(id(b))
            gmax[r] = max(gmax.get(r, 0.0), float(a['amax']))
        for b in bufs:
            m = gmax[find(id(b))]
            self.scales[id(b)] = 2.0 ** math.floor(math.log2(224.0 / m)) if m > 0 and math.isfinite(m) else 1.0

    def _scale(self, v):
        return self.scales.get(id(v.buf), 1.0) if v.buf is not None else 1.0

    def _cout_pad(self, cout, stem=False):
        if self.dt == L.DT_F32:
            return -(-cout // 64) * 64
        if self.dt == L.DT_FP8 and not stem:
            return -(-cout // 64) * 64
        if cout <= 32:
            return 32
        if cout <= 64:
            return 64
        return -(-cout // 128) * 128

    def _stem2_pairs(self):
        """Stem -> 3x3/s2 conv pairs that run as one ycx_stem_conv2 (the stem
        map stays in LDS): bf16, the stem's output read by that conv only."""
        pairs = {}
        if not (self.h16 or self.dt == L.DT_FP8) or not self.fuse_stem2:
            return pairs
        for nd in self.graph.nodes:
            if nd.kind != 'stem':
                continue
            v, p = nd.out, nd.p
            if v.role != 'act' or len(v.consumers) != 1 or v.buf is None or v.buf.c != v.c:
                continue
            c = v.consumers[0]
            q = c.p
            if c.kind != 'conv' or c.inputs[0] is not v or q['residual'] is not None or q['layout'] != L.OUT_NHWC:
                continue
            if not (p['k'] == 3 and p['p'] == 1 and p['s'] in (1, 2) and int(p['w'].shape[1]) == 3 and
                    int(p['w'].shape[0]) == 32 and p['layout'] == L.OUT_NHWC):
                continue
            if not (q['k'] == 3 and q['s'] == 2 and q['p'] == 1 and int(q['w'].shape[0]) <= 64 and
                    int(q['w'].shape[0]) % 8 == 0 and q['ho'] % 4 == 0 and q['wo'] % 32 == 0):
                continue
            if p['act'] != q['act']:  # the fused kernel is instantiated per (act, act) with both equal
                continue
            pairs[id(nd)] = c
        return pairs

    def _conv_pairs(self, pooled):
        """1x1 -> 1x1 chains that run as one ycx_conv2d_pair launch (tile 55): a 1x1 / s1
        conv with cin 64 / 128 / 256 and 256 output channels on a map large enough for the
        weight-resident kernel (>= 8 64-pixel tiles per CU), whose output a second 1x1 / s1
        conv (cin 256, cout_pad 128 / 256) reads directly; the first conv's output is still
        stored when anything else reads it (yolov7: layer 11 -> layer 14 at 160^2, layer 11
        also feeding the MP branch). 16-bit plans; YCX_NO_CONV_PAIR=1 keeps them apart.
        Returns {id(first conv): second conv}."""
        out = {}
        if not self.h16 or not self.fuse_pair or os.environ.get('YCX_NO_CONV_PAIR'):
            return out
        taken = set()

        def pointwise(nd):
            q = nd.p
            return (nd.kind == 'conv' and q['k'] == 1 and q['s'] == 1 and q['p'] == 0 and q['residual'] is None and
                    q['layout'] == L.OUT_NHWC and id(nd) not in pooled)

        for a in self.graph.nodes:
            if not pointwise(a) or id(a) in taken:
                continue
            x, v = a.inputs[0], a.out
            cin, cout = int(a.p['w'].shape[1]), int(a.p['w'].shape[0])
            if cin not in (64, 128, 256) or cout != 256 or v.role != 'act' or v.buf is None:
                continue
            if x.n * x.h * x.w < 8 * 64 * 256 or (x.role != 'input' and (x.coff % 8 or x.buf.c % 8)):
                continue
            if len(v.consumers) > 1 and (v.coff % 8 or v.buf.c % 8):  # y1 is stored: ycx_conv2d_pair's 16-B stores
                continue
            for b in v.consumers:
                if not pointwise(b) or b.inputs[0] is not v or id(b) in taken or id(b) in out:
                    continue
                cb = int(b.p['w'].shape[0])
                if self._cout_pad(cb) not in (128, 256) or cb % 8:
                    continue
                if b.out.role == 'act' and (b.out.coff % 8 or b.out.buf.c % 8):
                    continue
                out[id(a)] = b
                taken.update((id(a), id(b)))
                break
        return out

    def _pair_op(self, a, b):
        """One OP_CONV_PAIR for the chain a -> b (``_conv_pairs``)."""
        da, wa, ba, fa, shape = self._conv_parts(a)
        db, wb, bb, fb, _ = self._conv_parts(b)
        op = L.Op()
        op.kind = L.OP_CONV_PAIR
        op.d.pair[0], op.d.pair[1] = da, db
        idx = len(self.op_info)
        v = a.out
        store_a = len(v.consumers) > 1
        op.in_ = self._val_ptr(a.inputs[0], idx, 'in_')
        op.weight, op.bias = wa.data_ptr(), ba.data_ptr()
        op.weight2, op.bias2 = wb.data_ptr(), bb.data_ptr()
        op.out = self._val_ptr(v, idx, 'out') if store_a else None
        op.out2 = self._val_ptr(b.out, idx, 'out2')
        nbytes = (self._conv_bytes(da, wa, out_bytes=store_a) +
                  self._conv_bytes(db, wb) - db.n * db.h * db.w * db.cin * self.dtype.itemsize)  # y1 stays on chip
        self.op_info.append(dict(kind='conv_pair', name='wres1x1_pair', flops=fa + fb, shape=shape, parts=2,
                                 shape2=(db.n, db.h, db.w, db.cin, db.cout, 1, 1), bytes=nbytes))
        return op

    def _build(self):
        dev, dt = self.device, self.dtype
        self.buffers, self.params = [], []
        # packed tensors are named by the conv's position among the graph's conv / stem nodes,
        # not by packing order: which convs fuse (stem pair, 1x1 pair) varies with the batch
        # size and the A/B switches, and a prepack file is reused at any batch size
        self.packed = {}
        self._conv_index = {id(nd): i for i, nd in enumerate(
            nd for nd in self.graph.nodes if nd.kind in ('conv', 'stem'))}
        pairs = self._stem2_pairs()
        fused = {id(c) for c in pairs.values()}
        for b in self.activation_bufs():  # the stem maps of fused stem2 pairs stay in LDS
            b.tensor = torch.empty((b.n, b.h, b.w, b.c), dtype=dt, device=dev)
            self.buffers.append(b.tensor)
        ops, self.input_slots, self.output_slots, self.op_info = [], [], {}, []
        self._ksplit_ops = []  # (op index, workspace bytes) of the split-K convs
        self.conv_flops = 0
        cascades = self._pool_cascades()
        for c in cascades.values():
            fused.update(id(nd) for nd in c[1:])
        pooled = self._pool_convs()  # {id(conv): pool node} (the pool runs inside the conv)
        fused.update(id(nd) for nd in pooled.values())
        chains = self._conv_pairs(pooled)  # {id(first 1x1): second 1x1} (one launch each)
        fused.update(id(nd) for nd in chains.values())
        for node in self.graph.nodes:
            k = node.kind
            if id(node) in fused:
                continue
            if id(node) in pairs:
                ops.append(self._stem2_op(node, pairs[id(node)]))
            elif id(node) in chains:
                ops.append(self._pair_op(node, chains[id(node)]))
            elif k in ('conv', 'stem'):
                ops.append(self._conv_op(node, pool=pooled.get(id(node))))
            elif k == 'pool':
                ops.append(self._pool_op(node, levels=len(cascades.get(id(node), [node]))))
            elif k == 'up':  # an unfused upsample may write a slice of a concat buffer
                ops.append(self._copy_op(node.inputs[0], node.out, node.out.coff, scale=2))
            elif k == 'concat':
                for v, off in node.p['copies']:
                    ops.append(self._copy_op(v, node.out, off, scale=1))
            elif k == 'tonchw':
                ops.append(self._copy_op(node.inputs[0], node.out, 0, scale=1, nchw=True))
            else:
                raise AssertionError(k)
        self.n_ops = len(ops)
        self.ops = (L.Op * max(1, self.n_ops))(*ops)
        # one fp32 workspace for every split-K conv of the plan (they run in turn on its stream)
        nws = max([b for _, b in self._ksplit_ops], default=0)
        self.workspace = torch.empty(max(1, nws // 4), dtype=torch.float32, device=dev) if nws else None
        for i, _ in self._ksplit_ops:
            self.ops[i].workspace = self.workspace.data_ptr()
        self.head_params = []
        self.head_unstored = set()  # fused head ops that do not store raw logits (enable_head_decode)
        self.fixed_outputs = None
        self.static_input = None
        self._static_bound = False

    def _val_ptr(self, v, op_index, field):
        if v.role == 'input':
            self.input_slots.append((op_index, field))
            return None
        if v.role == 'output':
            self.output_slots.setdefault(id(v), []).append((op_index, field))
            return None
        return v.buf.tensor.data_ptr()

    def _conv_parts(self, node, bf16_weights=False, pool=None):
        """Packed weights/bias (kept alive in self.params) and the descriptor of a conv/stem node.
        bf16_weights: 16-bit packing whatever the plan dtype (the fp8 stem2 pair computes in bf16;
        an fp16 plan's pair in fp16).
        pool: the k2 s2 pool node feeding this 1x1 conv, fused into it (``_pool_convs``)."""
        p, x, out = node.p, node.inputs[0], node.out
        w64, b64 = p['w'], p['b']
        cout, cin, k = int(w64.shape[0]), int(w64.shape[1]), p['k']
        stem = node.kind == 'stem'
        cpad = self._cout_pad(cout, stem or bf16_weights)
        f8 = self.dt == L.DT_FP8
        if stem:  # [kh][kw][cin][cout_pad] fp32
            wshape, wdt = (k, k, cin, cpad), torch.float32
        elif bf16_weights:
            wshape, wdt = (cpad, k, k, cin), (torch.float16 if self.dt == L.DT_F16 else torch.bfloat16)
        elif f8:  # e4m3 rows of w * s_w[co], [cout_pad][kh*kw*cin padded to 128 B]
            wshape, wdt = (cpad, -(-k * k * cin // 128) * 128), torch.float8_e4m3fn
        else:     # [cout_pad][kh][kw][cin] in the activation dtype
            wshape, wdt = (cpad, k, k, cin), self.dtype
        bshape = (2 * cpad,) if (f8 and not stem and not bf16_weights) else (cpad,)
        # SiLU epilogues of the 16-bit / fp8 plans run on c' = -log2(e) c (YCX_ACT_SILU_PS): the weights
        # and bias are scaled here in float64 before their one rounding (fp8: the fp32 bias and dq rows,
        # so the e4m3 weights are unchanged); the fp32 parity plan keeps torch's silu(c) = c / (1 + e^-c)
        silu_ps = p['act'] == L.ACT_SILU and self.dt != L.DT_F32 and not _NO_SILU_PS
        i = 2 * self._conv_index[id(node)]
        if self.prepacked is not None:
            wt, bt = self.prepacked.get(f"p{i}"), self.prepacked.get(f"p{i + 1}")
            if wt is None or bt is None or tuple(wt.shape) != wshape or wt.dtype != wdt or \
                    tuple(bt.shape) != bshape or bt.dtype != torch.float32:
                raise ValueError(f"ycx: prepacked weights do not match this plan at tensor p{i}")
        else:
            wp = torch.zeros((cpad, cin, k, k), dtype=torch.float64)
            wp[:cout] = w64
            bp = torch.zeros(cpad, dtype=torch.float64)
            bp[:cout] = b64
            ks = L.SILU_PS_K if silu_ps else 1.0
            if not (f8 and not stem and not bf16_weights):
                wp, bp = wp * ks, bp * ks
            if stem:
                wt = wp.permute(2, 3, 1, 0).contiguous().to(torch.float32)
            elif bf16_weights:
                wt = wp.permute(0, 2, 3, 1).contiguous().to(wdt)
            elif f8:
                wt, sw = pack_fp8_weights(wp)
                bp = torch.cat([bp * ks, ks / (sw * self._scale(x))])  # dq[co] = 1 / (s_w[co] s_x), both x ks
            else:
                wt = wp.permute(0, 2, 3, 1).contiguous().to(self.dtype)
            bt = bp.to(torch.float32)
        wt = wt.to(self.device)
        bt = bt.to(self.device)
        self.params += [wt, bt]
        self.packed[f"p{i}"], self.packed[f"p{i + 1}"] = wt, bt
        d = L.ConvDesc()
        d.n, d.h, d.w, d.cin = x.n, x.h, x.w, cin
        if x.role == 'input':
            d.in_c_off, d.in_c_stride = 0, x.c
        else:
            d.in_c_off, d.in_c_stride = x.coff, x.buf.c
        if pool is not None:  # read the pool's (2h, 2w) input map instead of its output
            src = pool.inputs[0]
            d.in_c_off, d.in_c_stride, d.in_pool = src.coff, src.buf.c, 1
        d.ho, d.wo, d.cout, d.cout_pad = p['ho'], p['wo'], cout, cpad
        d.kh = d.kw = k
        d.stride, d.pad, d.act, d.leaky_slope = p['s'], p['p'], (L.ACT_SILU_PS if silu_ps else p['act']), p['slope']
        d.dtype, d.out_layout = self.dt, p['layout']
        if p['layout'] == L.OUT_NCHW_F32:
            d.out_c_off, d.out_c_stride = 0, cout
        else:
            d.out_c_off, d.out_c_stride = out.coff, out.buf.c
        r = p['residual']
        if r is not None:
            d.res_c_off, d.res_c_stride = r.coff, r.buf.c
        d.tile = 0
        d.out_scale = self._scale(out) if (f8 and p['layout'] != L.OUT_NCHW_F32) else 1.0
        d.res_scale = 1.0 / self._scale(r) if (f8 and r is not None) else 1.0
        flops = 2 * x.n * p['ho'] * p['wo'] * cout * cin * k * k
        self.conv_flops += flops
        return d, wt, bt, flops, (x.n, x.h, x.w, cin, cout, k, p['s'])

    def _conv_op(self, node, pool=None):
        x, out, r = node.inputs[0], node.out, node.p['residual']
        stem = node.kind == 'stem'
        d, wt, bt, flops, shape = self._conv_parts(node, pool=pool)
        op = L.Op()
        op.kind = L.OP_STEM if stem else L.OP_CONV
        op.d.conv = d
        idx = len(self.op_info)
        op.in_ = self._val_ptr(x if pool is None else pool.inputs[0], idx, 'in_')
        op.weight, op.bias = wt.data_ptr(), bt.data_ptr()
        op.out = self._val_ptr(out, idx, 'out')
        op.residual = r.buf.tensor.data_ptr() if r is not None else None
        tile = 0 if stem else int(L.lib.ycx_conv_pick_tile(ctypes.byref(d)))
        if not stem and tile in _TILE_MAP:  # development A/B only (YCX_TILE_MAP)
            cap, alts = _TILE_MAP[tile]
            bm, bn = _TILE_SHAPE.get(tile, (0, 0))
            if not bm or -(-d.cout_pad // bm) * -(-(d.n * d.ho * d.wo) // bn) < cap:
                for t in alts:
                    if (t not in (24, 25) or d.cout_pad % 256 == 0) and (pool is None or t in (16, 18)):
                        tile = d.tile = t
                        break
        name = 'stem' if stem else L.lib.ycx_conv_tile_name(tile).decode()
        if tile == 16 and d.stride == 2 and d.kh == 3 and d.kw == 3 and d.cin == 128 and pool is None:
            name += '+kcm'  # its own template instance (launch_glds: chunk-major K order), a row of its own in rocprof
        if not stem and pool is None and not _NO_KSPLIT:
            ks = int(L.lib.ycx_conv_pick_ksplit(ctypes.byref(d)))
            if ks > 1:  # split-K (r06): fp32 partials in the plan's workspace, then the ordered reduce launch
                d.k_split = ks
                self._ksplit_ops.append((len(self.op_info), int(L.lib.ycx_conv_workspace_size(ctypes.byref(d)))))
                name += f'+splitk{ks}'
        if pool is not None:
            name += '+maxpool_k2s2'
        op.d.conv = d  # ctypes copies a struct on assignment: store the final descriptor (tile map, k_split)
        kw = dict(stem=stem, pooled=pool is not None, residual=r is not None)
        nbytes = self._conv_bytes(d, wt, **kw)
        self.op_info.append(dict(kind=node.kind, name=name, flops=flops, shape=shape, parts=node.p.get('parts', 1),
                                 bytes=nbytes, out_bytes=nbytes - self._conv_bytes(d, wt, out_bytes=False, **kw)))
        return op

    def _conv_bytes(self, d, wt, stem=False, pooled=False, residual=False, out_bytes=True):
        """Algorithmic HBM bytes of one conv launch: its input map read once (the
        fp32 NCHW image for a stem; the 2x2-larger source map when an MP pool is
        fused in), the packed weights once, the residual once, the output written
        once (4x for the fused x2 upsample; fp32 for NCHW heads). The per-op
        roofline in bench.py prices each op against max(FLOP / MFMA peak, these
        bytes / HBM peak)."""
        isz = self.dtype.itemsize
        px_in = d.n * d.h * d.w * (4 if pooled else 1)
        b = px_in * d.cin * (4 if stem else isz)
        b += wt.numel() * wt.element_size()
        px_out = d.n * d.ho * d.wo
        if residual:
            b += px_out * d.cout * isz
        if out_bytes:
            if d.out_layout == L.OUT_NCHW_F32:
                b += px_out * d.cout * 4
            else:
                b += px_out * d.cout * isz * (4 if d.out_layout == L.OUT_NHWC_UP2 else 1)
        return int(b)

    def _stem2_op(self, stem, conv):
        ds, ws, bs, fs, _ = self._conv_parts(stem)
        dc, wc, bc, fc, shape = self._conv_parts(conv, bf16_weights=True)
        op = L.Op()
        op.kind = L.OP_STEM2
        op.d.pair[0], op.d.pair[1] = ds, dc
        idx = len(self.op_info)
        op.in_ = self._val_ptr(stem.inputs[0], idx, 'in_')
        op.weight, op.bias = ws.data_ptr(), bs.data_ptr()
        op.weight2, op.bias2 = wc.data_ptr(), bc.data_ptr()
        op.out = self._val_ptr(conv.out, idx, 'out')
        # the stem map stays in LDS: fp32 image in, both weight sets, the second conv's output out
        nbytes = (ds.n * ds.h * ds.w * ds.cin * 4 + ws.numel() * ws.element_size() + wc.numel() * wc.element_size() +
                  dc.n * dc.ho * dc.wo * dc.cout * self.dtype.itemsize)
        self.op_info.append(dict(kind='stem2', name='stem2_fused', flops=fs + fc, shape=shape, parts=2, bytes=nbytes))
        return op

    def _pool_cascades(self):
        """Chains of 'same' stride-1 pools (the SPPCSPC k5 cascade, `pyramid`), each pool
        reading the previous one's output, written to adjacent slices of one buffer: run as
        one ycx_maxpool launch with levels = chain length (bf16 / fp8 plans, HIP_CASCADE
        kernel), when the map's plane fits the kernel's LDS (``cascade_fits``; larger maps,
        e.g. the stride-32 map of a 1472^2 input, keep one launch per pool).
        Returns {id(first pool): [pool nodes]}."""
        if not (self.h16 or self.dt == L.DT_FP8) or os.environ.get('YCX_NO_POOL_CASCADE'):
            return {}
        nodes, out = self.graph.nodes, {}
        used = set()

        def same_pool(nd):
            p = nd.p
            return nd.kind == 'pool' and p['s'] == 1 and p['k'] % 2 == 1 and p['p'] == p['k'] // 2

        for i, a in enumerate(nodes):
            if id(a) in used or not same_pool(a) or a.out.role in ('input', 'output'):
                continue
            if not cascade_fits(a.inputs[0].h, a.inputs[0].w, a.inputs[0].c, self.dtype.itemsize):
                continue
            chain = [a]
            for b in nodes[i + 1:]:
                prev = chain[-1]
                if not (same_pool(b) and b.p['k'] == a.p['k'] and b.inputs[0] is prev.out and
                        b.out.buf is a.out.buf and b.out.coff == prev.out.coff + prev.out.c and
                        b.out.role not in ('input', 'output')):
                    break
                chain.append(b)
            if len(chain) > 1:
                out[id(a)] = chain
                used.update(id(nd) for nd in chain)
        return out

    def _pool_convs(self):
        """MP's k2 s2 pools (nets/common.py:25-31) whose map is read only by one 1x1 / s1
        conv: the conv pools its operand while staging it (ycx_conv_desc.in_pool, 16-bit
        plans, and fp8 plans where cin % 128 == 0), so the pooled map is never written.
        yolov7: all five MP pools. Returns {id(conv node): pool node}."""
        fp8 = self.dt == L.DT_FP8
        if not (self.h16 or fp8) or not self.fuse_pool or os.environ.get('YCX_NO_POOL_FUSE'):
            return {}
        out = {}
        for nd in self.graph.nodes:
            if nd.kind != 'pool':
                continue
            p, x, v = nd.p, nd.inputs[0], nd.out
            if not (p['k'] == 2 and p['s'] == 2 and p['p'] == 0 and x.h == 2 * v.h and x.w == 2 * v.w):
                continue
            if x.role != 'act' or v.role != 'act' or len(v.consumers) != 1 or x.coff % 8 or x.buf.c % 8:
                continue
            c = v.consumers[0]
            q = c.p
            if c.kind != 'conv' or c.inputs[0] is not v or not (q['k'] == 1 and q['s'] == 1 and q['p'] == 0):
                continue
            cin, cout = int(q['w'].shape[1]), int(q['w'].shape[0])
            if cin % (128 if fp8 else 64) or self._cout_pad(cout) % 64 or q['layout'] == L.OUT_NCHW_F32:
                continue
            if x.n * x.h * x.w * x.buf.c * (1 if fp8 else 2) >= (1 << 31) - 64:
                continue
            out[id(c)] = nd
        return out

    def _pool_op(self, node, levels=1):
        x, out, p = node.inputs[0], node.out, node.p
        d = L.PoolDesc()
        d.n, d.h, d.w, d.c, d.in_c_off, d.in_c_stride = x.n, x.h, x.w, x.c, x.coff, x.buf.c
        d.ho, d.wo, d.out_c_off, d.out_c_stride = out.h, out.w, out.coff, out.buf.c
        d.k, d.stride, d.pad, d.dtype, d.levels = p['k'], p['s'], p['p'], self.dt, levels
        op = L.Op()
        op.kind = L.OP_POOL
        op.d.pool = d
        op.in_, op.out = x.buf.tensor.data_ptr(), out.buf.tensor.data_ptr()
        name = f"maxpool_k{p['k']}s{p['s']}" + (f"_cascade{levels}" if levels > 1 else "")
        self.op_info.append(dict(kind='pool', name=name, flops=0,
                                 bytes=(x.n * (x.h * x.w + levels * out.h * out.w) * x.c * self.dtype.itemsize)))
        return op

    def _copy_op(self, x, out, off, scale, nchw=False):
        d = L.CopyDesc()
        d.n, d.h, d.w, d.c, d.in_c_off, d.in_c_stride = x.n, x.h, x.w, x.c, x.coff, x.buf.c
        d.scale, d.dtype = scale, self.dt
        op = L.Op()
        op.kind = L.OP_COPY
        idx = len(self.op_info)
        op.in_ = x.buf.tensor.data_ptr()
        d.dequant = 1.0 / self._scale(x) if self.dt == L.DT_FP8 else 1.0
        if nchw:
            d.out_c_off, d.out_c_stride, d.out_layout = 0, x.c, L.OUT_NCHW_F32
            op.out = self._val_ptr(out, idx, 'out')
        else:
            d.out_c_off, d.out_c_stride, d.out_layout = off, out.buf.c, L.OUT_NHWC
            op.out = out.buf.tensor.data_ptr()
        op.d.copy = d
        isz = self.dtype.itemsize
        nbytes = x.n * x.h * x.w * x.c * (isz + (4 if nchw else isz * scale * scale))
        self.op_info.append(dict(kind='copy', name='upsample2x' if scale == 2 else 'copy', flops=0, bytes=nbytes))
        return op

    # ------------------------------------------------------------------
    def _alloc_outputs(self):
        outs = [torch.empty((v.n, v.c, v.h, v.w), dtype=torch.float32, device=self.device) for v in self.out_vals]
        self._bind_outputs(outs)
        return outs

    def _bind_outputs(self, outs):
        for v, t in zip(self.out_vals, outs):
            for idx, field in self.output_slots.get(id(v), []):
                setattr(self.ops[idx], field, None if idx in self.head_unstored else t.data_ptr())

    # ---- fused Detect heads (decode + candidate filter in the head conv) ----
    def head_ops(self):
        """Op index of each output's producing conv, when every output is a bf16 or
        e4m3 Detect-head 1x1 conv the fused kernels cover (ycx_conv2d_head), else None."""
        if not (self.h16 or self.dt == L.DT_FP8):
            return None
        f8 = self.dt == L.DT_FP8
        idx = []
        for v in self.out_vals:
            slots = self.output_slots.get(id(v), [])
            if len(slots) != 1 or slots[0][1] != 'out':
                return None
            op = self.ops[slots[0][0]]
            d = op.d.conv
            if not (op.kind == L.OP_CONV and d.kh == 1 and d.kw == 1 and d.stride == 1 and d.pad == 0 and
                    d.act == L.ACT_NONE and d.out_layout == L.OUT_NCHW_F32 and d.cout <= 256 and
                    d.cin % (128 if f8 else 64) == 0 and d.in_c_off % (16 if f8 else 8) == 0 and
                    d.in_c_stride % (16 if f8 else 8) == 0):
                return None
            idx.append(slots[0][0])
        return idx

    def enable_head_decode(self, head_descs, cand, cand_rows, counts, keep_heads=True, status=None):
        """Turn the Detect-head convs into ycx_conv2d_head ops (decode_box + the
        candidate filter of detect.py:29-121 in the conv epilogue; candidates
        appended to cand / cand_rows / counts, which the caller zeroes before
        every forward). keep_heads: also store the raw fp32 NCHW logits.
        status: an int32 device tensor the head kernels set to
        YCX_HEAD_NONFINITE when a logit is inf / NaN (the fp16 range guard).
        Must precede capture(). Returns False when the plan does not qualify."""
        if self.graph_exec is not None:
            raise RuntimeError("ycx: enable_head_decode() after capture()")
        idx = self.head_ops()
        if idx is None or len(head_descs) != len(idx):
            return False
        for i, hd in zip(idx, head_descs):
            op = self.ops[i]
            conv = L.ConvDesc()
            ctypes.pointer(conv)[0] = op.d.conv
            if conv.cout_pad != 256:  # the head tile covers 256 output channels: zero-pad the weight rows
                wi = next(j for j, t in enumerate(self.params) if t.data_ptr() == op.weight)
                w, b = self.params[wi], self.params[wi + 1]
                w2 = torch.zeros((256,) + tuple(w.shape[1:]), dtype=w.dtype, device=w.device)
                if self.dt == L.DT_FP8:  # bias then dq, each [cout_pad]
                    b2 = torch.zeros((512,), dtype=b.dtype, device=b.device)
                    b2[:conv.cout] = b[:conv.cout]
                    b2[256:256 + conv.cout] = b[conv.cout_pad:conv.cout_pad + conv.cout]
                else:
                    b2 = torch.zeros((256,), dtype=b.dtype, device=b.device)
                    b2[:conv.cout] = b[:conv.cout]
                w2[:conv.cout] = w[:conv.cout]
                self.head_params += [w2, b2]   # self.params keeps the plan's shapes (prepack)
                op.weight, op.bias, conv.cout_pad = w2.data_ptr(), b2.data_ptr(), 256
            op.kind = L.OP_HEAD
            op.d.head.conv = conv
            op.d.head.head = hd
            op.cand, op.cand_rows, op.cand_counts = cand.data_ptr(), cand_rows.data_ptr(), counts.data_ptr()
            op.status = status.data_ptr() if status is not None else None
            tile = 39 if self.dt == L.DT_FP8 else 38
            self.op_info[i] = dict(self.op_info[i], name=L.lib.ycx_conv_tile_name(tile).decode(), kind='head')
            if not keep_heads:  # the logits never reach HBM (the candidates appended are ~KB)
                self.head_unstored.add(i)
                info = self.op_info[i]
                self.op_info[i] = dict(info, bytes=info['bytes'] - info.get('out_bytes', 0), out_bytes=0)
        if self.fixed_outputs is not None:
            self._bind_outputs(self.fixed_outputs)
        return True

    def _bind_input(self, x):
        if x.device != self.device or x.dtype != torch.float32 or not x.is_contiguous():
            x = x.to(self.device, torch.float32).contiguous()
        if tuple(x.shape) != self.shape:
            raise ValueError(f"ycx: engine built for {self.shape}, got {tuple(x.shape)}")
        for idx, field in self.input_slots:
            setattr(self.ops[idx], field, x.data_ptr())
        return x

    def _result(self, outs):
        return outs if self.is_list else outs[0]

    def run(self, x, events=None):
        """Eager forward: fresh output tensors every call (like the reference)."""
        x = self._bind_input(x)
        outs = self._alloc_outputs()
        self._static_bound = False  # the op array now points at this call's tensors
        ev = None
        if events is not None:
            ev = (ctypes.c_void_p * (self.n_ops + 1))(*[e.cuda_event for e in events])
        stream = L.stream_handle(self.device)
        L.check(L.lib.ycx_run_ops(self.ops, self.n_ops, stream, ev), "ycx_run_ops")
        return self._result(outs)

    # ---- static-I/O path for benchmarking / serving loops ----
    def bind_static(self, x):
        """Pin the plan to persistent input/output tensors (required by capture()).
        Idempotent: every caller of one engine shares the same static tensors
        (and the HIP graph captured on them)."""
        if self.fixed_outputs is None:
            self.static_input = self._bind_input(x)
            self.fixed_outputs = self._alloc_outputs()
            self._static_bound = True
        return self.static_input, self._result(self.fixed_outputs)

    def _ensure_static(self):
        if not self._static_bound:  # an eager run() re-pointed the op array
            self._bind_input(self.static_input)
            self._bind_outputs(self.fixed_outputs)
            self._static_bound = True

    def run_static(self, events=None):
        self._ensure_static()
        ev = None
        ops, n_ops = self.ops, self.n_ops
        if events is not None:  # per-op events: the plan's own op list
            ev = (ctypes.c_void_p * (self.n_ops + 1))(*[e.cuda_event for e in events])
        else:
            ops, n_ops = self._exec_ops()
        L.check(L.lib.ycx_run_ops(ops, n_ops, L.stream_handle(self.device), ev), "ycx_run_ops")
        return self._result(self.fixed_outputs)

    # ---- image-chunked prefix (experiment: keep the memory-bound high-resolution layers'
    # working set in the 256 MiB Infinity Cache by running them k images at a time) ----
    def _esize(self):
        return {L.DT_BF16: 2, L.DT_F16: 2, L.DT_F32: 4, L.DT_FP8: 1}[self.dt]

    def _chunk_op(self, op, i0, k):
        """A copy of ``op`` restricted to images [i0, i0 + k): every operand is image-major,
        so the restriction is n = k and a pointer offset per operand."""
        o = L.Op()
        ctypes.pointer(o)[0] = op
        es = self._esize()

        def shift(field, per_image):
            v = getattr(o, field)
            if v:
                setattr(o, field, v + i0 * per_image)

        if o.kind in (L.OP_CONV, L.OP_STEM, L.OP_STEM2):
            d = o.d.pair[1] if o.kind == L.OP_STEM2 else o.d.conv
            first = o.d.pair[0] if o.kind == L.OP_STEM2 else d
            if o.kind == L.OP_CONV:
                shift('in_', (4 if d.in_pool else 1) * d.h * d.w * d.in_c_stride * es)
            else:  # fp32 NCHW image
                shift('in_', first.cin * first.h * first.w * 4)
            if d.out_layout == L.OUT_NCHW_F32:
                shift('out', d.out_c_stride * d.ho * d.wo * 4)
            else:
                shift('out', (4 if d.out_layout == L.OUT_NHWC_UP2 else 1) * d.ho * d.wo * d.out_c_stride * es)
            shift('residual', d.ho * d.wo * d.res_c_stride * es)
            for dd in ((o.d.pair[0], o.d.pair[1]) if o.kind == L.OP_STEM2 else (o.d.conv,)):
                dd.n = k
        elif o.kind == L.OP_POOL:
            d = o.d.pool
            shift('in_', d.h * d.w * d.in_c_stride * es)
            shift('out', d.ho * d.wo * d.out_c_stride * es)
            d.n = k
        elif o.kind == L.OP_COPY:
            d = o.d.copy
            shift('in_', d.h * d.w * d.in_c_stride * es)
            if d.out_layout == L.OUT_NCHW_F32:
                shift('out', d.out_c_stride * d.h * d.w * 4)
            else:
                shift('out', d.scale * d.scale * d.h * d.w * d.out_c_stride * es)
            d.n = k
        else:
            raise ValueError("ycx: cannot chunk this op kind")
        return o

    @staticmethod
    def _op_out_h(op):
        if op.kind in (L.OP_CONV, L.OP_STEM, L.OP_HEAD):
            return op.d.conv.ho
        if op.kind == L.OP_STEM2:
            return op.d.pair[1].ho
        if op.kind == L.OP_POOL:
            return op.d.pool.ho
        return op.d.copy.h * op.d.copy.scale

    def _exec_ops(self):
        """The op array a forward runs: the plan, or with YCX_CHUNK='k:cut' its first ``cut``
        ops run k images at a time (all of them for images 0..k-1, then k..2k-1, ...)."""
        spec = os.environ.get('YCX_CHUNK')
        n = self.shape[0]
        if not spec:
            return self.ops, self.n_ops
        ks, cs = spec.split(':')
        k = int(ks)
        if cs.startswith('@'):  # '@H': every op up to the first whose output is below H rows
            hmin, cut = int(cs[1:]), 0
            while cut < self.n_ops and self._op_out_h(self.ops[cut]) >= hmin:
                cut += 1
        else:
            cut = min(int(cs), self.n_ops)
        if k <= 0 or k >= n or n % k or any(self.ops[i].kind == L.OP_HEAD for i in range(cut)):
            return self.ops, self.n_ops
        ops = [self._chunk_op(self.ops[i], i0, k) for i0 in range(0, n, k) for i in range(cut)]
        ops += [self.ops[i] for i in range(cut, self.n_ops)]
        self._chunked_ops = (L.Op * len(ops))(*ops)
        return self._chunked_ops, len(ops)

    def capture(self):
        """Capture the static plan into a HIP graph (one launch per forward)."""
        if self.fixed_outputs is None:
            raise RuntimeError("ycx: call bind_static() before capture()")
        if self.graph_exec is None:
            self._ensure_static()
            h = ctypes.c_void_p()
            s = torch.cuda.Stream(self.device)
            s.wait_stream(torch.cuda.current_stream(self.device))
            ops, n_ops = self._exec_ops()
            L.check(L.lib.ycx_graph_capture(ops, n_ops, s.cuda_stream, ctypes.byref(h)),
                    "ycx_graph_capture")
            torch.cuda.current_stream(self.device).wait_stream(s)
            self.graph_exec = h.value
        return self.graph_exec

    def replay(self):
        L.check(L.lib.ycx_graph_launch(self.graph_exec, L.stream_handle(self.device)), "ycx_graph_launch")
        return self._result(self.fixed_outputs)

    def close(self):
        if self.graph_exec is not None:
            L.lib.ycx_graph_destroy(self.graph_exec)
            self.graph_exec = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- introspection ----
    @property
    def flops_per_image(self):
        return self.conv_flops / self.shape[0]

    def summary(self):
        kinds = {}
        for info in self.op_info:
            kinds[info['kind']] = kinds.get(info['kind'], 0) + 1
        mem = sum(t.numel() * t.element_size() for t in self.buffers)
        return dict(ops=self.n_ops, kinds=kinds, activation_bytes=mem, gflop_per_image=self.flops_per_image / 1e9)
