"""YOLO model builder and the drop-in ``Model`` (nets/yolo.py semantics).

``parse_model`` restates the reference builder (nets/yolo.py:15-87): channel
bookkeeping ``c2 = make_divisible(c2 * width_multiple, 8)``, depth gain, repeat
insertion for CSP-type blocks, concat channel sums, head channel lists and the
save list. Unlike the reference it never calls ``eval`` on YAML strings: module
names come from a whitelist and arguments from a small safe parser
(``None``, ``nc``/``num_classes``, ``anchors``, ``nn.LeakyReLU(0.1)``,
``nn.SiLU()``, literals), SURVEY.md Appendix B.10.

``Model.forward`` runs inference only, through the HIP engine (``ycx.engine``):
the first call for a given (input shape, device, precision) lowers the module
tree to a static op plan with BN/RepConv folded and buffers pre-allocated.
Training is out of scope: ``forward`` in train mode raises.
"""
from __future__ import annotations

import ast
import math
import re
from copy import deepcopy
from enum import Enum

import torch
from torch import nn

from ..utils.helper_io import cvt_cfg
from .common import (SP, SPP, SPPCSPC, SPPF, MP, Bottleneck, BottleneckCSPA, BottleneckCSPB, BottleneckCSPC,
                     Concat, Conv, ImplicitA, ImplicitM, RepConv)
from .detect import Detect, IAuxDetect, IDetect


def make_divisible(x, divisor):
    return math.ceil(x / divisor) * divisor


_MODULES = {
    'Conv': Conv, 'MP': MP, 'SP': SP, 'Concat': Concat, 'SPPCSPC': SPPCSPC, 'RepConv': RepConv,
    'Bottleneck': Bottleneck, 'BottleneckCSPA': BottleneckCSPA, 'BottleneckCSPB': BottleneckCSPB,
    'BottleneckCSPC': BottleneckCSPC, 'SPP': SPP, 'SPPF': SPPF, 'ImplicitA': ImplicitA,
    'ImplicitM': ImplicitM, 'Detect': Detect, 'IDetect': IDetect, 'IAuxDetect': IAuxDetect,
    'nn.Conv2d': nn.Conv2d, 'nn.BatchNorm2d': nn.BatchNorm2d, 'nn.Upsample': nn.Upsample,
}
# Reference modules constructible by its parse_model but used by neither shipped
# YAML: named here so the error says "out of scope", not "unknown".
_OUT_OF_SCOPE = {
    'ReOrg', 'Chuncat', 'Shortcut', 'Foldcut', 'RobustConv', 'RobustConv2', 'GhostConv', 'Stem', 'DownC',
    'Res', 'ResX', 'Ghost', 'GhostSPPCSPC', 'GhostStem', 'dw_conv', 'Focus', 'Contract', 'Expand', 'Classify',
    'TransformerLayer', 'TransformerBlock', 'IBin', 'RepBottleneck',
} | {f'{p}{s}' for p in ('Res', 'ResX', 'RepRes', 'RepResX', 'Ghost', 'RepBottleneck')
     for s in ('CSPA', 'CSPB', 'CSPC')}

_CONV_LIKE = (nn.Conv2d, Conv, RepConv, SPP, SPPF, SPPCSPC, Bottleneck, BottleneckCSPA, BottleneckCSPB,
              BottleneckCSPC)
_CSP_LIKE = (SPPCSPC, BottleneckCSPA, BottleneckCSPB, BottleneckCSPC)
_ACTS = {'LeakyReLU': nn.LeakyReLU, 'SiLU': nn.SiLU, 'Identity': nn.Identity}
_CALL_RE = re.compile(r'^(?:nn\.)?(\w+)\((.*)\)$')


def _resolve_module(m):
    if not isinstance(m, str):
        return m
    if m in _MODULES:
        return _MODULES[m]
    base = m.split('.')[-1]
    if base in _OUT_OF_SCOPE or m in _OUT_OF_SCOPE:
        raise NotImplementedError(f"ycx: module '{m}' is out of scope for the HIP inference path (SURVEY.md §2)")
    raise ValueError(f"ycx: unknown module '{m}' in network config")


def _resolve_arg(a, nc, anchors):
    if not isinstance(a, str):
        return a
    if a == 'None':
        return None
    if a in ('nc', 'num_classes'):
        return nc
    if a == 'anchors':
        return anchors
    mt = _CALL_RE.match(a.strip())
    if mt and mt.group(1) in _ACTS:
        inner = mt.group(2).strip()
        params = [ast.literal_eval(p.strip()) for p in inner.split(',')] if inner else []
        return _ACTS[mt.group(1)](*params)
    try:
        return ast.literal_eval(a)
    except (ValueError, SyntaxError):
        return a  # e.g. 'nearest' (the reference's eval fails and keeps the string too)


def parse_model(d, ch, anchors, num_classes):
    """Network dict -> (nn.Sequential of layer modules tagged .i/.f/.type/.np, save list)."""
    nc, gd, gw = num_classes, d['depth_multiple'], d['width_multiple']
    na = (len(anchors[0]) // 2) if isinstance(anchors, list) else anchors
    no = na * (nc + 5)
    layers, save, c2 = [], [], ch[-1]
    for i, (f, n, m, args) in enumerate(d['backbone'] + d['head']):
        m = _resolve_module(m)
        args = [_resolve_arg(a, nc, anchors) for a in args]
        n = max(round(n * gd), 1) if n > 1 else n
        if m in _CONV_LIKE:
            c1, c2 = ch[f], args[0]
            if c2 != no:
                c2 = make_divisible(c2 * gw, 8)
            args = [c1, c2, *args[1:]]
            if m in _CSP_LIKE:
                args.insert(2, n)
                n = 1
        elif m is nn.BatchNorm2d:
            args = [ch[f]]
        elif m is Concat:
            c2 = sum(ch[x] for x in f)
        elif m in (Detect, IDetect, IAuxDetect):
            args.append([ch[x] for x in f])
            if isinstance(args[1], int):
                args[1] = [list(range(args[1] * 2))] * len(f)
        else:
            c2 = ch[f]
        m_ = nn.Sequential(*[m(*args) for _ in range(n)]) if n > 1 else m(*args)
        m_.i, m_.f = i, f
        m_.type = f"{m.__module__}.{m.__name__}"
        m_.np = sum(x.numel() for x in m_.parameters())
        save.extend(x % i for x in ([f] if isinstance(f, int) else f) if x != -1)
        layers.append(m_)
        if i == 0:
            ch = []
        ch.append(c2)
    return nn.Sequential(*layers), sorted(save)


class WeightInitial(Enum):
    NA = 0
    Random = 1


PRECISIONS = ('bf16', 'f32', 'fp8', 'fp16')


def _all_finite(outs):
    """One device reduction over every output tensor, one host read."""
    ts = [outs] if torch.is_tensor(outs) else [t for t in outs if torch.is_tensor(t)]
    if not ts:
        return True
    return bool(torch.stack([torch.isfinite(t).all() for t in ts]).all().item())


class Model(nn.Module):
    """Drop-in for nets/yolo.py ``Model`` (constructor :95-112, forward :143-153).

    forward(x: fp32 [N, C, H, W] on a ROCm device) -> the last layer's output:
    ``[P5, P4, P3]`` fp32 NCHW logits for a Detect head (nets/detect.py:38).
    ``precision`` selects the kernel dtype: 'fp16' (default: IEEE half
    activations and weights on the f16 MFMA, fp32 accumulate -- the bf16 kernels
    at the bf16 rate with an 11-bit significand, the mode that holds north_star's
    1e-3 of the reference's fp32 forward on box / confidence tensors; activations
    must stay inside the fp16 range, |a| < 65504 -- the range guard: a forward
    whose heads come out inf / NaN warns and re-plans this Model in 'bf16';
    a ``Detector`` flags it on the device and ``check()`` raises
    ``YcxRangeError``), 'bf16' (MFMA bf16, the BASELINE C2 bench
    configuration, ~1e-3), 'f32' (exact-fp32 MFMA) or 'fp8' (OCP
    e4m3 weights and activations on the block-scaled MFMA, fp32 accumulate; the
    activation scales come from ``calibrate_fp8``).
    """

    def __init__(self, model_cfg, anchors, num_classes, image_chan=3, weight_initial=WeightInitial.Random,
                 precision='fp16'):
        super().__init__()
        self.traced = False
        self.weight_initial = weight_initial
        self.anchors = anchors
        self.num_classes = num_classes
        self.image_chan = image_chan
        self.model, self.save = parse_model(deepcopy(cvt_cfg(model_cfg)), ch=[image_chan], anchors=anchors,
                                            num_classes=num_classes)
        self.set_precision(precision)
        self.initial_weights()

    # ---- reference API -------------------------------------------------
    def initial_weights(self):
        """nets/yolo.py:114-125: conv/linear W ~ N(0, 0.02); BN gamma ~ N(1, 0.02), beta = 0."""
        if self.weight_initial == WeightInitial.NA:
            return
        for m in self.modules():
            if isinstance(m, (nn.Conv2d, nn.Linear)):
                nn.init.normal_(m.weight, 0, 0.02)
            elif isinstance(m, (nn.BatchNorm2d, nn.GroupNorm)):
                nn.init.normal_(m.weight, 1.0, 0.02)
                nn.init.constant_(m.bias, 0)
            elif isinstance(m, (nn.Hardswish, nn.LeakyReLU, nn.ReLU, nn.ReLU6)):
                m.inplace = True
        self.invalidate(weights_changed=True)

    def print_info(self):
        n_p = sum(x.numel() for x in self.parameters())
        n_g = sum(x.numel() for x in self.parameters() if x.requires_grad)
        print('{0:5s} {1:40s} {2:9s} {3:12s} {4:20s} {5:10s} {6:10s}'.format(
            'layer', 'name', 'gradient', 'parameters', 'shape', 'mu', 'sigma'))
        for i, (name, p) in enumerate(self.named_parameters()):
            print('%5g %40s %9s %12g %20s %10.3g %10.3g' % (i, name, p.requires_grad, p.numel(), list(p.shape),
                                                            p.mean(), p.std()))
        print('total parameters: {0:7g} total gradients: {1:7g}'.format(n_p, n_g))

    def forward(self, x):
        if self.training:
            raise RuntimeError("ycx: Model is inference-only on the HIP path (training is out of scope); "
                               "call .eval() first")
        outs = self.engine_for(x.shape, x.device, slot=self.EAGER_SLOT).run(x)
        if self.precision == 'fp16' and not _all_finite(outs) and _all_finite(x):
            # the fp16 range guard: an activation past 65504 became inf at its producer's store and
            # reached the heads as inf / NaN (a non-finite input is passed through, as the
            # reference's fp32 forward does). The reference's fp32 forward has no such limit:
            # re-plan in bf16 (fp32's exponent range, 8-bit significand) for this and every later call.
            import warnings
            if (self.precision,) + tuple(int(v) for v in x.shape[2:]) in self._prepacked:
                # a bf16 re-plan would fold this module's own parameters, not the prepacked ones: raise
                # (as Detector.check does) rather than hand inf / NaN heads to a serving caller
                from .. import _lib
                raise _lib.YcxRangeError("ycx: the fp16 plan produced non-finite head logits on prepacked "
                                         "weights (an activation exceeds 65504); re-pack this checkpoint in "
                                         "'bf16' or 'f32'")
            warnings.warn("ycx: the fp16 plan overflowed (non-finite head logits: an activation exceeds "
                          "65504); switching this Model to precision='bf16' (about 1e-3 relative error, "
                          "use 'f32' for the 1e-3 parity mode)", RuntimeWarning, stacklevel=2)
            self.set_precision('bf16')
            return self.forward(x)
        head = self.model[-1]
        if isinstance(head, IDetect):  # eval branch: (z, x[:nl]) as nets/idetect.py:45, nets/iaux_detect.py:49
            from ..detect import idetect_outputs
            return idetect_outputs(head, outs, x.shape[2:])
        return outs

    # ---- engine management --------------------------------------------
    def set_precision(self, precision):
        if precision not in PRECISIONS:
            raise ValueError(f"ycx: precision must be one of {PRECISIONS}, got {precision!r}")
        self.precision = precision
        self.invalidate()
        return self

    def invalidate(self, weights_changed=False):
        """Drop compiled plans (packed weights); called when parameters change
        (then the fp8 calibration records are stale too)."""
        for eng in getattr(self, '_engines', {}).values():
            eng.close()
        self._engines = {}
        if weights_changed or not hasattr(self, '_fp8_amax'):
            self._fp8_amax = {}  # (H, W) -> calibration record
            self._prepacked = {}  # (precision, H, W) -> packed tensors (ycx.prepack)

    EAGER_SLOT = -1  # the engine behind forward(): never shared with a Detector

    def new_slot(self):
        """A slot id no other caller holds: every Detector (and every slot of a
        Pipelined/ConcurrentDetector) gets its own engine, i.e. its own
        activation buffers, static input and heads, so work in flight on one
        stream is never overwritten by another caller."""
        self._slot_counter = getattr(self, '_slot_counter', 0) + 1
        return 1000 + self._slot_counter

    def release_slot(self, shape, device, slot):
        """Drop the engine of one slot (its activation buffers, packed weights and
        HIP graph). Detectors call this from close() / their finaliser."""
        key = (tuple(int(s) for s in shape), str(torch.device(device)), self.precision, int(slot))
        eng = getattr(self, '_engines', {}).pop(key, None)
        if eng is not None:
            eng.close()
        return eng is not None

    def engine_for(self, shape, device, slot=0):
        """The compiled plan for (shape, device, precision); every distinct
        ``slot`` is an independent copy (own activation buffers). ``forward``
        uses ``EAGER_SLOT``; Detectors take fresh ids from ``new_slot``."""
        from ..engine import Engine
        shape = tuple(int(s) for s in shape)
        dev = torch.device(device)
        key = (shape, str(dev), self.precision, int(slot))
        eng = self._engines.get(key)
        if eng is None:
            amax = None
            if self.precision == 'fp8':
                amax = self._fp8_amax.get(shape[2:])
                if amax is None:
                    amax = self.calibrate_fp8(device=dev, hw=shape[2:])
            eng = Engine(self, shape, dev, self.precision, fp8_amax=amax,
                         prepacked=self._prepacked.get((self.precision,) + shape[2:]))
            self._engines[key] = eng
        return eng

    def calibrate_fp8(self, images=None, device=None, hw=None, n=4, seed=0):
        """fp8 activation calibration: one bf16 forward over ``images`` (fp32
        [N, C, H, W]) records max |activation| per buffer of the plan; every fp8
        engine for that (H, W) derives its power-of-two scales from it. Without
        images a seeded synthetic U[0,1) batch of ``n`` images at ``hw`` is used
        (no calibration set ships with the reference). Returns the record."""
        from ..engine import Engine
        from ..utils.synth import synthetic_images
        if images is None:
            if hw is None:
                raise ValueError("ycx: calibrate_fp8 needs images or hw=(H, W)")
            images = synthetic_images(n, self.image_chan, int(hw[0]), int(hw[1]), seed=seed)
        dev = torch.device(device) if device is not None else images.device
        images = images.to(dev, torch.float32).contiguous()
        # every buffer the fp8 plan stores must be written here: no fused MP pools, no 1x1 pairs
        # (a pair whose first output has one consumer keeps it on chip and never stores it)
        eng = Engine(self, tuple(images.shape), dev, 'bf16', fuse_pool=False, fuse_pair=False)
        try:
            eng.run(images)
            amax = [dict(c=int(b.c), amax=float(b.tensor.abs().max().float())) for b in eng.activation_bufs()]
        finally:
            eng.close()
        key = tuple(int(v) for v in images.shape[2:])
        self._fp8_amax[key] = amax
        for k in [k for k in self._engines if k[2] == 'fp8' and k[0][2:] == key]:
            self._engines.pop(k).close()
        return amax

    def save_prepacked(self, path, hw, precision=None, device='cuda'):
        """Write the folded, packed weights of the (precision, H, W) plan (and its
        fp8 calibration) to a safetensors file (ycx.prepack)."""
        from .. import prepack
        return prepack.save(self, path, hw, precision, device)

    def load_prepacked(self, path, strict=False):
        """Use the packed weights of a ycx.prepack file for its (precision, H, W)
        plan instead of folding this module's parameters, and switch to its
        precision. strict: the file must come from this module's current
        state_dict."""
        from .. import prepack
        meta, tensors = prepack.load(path)
        if strict and meta.get('state_dict_sha256') != prepack.state_dict_sha256(self):
            raise ValueError(f"ycx: {path} was packed from a different state_dict")
        hw = tuple(meta['hw'])
        self.set_precision(meta['precision'])
        self._prepacked[(meta['precision'],) + hw] = tensors
        if meta['precision'] == 'fp8':
            self._fp8_amax[hw] = meta['fp8_amax']
        return meta

    def load_state_dict(self, state_dict, strict=True, *args, **kwargs):
        r = super().load_state_dict(state_dict, strict, *args, **kwargs)
        self.invalidate(weights_changed=True)
        return r

    def _apply(self, fn, *args, **kwargs):
        r = super()._apply(fn, *args, **kwargs)
        self.invalidate()
        return r
