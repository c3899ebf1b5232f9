"""Layer modules of the YOLOv7 graph, as parameter holders for the HIP engine.

Each class keeps the constructor signature and the parameter/buffer attribute
names of the reference module it stands for, so a reference ``state_dict``
(e.g. the 558-key yolov7 schema) loads unchanged. The modules
hold no ``forward`` compute: ``Model.forward`` lowers the whole module tree to
a static plan of HIP kernels (``ycx.engine``), folding BatchNorm, RepConv
branches and ImplicitA/M into conv weight/bias on the way.

Reference: nets/common.py (line numbers cited per class).
"""
from __future__ import annotations

from torch import nn


def autopad(k, p=None):
    """'same' padding for odd kernels (nets/common.py:7-11)."""
    if p is None:
        p = k // 2 if isinstance(k, int) else [x // 2 for x in k]
    return p


class _Holder(nn.Module):
    """Base: calling a layer module directly is not a compute path."""

    def forward(self, *args, **kwargs):  # pragma: no cover - guard
        raise RuntimeError(f"ycx: {type(self).__name__} is lowered by Model.forward into HIP kernels; "
                           f"call the Model, not the layer")


class Conv(_Holder):
    """act(bn(conv2d(x))), bias-free conv, BN eps 1e-5 (nets/common.py:97-109)."""

    def __init__(self, c1, c2, k=1, s=1, p=None, g=1, act=True):
        super().__init__()
        self.conv = nn.Conv2d(c1, c2, k, s, autopad(k, p), groups=g, bias=False)
        self.bn = nn.BatchNorm2d(c2)
        self.act = nn.SiLU() if act is True else (act if isinstance(act, nn.Module) else nn.Identity())


class MP(_Holder):
    """MaxPool2d(k, k) (nets/common.py:25-31)."""

    def __init__(self, k=2):
        super().__init__()
        self.m = nn.MaxPool2d(kernel_size=k, stride=k)


class SP(_Holder):
    """MaxPool2d(k, s, k//2) (nets/common.py:34-40)."""

    def __init__(self, k=3, s=1):
        super().__init__()
        self.m = nn.MaxPool2d(kernel_size=k, stride=s, padding=k // 2)


class Concat(_Holder):
    """Channel concat (nets/common.py:54-60); never materialised on device."""

    def __init__(self, dimension=1):
        super().__init__()
        self.d = dimension


class Bottleneck(_Holder):
    """x + cv2(cv1(x)) when shortcut and c1 == c2 (nets/common.py:199-209)."""

    def __init__(self, c1, c2, shortcut=True, g=1, e=0.5):
        super().__init__()
        c_ = int(c2 * e)
        self.cv1 = Conv(c1, c_, 1, 1)
        self.cv2 = Conv(c_, c2, 3, 1, g=g)
        self.add = shortcut and c1 == c2


class SPP(_Holder):
    """cv2(cat[x, mp5, mp9, mp13](cv1 x)) (nets/common.py:185-196)."""

    def __init__(self, c1, c2, k=(5, 9, 13)):
        super().__init__()
        c_ = c1 // 2
        self.cv1 = Conv(c1, c_, 1, 1)
        self.cv2 = Conv(c_ * (len(k) + 1), c2, 1, 1)
        self.m = nn.ModuleList([nn.MaxPool2d(kernel_size=x, stride=1, padding=x // 2) for x in k])


class SPPCSPC(_Holder):
    """CSP spatial pyramid pooling block of yolov7 layer 51 (nets/common.py:248-266)."""

    def __init__(self, c1, c2, n=1, shortcut=False, g=1, e=0.5, k=(5, 9, 13)):
        super().__init__()
        c_ = int(2 * c2 * e)
        self.cv1 = Conv(c1, c_, 1, 1)
        self.cv2 = Conv(c1, c_, 1, 1)
        self.cv3 = Conv(c_, c_, 3, 1)
        self.cv4 = Conv(c_, c_, 1, 1)
        self.m = nn.ModuleList([nn.MaxPool2d(kernel_size=x, stride=1, padding=x // 2) for x in k])
        self.cv5 = Conv(4 * c_, c_, 1, 1)
        self.cv6 = Conv(c_, c_, 3, 1)
        self.cv7 = Conv(2 * c_, c2, 1, 1)


class BottleneckCSPA(_Holder):
    """cv3(cat[m(cv1 x), cv2 x]) (nets/common.py:294-307)."""

    def __init__(self, c1, c2, n=1, shortcut=True, g=1, e=0.5):
        super().__init__()
        c_ = int(c2 * e)
        self.cv1 = Conv(c1, c_, 1, 1)
        self.cv2 = Conv(c1, c_, 1, 1)
        self.cv3 = Conv(2 * c_, c2, 1, 1)
        self.m = nn.Sequential(*[Bottleneck(c_, c_, shortcut, g, e=1.0) for _ in range(n)])


class BottleneckCSPB(_Holder):
    """x1 = cv1 x; cv3(cat[m(x1), cv2 x1]) (nets/common.py:310-324)."""

    def __init__(self, c1, c2, n=1, shortcut=False, g=1, e=0.5):
        super().__init__()
        c_ = int(c2)
        self.cv1 = Conv(c1, c_, 1, 1)
        self.cv2 = Conv(c_, c_, 1, 1)
        self.cv3 = Conv(2 * c_, c2, 1, 1)
        self.m = nn.Sequential(*[Bottleneck(c_, c_, shortcut, g, e=1.0) for _ in range(n)])


class BottleneckCSPC(_Holder):
    """cv4(cat[cv3(m(cv1 x)), cv2 x]) (nets/common.py:327-341)."""

    def __init__(self, c1, c2, n=1, shortcut=True, g=1, e=0.5):
        super().__init__()
        c_ = int(c2 * e)
        self.cv1 = Conv(c1, c_, 1, 1)
        self.cv2 = Conv(c1, c_, 1, 1)
        self.cv3 = Conv(c_, c_, 1, 1)
        self.cv4 = Conv(2 * c_, c2, 1, 1)
        self.m = nn.Sequential(*[Bottleneck(c_, c_, shortcut, g, e=1.0) for _ in range(n)])


class ImplicitA(_Holder):
    """Learned additive channel bias (nets/common.py:416-426)."""

    def __init__(self, channel, mean=0., std=.02):
        super().__init__()
        import torch
        self.channel, self.mean, self.std = channel, mean, std
        self.implicit = nn.Parameter(torch.zeros(1, channel, 1, 1))
        nn.init.normal_(self.implicit, mean=self.mean, std=self.std)


class ImplicitM(_Holder):
    """Learned multiplicative channel scale (nets/common.py:429-439)."""

    def __init__(self, channel, mean=0., std=.02):
        super().__init__()
        import torch
        self.channel, self.mean, self.std = channel, mean, std
        self.implicit = nn.Parameter(torch.ones(1, channel, 1, 1))
        nn.init.normal_(self.implicit, mean=self.mean, std=self.std)


class RepConv(_Holder):
    """RepVGG block: act(BN(conv3x3) + BN(conv1x1) [+ BN(x)]) (nets/common.py:442-486).

    The engine always runs the re-parameterised single 3x3 conv; the branch
    folding restates get_equivalent_kernel_bias / _fuse_bn_tensor
    (nets/common.py:488-529)."""

    def __init__(self, c1, c2, k=3, s=1, p=None, g=1, act=True, deploy=False):
        super().__init__()
        assert k == 3
        assert autopad(k, p) == 1
        self.deploy = deploy
        self.groups = g
        self.in_channels = c1
        self.out_channels = c2
        self.stride = s
        padding_11 = autopad(k, p) - k // 2
        self.act = nn.SiLU() if act is True else (act if isinstance(act, nn.Module) else nn.Identity())
        if deploy:
            self.rbr_reparam = nn.Conv2d(c1, c2, k, s, autopad(k, p), groups=g, bias=True)
        else:
            self.rbr_identity = nn.BatchNorm2d(num_features=c1) if c2 == c1 and s == 1 else None
            self.rbr_dense = nn.Sequential(nn.Conv2d(c1, c2, k, s, autopad(k, p), groups=g, bias=False),
                                           nn.BatchNorm2d(num_features=c2))
            self.rbr_1x1 = nn.Sequential(nn.Conv2d(c1, c2, 1, s, padding_11, groups=g, bias=False),
                                         nn.BatchNorm2d(num_features=c2))


class SPPF(_Holder):
    """cv2(cat[x, m x, m m x, m m m x]) with k=5 (nets/common.py:771-784)."""

    def __init__(self, c1, c2, k=5):
        super().__init__()
        c_ = c1 // 2
        self.cv1 = Conv(c1, c_, 1, 1)
        self.cv2 = Conv(c_ * 4, c2, 1, 1)
        self.m = nn.MaxPool2d(kernel_size=k, stride=1, padding=k // 2)
