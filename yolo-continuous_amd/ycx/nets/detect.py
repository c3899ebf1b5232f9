"""Detection heads as parameter holders (lowered to HIP convs by the engine).

Detect  — nets/detect.py:4-38: three 1x1 convs with bias; eval returns the raw
          logits [P5, P4, P3] (NCHW fp32), no decode.
IDetect — nets/idetect.py:7-50: ImplicitA -> 1x1 conv -> ImplicitM, reshaped to
          (bs, na, ny, nx, no); in eval also the decoded boxes in pixels. The
          reference leaves ``stride`` as None so its eval raises TypeError
          (SURVEY.md Appendix B.7); here the strides default to
          image_size / ny per level (documented deviation).
IAuxDetect — nets/iaux_detect.py:7-49: IDetect's main heads on x[:nl] plus
          auxiliary 1x1 heads ``m2`` on x[nl:]. Eval returns
          (cat(z, 1), x[:nl]): the aux maps are computed and discarded
          (:32-33, :49), so the engine lowers only the main heads and the aux
          branch is dead code it never launches.
"""
from __future__ import annotations

import torch
from torch import nn

from .common import ImplicitA, ImplicitM, _Holder


class Detect(_Holder):
    def __init__(self, num_classes=80, anchors=(), ch=()):
        super().__init__()
        self.num_classes = num_classes
        self.len_output = num_classes + 5
        self.num_layers = len(anchors)
        self.num_anchors_each_layer = len(anchors[0]) // 2
        out_c = self.num_anchors_each_layer * self.len_output
        # Attribute names = state_dict keys of the reference (model.N.yolo_head_P*).
        self.yolo_head_P3 = nn.Conv2d(ch[0], out_c, 1)
        self.yolo_head_P4 = nn.Conv2d(ch[1], out_c, 1)
        self.yolo_head_P5 = nn.Conv2d(ch[2], out_c, 1)
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.normal_(m.weight, 0, 0.01)

    def heads_in_output_order(self):
        """(conv, input position) pairs in the order the reference returns them."""
        return [(self.yolo_head_P5, 2), (self.yolo_head_P4, 1), (self.yolo_head_P3, 0)]


class IDetect(_Holder):
    stride = None

    def __init__(self, nc=80, anchors=(), ch=()):
        super().__init__()
        self.nc = nc
        self.no = nc + 5
        self.nl = len(anchors)
        self.na = len(anchors[0]) // 2
        a = torch.tensor(anchors).float().view(self.nl, -1, 2)
        self.register_buffer('anchors', a)
        self.register_buffer('anchor_grid', a.clone().view(self.nl, 1, -1, 1, 1, 2))
        self.m = nn.ModuleList(nn.Conv2d(x, self.no * self.na, 1) for x in ch)
        self.ia = nn.ModuleList(ImplicitA(x) for x in ch)
        self.im = nn.ModuleList(ImplicitM(self.no * self.na) for _ in ch)


class IAuxDetect(IDetect):
    """Schema of nets/iaux_detect.py:11-25 (state_dict keys anchors, anchor_grid,
    m.*, m2.*, ia.*, im.*). ``ch`` lists the main inputs then the aux inputs."""

    def __init__(self, nc=80, anchors=(), ch=()):
        nl = len(anchors)
        super().__init__(nc, anchors, ch[:nl])
        self.m2 = nn.ModuleList(nn.Conv2d(x, self.no * self.na, 1) for x in ch[nl:])
