"""Plan YAML (cfg/train_plan.py:10-65), inference subset.

Reads the keys ``predict`` needs (device, image_size, image_chan, labels,
anchors, anchors_mask, model_cfg, save_dir/save_name) with yaml.safe_load;
training keys are kept as attributes when present and ignored otherwise.
``model_cfg`` paths that do not exist (the reference plans carry Windows
paths) fall back to the packaged net of the same
name (ycx/cfg/net/*.json).
"""
from __future__ import annotations

import os

import yaml


class TrainPlan(object):
    def __init__(self, cfg_file):
        with open(cfg_file, 'r') as f:
            cfg = yaml.safe_load(f)
        self.cfg_file = cfg
        self.device = "{}".format(cfg.get('device', 0))
        self.image_size = cfg['image_size']
        self.image_chan = cfg.get('image_chan', 3)
        self.labels = cfg['labels']
        self.num_labels = len(self.labels)
        self.model_cfg = self._resolve_net(cfg['model_cfg'])
        self.anchors = cfg['anchors']
        self.anchors_mask = cfg['anchors_mask']
        self.save_dir = cfg.get('save_dir', '.')
        self.save_name = cfg.get('save_name', 'model')
        self.save_path = os.path.join(self.save_dir, "{}.pth".format(self.save_name))
        for k, v in cfg.items():  # training hyper-parameters: carried, unused
            if not hasattr(self, k):
                setattr(self, k, v)

    @staticmethod
    def _resolve_net(path):
        if os.path.exists(str(path)):
            return path
        base = str(path).replace('\\', '/').split('/')[-1]
        return os.path.splitext(base)[0]  # cvt_cfg resolves bare names to ycx/cfg/net/<name>.json

    def __str__(self):
        info = "-" * 20 + type(self).__name__ + "-" * 20 + "\r\n"
        for key, value in self.__dict__.items():
            if key != 'cfg_file':
                info += "%20s :\t%s\r\n" % (key, value)
        return info
