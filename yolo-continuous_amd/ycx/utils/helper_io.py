"""Config I/O (utils/helper_io.py:7-26 semantics) with a safe YAML loader.

``cvt_cfg`` accepts a dict, a YAML path (SafeLoader) or a JSON path. Network
configs shipped with this package live in ``ycx/cfg/net/*.json``; they are the
reference's network YAMLs converted to JSON by tests/golden/make_golden.py.
"""
from __future__ import annotations

import glob
import json
import os
from pathlib import Path

import yaml

NET_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "cfg", "net")


def check_file(file):
    """Return ``file`` if it exists, else the unique recursive match under cwd."""
    if Path(file).is_file() or file == '':
        return file
    files = glob.glob('./**/' + str(file), recursive=True)
    assert len(files), f'File Not Found: {file}'
    assert len(files) == 1, f"Multiple files match '{file}', specify exact path: {files}"
    return files[0]


def cvt_cfg(cfg):
    """dict -> dict; *.json / *.yaml path -> dict. Bare net names ('yolov7',
    'yolov7-tiny') resolve to the packaged configs."""
    if isinstance(cfg, dict):
        return cfg
    path = str(cfg)
    if not os.path.exists(path):
        cand = os.path.join(NET_DIR, os.path.splitext(os.path.basename(path))[0] + ".json")
        if os.path.exists(cand):
            path = cand
    with open(path) as f:
        if path.endswith(".json"):
            return json.load(f)
        return yaml.load(f, Loader=yaml.SafeLoader)
