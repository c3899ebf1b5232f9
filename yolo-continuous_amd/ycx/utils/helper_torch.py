"""Device selection (utils/helper_torch.py:23-45 semantics) for ROCm.

``select_device('0')`` -> cuda:0 (HIP), asserting a device is visible, like the
reference. Unlike the reference it does not rewrite CUDA_VISIBLE_DEVICES /
HIP_VISIBLE_DEVICES (that is the launcher's job with one process per GPU).
'cpu' is accepted for API compatibility but the HIP model path will refuse it.
"""
from __future__ import annotations

import time

import torch


def timer(func):
    def wrapper(*args, **kwargs):
        t0 = time.time()
        r = func(*args, **kwargs)
        print('{0} cost:\t{1:.3f}s'.format(func.__name__, time.time() - t0))
        return r
    return wrapper


def select_device(device='', batch_size=None):
    device = str(device).strip().lower()
    if device == 'cpu':
        return torch.device('cpu')
    assert torch.cuda.is_available(), f'ROCm device unavailable, invalid device {device!r} requested'
    n = torch.cuda.device_count()
    if n > 1 and batch_size:
        assert batch_size % n == 0, f'batch-size {batch_size} not multiple of GPU count {n}'
    idx = 0
    if device and device not in ('cuda',):
        idx = int(device.split(',')[0].replace('cuda:', ''))
    return torch.device(f'cuda:{idx}')
