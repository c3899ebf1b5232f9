"""Seeded, platform-independent synthetic weights and inputs.

No checkpoint exists for the reference and its own init gives bias-dominated,
near-constant heads (nets/yolo.py:114-125), so parity fixtures and the bench
use this recipe instead. Every tensor gets its own splitmix64 stream keyed by
(seed, state_dict key); normals are Box-Muller in float64, rounded to fp32.

  conv weight         N(0, 2 / fan_in)            (He; keeps O(1) activations)
  conv bias           0.1 N                       (Detect/IDetect heads)
  BN weight / bias    1 + 0.1 N / 0.1 N
  BN running_mean     0.1 N
  BN running_var      1 + 0.5 U
  ImplicitA / M       0.02 N / 1 + 0.02 N
  num_batches_tracked 0;  anchors buffers keep their values
"""
from __future__ import annotations

import zlib

import numpy as np
import torch
from torch import nn

_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def splitmix64(seed: int, n: int) -> np.ndarray:
    """n outputs of the splitmix64 sequence started at ``seed`` (uint64)."""
    with np.errstate(over='ignore'):
        idx = np.arange(1, n + 1, dtype=np.uint64)
        z = np.uint64(seed & 0xFFFFFFFFFFFFFFFF) + idx * np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return z


def uniform(seed: int, n: int) -> np.ndarray:
    """U[0, 1) float64 with 53 random bits."""
    return (splitmix64(seed, n) >> np.uint64(11)).astype(np.float64) * (1.0 / 9007199254740992.0)


def normal(seed: int, n: int) -> np.ndarray:
    u = uniform(seed, 2 * ((n + 1) // 2)).reshape(-1, 2)
    r = np.sqrt(-2.0 * np.log1p(-u[:, 0]))
    t = 2.0 * np.pi * u[:, 1]
    return np.stack([r * np.cos(t), r * np.sin(t)], 1).reshape(-1)[:n]


def tensor_seed(seed: int, key: str) -> int:
    return (seed * 0x100000001B3 + zlib.crc32(key.encode())) & 0xFFFFFFFFFFFFFFFF


def synthetic_state_dict(model: nn.Module, seed: int = 0) -> dict:
    """A full state_dict for ``model`` following the recipe above."""
    owners = dict(model.named_modules())
    out = {}
    for key, t in model.state_dict().items():
        mod_name, _, leaf = key.rpartition('.')
        owner = owners.get(mod_name)
        s = tensor_seed(seed, key)
        n = t.numel()
        if leaf == 'num_batches_tracked':
            v = np.zeros(n)
        elif leaf == 'running_var':
            v = 1.0 + 0.5 * uniform(s, n)
        elif leaf == 'running_mean':
            v = 0.1 * normal(s, n)
        elif isinstance(owner, (nn.BatchNorm2d, nn.GroupNorm)):
            v = (1.0 + 0.1 * normal(s, n)) if leaf == 'weight' else 0.1 * normal(s, n)
        elif isinstance(owner, nn.Conv2d) and leaf == 'weight':
            fan_in = t.shape[1] * t.shape[2] * t.shape[3]
            v = normal(s, n) * np.sqrt(2.0 / fan_in)
        elif isinstance(owner, nn.Conv2d) and leaf == 'bias':
            v = 0.1 * normal(s, n)
        elif leaf == 'implicit':
            is_mul = type(owner).__name__ == 'ImplicitM'
            v = (1.0 if is_mul else 0.0) + 0.02 * normal(s, n)
        else:  # registered buffers such as IDetect anchors keep their values
            out[key] = t.detach().clone()
            continue
        out[key] = torch.from_numpy(v.reshape(tuple(t.shape))).to(t.dtype)
    return out


def synthetic_images(n: int, c: int, h: int, w: int, seed: int = 0) -> torch.Tensor:
    """U[0, 1) fp32 images [n, c, h, w] (the bench / fixture input recipe)."""
    return torch.from_numpy(uniform(tensor_seed(seed, 'images'), n * c * h * w).astype(np.float32)).reshape(n, c, h, w)


def synthetic_head_logits(shapes, nc: int, na: int = 3, seed: int = 0, obj_shift: float = -3.0):
    """N(0, 1) fp32 head logits [bs, na*(5+nc), h, w] per (bs, h, w) in ``shapes``
    with the objectness logit shifted by ``obj_shift`` (the G3 decode/NMS recipe)."""
    outs = []
    for i, (bs, h, w) in enumerate(shapes):
        v = normal(tensor_seed(seed, f'head{i}'), bs * na * (5 + nc) * h * w).astype(np.float32)
        v = v.reshape(bs, na, 5 + nc, h, w)
        v[:, :, 4] += np.float32(obj_shift)
        outs.append(torch.from_numpy(v.reshape(bs, na * (5 + nc), h, w).copy()))
    return outs
