"""Data-parallel inference across the GPUs of one node.

Images are independent (the reference loops per image, detect.py:105-106), so
each rank runs the whole hot path on its own contiguous shard of the batch and
the only collective is ONE all-gather of the fixed-size padded detections
(+ keep rows + counts) over RCCL/xGMI. Gathered rank-major = original image
order, which is the order of the reference's ``output`` list (detect.py:105).
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def shard(global_batch: int, rank: int, world: int) -> slice:
    """Contiguous shard of a global batch for ``rank`` (sizes differ by <= 1)."""
    q, r = divmod(global_batch, world)
    lo = rank * q + min(rank, r)
    return slice(lo, lo + q + (1 if rank < r else 0))


def _gather(t: torch.Tensor, group=None) -> torch.Tensor:
    world = dist.get_world_size(group)
    out = t.new_empty((world * t.shape[0],) + tuple(t.shape[1:]))
    if dist.get_backend(group) == "nccl":  # RCCL: one flat collective into the output
        dist.all_gather_into_tensor(out, t.contiguous(), group=group)
    else:  # gloo (CPU tests)
        dist.all_gather(list(out.chunk(world)), t.contiguous(), group=group)
    return out


def gather_detections(dets: torch.Tensor, counts: torch.Tensor, keep_rows: torch.Tensor | None = None,
                      group=None):
    """All-gather per-rank ``dets [n, max_det, 7]``, ``counts [n]`` (and
    optionally ``keep_rows [n, max_det]``). Every rank must pass the same n."""
    g_dets = _gather(dets, group)
    g_cnt = _gather(counts, group)
    g_keep = _gather(keep_rows, group) if keep_rows is not None else None
    return g_dets, g_cnt, g_keep


def to_output_list(dets: torch.Tensor, counts: torch.Tensor):
    """Padded device result -> the reference's ``output`` list: per image an
    ``np.float32 (K, 7)`` array, or None when nothing survived (detect.py:105,137)."""
    d = dets.detach().cpu().numpy()
    c = counts.detach().cpu().numpy()
    return [d[i, :int(c[i])].copy() if c[i] > 0 else None for i in range(d.shape[0])]
