"""Data-parallel inference across the GPUs of one node.

Images are independent (the reference loops per image, detect.py:105-106), so
each rank runs the whole hot path on its own contiguous shard of the batch and
the only collective is ONE all-gather of the fixed-size padded detections
(+ keep rows + counts) over RCCL/xGMI. Gathered rank-major = original image
order, which is the order of the reference's ``output`` list (detect.py:105).
"""
from __future__ import annotations

import warnings

import numpy as np
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


class OutputList(list):
    """The reference's ``output`` list (per image ``np.float32 (K, 7)`` or None)
    plus what the padded device result could not hold: ``counts`` = the
    survivors NMS found per image (the reference keeps all of them,
    detect.py:130-137), ``truncated`` = per image, True when counts > max_det
    and only the first max_det rows (class-ordered, score-descending within a
    class) are in the list."""

    def __init__(self, rows, counts, truncated):
        super().__init__(rows)
        self.counts = counts
        self.truncated = truncated

    @property
    def any_truncated(self):
        return bool(any(self.truncated))


def to_output_list(dets: torch.Tensor, counts: torch.Tensor, warn: bool = True):
    """Padded device result ``dets [n, max_det, 7]`` + uncapped ``counts [n]``
    -> the reference's ``output`` list (detect.py:105,137): per image
    ``min(count, max_det)`` rows, or None when nothing survived. Never a slice
    that disagrees silently with the count: the result carries the raw counts
    and a per-image ``truncated`` flag, and a warning names the images that
    lost rows (raise ``max_det`` to keep them all)."""
    d = dets.detach().cpu().numpy()
    c = counts.detach().cpu().numpy().astype(np.int64)
    max_det = d.shape[1]
    rows = [d[i, :min(int(c[i]), max_det)].copy() if c[i] > 0 else None for i in range(d.shape[0])]
    trunc = [bool(v > max_det) for v in c]
    if warn and any(trunc):
        lost = [(i, int(c[i])) for i, t in enumerate(trunc) if t]
        warnings.warn(f"ycx: max_det={max_det} truncated the detections of {len(lost)} image(s) "
                      f"(image, survivors): {lost[:8]}", RuntimeWarning, stacklevel=2)
    return OutputList(rows, c, trunc)
