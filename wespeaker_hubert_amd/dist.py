"""Multi-GPU plumbing for the extraction path (one process per GPU).

* `shard_bounds` / `shard_lines`: the contiguous data-list split of
  tools/extract_embedding.sh:40-42 (`split -l $((N/nj + 1))`), rank r takes
  lines [r*per, (r+1)*per) — concatenating the per-rank scps in rank order
  preserves input order.  No collective on the data path.
* `allreduce_sums`: the only collective of the north-star pipeline — the
  cohort / mean-vector statistics of AS-Norm (bin/score.py:25-35,
  tools/vector_mean.py:24-53) summed over ranks with torch.distributed
  (RCCL over xGMI for "nccl" on ROCm; gloo on CPU for tests).  Sums and
  counts travel in float64, so the result is independent of the shard split
  up to f64 rounding.
"""
from __future__ import annotations

import os
from typing import List, Sequence, Tuple

import torch


def world() -> Tuple[int, int]:
    if torch.distributed.is_available() and torch.distributed.is_initialized():
        return torch.distributed.get_rank(), torch.distributed.get_world_size()
    return int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1"))


def shard_bounds(n: int, rank: int, world_size: int) -> Tuple[int, int]:
    per = n // world_size + 1
    lo = min(n, rank * per)
    return lo, min(n, lo + per)


def shard_lines(lines: Sequence[str], rank: int, world_size: int) -> List[str]:
    lo, hi = shard_bounds(len(lines), rank, world_size)
    return list(lines[lo:hi])


def allreduce_sums(acc: torch.Tensor, cnt: torch.Tensor, force: bool = False) -> Tuple[torch.Tensor, torch.Tensor]:
    """In-place SUM all-reduce of per-group embedding sums [G, D] and counts [G]
    (one fused buffer -> one collective).  A world of one returns at once unless
    `force` (the hardware check of the RCCL path on a one-GPU box)."""
    if not (torch.distributed.is_available() and torch.distributed.is_initialized()):
        return acc, cnt
    if torch.distributed.get_world_size() == 1 and not force:
        return acc, cnt
    buf = torch.cat([acc.reshape(-1), cnt.reshape(-1)]).to(torch.float64)
    if torch.distributed.get_backend() == "gloo":  # gloo reduces host tensors (CPU tests, 1-GPU rehearsal)
        buf = buf.cpu()
    torch.distributed.all_reduce(buf, op=torch.distributed.ReduceOp.SUM)
    acc.copy_(buf[:acc.numel()].view_as(acc))
    cnt.copy_(buf[acc.numel():].view_as(cnt))
    return acc, cnt
