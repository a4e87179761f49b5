"""Multi-GPU frame tiling: one process per GPU, interleaved 8-row strips
(strip s -> rank s mod N), one gather to rank 0 over RCCL (torch.distributed "nccl" backend), then
the un-interleave on rank 0 (rt_assemble_strips on the GPU; assemble_host is its host twin for
CPU tests). Every rank holds the full scene and builds the same LBVH, so nothing but the finished
strips crosses xGMI: ~8.3 MB per 1080p frame (33 MB at 4K) into the root.
"""
from __future__ import annotations

from typing import List, Optional

import numpy as np

from . import strip_rows, strip_rows_per_rank

STRIP_ROWS = 8


def rank_rows(height: int, world: int, rank: int, strip: int = STRIP_ROWS) -> np.ndarray:
    """Global rows rank `rank` renders, in output order (its compact buffer's row order)."""
    return strip_rows(height, world, rank, strip)


def padded_rows(height: int, world: int, strip: int = STRIP_ROWS) -> int:
    """Rows of every rank's send buffer: the gather needs equal-sized pieces."""
    return strip_rows_per_rank(height, world, strip)


def gather_parts(gathered, world: int, rank: int, dst: int = 0) -> Optional[List]:
    """The per-rank views of `gathered` dist.gather fills on dst (None elsewhere); built once per
    buffer, not per frame (each view costs a Python call on the frame loop's critical path)."""
    return [gathered[r] for r in range(world)] if rank == dst else None


def gather_strips(local, world: int, rank: int, gathered: Optional[object] = None, dst: int = 0,
                  parts: Optional[List] = None):
    """dist.gather of the per-rank compact buffers into `gathered` (world x rows x W x 4) on dst."""
    import torch.distributed as dist

    if parts is None and rank == dst:
        parts = gather_parts(gathered, world, rank, dst)
    dist.gather(local, parts if rank == dst else None, dst=dst)
    return gathered if rank == dst else None


def assemble_host(gathered: np.ndarray, height: int, world: int, strip: int = STRIP_ROWS) -> np.ndarray:
    """Host twin of rt_assemble_strips: rank-major padded strips -> H x W x C frame."""
    out = np.empty((height,) + gathered.shape[2:], gathered.dtype)
    for y in range(height):
        s, within = divmod(y, strip)
        rank, local_strip = s % world, s // world
        out[y] = gathered[rank, local_strip * strip + within]
    return out
