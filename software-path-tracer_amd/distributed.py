"""Multi-GPU plumbing for the row-sharded integrator.

One process per GPU (torch.distributed; backend "nccl" = RCCL over xGMI on the GPU box, "gloo" in the
CPU tests). Rows are dealt round-robin: row y belongs to rank y % world, so cheap sky rows and costly
box rows spread evenly and every pixel's samples stay on one rank (bit-identical to one GPU). The only
exchange is a single gather of the per-rank float RGBA accumulation shards to rank 0, each padded to
ceil(H / world) rows so the collective moves equal-sized buffers, followed by a device-side
de-interleave (spt_assemble_rows) on the root.
"""
from __future__ import annotations

from typing import List, Optional

import numpy as np


def rows_of(height: int, rank: int, world: int) -> List[int]:
    return list(range(rank, height, world))


def rows_max(height: int, world: int) -> int:
    return (height + world - 1) // world


def gather_to_root(send, world: int, rank: int):
    """torch.distributed.gather of equal-sized shard tensors to rank 0; returns the list on rank 0."""
    import torch.distributed as dist

    gather_list = [send.new_empty(send.shape) for _ in range(world)] if rank == 0 else None
    dist.gather(send, gather_list, dst=0)
    return gather_list


def pad_shard(accum_rows: np.ndarray, height: int, world: int) -> np.ndarray:
    """(n_rows, W, 4) shard -> flat float32 of rows_max * W * 4 (zero padded)."""
    n_rows, w, _ = accum_rows.shape
    out = np.zeros((rows_max(height, world), w, 4), np.float32)
    out[:n_rows] = accum_rows
    return out.reshape(-1)


def assemble_rows_host(gathered: np.ndarray, width: int, height: int, world: int) -> np.ndarray:
    """Host restatement of k_assemble_rows: out[y] = shard[y % world][y // world]."""
    g = np.asarray(gathered, np.float32).reshape(world, rows_max(height, world), width, 4)
    out = np.empty((height, width, 4), np.float32)
    for y in range(height):
        out[y] = g[y % world, y // world]
    return out
