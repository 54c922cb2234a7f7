"""Multi-GPU framebuffer tiling and gather.

Rows are interleaved over the ranks (row y -> rank y mod N) so cheap sky rows and expensive
ground rows spread evenly; RNG seeds depend only on the global pixel index (initRandState.cu:16),
so any tiling reproduces the single-GPU image bit for bit.  After rendering, each rank's rows are
gathered to rank 0 with one collective (RCCL over xGMI with the "nccl" backend, or gloo on CPU)
and un-interleaved there.  No other data-path communication exists.
"""
from __future__ import annotations


def rows_of(height: int, rank: int, world: int) -> int:
    return (height - rank + world - 1) // world if rank < height else 0


def max_rows(height: int, world: int) -> int:
    return (height + world - 1) // world


def gather_framebuffer(local, height: int, rank: int, world: int, recv=None, full=None):
    """Gather the (max_rows, W, 4) per-rank buffers to rank 0 and un-interleave into (H, W, 4).

    `local` holds this rank's rows in its first rows_of(height, rank, world) rows.  Returns the
    full image on rank 0 (None elsewhere).  `recv` / `full` may be preallocated.
    """
    import torch
    import torch.distributed as dist

    if rank == 0:
        if recv is None:
            recv = [torch.empty_like(local) for _ in range(world)]
        dist.gather(local, recv, dst=0)
        if full is None:
            full = torch.empty((height,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
        for r in range(world):
            full[r::world] = recv[r][: rows_of(height, r, world)]
        return full
    dist.gather(local, None, dst=0)
    return None
