"""Multi-GPU framebuffer tiling and gather across processes (bench.py --gpus N).

The image is cut into bands of `band_rows` rows and band b goes to rank b mod N, so cheap sky
bands and expensive ground bands spread evenly over the ranks, and with band_rows = 8 every 8x8
tile a rank renders is a spatially coherent 8x8 tile of the image (with band_rows = 1 -- plain row
interleaving -- a rank's 8x8 tile spans 8N image rows and its primary rays lose their coherence).
RNG seeds depend only on the global pixel index (initRandState.cu:16), so every tiling reproduces
the single-GPU image bit for bit.  After rendering, each rank's rows are gathered to rank 0 with one
collective (RCCL over xGMI with the "nccl" backend, or gloo on CPU) and scattered into the image
there.  No other data-path communication exists.  The same partition runs in one process over
several devices in the native layer (pt_group_*, include/pt_hip.h).
"""
from __future__ import annotations

DEFAULT_BAND_ROWS = 8


def rows_of(height: int, rank: int, world: int, band_rows: int = 1) -> int:
    """Local rows of `rank` (= pt_band_rows of the native layer)."""
    rows = 0
    b = rank
    while b * band_rows < height:
        rows += min(band_rows, height - b * band_rows)
        b += world
    return rows


def max_rows(height: int, world: int, band_rows: int = 1) -> int:
    return max(rows_of(height, r, world, band_rows) for r in range(world))


def global_rows(height: int, rank: int, world: int, band_rows: int = 1):
    """Image row of each local row of `rank`, in local order."""
    out = []
    b = rank
    while b * band_rows < height:
        out.extend(range(b * band_rows, min((b + 1) * band_rows, height)))
        b += world
    return out


def gather_framebuffer(local, height: int, rank: int, world: int, recv=None, full=None, band_rows: int = 1,
                       index=None):
    """Gather the (max_rows, W, 4) per-rank buffers to rank 0 and scatter them into (H, W, 4).

    `local` holds this rank's rows in its first rows_of(height, rank, world, band_rows) rows.
    Returns the full image on rank 0 (None elsewhere).  `recv`, `full` and `index` (per-rank
    LongTensors of global_rows on local's device) may be preallocated.
    """
    import torch
    import torch.distributed as dist

    if rank == 0:
        if recv is None:
            recv = [torch.empty_like(local) for _ in range(world)]
        dist.gather(local, recv, dst=0)
        if full is None:
            full = torch.empty((height,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
        native = (local.device.type == "cuda" and local.dtype == torch.float32 and local.dim() == 3
                  and int(local.shape[-1]) == 4 and full.dtype == torch.float32 and full.is_contiguous()
                  and all(t.is_contiguous() and t.dtype == torch.float32 for t in recv))
        if native:
            # on the GPU the scatter is the native unpermute kernel -- the same one pt_group_gather
            # runs after its RCCL gather -- so both multi-GPU front ends assemble the image identically.
            # It moves float4 rows, so only a contiguous (rows, W, 4) float32 framebuffer takes it;
            # anything else takes the index copy below.
            from . import _native as N
            width = int(local.shape[1])
            for r in range(world):
                rc = N.hip().pt_unpermute_bands(int(local.device.index or 0), full.data_ptr(), recv[r].data_ptr(), width,
                                                int(height), int(band_rows), r, int(world))
                if rc != 0:
                    raise RuntimeError(f"pt_unpermute_bands failed ({rc})")
            return full
        # CPU tensors (the gloo tests) and other layouts: the same row map (global_rows), as a torch index copy
        for r in range(world):
            idx = index[r] if index is not None else torch.tensor(global_rows(height, r, world, band_rows),
                                                                  dtype=torch.long, device=local.device)
            full.index_copy_(0, idx, recv[r][: idx.numel()])
        return full
    dist.gather(local, None, dst=0)
    return None
