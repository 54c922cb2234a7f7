"""Multi-GPU tiling + framebuffer gather on CPU with the gloo backend.

Each rank renders its row bands (band b of band_rows rows -> rank b mod N) with the oracle (standing in for a
GPU here; the GPU tile path is covered bit-exactly by test_gpu_parity.py::test_row_tiles_*), pads
to the common row count, and pathtracercuda_amd.distributed.gather_framebuffer assembles the image
on rank 0 -- the same function bench.py runs over RCCL.  The result must equal the single-device
render bit for bit.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import pyoracle as po
from pathtracercuda_amd.distributed import gather_framebuffer, global_rows, max_rows, rows_of


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, scene, W, H, band, out_path):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        sc = po.load_scene(scene, W, H)
        r = po.OracleRenderer(sc, W, H, rank, world, threads=1, band_rows=band)
        r.render(sc.camera, 2, True, chunks=2)
        assert r.rows == rows_of(H, rank, world, band)
        local = torch.zeros((max_rows(H, world, band), W, 4), dtype=torch.float32)
        local[: r.rows] = torch.from_numpy(r.accum)
        full = gather_framebuffer(local, H, rank, world, band_rows=band)
        if rank == 0:
            np.save(out_path, full.numpy())
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,H,band", [(2, 24, 1), (2, 23, 1), (3, 17, 1), (2, 37, 8), (3, 41, 8), (2, 9, 8)])
def test_gather_band_tiles_bitexact(tmp_path, scenes, world, H, band):
    W = 20
    scene = scenes / "cornell_box.scene.json"
    out = tmp_path / "full.npy"
    mp.spawn(_worker, args=(world, _free_port(), scene, W, H, band, str(out)), nprocs=world, join=True)
    full = np.load(out)
    sc = po.load_scene(scene, W, H)
    ref = po.OracleRenderer(sc, W, H, threads=1)
    ref.render(sc.camera, 2, True, chunks=2)
    assert np.array_equal(full.view(np.uint32), ref.accum.view(np.uint32))


@pytest.mark.parametrize("band", [1, 2, 8, 16])
def test_band_partition_covers_image_once(band):
    # every image row belongs to exactly one rank; the Python partition, the native one
    # (pt_band_rows, libpt_hip.so) and the oracle's (or_view_rows) agree
    from pathtracercuda_amd import _native as N
    for H in (1, 7, 8, 9, 64, 1080, 1528, 2160, 3056):
        for world in (1, 2, 3, 8):
            seen = []
            for r in range(world):
                g = global_rows(H, r, world, band)
                assert len(g) == rows_of(H, r, world, band)
                assert int(N.hip().pt_band_rows(H, band, r, world)) == len(g)
                assert po.rows_of(H, r, world, band) == len(g)
                seen += g
            assert sorted(seen) == list(range(H))
