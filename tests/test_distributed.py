"""Multi-GPU tiling + framebuffer gather on CPU with the gloo backend.

Each rank renders its interleaved rows (row y -> rank y mod N) with the oracle (standing in for a
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
from pathtracercuda_amd.distributed import gather_framebuffer, max_rows, rows_of


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, scene, W, H, out_path):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        sc = po.load_scene(scene, W, H)
        r = po.OracleRenderer(sc, W, H, rank, world, threads=1)
        r.render(sc.camera, 2, True, chunks=2)
        assert r.rows == rows_of(H, rank, world)
        local = torch.zeros((max_rows(H, world), W, 4), dtype=torch.float32)
        local[: r.rows] = torch.from_numpy(r.accum)
        full = gather_framebuffer(local, H, rank, world)
        if rank == 0:
            np.save(out_path, full.numpy())
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,H", [(2, 24), (2, 23), (3, 17)])
def test_gather_interleaved_tiles_bitexact(tmp_path, scenes, world, H):
    W = 20
    scene = scenes / "cornell_box.scene.json"
    out = tmp_path / "full.npy"
    mp.spawn(_worker, args=(world, _free_port(), scene, W, H, str(out)), nprocs=world, join=True)
    full = np.load(out)
    sc = po.load_scene(scene, W, H)
    ref = po.OracleRenderer(sc, W, H, threads=1)
    ref.render(sc.camera, 2, True, chunks=2)
    assert np.array_equal(full.view(np.uint32), ref.accum.view(np.uint32))
