"""Benchmark: Msamples/s of the path-tracing hot path (BASELINE.json metric, config C3).

Workload (one "step"): generated_scene.json (484 quadrics + synthetic HDR sky) at 1920x1080,
1024 spp as the reference's headless loop renders it -- 128 render() calls of 8 spp
(main.cpp:272-279) -- executed as one chunked launch per GPU (bit-identical to 128 launches,
tests/test_gpu_parity.py).  Inputs are resident on the GPU before the timed region (scene, BVH,
sky texture, RNG state, accumulation buffer).

N GPUs (torchrun, one process per GPU, RCCL): the image rows are interleaved over the ranks
(row r -> rank r mod N), each rank renders its rows, and the HDR framebuffer is gathered to rank 0
over RCCL inside the timed region.  Default weak scaling: each GPU keeps one 1080p frame's worth of
pixels (the image grows by sqrt(N) per axis: 2720x1528, 3840x2160 (= C4), 5432x3056 at 1024 spp);
`--scaling strong` renders the same 1080p image for every N.  A pixel's samples are one serial
XORWOW stream, so strong scaling of a 1080p frame is bounded by its most expensive 8x8 tile
(DESIGN.md "Multi-GPU"; tools/scale_sim.py).

Printed JSON line (rank 0): value = samples of the whole image / step time; roofline = the trace
kernel's algorithmic bytes (counted node/prim/material/sky reads + per-pixel
state traffic, measured with the instrumented kernel on this workload) / its HIP-event time vs
8.0 TB/s HBM; cpu_baseline = the oracle (CPU restatement) on a bounded sample of this workload.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import pathlib
import sys
import time

ROOT = pathlib.Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

HBM_PEAK_GBS = 8000.0      # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
NODE_B, PRIM_B, MAT_B, SKY_B = 32, 96, 40, 64            # SURVEY.md §8(d) per-event bytes
PIXEL_STATE_B = 16 + 16 + 24 + 24                          # accum RMW + XORWOW state RMW, per pixel per launch


def parse_args():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=3)
    p.add_argument("--warmup", type=int, default=1)
    p.add_argument("--scene", default=str(ROOT / "scenes" / "generated_scene.scene.json"))
    p.add_argument("--width", type=int, default=1920)
    p.add_argument("--height", type=int, default=1080)
    p.add_argument("--spp", type=int, default=1024)
    p.add_argument("--chunk", type=int, default=8)
    p.add_argument("--cpu-baseline", type=int, default=1, help="time the oracle on a bounded sample (rank 0, N=1)")
    p.add_argument("--scaling", choices=["weak", "strong"], default="weak",
                   help="weak: per-GPU work fixed (image grows with N); strong: the same 1080p image for every N")
    p.add_argument("--cpu-threads", type=int, default=0)
    p.add_argument("--cpu-spp", type=int, default=192)
    return p.parse_args()


def algorithmic_bytes(stats: dict, pixels: int, launches: int) -> float:
    return (NODE_B * stats["node_tests"] + PRIM_B * stats["prim_tests"] + MAT_B * stats["hits"]
            + SKY_B * stats["sky_lookups"] + PIXEL_STATE_B * pixels * launches)


def load_pmc_traffic(workload: str):
    """Per-launch HBM bytes of the trace kernel from the committed rocprofv3 --pmc summary, and the
    issue utilisation of the same launch over shader-active cycles (GRBM_GUI_ACTIVE summed over the
    8 XCDs): VALU = wave64 VALU instructions x 2 cycles (CDNA4 SIMD-32 throughput,
    MI355X_MICROARCH.md cycle table) over 1024 SIMDs; SALU = scalar instructions per CU-cycle (one
    scalar unit per CU, shared by its 4 SIMDs)."""
    for f in sorted((ROOT / "profiles").glob("*pmc_traffic*.json"), reverse=True):
        try:
            d = json.loads(f.read_text())
        except (OSError, ValueError):
            continue
        if d.get("workload") == workload and d.get("bytes_per_launch"):
            c = d.get("counters", {})
            util = {}
            cyc = c.get("GRBM_GUI_ACTIVE", 0) / 8.0
            if cyc and c.get("SQ_INSTS_VALU"):
                util["valu_util"] = round(2.0 * c["SQ_INSTS_VALU"] / (1024.0 * cyc), 3)
            if cyc and c.get("SQ_INSTS_SALU"):
                util["salu_per_cu_cycle"] = round(c["SQ_INSTS_SALU"] / (256.0 * cyc), 3)
            return float(d["bytes_per_launch"]), f.name, util
    return None, None, {}


def cpu_baseline(args, W, H):
    """Oracle (plain-C restatement, pthreads) on a bounded sample of the same workload."""
    from oracle import pyoracle as po
    threads = args.cpu_threads or min(16, len(os.sched_getaffinity(0)))
    stride = 1                     # the full 1080p frame, fewer samples per pixel (~10 s of CPU work)
    sc = po.load_scene(args.scene, W, H)
    r = po.OracleRenderer(sc, W, H, 0, stride, threads=threads)
    spp = min(args.chunk, args.cpu_spp)
    chunks = max(1, args.cpu_spp // spp)
    t0 = time.perf_counter()
    r.render(sc.camera, spp, True, chunks=chunks)
    dt = time.perf_counter() - t0
    samples = r.rows * W * spp * chunks
    return {"value": round(samples / dt / 1e6, 3), "unit": "Msamples/s", "cores": threads, "kind": "port",
            "sample": f"{W}x{H} rows 0::{stride} ({r.rows} rows) x {spp * chunks} spp = {samples} samples, "
                      f"{dt:.1f} s on {threads} threads"}


def main():
    args = parse_args()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world == 1 and args.gpus > 1:
        print(f"bench.py: --gpus {args.gpus} needs one process per GPU (torch.distributed.run "
              f"--nproc-per-node {args.gpus}); running on 1 GPU", file=sys.stderr)
    n = max(1, world)
    W, H, spp, chunk = args.width, args.height, args.spp, args.chunk
    if args.scaling == "weak" and n > 1:
        # weak scaling: every GPU keeps one 1080p frame's worth of pixels; the image grows by
        # sqrt(N) per axis (N = 4 is 3840x2160, the C4 resolution), rows interleaved over ranks
        W = int(round(W * math.sqrt(n) / 8.0)) * 8
        H = int(round(H * math.sqrt(n) / 8.0)) * 8
    chunks = spp // chunk
    assert chunks * chunk == spp, "spp must be a multiple of --chunk"

    import torch
    import torch.distributed as dist
    import pathtracercuda_amd as pa

    dist_on = world > 1
    if dist_on:
        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
    device = local_rank
    pt = pa.Pathtracer(W, H, device=device, row_offset=rank if dist_on else 0, row_stride=n if dist_on else 1)
    cam = pt.load_scene(args.scene)
    rows_max = (H + n - 1) // n
    if dist_on:
        send = torch.zeros((rows_max, W, 4), dtype=torch.float32, device=f"cuda:{local_rank}")
        recv = [torch.zeros_like(send) for _ in range(n)] if rank == 0 else None
        full = torch.empty((H, W, 4), dtype=torch.float32, device=f"cuda:{local_rank}") if rank == 0 else None

    from pathtracercuda_amd.distributed import gather_framebuffer

    def gather():
        # RCCL framebuffer gather over xGMI + unpermute of the interleaved rows on rank 0
        pt.copy_accum_to_device(send.data_ptr(), send.numel() * 4)
        gather_framebuffer(send, H, rank, n, recv=recv, full=full)

    def step():
        ms = pt.render_raw(cam, chunk, chunks, True)
        if dist_on:
            gather()
        return ms

    def barrier_sync():
        torch.cuda.synchronize(device)
        if dist_on:
            dist.barrier()

    # instrumented run (not timed): algorithmic byte count of this workload, 1 chunk.  Counted
    # with the non-speculative child-box kernel, whose node/primitive tests are the reference's
    # (the speculative variant adds node tests of its own); then back to automatic selection.
    pt.set_kernel_variant(20)
    stats = pt.render_instrumented(cam, chunk, 1, True)
    pt.set_kernel_variant(0)    # (that launch also recorded the tile costs: every timed launch is cost-ordered)
    samples_per_chunk = stats["samples"]
    for _ in range(args.warmup):
        step()
    barrier_sync()
    t0 = time.perf_counter()
    kernel_ms = 0.0
    for _ in range(args.steps):
        kernel_ms += step()
    barrier_sync()
    elapsed = time.perf_counter() - t0
    if dist_on:
        t = torch.tensor([elapsed, kernel_ms], dtype=torch.float64, device=f"cuda:{local_rank}")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, kernel_ms = float(t[0]), float(t[1])
        st = torch.tensor([stats[k] for k in ("node_tests", "prim_tests", "hits", "sky_lookups", "samples")],
                          dtype=torch.float64, device=f"cuda:{local_rank}")
        dist.all_reduce(st)
        stats = dict(zip(("node_tests", "prim_tests", "hits", "sky_lookups", "samples"), [float(x) for x in st]))
        samples_per_chunk = stats["samples"]

    total_samples = W * H * spp * args.steps
    ms_per_step = elapsed * 1e3 / args.steps
    value = total_samples / elapsed / 1e6
    # roofline of the trace kernel: algorithmic bytes of one launch (= one step per GPU)
    launch_bytes = algorithmic_bytes(stats, 0, 0) * chunks + PIXEL_STATE_B * W * H   # whole image per step
    per_gpu_bytes = launch_bytes / n
    avg_launch_s = kernel_ms / args.steps / 1e3
    achieved = per_gpu_bytes / avg_launch_s / 1e9
    workload = f"generated_scene {W}x{H} {spp}spp chunk{chunk}"
    traffic, traffic_src, util = load_pmc_traffic(workload)
    out = {
        "metric": "Msamples/sec + achieved HBM GB/s, 1080p 1024spp, 1/2/4/8 MI355X",
        "value": round(value, 3),
        "unit": "Msamples/s",
        "n_gpus": n,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 3),
        "higher_is_better": True,
        "scaling": args.scaling,
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic sky (scenes/skybox.hdr), reference scene generated_scene.json",
        "config": {"workload": workload, "scene": "generated_scene.json (484 quadrics)", "width": W, "height": H,
                   "spp": spp, "render_calls_per_step": chunks, "parallelism": f"rows interleaved x{n}, RCCL gather",
                   "per_gpu_pixels": (W * H + n - 1) // n},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                     "kernel": "trace_kernel", "avg_launch_ms": round(avg_launch_s * 1e3, 3),
                     "bytes_per_sample": round(launch_bytes / (W * H * spp), 1),
                     "traffic_source": traffic_src,
                     # the algorithmic bytes are served from LDS and L2 (traffic = HBM bytes measured);
                     # the kernel is issue/latency-bound: VALU and scalar-unit use from the same profile
                     "hbm_frac_measured": (round(traffic / avg_launch_s / 1e9 / HBM_PEAK_GBS, 5) if traffic else None),
                     **util},
        "cpu_baseline": None,
    }
    if rank == 0 and n == 1 and args.cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(args, W, H)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist_on:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
