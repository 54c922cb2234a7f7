"""Benchmark: Msamples/s of the path-tracing hot path (BASELINE.json metric).

Workloads (SURVEY.md §8 config labels; one "step" = one pass of the hot path over the workload):
  C3 (default)  generated_scene.json (484 quadrics + synthetic HDR sky), 1920x1080, 1024 spp
  C2            cornell_box.json, 512x512, 64 spp
  C4            generated_scene.json, 3840x2160, 4096 spp
  C5            100,490 random quadrics (tools/make_stress_scene.py, seeded), 1920x1080, 4096 spp
Every workload runs as the reference's headless loop renders it -- render() calls of 8 spp
(main.cpp:272-279) -- executed as one chunked launch per GPU (bit-identical to the call loop,
tests/test_gpu_parity.py).  Inputs are resident on the GPU before the timed region (scene, BVH,
sky texture, RNG state, accumulation buffer).

N GPUs, two launch modes, one partition (8-row bands, band b -> GPU b mod N):
  * torch.distributed.run (WORLD_SIZE > 1, one process per GPU, RCCL): each rank renders its bands
    and the HDR framebuffer is gathered to rank 0 over RCCL inside the timed region
    (pathtracercuda_amd/distributed.py);
  * `python bench.py --gpus N` without a launcher: the product's in-process multi-device Pathtracer
    (pt_group_*: one context and host thread per GPU, ncclCommInitAll, grouped ncclSend/ncclRecv +
    unpermute kernel -- the boundary that replaces Pathtracer.cpp:40's single device); the timed
    step is pt_group_render + pt_group_gather.  Fewer than N visible GPUs is an error (exit 2);
    `--group 1` runs this path at N = 1 too.
Scaling.  The headline is the metric's own workload at every N: strong scaling of the fixed
1920x1080 x 1024 spp image (BASELINE.json metric "1080p 1024spp, 1/2/4/8 MI355X"), value = all
samples / the slowest rank's step time.  At N > 1 a weak-scaling record is added beside it
(`secondary`: every GPU keeps one C3 frame's worth of pixels, the image grows by sqrt(N) per axis),
so both are on the driver's clock; `--scaling weak` swaps them.  Also at N > 1: C2, C4 (the 4K x
4096 image BASELINE tiles across 8 GPUs) and C5 on the same N GPUs, strong scaling each
(`--configs-n 0` drops them).  At N = 1 the two coincide, and the
secondary records are the reference's unchanged call loop on C3 (128 separate render(cam, 8, i == 0)
calls through the drop-in Pathtracer, main.cpp:272-279), a cold one-shot C3 render (fresh context,
cost pre-pass included), C2 and C5, each C2/C5 with its roofline and CPU baseline (`--extra ''` drops
C5, `--secondary 0` turns all secondary records off).

Printed JSON line (rank 0): value = samples of the whole workload / step time.  roofline: the
trace kernel is bound by VALU issue -- achieved = its wave64 VALU instructions per
launch (rocprofv3 PMC profile of the same workload, profiles/) / its live HIP-event launch time,
peak = 1,024 SIMD-32 x 2.4 GHz / 2 cycles per wave64 instruction; traffic = measured HBM bytes per
launch (same profile); the SURVEY §8(d) algorithmic bytes (served from LDS/L1/L2, not HBM) are
reported as lds_l2_effective_GBs.  cpu_baseline = the oracle (CPU restatement, -O3) on every
allowed core of this host, on a time-bounded sample of the same workload.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import pathlib
import platform
import sys
import tempfile
import time

ROOT = pathlib.Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

METRIC = "Msamples/sec + achieved HBM GB/s, 1080p 1024spp, 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0                 # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
SIMDS, CLOCK_HZ = 1024, 2.4e9         # 256 CUs x 4 SIMD-32; max engine clock (MI355X_MICROARCH.md)
VALU_PEAK_G = SIMDS * CLOCK_HZ / 2 / 1e9   # wave64 VALU instructions per second: 2 cycles each on SIMD-32
NODE_B, PRIM_B, MAT_B, SKY_B = 32, 96, 40, 64            # SURVEY.md §8(d) per-event bytes
PIXEL_STATE_B = 16 + 16 + 24 + 24                          # accum RMW + XORWOW state RMW, per pixel per launch
CHUNK = 8                                                  # spp per render() call (main.cpp:272)

CONFIGS = {
    "C2": {"scene": "cornell_box", "width": 512, "height": 512, "spp": 64},
    "C3": {"scene": "generated_scene", "width": 1920, "height": 1080, "spp": 1024},
    "C4": {"scene": "generated_scene", "width": 3840, "height": 2160, "spp": 4096},
    "C5": {"scene": "stress_100k", "width": 1920, "height": 1080, "spp": 4096},
}


def parse_args(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=3)
    p.add_argument("--warmup", type=int, default=1)
    p.add_argument("--config", choices=sorted(CONFIGS), default="C3")
    p.add_argument("--spp", type=int, default=0, help="override the config's spp (multiple of 8)")
    p.add_argument("--scaling", choices=["weak", "strong"], default="strong",
                   help="strong (default): the same 1080p workload for every N; weak: the image grows by sqrt(N) per axis")
    p.add_argument("--band-rows", type=int, default=8, help="rows per band of the multi-GPU partition")
    p.add_argument("--secondary", type=int, default=1,
                   help="N=1: add the C2 and --extra records; N>1: add the other scaling mode's record")
    p.add_argument("--cpu-baseline", type=int, default=1, help="time the oracle on a bounded sample (rank 0, N=1)")
    p.add_argument("--cpu-seconds", type=float, default=15.0, help="target length of the CPU baseline run")
    p.add_argument("--cpu-threads", type=int, default=0, help="0 = every core this process may use")
    p.add_argument("--call-loop", type=int, default=1,
                   help="N=1, C3: also time the reference's unchanged 128-call loop (secondary record)")
    p.add_argument("--cold", type=int, default=1,
                   help="N=1, C3: also time a cold one-shot render (fresh context, pre-pass included; secondary record)")
    p.add_argument("--configs-n", type=int, default=1,
                   help="N>1: also time C2, C4 and C5 on the N GPUs (strong scaling; secondary records); 2: at N=1 too (test)")
    p.add_argument("--extra", default="C5", help="N=1: secondary records after C2 (comma-separated labels; '' = none)")
    p.add_argument("--group", type=int, default=-1,
                   help="in-process device group (pt_group_*): 1 = always, 0 = never, -1 = when --gpus > 1 "
                        "without a launcher")
    return p.parse_args(argv)


def resolve_mode(gpus: int, world: int, group: int, visible) -> str:
    """Which path times the step: "torchrun" (one process per GPU, WORLD_SIZE > 1), "group" (this
    process drives --gpus devices through pt_group_*), or "single".  `visible` is a callable giving
    the number of visible GPUs (queried only for the group path).  Never silently runs fewer GPUs
    than asked: a mismatch raises SystemExit(2) with the reason."""
    if gpus < 1:
        print("bench.py: --gpus must be >= 1", file=sys.stderr)
        raise SystemExit(2)
    if world > 1:
        if gpus not in (1, world):
            print(f"bench.py: --gpus {gpus} but WORLD_SIZE={world}", file=sys.stderr)
            raise SystemExit(2)
        return "torchrun"
    if group == 0 and gpus > 1:
        print(f"bench.py: --gpus {gpus} with --group 0 needs one process per GPU (torch.distributed.run "
              f"--nproc-per-node {gpus})", file=sys.stderr)
        raise SystemExit(2)
    if gpus > 1 or group == 1:
        n = int(visible())
        if n < gpus:
            print(f"bench.py: --gpus {gpus} but only {n} GPU(s) are visible", file=sys.stderr)
            raise SystemExit(2)
        return "group"
    return "single"


def scene_path(name: str) -> str:
    if name == "stress_100k":
        p = pathlib.Path(tempfile.gettempdir()) / "pt_stress_100k.json"
        if not p.exists():
            import importlib.util
            spec = importlib.util.spec_from_file_location("mss", ROOT / "tools" / "make_stress_scene.py")
            mod = importlib.util.module_from_spec(spec)
            spec.loader.exec_module(mod)
            # every rank of a multi-GPU run may write it: each writes its own file and renames it
            tmp = p.with_name(f"{p.name}.{os.getpid()}.tmp")
            mod.write_scene(tmp, grid=317, skybox=str(ROOT / "scenes" / "skybox.hdr"))
            os.replace(tmp, p)
        return str(p)
    return str(ROOT / "scenes" / f"{name}.scene.json")


def workload_name(cfg: dict, W: int, H: int, spp: int) -> str:
    return f"{cfg['scene']} {W}x{H} {spp}spp chunk{CHUNK}"


def algorithmic_bytes(stats: dict) -> float:
    return (NODE_B * stats["node_tests"] + PRIM_B * stats["prim_tests"] + MAT_B * stats["hits"]
            + SKY_B * stats["sky_lookups"])


def kernel_source_sha() -> str:
    """sha256 (16 hex) of what the trace kernel is built from -- its sources, the headers under
    include/ and the hipcc flags of the Makefile (HIPFLAGS; e.g. -fno-slp-vectorize moved C3 by
    4.6 %): a committed PMC profile records the same digest, so a profile of another binary cannot
    pair with this build unnoticed."""
    import hashlib
    import re
    h = hashlib.sha256()
    src = ROOT / "pathtracercuda_amd" / "csrc"      # (a build snapshot for A/Bs holds no sources)
    for f in [src / "pt_kernels.hip"] + sorted(src.glob("*.h")):
        if f.exists():
            h.update(f.read_bytes())
    for f in sorted((ROOT / "include").glob("*.h")):
        h.update(f.read_bytes())
    mk = (ROOT / "Makefile").read_text() if (ROOT / "Makefile").exists() else ""
    m = re.search(r"^HIPFLAGS \?=(.*?)(?<!\\)\n", mk, re.S | re.M)
    h.update((m.group(1) if m else "").encode())
    return h.hexdigest()[:16]


def load_profile(workload: str):
    """Per-launch counters of the trace kernel from the newest committed rocprofv3 --pmc summary of
    this workload (profiles/*pmc_traffic*.json): HBM bytes (FETCH_SIZE x2 + WRITE_SIZE, gfx950
    correction), wave64 VALU and scalar instructions, shader-active cycles (GRBM_GUI_ACTIVE summed
    over the 8 XCDs)."""
    for f in sorted((ROOT / "profiles").glob("*pmc_traffic*.json"), reverse=True):
        try:
            d = json.loads(f.read_text())
        except (OSError, ValueError):
            continue
        if d.get("workload") == workload and d.get("bytes_per_launch"):
            return d, f.name
    return None, None


def cpu_info():
    model = platform.processor() or ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            quota = float(q) / float(per)
    except (OSError, ValueError):
        pass
    return model, quota


def cpu_baseline(args, cfg, W, H):
    """The oracle (plain-C restatement of the reference's trace(), -O3 timing build, pthreads with
    dynamic row scheduling) on every core this process may use, over the full image at a reduced
    spp chosen from a pilot run so the run lasts about --cpu-seconds."""
    from oracle import pyoracle as po
    affinity = len(os.sched_getaffinity(0))
    model, quota = cpu_info()
    # every core this process may use: the affinity mask, capped by the cgroup's CPU quota (on the
    # GPU hosts 256 logical CPUs are visible but the job's cgroup grants 16 -- more threads than
    # that only time-slice the same 16 CPUs; measured 36 Msamples/s at 256 threads vs ~50 at 16)
    threads = args.cpu_threads or (min(affinity, max(1, int(math.ceil(quota)))) if quota else affinity)
    sc = po.load_scene(scene_path(cfg["scene"]), W, H)
    pilot = po.OracleRenderer(sc, W, H, 0, max(1, H // (4 * threads)), threads=threads, fast=True)
    t0 = time.perf_counter()
    pilot.render(sc.camera, CHUNK, True, chunks=1)
    rate = pilot.rows * W * CHUNK / max(time.perf_counter() - t0, 1e-6)
    chunks = max(1, min(cfg["spp"] // CHUNK, int(args.cpu_seconds * rate / (W * H * CHUNK))))
    r = po.OracleRenderer(sc, W, H, threads=threads, fast=True)
    t0 = time.perf_counter()
    r.render(sc.camera, CHUNK, True, chunks=chunks)
    dt = time.perf_counter() - t0
    samples = W * H * CHUNK * chunks
    return {"value": round(samples / dt / 1e6, 3), "unit": "Msamples/s", "cores": threads, "kind": "port",
            "sample": f"{cfg['scene']} {W}x{H} x {CHUNK * chunks} spp (of {cfg['spp']}) = {samples} samples, "
                      f"{dt:.1f} s on {threads} threads",
            "per_core": round(samples / dt / 1e6 / threads, 3),
            "cpu_model": model, "host_logical_cpus": os.cpu_count(), "affinity_cpus": affinity, "cgroup_cpu_limit": quota,
            "build": "oracle/liboracle_fast.so: gcc -O3 -march=x86-64-v3 -ffp-contract=off (bit-identical to the checker)"}


class Run:
    """One workload on this rank: the renderer (one context, or the in-process device group), the
    camera, the gather buffers of the torchrun path."""

    def __init__(self, cfg, W, H, spp, rank, n, local_rank, band_rows, mode):
        import pathtracercuda_amd as pa
        from pathtracercuda_amd.distributed import global_rows, max_rows

        self.cfg, self.W, self.H, self.spp = cfg, W, H, spp
        self.rank, self.n, self.mode = rank, n, mode
        self.dist_on = mode == "torchrun"
        self.chunks = spp // CHUNK
        assert self.chunks * CHUNK == spp, "spp must be a multiple of 8"
        self.band_rows = band_rows if mode != "single" else 1
        self.gather_ms = 0.0
        if mode == "group":
            # the product's multi-device Pathtracer: one context per GPU, RCCL communicators from
            # ncclCommInitAll.  RCCL prints its version banner on stdout; it goes to stderr here so
            # that stdout carries only the JSON line
            sys.stdout.flush()
            saved = os.dup(1)
            os.dup2(2, 1)
            try:
                self.pt = pa.Pathtracer(W, H, devices=list(range(n)), band_rows=self.band_rows)
            finally:
                os.dup2(saved, 1)
                os.close(saved)
        else:
            self.pt = pa.Pathtracer(W, H, device=local_rank, row_offset=rank if self.dist_on else 0,
                                    row_stride=n if self.dist_on else 1, band_rows=self.band_rows)
        self.cam = self.pt.load_scene(scene_path(cfg["scene"]))
        if self.dist_on:
            import torch
            dev = f"cuda:{local_rank}"
            self.send = torch.zeros((max_rows(H, n, self.band_rows), W, 4), dtype=torch.float32, device=dev)
            self.recv = [torch.zeros_like(self.send) for _ in range(n)] if rank == 0 else None
            self.full = torch.empty((H, W, 4), dtype=torch.float32, device=dev) if rank == 0 else None
            self.index = ([torch.tensor(global_rows(H, r, n, self.band_rows), dtype=torch.long, device=dev)
                           for r in range(n)] if rank == 0 else None)

    def instrument(self):
        # one untimed 8-spp chunk with the non-speculative child-box kernel, whose node/primitive
        # tests are the reference's, for the algorithmic byte count and the lane utilisation; the
        # launch also records the tile costs, so every timed launch runs in cost order.  A device
        # group counts on a one-device context of the whole image (the counts are per sample and do
        # not depend on the partition); its own contexts get their cost order from the warm-up.
        import pathtracercuda_amd as pa
        pt = pa.Pathtracer(self.W, self.H, device=0) if self.mode == "group" else self.pt
        cam = pt.load_scene(scene_path(self.cfg["scene"])) if self.mode == "group" else self.cam
        pt.set_kernel_variant(20)
        st = pt.render_instrumented(cam, CHUNK, 1, True)
        pt.set_kernel_variant(0)
        # the lane utilisation of the kernel that is timed: the same chunk with the default variant
        # (its lanes run the same tests; only the wave schedule differs)
        sd = pt.render_instrumented(cam, CHUNK, 1, True)
        st.update({"d_" + k: v for k, v in sd.items() if k in LANE_KEYS})
        if self.mode == "group":
            pt.close()
        return st

    def step(self):
        ms = self.pt.render_raw(self.cam, CHUNK, self.chunks, True)
        if self.mode == "group":
            # RCCL gather of every device's bands to device 0 + unpermute (pt_group_gather)
            self.gather_ms += self.pt.gather()
        elif self.dist_on:
            from pathtracercuda_amd.distributed import gather_framebuffer
            # RCCL framebuffer gather over xGMI + scatter of the bands on rank 0
            self.pt.copy_accum_to_device(self.send.data_ptr(), self.send.numel() * 4)
            gather_framebuffer(self.send, self.H, self.rank, self.n, recv=self.recv, full=self.full,
                               band_rows=self.band_rows, index=self.index)
        return ms

    def close(self):
        self.pt.close()


class CallLoopRun(Run):
    """The reference's headless loop unchanged (main.cpp:272-279): spp / 8 separate
    Pathtracer::render(camera, 8, i == 0) calls per step through the C++ drop-in (libpt_host ->
    pt_render: one launch per call, synchronous like Pathtracer.cpp:162-227).  step() returns the
    sum of getTiming() over the calls -- the loop's totalGpuTime."""

    def step(self):
        total = 0.0
        for i in range(self.chunks):
            self.pt.render(self.cam, CHUNK, i == 0)
            total += self.pt.get_timing()
        return total


def cold_one_shot(cfg, W, H, spp, local_rank, use_torch, warm_step_s, reps=3):
    """A one-shot render the way `pathtracer -w W -h H -spp SPP` runs it (main.cpp:262-295): a fresh
    context (Pathtracer ctor, scene load: untimed), then ONE render of the whole workload with no tile
    costs yet -- the built-in cost pre-pass, its sort and the launch in the pre-pass's order, all
    inside the timed call.  `reps` fresh contexts; the kernel module is already loaded in this process."""
    import pathtracercuda_amd as pa
    walls, gpus = [], []
    for _ in range(reps):
        pt = pa.Pathtracer(W, H, device=local_rank)
        cam = pt.load_scene(scene_path(cfg["scene"]))
        if use_torch:
            import torch
            torch.cuda.synchronize(local_rank)
        t0 = time.perf_counter()
        gpus.append(pt.render_raw(cam, CHUNK, spp // CHUNK, True))
        walls.append(time.perf_counter() - t0)
        pt.close()
    med = sorted(walls)[len(walls) // 2]
    return {"label": "C3 cold one-shot", "value": round(W * H * spp / med / 1e6, 3), "unit": "Msamples/s",
            "ms_per_step": round(med * 1e3, 3), "runs_ms": [round(w * 1e3, 3) for w in walls],
            "gpu_ms": [round(g, 3) for g in gpus], "cold_over_warm": round(med / warm_step_s, 4),
            "workload": workload_name(cfg, W, H, spp) + ", first launch of a fresh context",
            "what": "fresh Pathtracer + scene load (untimed), then one render_raw of the whole workload: cost "
                    "pre-pass + device sort + the launch in that order (wall time of the call; median of "
                    f"{reps} fresh contexts); cold_over_warm = its time / the headline's step time"}


def timed(run, steps, warmup, local_rank, dist_on, use_torch=True):
    if not use_torch:
        # the in-process device group (main): pt_group_render / pt_group_gather return after every
        # device's stream is idle, and so does pt_render on a plain context (hipEventSynchronize),
        # so the calls are their own barrier
        def barrier_sync():
            pass
    else:
        import torch
        import torch.distributed as dist

        def barrier_sync():
            torch.cuda.synchronize(local_rank)
            if dist_on:
                dist.barrier()

    for _ in range(warmup):
        run.step()
    barrier_sync()
    run.gather_ms = 0.0
    t0 = time.perf_counter()
    kernel_ms = 0.0
    for _ in range(steps):
        kernel_ms += run.step()
    barrier_sync()
    elapsed = time.perf_counter() - t0
    if dist_on:
        import torch
        import torch.distributed as dist
        t = torch.tensor([elapsed, kernel_ms], dtype=torch.float64, device=f"cuda:{local_rank}")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, kernel_ms = float(t[0]), float(t[1])
    return elapsed, kernel_ms


LANE_KEYS = ("node_tests", "prim_tests", "hits", "sky_lookups", "segments", "wave_node_iters", "wave_prim_iters",
             "wave_hits", "wave_sky", "leaf_rounds", "family_execs", "family_execs_compacted", "leaf_round_lanes",
             "leaf_pairs", "family_execs_compacted_in_round", "repairs")


def lane_utilisation(st):
    """SIMD efficiency of each phase of the instrumented launch: lane-level events / (64 x wave-level
    executions).  An interior child-box visit counts two node tests per lane and one wave tick; the
    root test of each segment counts one of each."""
    def ratio(lanes, waves):
        return round(lanes / (64.0 * waves), 3) if waves else None
    if "d_hits" in st:                     # the default kernel's instrumented chunk (Run.instrument)
        st = {k: st["d_" + k] for k in LANE_KEYS}
    visits = (st["node_tests"] + st["segments"]) / 2.0
    out = {"interior_walk": ratio(visits, st["wave_node_iters"]), "leaf_tests": ratio(st["prim_tests"], st["wave_prim_iters"]),
           "hit_shading": ratio(st["hits"], st["wave_hits"]), "sky_shading": ratio(st["sky_lookups"], st["wave_sky"])}
    if st.get("family_execs"):
        # leaf tests per shape-family path (plane / cube / quadric): lane utilisation of the family
        # paths as run, and the executions a perfect cross-lane compaction by family would need
        out["leaf_family_paths"] = ratio(st["prim_tests"], st["family_execs"])
        out["leaf_family_execs_per_round"] = round(st["family_execs"] / max(st["leaf_rounds"], 1), 3)
        out["leaf_family_execs_per_round_compacted"] = round(st["family_execs_compacted"] / max(st["leaf_rounds"], 1), 3)
    if st.get("leaf_round_lanes"):
        # the lanes a leaf round has to work with: compaction can only move pairs onto lanes in the round
        r = max(st["leaf_rounds"], 1)
        out["leaf_round_lanes"] = round(st["leaf_round_lanes"] / r, 2)
        out["leaf_round_pairs"] = round(st["leaf_pairs"] / r, 2)
        out["leaf_family_execs_per_round_compacted_in_round"] = round(st["family_execs_compacted_in_round"] / r, 3)
    return out


def record(cfg, run, elapsed, kernel_ms, steps, st, n, with_profile=True):
    W, H, spp = run.W, run.H, run.spp
    total_samples = W * H * spp * steps
    avg_launch_s = kernel_ms / steps / 1e3
    samples_launch = W * H * spp / n                              # per GPU
    alg = algorithmic_bytes(st) / max(st["samples"], 1) * samples_launch + PIXEL_STATE_B * W * H / n
    workload = workload_name(cfg, W, H, spp)
    prof, src = load_profile(workload) if with_profile else (None, None)
    if prof is None and with_profile:      # e.g. weak scaling: the same scene's base workload, per sample
        prof, src = load_profile(workload_name(cfg, cfg["width"], cfg["height"], cfg["spp"]))
    scale = 1.0
    if prof:                               # the profile is one whole-image launch on one GPU
        dims, pspp = prof["workload"].split()[1], prof["workload"].split()[2]
        pw, ph = (int(x) for x in dims.split("x"))
        scale = samples_launch / (pw * ph * int(pspp[:-3]))
    roof = {"bound": "valu_issue", "achieved": None, "peak": round(VALU_PEAK_G, 1), "unit": "G wave64-VALU-instr/s",
            "frac": None, "traffic": None, "kernel": "trace_kernel", "avg_launch_ms": round(avg_launch_s * 1e3, 3),
            "lds_l2_effective_GBs": round(alg / avg_launch_s / 1e9, 1),
            "bytes_per_sample": round(alg / samples_launch, 1),
            "segments_per_sample": round(st["segments"] / max(st["samples"], 1), 3),
            # leaf rounds whose sphere test raised t_max (Hittable.inl:152-158) and rebuilt the pending
            # far children (repair_pending), in the default kernel's instrumented chunk
            "rise_repairs_per_Msample": (round(st["d_repairs"] / max(st["samples"], 1) * 1e6, 3)
                                         if "d_repairs" in st else None),
            "lane_utilisation": lane_utilisation(st)}
    if prof:
        c = prof["counters"]
        valu = c["SQ_INSTS_VALU"] * scale
        cyc = c.get("GRBM_GUI_ACTIVE", 0) / 8.0
        roof.update({
            "achieved": round(valu / avg_launch_s / 1e9, 1),
            "frac": round(valu / avg_launch_s / 1e9 / VALU_PEAK_G, 4),
            "traffic": round(prof["bytes_per_launch"] * scale),
            "valu_instr_per_launch": round(valu),
            "valu_busy_measured": round(2.0 * c["SQ_INSTS_VALU"] / (SIMDS * cyc), 3) if cyc else None,
            "salu_per_cu_cycle": round(c["SQ_INSTS_SALU"] / (256.0 * cyc), 3) if cyc and c.get("SQ_INSTS_SALU") else None,
            "hbm_GBs_measured": round(prof["bytes_per_launch"] * scale / avg_launch_s / 1e9, 1),
            "hbm_frac_measured": round(prof["bytes_per_launch"] * scale / avg_launch_s / 1e9 / HBM_PEAK_GBS, 5),
            "profile": src + ("" if scale == 1.0 else f" (per-launch counts x {scale:.4f}: this GPU's share)"),
            "profile_commit": prof.get("commit"),
            "profile_kernel_sha": prof.get("kernel_sha"),
            "profile_matches_build": prof.get("kernel_sha") == kernel_source_sha(),
        })
    return {"value": round(total_samples / elapsed / 1e6, 3), "unit": "Msamples/s", "ms_per_step": round(elapsed * 1e3 / steps, 3),
            "workload": workload, "roofline": roof}


def main():
    args = parse_args()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))

    def visible():
        import pathtracercuda_amd as pa
        return pa.device_count()

    mode = resolve_mode(args.gpus, world, args.group, visible)
    n = world if mode == "torchrun" else (args.gpus if mode == "group" else 1)
    cfg = CONFIGS[args.config]
    W, H, spp = cfg["width"], cfg["height"], args.spp or cfg["spp"]
    if args.scaling == "weak" and n > 1:
        W = int(round(W * math.sqrt(n) / 8.0)) * 8
        H = int(round(H * math.sqrt(n) / 8.0)) * 8

    dist_on = mode == "torchrun"
    if mode != "group":
        # the torchrun and single-GPU paths time with torch's events and barriers; the device-group
        # path synchronises every device in its own calls (torch is still loaded, by _native.hip(),
        # so the process keeps a single HIP runtime: INTEGRATION.md §4)
        import torch
        import torch.distributed as dist
    if dist_on:
        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))

    def stats_all(st):
        if not dist_on:
            return st
        keys = ("node_tests", "prim_tests", "hits", "sky_lookups", "samples", "segments", "wave_node_iters",
                "wave_prim_iters", "wave_hits", "wave_sky") + tuple("d_" + k for k in LANE_KEYS if "d_" + k in st)
        t = torch.tensor([st[k] for k in keys], dtype=torch.float64, device=f"cuda:{local_rank}")
        dist.all_reduce(t)
        return dict(zip(keys, [float(x) for x in t]))

    use_torch = mode != "group"        # decided by the process's launch mode, for every record below
    run = Run(cfg, W, H, spp, rank, n, local_rank, args.band_rows, mode)
    st = stats_all(run.instrument())
    elapsed, kernel_ms = timed(run, args.steps, args.warmup, local_rank, dist_on, use_torch)
    main_rec = record(cfg, run, elapsed, kernel_ms, args.steps, st, n)
    gather_ms = run.gather_ms
    run.close()
    part = {"torchrun": f"{args.band_rows}-row bands interleaved x{n}, one process per GPU, RCCL gather (torch.distributed)",
            "group": f"{args.band_rows}-row bands interleaved x{n}, in-process device group (pt_group_*), RCCL gather",
            "single": "1 GPU"}[mode]
    out = {
        "metric": METRIC,
        "value": main_rec["value"],
        "unit": "Msamples/s",
        "n_gpus": n,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": main_rec["ms_per_step"],
        "higher_is_better": True,
        "scaling": args.scaling,
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic sky (scenes/skybox.hdr); reference scene files (scenes/)",
        "config": {"workload": main_rec["workload"], "label": args.config, "scene": cfg["scene"], "width": W,
                   "height": H, "spp": spp, "render_calls_per_step": spp // CHUNK, "parallelism": part,
                   "launch_mode": mode, "per_gpu_pixels": (W * H + n - 1) // n},
        "roofline": main_rec["roofline"],
        "cpu_baseline": None,
    }
    if mode == "group":
        out["group_timing"] = {"kernel_ms_per_step": round(kernel_ms / args.steps, 3),
                               "gather_ms_per_step": round(gather_ms / args.steps, 3)}
    def all_ok(ok):
        """Every rank's verdict on a local phase: the next phase makes collective calls,
        so all ranks run it or none does -- a rank that failed alone must not leave the others
        blocked in a collective, or pair their collectives with the next record's."""
        if not dist_on:
            return ok
        t = torch.tensor([1 if ok else 0], dtype=torch.int32, device=f"cuda:{local_rank}")
        dist.all_reduce(t, op=dist.ReduceOp.MIN)
        return bool(t.item())

    def strong_records():
        """C2, C4 and C5 on this run's N GPUs (strong scaling of each fixed workload)."""
        recs = []
        # the other BASELINE configurations on the same N GPUs, each a fixed workload (strong
        # scaling): cornell (C2), the 4K x 4096 image BASELINE tiles across 8 GPUs (C4) and the
        # 100k-quadric stress scene (C5)
        for label in (("C2", "C4", "C5") if args.configs_n else ()):
            if label == args.config:
                continue
            c = CONFIGS[label]
            name = f"{label} strong scaling ({c['width']}x{c['height']} x {c['spp']} spp on {n} GPUs)"
            # local phase (context, scene, instrumented chunks: no collective), then one agreement
            rc, raw, err = None, None, None
            try:
                rc = Run(c, c["width"], c["height"], c["spp"], rank, n, local_rank, args.band_rows, mode)
                raw = rc.instrument()
            except Exception as e:     # a secondary record never costs the headline line
                err = f"{type(e).__name__}: {e}"
            if not all_ok(err is None):
                if rc is not None:
                    rc.close()
                recs.append({"label": name, "error": err or "failed on another rank"})
                continue
            # collective phase: every rank is here.  (A failure inside it on one rank alone leaves
            # the others in the step's gather until the process group's timeout.)
            try:
                stc = stats_all(raw)
                csteps = max(args.steps, 10) if label == "C2" else min(args.steps, 2)
                ec, kc = timed(rc, csteps, 2, local_rank, dist_on, use_torch)
                recc = record(c, rc, ec, kc, csteps, stc, n)
                rc.close()
            except Exception as e:
                recs.append({"label": name, "error": f"{type(e).__name__}: {e}"})
                continue
            recc["label"] = name
            recc["scaling"] = "strong"
            recs.append(recc)
        return recs

    if args.secondary:
        if n == 1:
            recs = []
            if args.config == "C3" and args.call_loop:
                # the reference's unchanged call loop on the headline workload
                rl = CallLoopRun(cfg, W, H, spp, 0, 1, local_rank, 1, "single")
                el, kl = timed(rl, args.steps, args.warmup, local_rank, False, use_torch)
                rl.close()
                recs.append({"label": "C3 call loop", "value": round(W * H * spp * args.steps / el / 1e6, 3),
                             "unit": "Msamples/s", "ms_per_step": round(el * 1e3 / args.steps, 3),
                             "gpu_ms_per_step": round(kl / args.steps, 3),
                             "fused_over_loop": round(el / elapsed, 4),
                             "workload": workload_name(cfg, W, H, spp) + " as " + str(spp // CHUNK) + " render() calls",
                             "what": "main.cpp:272-279 unchanged: Pathtracer::render(cam, 8, i == 0) per call, one "
                                     "synchronous launch each (libpt_host -> pt_render); gpu_ms_per_step = sum of "
                                     "getTiming() (the loop's totalGpuTime); fused_over_loop = loop step time / "
                                     "headline (one chunked launch) step time"})
            if args.config == "C3" and args.cold:
                recs.append(cold_one_shot(cfg, W, H, spp, local_rank, use_torch, elapsed / args.steps))
            for label in ("C2",) + tuple(x for x in args.extra.split(",") if x):
                c2 = CONFIGS[label]
                r2 = Run(c2, c2["width"], c2["height"], c2["spp"], 0, 1, local_rank, 1, "single")
                st2 = r2.instrument()
                k2steps = max(args.steps, 20) if label == "C2" else args.steps   # C2: 4.4 ms steps
                e2, k2 = timed(r2, k2steps, args.warmup, local_rank, False, use_torch)
                rec2 = record(c2, r2, e2, k2, k2steps, st2, 1)
                r2.close()
                rec2["label"] = label
                if rank == 0 and args.cpu_baseline:
                    rec2["cpu_baseline"] = cpu_baseline(args, c2, c2["width"], c2["height"])
                recs.append(rec2)
            if args.configs_n == 2:         # test hook: the N > 1 records' code path on one GPU
                recs += strong_records()
            out["secondary"] = recs
        else:
            other = "strong" if args.scaling == "weak" else "weak"
            Ww, Hw = cfg["width"], cfg["height"]
            if other == "weak":
                Ww = int(round(cfg["width"] * math.sqrt(n) / 8.0)) * 8
                Hw = int(round(cfg["height"] * math.sqrt(n) / 8.0)) * 8
            rw = Run(cfg, Ww, Hw, spp, rank, n, local_rank, args.band_rows, mode)
            stw = stats_all(rw.instrument())
            ew, kw = timed(rw, min(args.steps, 3), 1, local_rank, dist_on, use_torch)
            recw = record(cfg, rw, ew, kw, min(args.steps, 3), stw, n)
            rw.close()
            recw["label"] = (f"{args.config} weak scaling (image {Ww}x{Hw}: one {cfg['width']}x{cfg['height']} frame per GPU)"
                             if other == "weak" else f"{args.config} strong scaling (the fixed {Ww}x{Hw} image on {n} GPUs)")
            recw["scaling"] = other
            recs = [recw]
            recs += strong_records()
            out["secondary"] = recs
    if rank == 0 and n == 1 and args.cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(args, cfg, W, H)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist_on:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
