"""A/B timing of the trace-kernel variants in one process (interleaved rounds), with a bit-exact
cross-check of every variant's accumulation against variant 1.  Usage on the GPU box:
    python tools/ab_variants.py [--spp 64] [--rounds 5] [--variants 1,2,3,4,5] [--scene ...]
"""
import argparse
import json
import pathlib
import sys
import time

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import pathtracercuda_amd as pa  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default=str(ROOT / "scenes/generated_scene.scene.json"))
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--spp", type=int, default=64)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--variants", default="1,2,3,4,5")
    ap.add_argument("--schedules", default="0", help="tile schedules to cross with the variants (0 sorted, 1 row-major)")
    ap.add_argument("--n", type=int, default=1, help="render one rank's share of an N-way 8-row band partition")
    ap.add_argument("--rank", type=int, default=0)
    ap.add_argument("--groups", type=int, default=1, help="sample groups: 1 = off (plain launches), 0 = automatic")
    ap.add_argument("--ahead", type=int, default=0, help="run-ahead across launches (pt_set_run_ahead): 0 automatic, 1 off")
    ap.add_argument("--block", type=int, default=1,
                    help="launches per variant per round; with > 1 the first of each block (after a switch) is dropped")
    ap.add_argument("--check", type=int, default=1, help="assert every variant bit-identical (0 for A/B-only variants)")
    a = ap.parse_args()
    if a.scene == "stress_100k":                   # C5's generated scene (bench.scene_path)
        import bench
        a.scene = bench.scene_path("stress_100k")
    vs = [(int(v), int(m)) for v in a.variants.split(",") for m in a.schedules.split(",")]
    pt = (pa.Pathtracer(a.width, a.height, row_offset=a.rank, row_stride=a.n, band_rows=8) if a.n > 1
          else pa.Pathtracer(a.width, a.height))
    pt.set_sample_groups(a.groups)
    pt.set_run_ahead(a.ahead)
    cam = pt.load_scene(a.scene)
    chunks = a.spp // 8
    ref = None
    times = {v: [] for v in vs}
    ran = {}
    for v, m in vs:                                # correctness first: every variant bit-identical
        pt.set_kernel_variant(v)
        pt.set_schedule(m)
        st = pt.rng_state()
        pt.render_raw(cam, 8, 1, True)             # schedule 0: records the tile costs
        pt.set_rng_state(st)
        pt.render_raw(cam, 8, 1, True)             # ... and this launch runs in cost order
        acc = pt.accum()
        pt.set_rng_state(st)
        if ref is None:
            ref = acc
        assert not a.check or np.array_equal(acc.view(np.uint32), ref.view(np.uint32)), f"variant {v} schedule {m} differs"
    for r in range(a.rounds):
        for v, m in vs:
            pt.set_kernel_variant(v)
            if len(a.schedules.split(",")) > 1:
                pt.set_schedule(m)
                pt.render_raw(cam, 8, 1, True)     # records the tile costs for mode 0
            for b in range(a.block):
                ms = pt.render_raw(cam, 8, chunks, True)
                if b or a.block == 1:            # blocks: the first launch after a switch is not kept
                    times[(v, m)].append(ms)
            ran[(v, m)] = pt.last_variant
    samples = a.width * pt.rows * a.spp
    out = {}
    for v, m in vs:
        t = np.array(times[(v, m)])
        key = f"{v}" + ("" if len(a.schedules.split(",")) == 1 else f"/s{m}")
        out[key] = {"median_ms": float(np.median(t)), "min_ms": float(t.min()), "ran": ran[(v, m)], "ms": [round(x, 2) for x in t],
                    "Msamples_s": round(samples / (np.median(t) / 1e3) / 1e6, 1)}
    print(json.dumps({"scene": pathlib.Path(a.scene).name, "image": f"{a.width}x{a.height}", "spp": a.spp,
                      "n": a.n, "rank": a.rank, "variants": out}))


if __name__ == "__main__":
    main()
