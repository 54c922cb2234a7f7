"""Launch-sequence probe for the slowdown after a kernel-variant switch (VERDICT r05 "do this" 5).

Renders one rank's share of an N-way 8-row band partition (default: the C4 N = 8 share, rank 2)
with a given sequence of kernel variants, one plain launch each, and prints one JSON line with
every launch's variant, time, the cost-order state it ran with and the tile costs it recorded.
Run it under `rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VALU --kernel-trace` to get each
dispatch's engine clock (GRBM_GUI_ACTIVE / duration) next to its work (tools/switch_summary.py).

    python tools/switch_probe.py --seq 60,40,40,40,60,60,40,40 [--n 8 --rank 2 --spp 4096]
    --fresh-order 1: before every launch after a switch, rebuild the cost order from a launch of
                     the new variant (separates "order measured under the other variant" from the rest)
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
    ap.add_argument("--width", type=int, default=3840)
    ap.add_argument("--height", type=int, default=2160)
    ap.add_argument("--spp", type=int, default=4096)
    ap.add_argument("--n", type=int, default=8)
    ap.add_argument("--rank", type=int, default=2)
    ap.add_argument("--seq", default="60,40,40,40,60,60,40,40,40")
    ap.add_argument("--gap", type=float, default=0.0, help="seconds of idle host time before every launch")
    a = ap.parse_args()
    pt = pa.Pathtracer(a.width, a.height, row_offset=a.rank, row_stride=a.n, band_rows=8)
    pt.set_sample_groups(1)
    pt.set_run_ahead(1)
    cam = pt.load_scene(a.scene)
    chunks = a.spp // 8
    seq = [int(v) for v in a.seq.split(",")]
    # warm-up: one cold launch of the first variant (records the first cost order)
    pt.set_kernel_variant(seq[0])
    pt.render_raw(cam, 8, chunks, True)
    out = []
    prev = seq[0]
    for i, v in enumerate(seq):
        pt.set_kernel_variant(v)
        if a.gap:
            time.sleep(a.gap)
        costs_before = pt.tile_costs().astype(np.float64).ravel()
        t0 = time.perf_counter()
        ms = pt.render_raw(cam, 8, chunks, True)
        wall = (time.perf_counter() - t0) * 1e3
        costs = pt.tile_costs().astype(np.float64).ravel()
        # rank correlation of the order this launch ran in (previous launch's costs) with its own costs
        rb = np.argsort(np.argsort(-costs_before))
        ra = np.argsort(np.argsort(-costs))
        rho = float(np.corrcoef(rb, ra)[0, 1]) if costs.size > 1 else 1.0
        out.append({"i": i, "variant": v, "ran": pt.last_variant, "after": prev, "ms": round(ms, 2),
                    "wall_ms": round(wall, 2), "max_tile_Mcyc": round(float(costs.max()) / 1e6, 2),
                    "sum_tile_Gcyc": round(float(costs.sum()) / 1e9, 3), "order_rank_rho": round(rho, 4)})
        prev = v
        print(json.dumps(out[-1]), flush=True)
    print(json.dumps({"probe": "switch", "n": a.n, "rank": a.rank, "image": f"{a.width}x{a.height}", "spp": a.spp,
                      "launches": out}))


if __name__ == "__main__":
    main()
