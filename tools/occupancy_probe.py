"""How much faster does one tile's sample chain run with fewer waves per SIMD?  (The premise of
reserving CUs for the most expensive tiles: DESIGN.md §5)

Renders the same image at several persistent-grid occupancies (pt_set_occupancy: workgroups of four
waves per CU = waves per SIMD) and compares every tile's recorded shader-clock time with its time at
the default occupancy, overall and for the most expensive tiles.  Usage on the GPU box:
    python tools/occupancy_probe.py [--width 1920 --height 1080 --spp 256 --occ 1,2,3,5]
"""
import argparse
import json
import pathlib
import sys

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import pathtracercuda_amd as pa  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default=str(ROOT / "scenes/generated_scene.scene.json"))
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--spp", type=int, default=256)
    ap.add_argument("--occ", default="5,3,2,1")
    ap.add_argument("--n", type=int, default=1, help="one rank's share of an N-way 8-row band partition")
    a = ap.parse_args()
    pt = (pa.Pathtracer(a.width, a.height, row_offset=0, row_stride=a.n, band_rows=8) if a.n > 1
          else pa.Pathtracer(a.width, a.height))
    pt.set_sample_groups(1)
    cam = pt.load_scene(a.scene)
    st = pt.rng_state()
    pt.render_raw(cam, 8, 1, True)                   # tile costs -> cost order
    res, base = {}, None
    for occ in [int(x) for x in a.occ.split(",")]:
        pt.set_occupancy(0 if occ >= 5 else occ)
        pt.set_rng_state(st)
        ms = pt.render_raw(cam, 8, a.spp // 8, True)
        cost = pt.tile_costs().ravel().astype(np.float64) / 2.4e6          # ms at 2.4 GHz
        if base is None:
            base = cost
            order = np.argsort(-base)
        top = order[:max(1, len(order) // 100)]
        r = base / np.maximum(cost, 1e-9)
        res[occ] = {"launch_ms": round(ms, 2), "tile_ms_mean": round(float(cost.mean()), 3),
                    "tile_ms_max": round(float(cost.max()), 3),
                    "speedup_vs_default_all_median": round(float(np.median(r)), 3),
                    "speedup_vs_default_top1pct_median": round(float(np.median(r[top])), 3),
                    "top1pct_tile_ms_mean": round(float(cost[top].mean()), 3)}
        print(json.dumps({occ: res[occ]}), flush=True)
    print(json.dumps({"image": f"{a.width}x{a.height}", "n": a.n, "spp": a.spp, "tiles": int(base.size),
                      "by_waves_per_simd": res}))


if __name__ == "__main__":
    main()
