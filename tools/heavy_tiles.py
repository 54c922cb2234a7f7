"""Idle lanes in the most expensive tiles (VERDICT r03 "do this" 1: lane idle vs contention).

Renders one rank's share of the 8-row band partition (or the whole image) with the instrumented
default kernel after a plain launch has built the cost order, and reports per tile the fraction of
lane time spent done while the tile still ran (pt_read_tile_idle / pt_read_tile_costs), for the
heaviest 1 % / 0.1 % of tiles and for all tiles.
    python tools/heavy_tiles.py [--width 3840 --height 2160 --n 8 --rank 0 --spp 4096 --variant 0]
"""
import argparse
import json
import pathlib
import sys

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import pathtracercuda_amd as pa  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--scene", default=str(ROOT / "scenes/generated_scene.scene.json"))
ap.add_argument("--width", type=int, default=3840)
ap.add_argument("--height", type=int, default=2160)
ap.add_argument("--n", type=int, default=8)
ap.add_argument("--rank", type=int, default=0)
ap.add_argument("--spp", type=int, default=4096)
ap.add_argument("--variants", default="0")
a = ap.parse_args()
pt = (pa.Pathtracer(a.width, a.height, row_offset=a.rank, row_stride=a.n, band_rows=8) if a.n > 1
      else pa.Pathtracer(a.width, a.height))
pt.set_sample_groups(1)
cam = pt.load_scene(a.scene)
out = {"image": f"{a.width}x{a.height}", "n": a.n, "rank": a.rank, "spp": a.spp, "variants": {}}
for v in [int(x) for x in a.variants.split(",")]:
    pt.set_kernel_variant(v)
    st = pt.rng_state()
    ms = pt.render_raw(cam, 8, a.spp // 8, True)          # builds / refines the cost order
    plain = pt.tile_costs().astype(np.float64).ravel()
    pt.set_rng_state(st)
    s = pt.render_instrumented(cam, 8, a.spp // 8, True)
    cost = pt.tile_costs().astype(np.float64).ravel()
    idle = pt.tile_idle().astype(np.float64).ravel()
    ok = cost > 0
    frac = np.where(ok, idle / np.maximum(cost, 1.0), 0.0)
    order = np.argsort(-cost)
    res = {"plain_ms": round(ms, 2), "instrumented_ms": round(s["ms"], 2), "tiles": int(ok.sum())}
    for name, k in (("top_0.1pct", max(1, ok.sum() // 1000)), ("top_1pct", max(1, ok.sum() // 100)),
                    ("top_10pct", max(1, ok.sum() // 10)), ("all", int(ok.sum()))):
        sel = order[:k]
        res[name] = {"tiles": int(k), "idle_frac_mean": round(float(frac[sel].mean()), 4),
                     "idle_frac_max": round(float(frac[sel].max()), 4),
                     "cycles_mean_instrumented": round(float(cost[sel].mean())),
                     "cycles_mean_plain": round(float(np.sort(plain)[::-1][:k].mean()))}
    res["plain_tile_ms_max_at_2.4GHz"] = round(float(plain.max()) / 2.4e9 * 1e3, 2)   # s_memtime: shader clock
    out["variants"][v] = res
print(json.dumps(out))
