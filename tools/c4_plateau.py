"""Tile-cost plateau of one rank's share (default: C4 at N = 8, rank 0, 8-row bands): the launch time
against its heaviest tiles' times (per-tile shader cycles recorded by the kernel, s_memtime,
shader clock -> ms), to size a head-of-order split (how many tiles run longer than a target).
    python tools/c4_plateau.py [--n 8 --rank 0 --width 3840 --height 2160 --spp 4096] [--launches 3]
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
ap.add_argument("--n", type=int, default=8)
ap.add_argument("--rank", type=int, default=0)
ap.add_argument("--width", type=int, default=3840)
ap.add_argument("--height", type=int, default=2160)
ap.add_argument("--spp", type=int, default=4096)
ap.add_argument("--launches", type=int, default=3)
ap.add_argument("--clock-mhz", type=float, default=2400.0, help="s_memtime rate (shader clock; reproduces kernel times, profiles/r02_c4_tile_costs.json)")
ap.add_argument("--scene", default=str(ROOT / "scenes/generated_scene.scene.json"))
a = ap.parse_args()
pt = pa.Pathtracer(a.width, a.height, row_offset=a.rank, row_stride=a.n, band_rows=8)
cam = pt.load_scene(a.scene)
out = {"share": f"{a.width}x{a.height}x{a.spp} N={a.n} rank {a.rank}", "launch_ms": []}
for i in range(a.launches):
    out["launch_ms"].append(round(pt.render_raw(cam, 8, a.spp // 8, True), 2))
c = np.sort(pt.tile_costs().ravel().astype(np.float64) / (a.clock_mhz * 1e3))[::-1]
slots = 256 * 4 * 5
out.update({"tiles": int(c.size), "sum_over_slots_ms": round(float(c.sum()) / slots, 1),
            "top_ms": {k: round(float(c[k - 1]), 1) for k in (1, 10, 50, 100, 200, 500, 1000, 2000) if k <= c.size},
            "tiles_above_ms": {t: int((c > t).sum()) for t in (300, 350, 400, 420, 450)},
            "work_share_top": {k: round(float(c[:k].sum() / c.sum()), 4) for k in (100, 200, 500, 1000) if k <= c.size}})
print(json.dumps(out))
