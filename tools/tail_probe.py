"""Launch-tail probe of one tile of a multi-GPU partition (GPU box): renders rank r's share of an
image (8-row bands over N ranks) with the cost order, and reports the kernel time and the distribution of per-tile cycle counts.  Usage:
    python tools/tail_probe.py [--width 1920 --height 1080 --spp 1024 --n 8 --rank 0] 
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
ap.add_argument("--width", type=int, default=1920)
ap.add_argument("--height", type=int, default=1080)
ap.add_argument("--spp", type=int, default=1024)
ap.add_argument("--n", type=int, default=8)
ap.add_argument("--rank", type=int, default=0)
ap.add_argument("--band", type=int, default=8)
ap.add_argument("--reps", type=int, default=2)
ap.add_argument("--scene", default=str(ROOT / "scenes/generated_scene.scene.json"))
ap.add_argument("--save", default="", help="write the last run's tile-cost map (.npy)")
a = ap.parse_args()
pt = pa.Pathtracer(a.width, a.height, row_offset=a.rank, row_stride=a.n, band_rows=a.band)
cam = pt.load_scene(a.scene)
pt.render_raw(cam, 8, 1, True)
out = {"image": f"{a.width}x{a.height}", "spp": a.spp, "n": a.n, "rank": a.rank, "tiles": int(((a.width + 7) // 8) * ((pt.rows + 7) // 8)),
       "runs": {}}
for rep in range(a.reps):
    for p in [0]:
        ms = pt.render_raw(cam, 8, a.spp // 8, True)
        c = pt.tile_costs().astype(np.float64).ravel()
        c = c[c > 0]
        q = np.percentile(c, [50, 90, 99, 99.9, 100])
        out["runs"].setdefault(str(p), []).append({"ms": round(ms, 2), "tile_Mcycles_p50_p90_p99_p999_max": [round(x / 1e6, 2) for x in q],
                                                   "tile_Mcycles_mean": round(c.mean() / 1e6, 2)})
        print(json.dumps({p: out["runs"][str(p)][-1]}), flush=True)
if a.save:
    np.save(a.save, pt.tile_costs())
print(json.dumps(out))
