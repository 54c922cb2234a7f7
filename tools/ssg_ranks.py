"""Launch-to-launch variation of the 1080p strong-scaling shares under speculative sample groups:
every rank's share of an N-way 8-row band partition, rendered in turn on one GPU (one context at a
time), several timed launches each, with how each grouped launch went (groups, patch rounds, dead
ends).  Run under rocprofv3 --kernel-trace to split the launches into their kernels.
    python tools/ssg_ranks.py [--n 8 --spp 1024 --launches 6 --groups 0]
"""
import argparse
import json
import pathlib
import sys

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import pathtracercuda_amd as pa  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--width", type=int, default=1920)
ap.add_argument("--height", type=int, default=1080)
ap.add_argument("--spp", type=int, default=1024)
ap.add_argument("--n", type=int, default=8)
ap.add_argument("--ranks", default="")
ap.add_argument("--launches", type=int, default=6)
ap.add_argument("--groups", type=int, default=0, help="0 = automatic, 1 = off, G >= 2 forced")
ap.add_argument("--scene", default=str(ROOT / "scenes/generated_scene.scene.json"))
a = ap.parse_args()
ranks = [int(x) for x in a.ranks.split(",")] if a.ranks else list(range(a.n))
out = {"image": f"{a.width}x{a.height}", "spp": a.spp, "n": a.n, "groups_mode": a.groups, "ranks": {}}
for r in ranks:
    pt = pa.Pathtracer(a.width, a.height, row_offset=r, row_stride=a.n, band_rows=8)
    pt.set_sample_groups(a.groups)
    cam = pt.load_scene(a.scene)
    pt.render_raw(cam, 8, a.spp // 8, True)                  # cost order, group statistics
    pt.render_raw(cam, 8, a.spp // 8, True)
    runs = []
    for _ in range(a.launches):
        ms = pt.render_raw(cam, 8, a.spp // 8, True)
        g = pt.group_stats() if pt.last_sample_groups else {}
        runs.append({"ms": round(ms, 2), "groups": pt.last_sample_groups, "patch_rounds": g.get("patch_rounds"),
                     "dead_ends": g.get("dead_ends")})
    out["ranks"][r] = {"rows": pt.rows, "runs": runs}
    print(json.dumps({r: out["ranks"][r]}), flush=True)
    pt.close()
print(json.dumps(out))
