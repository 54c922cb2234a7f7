"""Head groups on one rank's share (pt_set_head_groups): launch times and the group statistics of
each launch (G, patch rounds, dead ends after each fold round); run under rocprofv3 --kernel-trace to
see the grouped kernel, the plain remainder, folds, patch rounds and resume side by side.
    python tools/head_probe.py --n 8 --width 3840 --height 2160 --spp 4096 --head 64 --groups 2
"""
import argparse
import json
import pathlib
import sys

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import pathtracercuda_amd as pa  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--scene", default=str(ROOT / "scenes/generated_scene.scene.json"))
ap.add_argument("--width", type=int, default=1920)
ap.add_argument("--height", type=int, default=1080)
ap.add_argument("--spp", type=int, default=1024)
ap.add_argument("--n", type=int, default=1)
ap.add_argument("--head", type=int, default=64)
ap.add_argument("--groups", type=int, default=2)
ap.add_argument("--launches", type=int, default=3)
a = ap.parse_args()
pt = (pa.Pathtracer(a.width, a.height, row_offset=0, row_stride=a.n, band_rows=8) if a.n > 1
      else pa.Pathtracer(a.width, a.height))
pt.set_sample_groups(1)
cam = pt.load_scene(a.scene)
st = pt.rng_state()
out = {"plain": [], "head": [], "stats": []}
pt.render_raw(cam, 8, a.spp // 8, True)                 # cost order from a full launch
for _ in range(a.launches):
    pt.set_head_groups(1)
    pt.set_rng_state(st)
    out["plain"].append(round(pt.render_raw(cam, 8, a.spp // 8, True), 2))
    pt.set_head_groups(2, a.head, a.groups)
    pt.set_rng_state(st)
    out["head"].append(round(pt.render_raw(cam, 8, a.spp // 8, True), 2))
    out["stats"].append(pt.group_stats())
print(json.dumps(out), flush=True)
pt.close()
