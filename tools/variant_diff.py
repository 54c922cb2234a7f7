"""Locate the first divergence between two trace-kernel variants on a full image (GPU box, debugging).

Two contexts render the same render() calls (8 spp each) with variants A and B, compared after every
call; at the first call with differing pixels the pixels' rows are rendered by the oracle (CPU
restatement) with the same calls, which tells which variant left the reference's bits.
    python tools/variant_diff.py [--a 40 --b 60 --calls 128 --width 1920 --height 1080]
"""
import argparse
import json
import pathlib
import sys

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import pathtracercuda_amd as pa  # noqa: E402
from oracle import pyoracle as po  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--scene", default=str(ROOT / "scenes/generated_scene.scene.json"))
ap.add_argument("--width", type=int, default=1920)
ap.add_argument("--height", type=int, default=1080)
ap.add_argument("--a", type=int, default=40)
ap.add_argument("--b", type=int, default=60)
ap.add_argument("--calls", type=int, default=128)
ap.add_argument("--spp", type=int, default=8)
a = ap.parse_args()
ctx = {}
for v in (a.a, a.b):
    pt = pa.Pathtracer(a.width, a.height)
    cam = pt.load_scene(a.scene)
    pt.set_kernel_variant(v)
    pt.set_strip_units(1)
    ctx[v] = (pt, cam)
out = {"a": a.a, "b": a.b, "first_call": None}
for i in range(a.calls):
    for v in (a.a, a.b):
        pt, cam = ctx[v]
        pt.render(cam, a.spp, i == 0)
    ra, rb = (ctx[v][0].accum().view(np.uint32) for v in (a.a, a.b))
    if not np.array_equal(ra, rb):
        bad = np.argwhere((ra != rb).any(-1))
        out["first_call"] = i
        out["pixels"] = int(len(bad))
        out["where"] = [[int(y), int(x)] for y, x in bad[:16]]
        y, x = (int(t) for t in bad[0])
        osc = po.load_scene(pathlib.Path(a.scene), a.width, a.height)
        ref = po.OracleRenderer(osc, a.width, a.height, y, a.height)      # row y only
        ref.render(osc.camera, a.spp, True, chunks=1)
        if i:
            ref.render(osc.camera, a.spp, False, chunks=i)
        o = ref.accum[0, x].view(np.uint32)
        out["pixel"] = [y, x]
        out["oracle"] = [float(t) for t in ref.accum[0, x]]
        out["A"] = [float(t) for t in ra[y, x].view(np.float32)]
        out["B"] = [float(t) for t in rb[y, x].view(np.float32)]
        out["A_matches_oracle"] = bool(np.array_equal(ra[y, x], o))
        out["B_matches_oracle"] = bool(np.array_equal(rb[y, x], o))
        break
print(json.dumps(out))
