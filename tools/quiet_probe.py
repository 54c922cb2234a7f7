"""Quiet head CUs (pt_set_quiet_heads) on one rank's share: launch time and the heaviest tiles' times
for each setting, interleaved in rounds on one context (same cost order throughout).
    python tools/quiet_probe.py [--n 8 --rank 2 --width 3840 --height 2160 --spp 4096]
                                [--settings 0:0,64:2,64:1] [--rounds 3]
A setting is CUS:BESIDE[:P3] (0:0 = off; P3: issue priority 3 for the first P3 positions only, the
rest graded by quarter as by default).  Tile times are per-tile shader cycles (s_memtime) at 2.4 GHz;
"heads" are the 4 x CUS heaviest tiles of the order's source launch (a plain launch).
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
ap.add_argument("--rank", type=int, default=2)
ap.add_argument("--width", type=int, default=3840)
ap.add_argument("--height", type=int, default=2160)
ap.add_argument("--spp", type=int, default=4096)
ap.add_argument("--settings", default="0:0,64:2,64:1")
ap.add_argument("--rounds", type=int, default=3)
ap.add_argument("--scene", default=str(ROOT / "scenes/generated_scene.scene.json"))
a = ap.parse_args()
settings = [tuple(int(x) for x in (s + ":-1").split(":")[:3]) for s in a.settings.split(",")]
pt = pa.Pathtracer(a.width, a.height, row_offset=a.rank, row_stride=a.n, band_rows=8)
cam = pt.load_scene(a.scene)
chunks = a.spp // 8
cold = [round(pt.render_raw(cam, 8, chunks, True), 2) for _ in range(2)]   # cold start, then its order rebuild
ref = pt.tile_costs().ravel().astype(np.float64) / 2.4e6
rank = np.argsort(-ref, kind="stable")
def key(c, b, p):
    return f"{c}:{b}" + (f":{p}" if p >= 0 else "")


res = {key(c, b, p): {"ms": [], "head_max_ms": [], "rest_max_ms": [], "rest_max_pos": [], "band_max_ms": []}
       for c, b, p in settings}
n = ref.size
pos_of = np.empty(n, np.int64)
pos_of[rank] = np.arange(n)
bands = [0, 256, 512, 1024, 2048, 4096, n]
for r in range(a.rounds):
    for c, b, p in settings:
        pt.set_quiet_heads(c, b)
        if p >= 0:
            pt.set_issue_priority(2, p, max(p, n // 2), max(p, n - n // 4))
        else:
            pt.set_issue_priority(0)
        ms = pt.render_raw(cam, 8, chunks, True)
        t = pt.tile_costs().ravel().astype(np.float64) / 2.4e6
        h = rank[:4 * c]
        rest = rank[4 * c:]
        e = res[key(c, b, p)]
        e["ms"].append(round(ms, 2))
        e["head_max_ms"].append(round(float(t[h].max()), 1) if c else None)
        e["rest_max_ms"].append(round(float(t[rest].max()), 1))
        e["rest_max_pos"].append(int(pos_of[rest[np.argmax(t[rest])]]))
        ts = t[rank]
        e["band_max_ms"].append([round(float(ts[lo:hi].max()), 1) for lo, hi in zip(bands, bands[1:]) if lo < hi])
        print(json.dumps({"round": r, "setting": key(c, b, p), "ms": round(ms, 2), "variant": pt.last_variant, "quiet": pt.last_quiet_heads}), flush=True)
pt.set_quiet_heads(0, 0)
out = {"share": f"{a.width}x{a.height}x{a.spp} N={a.n} rank {a.rank}", "tiles": int(ref.size), "cold_ms": cold,
       "variant": pt.last_variant, "settings": res}
for k, e in res.items():
    e["median_ms"] = float(np.median(e["ms"]))
print(json.dumps(out))
