"""Head groups (pt_set_head_groups) on one rank's share (default: C4 at N = 8, rank 0): warm launch
times for head settings, interleaved rounds in one process, results checked bit-identical.
A setting is K:G (K = -1 off, 0 automatic, K > 0 forced head tiles; G groups).
    python tools/head_probe.py [--settings -1:2,0:2,128:2,256:2,256:3] [--rounds 3] [--n 8 --rank 0]
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
ap.add_argument("--rounds", type=int, default=3)
ap.add_argument("--settings", default="-1:2,0:2,128:2,256:2,256:3")
ap.add_argument("--scene", default=str(ROOT / "scenes/generated_scene.scene.json"))
a = ap.parse_args()
pt = pa.Pathtracer(a.width, a.height, row_offset=a.rank, row_stride=a.n, band_rows=8)
cam = pt.load_scene(a.scene)
pt.set_head_groups(-1, 2)
st = pt.rng_state()
pt.render_raw(cam, 8, a.spp // 8, True)            # cold launch: cost order
pt.set_rng_state(st)
pt.render_raw(cam, 8, a.spp // 8, True)            # order rebuilt without priority
sets = [tuple(int(x) for x in t.split(":")) for t in a.settings.split(",")]
res = {f"{k}:{g}": {"ms": [], "head": []} for k, g in sets}
ref = None
ok = True
for r in range(a.rounds):
    for k, g in sets:
        pt.set_head_groups(k, g)
        pt.set_rng_state(st)
        ms = pt.render_raw(cam, 8, a.spp // 8, True)
        res[f"{k}:{g}"]["ms"].append(round(ms, 2))
        res[f"{k}:{g}"]["head"].append(pt.last_head_tiles)
        acc = pt.accum().view(np.uint32)
        if ref is None:
            ref = acc.copy()
        ok = ok and np.array_equal(acc, ref)
        gs = pt.group_stats() if pt.last_head_tiles else {}
        extra = {}
        costs = np.sort(pt.tile_costs().ravel().astype(np.float64) / 2.4e6)[::-1]    # ms (2.4 GHz)
        extra["top_tile_ms"] = [round(float(x), 1) for x in costs[:5]]
        if pt.last_head_tiles:
            hk = pt.last_head_tiles
            cnt = pt.group_log_counts()[:hk]                   # (head tiles, items, 64 lanes), order positions
            per_item = cnt.max(axis=2)                         # slowest lane's samples per item
            extra["item_max_samples_median"] = [int(np.median(per_item[:, j])) for j in range(per_item.shape[1])]
            extra["item_max_samples_max"] = [int(per_item[:, j].max()) for j in range(per_item.shape[1])]
            extra["items_at_cap"] = int((per_item >= a.spp).sum())
        print(json.dumps({"round": r, "setting": f"{k}:{g}", "ms": round(ms, 2), "head": pt.last_head_tiles,
                          "group_stats": gs, **extra}), flush=True)
out = {"share": f"{a.width}x{a.height}x{a.spp} N={a.n} rank {a.rank}", "bit_identical": bool(ok), "settings": {}}
for key, d in res.items():
    out["settings"][key] = {"ms_median": float(np.median(d["ms"])), "ms": d["ms"], "head_tiles": d["head"]}
print(json.dumps(out))
