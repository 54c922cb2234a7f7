"""Speculative sample groups on one rank's share of an image (GPU box): kernel time with groups and
without, and how the groups went -- samples logged per item relative to the nominal group length,
the per-item maximum over lanes (what sets an item's duration), and the resume pass.
    python tools/ssg_probe.py [--width 1920 --height 1080 --spp 1024 --n 8 --rank 0 --groups 0]
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
ap.add_argument("--groups", type=int, default=0, help="0 = automatic, G >= 2 forced")
ap.add_argument("--scene", default=str(ROOT / "scenes/generated_scene.scene.json"))
ap.add_argument("--reps", type=int, default=2, help="timed launches after the cold one")
ap.add_argument("--lookback", default="d",
                help="comma-separated far:near second-phase lookbacks of the grouped runs (set_group_lookback; "
                     "'d' = the library's default)")
a = ap.parse_args()
res = {"image": f"{a.width}x{a.height}", "spp": a.spp, "n": a.n, "rank": a.rank}
runs = [("plain", 1, "d")] + [("groups" if cfg == "d" else f"groups_look{cfg}", a.groups, cfg) for cfg in a.lookback.split(",")]
for name, mode, cfg in runs:
    pt = pa.Pathtracer(a.width, a.height, row_offset=a.rank, row_stride=a.n, band_rows=8)
    pt.set_sample_groups(mode)
    if cfg != "d":
        pt.set_group_lookback(*(int(x) for x in cfg.split(":")))
    cam = pt.load_scene(a.scene)
    pt.render_raw(cam, 8, a.spp // 8, True)
    ms, st = [], []
    for _ in range(a.reps):
        ms.append(pt.render_raw(cam, 8, a.spp // 8, True))
        st.append(pt.group_stats() if pt.last_sample_groups else None)
    r = {"ms": [round(x, 2) for x in ms], "groups": pt.last_sample_groups, "stats_by_rep": st}
    if pt.last_sample_groups:
        G = pt.last_sample_groups
        nom = a.spp // G
        c = pt.group_log_counts().astype(np.int64)           # tiles x G x 64
        act = c > 0
        itemmax = c.max(-1)
        r.update({"nominal": nom,
                  "lane_count_over_nominal_p50_p99_max": [round(float(np.percentile(c[act], q)) / nom, 3) for q in (50, 99, 100)],
                  "item_max_over_nominal_p50_p99_max": [round(float(np.percentile(itemmax[itemmax > 0], q)) / nom, 3) for q in (50, 99, 100)],
                  "lanes_over_2x": int((c > 2 * nom).sum()), "lanes_at_cap": int((c >= c.max()).sum()),
                  "logged_samples_over_needed": round(float(c.sum()) / (pt.rows * a.width * a.spp), 3),
                  "stats": pt.group_stats()})
        by_g = [round(float(c[:, g][c[:, g] > 0].mean()) / nom, 3) if (c[:, g] > 0).any() else 0 for g in range(2 * G - 1)]
        r["mean_count_by_group"] = by_g
        # slot time in samples: an item holds its wave slot for its slowest lane's count; dead lanes
        # (no second phase, stopped early) idle beside it
        live = [round(float((c[:, j] > 0).mean()), 3) for j in range(2 * G - 1)]
        eff = [round(float(c[:, j].sum()) / max(1.0, float(64 * c[:, j].max(-1).sum())), 3) for j in range(2 * G - 1)]
        r["live_lane_frac_by_item"] = live
        r["slot_efficiency_by_item"] = eff
        r["slot_efficiency"] = round(float(c.sum()) / float(64 * itemmax.sum()), 3)
        r["slot_samples_over_needed"] = round(float(64 * itemmax.sum()) / (pt.rows * a.width * a.spp), 3)
    res[name] = r
    print(json.dumps(r), flush=True)
    pt.close()
print(json.dumps(res))
