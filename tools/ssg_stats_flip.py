"""Do a rank share's guess statistics alternate between grouped launches?  (GPU box, diagnostics.)
Renders the 1080p N = 8 rank-0 share with sample groups several times (cold launch first) and after
each launch reads the group stats (patch rounds, dead ends) and the per-pixel guess statistics the
next launch uses (draw pairs per sample m, odd-length fraction, variance); reports, per launch, how
many pixels changed their parity class (odd fraction < 6 %: a second phase) and the largest changes
of m against the previous launch.
    python tools/ssg_stats_flip.py [--n 8 --rank 0 --reps 6]
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
ap.add_argument("--reps", type=int, default=6)
ap.add_argument("--spp", type=int, default=1024)
a = ap.parse_args()
pt = pa.Pathtracer(1920, 1080, row_offset=a.rank, row_stride=a.n, band_rows=8)
cam = pt.load_scene(str(ROOT / "scenes/generated_scene.scene.json"))
out = []
prev = None
for i in range(a.reps + 1):
    ms = pt.render_raw(cam, 8, a.spp // 8, True)
    m, odd, var = (pt.group_fold_word(w).copy() for w in (19, 20, 21))
    fin = pt.group_fold_word(16) >> 8                  # fold round in which each pixel finished
    rec = {"launch": i, "ms": round(ms, 2), "stats": pt.group_stats()}
    if prev is not None:
        # the pixels that needed two or more patch rounds, with the statistics their guesses used
        late = np.argwhere(fin >= 2)
        pm, podd, _ = prev
        fdone, foff, fh = (pt.group_fold_word(w) for w in (7, 8, 9))
        G = pt.last_sample_groups
        rec["late_pixels"] = [{"pixel": [int(y), int(x)], "round": int(fin[y, x]), "m_used": round(float(pm[y, x]), 4),
                               "odd_used": round(float(podd[y, x]), 4), "m_after": round(float(m[y, x]), 4),
                               "odd_after": round(float(odd[y, x]), 4),
                               "last_dead_end": {"done": int(fdone[y, x]), "off": int(foff[y, x]), "h": int(fh[y, x])},
                               "group_starts_even_lattice": [2 * int(g * (a.spp // G) * float(pm[y, x]) / 2 + 0.5)
                                                             for g in range(1, G)]}
                              for y, x in late[:8]]
    if prev is not None:
        pm, podd, pvar = prev
        stable, pstable = odd < 0.06, podd < 0.06
        dm = np.abs(m - pm)
        rec["parity_class_flips"] = int((stable != pstable).sum())
        rec["m_change_p99_max"] = [round(float(np.percentile(dm, 99)), 4), round(float(dm.max()), 4)]
        worst = np.argsort(dm.ravel())[-4:][::-1]
        rec["worst"] = [{"pixel": [int(q // pt.width), int(q % pt.width)], "m": [float(pm.ravel()[q]), float(m.ravel()[q])],
                         "odd": [float(podd.ravel()[q]), float(odd.ravel()[q])]} for q in worst]
    prev = (m, odd, var)
    out.append(rec)
    print(json.dumps(rec), flush=True)
print(json.dumps({"n": a.n, "rank": a.rank, "launches": out}))
