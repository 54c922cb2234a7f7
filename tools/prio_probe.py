"""Issue-priority schedules on one rank's share, interleaved in rounds on one context (same cost order
throughout): launch time, and with --trace the last tile ends per position band (per-CU clocks).
    python tools/prio_probe.py [--n 8 --rank 2 --width 3840 --height 2160 --spp 4096]
                               [--settings a,5120/8160/12240@3210] [--rounds 3] [--trace]
A setting is "a" (automatic) or B0/B1/B2: positions < B0 at priority 3, < B1 at 2, < B2 at 1, the rest
at 0 (pt_set_issue_priority mode 2).  (Other level orders per band, quiet head CUs and a two-ended
queue were probed with this tool at commit 3c9fd51, profiles/r06_schedule_trace.json.)  --trace runs
the instrumented build (the plain kernel carries no trace code): same schedule rules, ~15 % slower.  Bounds may be written as fractions of the tiles
(e.g. 0.25).
"""
import argparse
import json
import pathlib
import re
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
ap.add_argument("--settings", default="a")
ap.add_argument("--rounds", type=int, default=3)
ap.add_argument("--trace", action="store_true")
ap.add_argument("--variant", type=int, default=0, help="kernel variant of the timed launches (0 = automatic)")
ap.add_argument("--out", default="", help="with --trace: .npz of the last round's per-tile start, duration, hardware ids")
ap.add_argument("--scene", default=str(ROOT / "scenes/generated_scene.scene.json"))
a = ap.parse_args()
pt = pa.Pathtracer(a.width, a.height, row_offset=a.rank, row_stride=a.n, band_rows=8)
cam = pt.load_scene(a.scene)
chunks = a.spp // 8
cold = [round(pt.render_raw(cam, 8, chunks, True), 2) for _ in range(2)]   # cold start, then its order rebuild
ref = pt.tile_costs().ravel()
n = ref.size
pos_of = np.empty(n, np.int64)
pos_of[np.argsort(-ref.astype(np.int64), kind="stable")] = np.arange(n)


def apply(tok):
    m = re.fullmatch(r"([\d.]+)/([\d.]+)/([\d.]+)", tok)
    if tok == "a":
        pt.set_issue_priority(0)
        return
    if not m:
        raise SystemExit(f"bad setting {tok}")
    b = [int(float(x) * n) if "." in x else int(x) for x in m.groups()[:3]]
    pt.set_issue_priority(2, *b)


def ends(tr, dur):
    """Tile end times (ms) with each CU's clock zeroed at its first tile start (s_memtime is per CU and
    wraps at 2^32 cycles)."""
    W = 2.0 ** 32 / 2.4e6
    st = tr[:, 0].astype(np.float64) / 2.4e6
    hw = tr[:, 1]
    cu = (hw >> 16) << 8 | ((hw & 0xffff) >> 8)
    for x in np.unique(cu):
        m = np.where(cu == x)[0]
        v = np.sort(st[m] % W)
        i = int(np.argmax(np.diff(np.r_[v, v[0] + W])))
        st[m] = (st[m] - v[(i + 1) % len(v)]) % W
    return st, st + dur


settings = a.settings.split(",")
SAVE = {}
pt.set_kernel_variant(a.variant)
res = {s: {"ms": []} for s in settings}
bands = [0, 1024, 2048, 3072, 4096, 5120, 6144, 8192, 12288, n]
pt.set_tile_trace(a.trace)
for r in range(a.rounds):
    for s in settings:
        apply(s)
        ms = pt.render_instrumented(cam, 8, chunks, True)["ms"] if a.trace else pt.render_raw(cam, 8, chunks, True)
        e = res[s]
        e["ms"].append(round(ms, 2))
        if a.trace:
            dur = pt.tile_costs().ravel().astype(np.float64) / 2.4e6
            st, en = ends(pt.tile_trace().reshape(-1, 2), dur)
            order = np.argsort(pos_of)
            e.setdefault("band_end_max", []).append(
                [round(float(en[order[lo:hi]].max()), 1) for lo, hi in zip(bands, bands[1:]) if lo < hi])
            e.setdefault("band_dur_med", []).append(
                [round(float(np.median(dur[order[lo:hi]])), 1) for lo, hi in zip(bands, bands[1:]) if lo < hi])
            hw = pt.tile_trace().reshape(-1, 2)[:, 1]
            last = np.argsort(-en)[:10]
            e["last"] = [[int(pos_of[i]), round(float(st[i]), 1), round(float(dur[i]), 1), int(hw[i] & 15)] for i in last]
            SAVE[s] = (st, dur, hw)
        print(json.dumps({"round": r, "setting": s, "ms": round(ms, 2), "variant": pt.last_variant}), flush=True)
apply("a")
if a.out and SAVE:
    arrs = {"pos_of": pos_of}
    for i, (k, (st, dur, hw)) in enumerate(SAVE.items()):
        arrs.update({f"start_{i}": st, f"dur_{i}": dur, f"hw_{i}": hw})
    np.savez_compressed(a.out, settings=np.array(list(SAVE)), **arrs)
for e in res.values():
    e["median_ms"] = float(np.median(e["ms"]))
print(json.dumps({"share": f"{a.width}x{a.height}x{a.spp} N={a.n} rank {a.rank}", "tiles": n, "cold_ms": cold,
                  "bands": bands, "settings": res}))
