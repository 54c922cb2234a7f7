"""Launch time of one workload under several tile schedules, interleaved rounds in one process,
results checked bit-identical against the first schedule.  A schedule is a comma-free token:
    p<K>                 issue priority 3 for the first K positions of the cost order (pt_set_issue_priority)
    f<F>                 the same for the first F percent of the positions
    q                    graded: priority 3 / 2 / 1 / 0 by quarter of the order
    g<A>_<B>_<C>         graded: priority 3 below A %, 2 below B %, 1 below C % of the positions
    a                    the automatic policy (graded by quarter since it was measured; "a" meant off before)
    o                    off: priority 0 for every position
(The round-3 split-launch tokens r<R>w<W>[k<K>] measured the CU-masked split launches of commit
2ac067f; the knob was removed after profiles/r03_schedule_sweep.json.)
Usage on the GPU box:
    python tools/sched_probe.py [--width 1920 --height 1080 --spp 1024 --n 1] --scheds a,p4096,f25,q
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


def apply(pt, tok, tiles):
    if tok in ("a", "o"):
        pt.set_issue_priority(0 if tok == "a" else 1)
        return
    if tok == "q":
        pt.set_issue_priority(2, tiles // 4, tiles // 2, 3 * tiles // 4)
        return
    g = re.fullmatch(r"g(\d+)_(\d+)_(\d+)", tok)
    if g:                                              # graded, bounds in percent of the positions
        pt.set_issue_priority(2, *(tiles * int(x) // 100 for x in g.groups()))
        return
    m = re.fullmatch(r"([pf])(\d+)", tok)
    if not m:
        raise SystemExit(f"bad schedule {tok}")
    kind, p = m.groups()
    K = int(p) if kind == "p" else tiles * int(p) // 100
    pt.set_issue_priority(2, K, K, K)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default=str(ROOT / "scenes/generated_scene.scene.json"))
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--spp", type=int, default=1024)
    ap.add_argument("--n", type=int, default=1, help="a rank's share of an N-way 8-row band partition")
    ap.add_argument("--rank", type=int, default=0)
    ap.add_argument("--scheds", default="p0,p256")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--groups", type=int, default=1, help="sample groups: 1 = off, 0 = automatic")
    a = ap.parse_args()
    pt = (pa.Pathtracer(a.width, a.height, row_offset=a.rank, row_stride=a.n, band_rows=8) if a.n > 1
          else pa.Pathtracer(a.width, a.height))
    pt.set_sample_groups(a.groups)
    cam = pt.load_scene(a.scene)
    st = pt.rng_state()
    pt.render_raw(cam, 8, 2, True)                      # cost order
    scheds = a.scheds.split(",")
    times = {k: [] for k in scheds}
    tails = {k: [] for k in scheds}
    order = None
    ref = None
    for r in range(a.rounds):
        for k in (scheds if r % 2 == 0 else scheds[::-1]):
            apply(pt, k, ((a.width + 7) // 8) * ((pt.rows + 7) // 8))
            pt.set_rng_state(st)
            times[k].append(pt.render_raw(cam, 8, a.spp // 8, True))
            cost = pt.tile_costs().ravel().astype(np.float64) / 2.4e6          # ms at 2.4 GHz
            if order is None:
                order = np.argsort(-cost)[: max(1, cost.size // 100)]          # the first schedule's top 1 %
            tails[k].append((float(cost.max()), float(cost[order].mean()), float(cost.mean())))
            acc = pt.accum().view(np.uint32)
            if ref is None:
                ref = acc.copy()
            assert np.array_equal(acc, ref), f"{k}: results differ"
    tiles = ((a.width + 7) // 8) * ((pt.rows + 7) // 8)
    print(json.dumps({"image": f"{a.width}x{a.height}", "n": a.n, "spp": a.spp, "tiles": tiles,
                      "groups": pt.last_sample_groups, "ms_min": {k: round(min(v), 2) for k, v in times.items()},
                      "ms_all": {k: [round(x, 2) for x in v] for k, v in times.items()},
                      "tile_ms_max_top1pct_mean": {k: [round(float(np.mean([t[i] for t in v])), 2) for i in range(3)]
                                                   for k, v in tails.items()}}), flush=True)


if __name__ == "__main__":
    main()
