"""Sweep of the issue-priority knob (pt_set_priority_slots): launch time of one workload with the
waves on the first K positions of the cost order at raised priority, for several K, interleaved
rounds in one process, results checked bit-identical against K = 0.  Usage on the GPU box:
    python tools/prio_probe.py [--width 1920 --height 1080 --spp 1024 --n 1 --ks 0,64,256,1024]
"""
import argparse
import json
import pathlib
import sys

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import pathtracercuda_amd as pa  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default=str(ROOT / "scenes/generated_scene.scene.json"))
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--spp", type=int, default=1024)
    ap.add_argument("--n", type=int, default=1, help="rank 0's share of an N-way 8-row band partition")
    ap.add_argument("--ks", default="0,32,128,512,2048")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--groups", type=int, default=1, help="sample groups: 1 = off, 0 = automatic")
    a = ap.parse_args()
    pt = (pa.Pathtracer(a.width, a.height, row_offset=0, row_stride=a.n, band_rows=8) if a.n > 1
          else pa.Pathtracer(a.width, a.height))
    pt.set_sample_groups(a.groups)
    cam = pt.load_scene(a.scene)
    st = pt.rng_state()
    pt.render_raw(cam, 8, 2, True)                      # cost order
    ks = [int(k) for k in a.ks.split(",")]
    times = {k: [] for k in ks}
    ref = None
    for r in range(a.rounds):
        for k in (ks if r % 2 == 0 else ks[::-1]):
            pt.set_priority_slots(k)
            pt.set_rng_state(st)
            times[k].append(pt.render_raw(cam, 8, a.spp // 8, True))
            acc = pt.accum().view(np.uint32)
            if ref is None:
                ref = acc.copy()
            assert np.array_equal(acc, ref), f"K={k}: results differ"
    tiles = ((a.width + 7) // 8) * ((pt.rows + 7) // 8)
    out = {"image": f"{a.width}x{a.height}", "n": a.n, "spp": a.spp, "tiles": tiles, "groups": pt.last_sample_groups,
           "ms_min": {k: round(min(v), 2) for k, v in times.items()},
           "ms_all": {k: [round(x, 2) for x in v] for k, v in times.items()}}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
