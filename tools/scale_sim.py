"""Single-GPU projection of multi-GPU strong scaling: renders every rank's exact share of the image
(the tile `bench.py --gpus N` gives rank r) on one MI355X, one after another, and compares the
slowest rank's kernel time with 1/N of the full-image time.  Two partitions side by side:
  rows   band_rows = 1: row y -> rank y mod N (round 1's partition)
  bands  band_rows = 8: 8-row band b -> rank b mod N (the default since round 2)
The RCCL gather (~0.1 ms for a C4 frame) is not included.  Usage on the GPU box:
    python tools/scale_sim.py [--width 3840 --height 2160 --spp 4096] [--ns 2,4,8] [--runs 3]
"""
import argparse
import json
import pathlib
import sys

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import pathtracercuda_amd as pa  # noqa: E402


SSG = 0
GROUPS = {}


RUNS = 1


def run(W, H, off, stride, band, spp, scene):
    """Warm launch times of one share: a cold launch (cost order, draw-pair guesses), then RUNS
    launches; returns the list."""
    pt = pa.Pathtracer(W, H, row_offset=off, row_stride=stride, band_rows=band)
    pt.set_sample_groups(SSG)
    cam = pt.load_scene(scene)
    pt.render_raw(cam, 8, spp // 8, True)
    ms = [pt.render_raw(cam, 8, spp // 8, True) for _ in range(RUNS)]
    GROUPS[(stride, off)] = pt.last_sample_groups
    pt.close()
    return ms


def med(x):
    x = sorted(x)
    return x[len(x) // 2] if len(x) % 2 else 0.5 * (x[len(x) // 2 - 1] + x[len(x) // 2])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ns", default="2,4,8")
    ap.add_argument("--spp", type=int, default=4096)
    ap.add_argument("--width", type=int, default=3840)
    ap.add_argument("--height", type=int, default=2160)
    ap.add_argument("--scene", default=str(ROOT / "scenes/generated_scene.scene.json"))
    ap.add_argument("--partitions", default="rows:1,bands:8")
    ap.add_argument("--ssg", type=int, default=0, help="speculative sample groups: 0 = automatic, 1 = off")
    ap.add_argument("--runs", type=int, default=1,
                    help="warm launches per share: efficiency from the median of each rank (and the min/max spread)")
    a = ap.parse_args()
    global SSG, RUNS
    SSG, RUNS = a.ssg, a.runs
    fulls = run(a.width, a.height, 0, 1, 1, a.spp, a.scene)
    full = med(fulls)
    out = {"image": f"{a.width}x{a.height}", "spp": a.spp, "ssg_mode": a.ssg, "runs": a.runs, "full_ms": round(full, 2),
           "full_ms_runs": [round(x, 2) for x in fulls], "full_groups": GROUPS.get((1, 0), 0), "partitions": {}}
    for part in a.partitions.split(","):
        name, band = part.split(":")
        res = {}
        for n in [int(x) for x in a.ns.split(",")]:
            ranks = [run(a.width, a.height, r, n, int(band), a.spp, a.scene) for r in range(n)]
            meds = [med(x) for x in ranks]
            worst = max(meds)
            res[n] = {"rank_ms": [round(x, 2) for x in meds], "rank_ms_runs": [[round(v, 2) for v in x] for x in ranks],
                      "rank_ms_max": round(worst, 2), "ideal_ms": round(full / n, 2),
                      "efficiency": round(full / n / worst, 3), "speedup": round(full / worst, 2),
                      # spread: the slowest rank's time in the best and the worst of its runs
                      "efficiency_min": round(full / n / max(max(x) for x in ranks), 3),
                      "efficiency_max": round(full / n / max(min(x) for x in ranks), 3),
                      "groups": GROUPS.get((n, 0), 0)}
            print(json.dumps({name: {n: res[n]}}), flush=True)
        out["partitions"][name] = {"band_rows": int(band), "per_n": res}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
