"""Single-GPU estimate of strong-scaling efficiency: renders one rank's share of the bench image
(rows y = r + k*N, exactly what rank r renders in `bench.py --gpus N`) and compares its time with
1/N of the full-frame time.  Usage on the GPU box:
    python tools/scale_sim.py [--ns 1,2,4,8] [--spp 1024]
"""
import argparse
import json
import pathlib
import sys

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import pathtracercuda_amd as pa  # noqa: E402


def run(W, H, off, stride, spp, scene, schedule):
    pt = pa.Pathtracer(W, H, row_offset=off, row_stride=stride)
    pt.set_schedule(schedule)
    cam = pt.load_scene(scene)
    pt.render_raw(cam, 8, 1, True)                       # records tile costs -> sorted order
    ms = [pt.render_raw(cam, 8, spp // 8, True) for _ in range(2)]
    return min(ms)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ns", default="1,2,4,8")
    ap.add_argument("--spp", type=int, default=1024)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--scene", default=str(ROOT / "scenes/generated_scene.scene.json"))
    ap.add_argument("--schedule", type=int, default=0, help="pt_set_schedule mode (0 sorted tiles, 2 scattered)")
    a = ap.parse_args()
    full = run(a.width, a.height, 0, 1, a.spp, a.scene, a.schedule)
    out = {"schedule": a.schedule, "full_ms": round(full, 2), "per_n": {}}
    for n in [int(x) for x in a.ns.split(",")]:
        worst = max(run(a.width, a.height, r, n, a.spp, a.scene, a.schedule) for r in ([0, n - 1] if n > 1 else [0]))
        out["per_n"][n] = {"rank_ms_max": round(worst, 2), "ideal_ms": round(full / n, 2),
                           "efficiency": round(full / n / worst, 3)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
