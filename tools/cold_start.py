"""First-launch (cold) throughput of a one-shot render (GPU box): a fresh context renders the
workload once -- with the built-in cost pre-pass (default), with row-major tiles (pt_set_schedule 1,
round 1's cold behaviour), and warm (cost order from a previous launch of the same camera).
    python tools/cold_start.py [--width 1920 --height 1080 --spp 1024]
"""
import argparse
import json
import pathlib
import sys

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import pathtracercuda_amd as pa  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--width", type=int, default=1920)
ap.add_argument("--height", type=int, default=1080)
ap.add_argument("--spp", type=int, default=1024)
ap.add_argument("--reps", type=int, default=2)
ap.add_argument("--scene", default=str(ROOT / "scenes/generated_scene.scene.json"))
a = ap.parse_args()
samples = a.width * a.height * a.spp
res = {"image": f"{a.width}x{a.height}", "spp": a.spp, "runs": []}
for rep in range(a.reps):
    row = {}
    for mode in ("cold_prepass", "cold_row_major", "warm_sorted"):
        pt = pa.Pathtracer(a.width, a.height)
        cam = pt.load_scene(a.scene)
        if mode == "cold_row_major":
            pt.set_schedule(1)
        if mode == "warm_sorted":
            pt.render_raw(cam, 8, 1, True)
        ms = pt.render_raw(cam, 8, a.spp // 8, True)       # gpu_ms includes the pre-pass when it runs
        row[mode] = {"ms": round(ms, 2), "Msamples_s": round(samples / ms / 1e3, 1)}
        pt.close()
    res["runs"].append(row)
    print(json.dumps(row), flush=True)
print(json.dumps(res))
