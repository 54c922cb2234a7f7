"""One timed launch of a bench workload with a chosen trace-kernel variant (for rocprofv3 --pmc
passes and A/Bs on the GPU box):
    python tools/one_launch.py --variant 46 [--width 1920 --height 1080 --spp 1024 --scene generated_scene]
"""
import argparse
import json
import pathlib
import sys

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import pathtracercuda_amd as pa  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--variant", type=int, default=0)
ap.add_argument("--width", type=int, default=1920)
ap.add_argument("--height", type=int, default=1080)
ap.add_argument("--spp", type=int, default=1024)
ap.add_argument("--reps", type=int, default=1)
ap.add_argument("--scene", default="generated_scene")
a = ap.parse_args()
pt = pa.Pathtracer(a.width, a.height)
cam = pt.load_scene(str(ROOT / "scenes" / f"{a.scene}.scene.json"))
pt.set_kernel_variant(a.variant)
pt.render_raw(cam, 8, 1, True)                 # records the tile costs: later launches run cost-sorted
for _ in range(a.reps):
    ms = pt.render_raw(cam, 8, a.spp // 8, True)
    print(json.dumps({"variant": a.variant, "ms": round(ms, 3),
                      "Msamples_s": round(a.width * a.height * a.spp / ms / 1e3, 1)}), flush=True)
pt.close()
