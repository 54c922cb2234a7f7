"""Short render of the bench scene for PC sampling / profiling: generated_scene at 1080p, one
launch of `--chunks` 8-spp render() calls with the default kernel variant (or --variant)."""
import argparse
import pathlib
import sys

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import pathtracercuda_amd as pa  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--scene", default=str(ROOT / "scenes/generated_scene.scene.json"))
ap.add_argument("--chunks", type=int, default=8)
ap.add_argument("--variant", type=int, default=0)
ap.add_argument("--launches", type=int, default=2)
a = ap.parse_args()
pt = pa.Pathtracer(1920, 1080)
cam = pt.load_scene(a.scene)
if a.variant:
    pt.set_kernel_variant(a.variant)
pt.render_raw(cam, 8, 1, True)                 # records tile costs
for _ in range(a.launches):
    ms = pt.render_raw(cam, 8, a.chunks, True)
    print(f"{ms:.2f} ms, {1920 * 1080 * 8 * a.chunks / ms / 1e3:.1f} Msamples/s", flush=True)
