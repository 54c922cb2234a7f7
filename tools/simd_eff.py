"""SIMD efficiency of each phase of the trace kernel (instrumented variant): lane-level events
divided by 64 x wave-level executions, cycle shares of the phases, and the leaf-round counters
(bench.lane_utilisation).  Usage: python tools/simd_eff.py [--scene ...] [--variants 40,...]"""
import argparse
import json
import pathlib
import sys

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import pathtracercuda_amd as pa  # noqa: E402
from bench import lane_utilisation  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--scene", default=str(ROOT / "scenes/generated_scene.scene.json"))
ap.add_argument("--width", type=int, default=1920)
ap.add_argument("--height", type=int, default=1080)
ap.add_argument("--variants", default="40")
ap.add_argument("--spp", type=int, default=8)
ap.add_argument("--chunks", type=int, default=1)
a = ap.parse_args()
if a.scene == "stress_100k":                       # C5's generated scene (bench.scene_path)
    import bench  # noqa: E402
    a.scene = bench.scene_path("stress_100k")
pt = pa.Pathtracer(a.width, a.height)
cam = pt.load_scene(a.scene)
res = {}
for v in [int(x) for x in a.variants.split(",")]:
    pt.set_kernel_variant(v)
    st = pt.render_instrumented(cam, a.spp, a.chunks, True)
    eff = {k: round(st[l] / (64.0 * st[w]), 3) if st[w] else None for k, l, w in [
        ("node", "node_tests", "wave_node_iters"), ("prim", "prim_tests", "wave_prim_iters"),
        ("hit_shade", "hits", "wave_hits"), ("sky", "sky_lookups", "wave_sky"), ("segment", "segments", "wave_segments")]}
    per_sample = {k: round(st[k] / st["samples"], 3) for k in ("node_tests", "prim_tests", "hits", "sky_lookups", "segments",
                                                                "wave_node_iters", "wave_prim_iters", "wave_hits", "wave_sky", "wave_segments")}
    tot = st["cycles_total"] or 1
    shares = {k: round(st[k] / tot, 3) for k in ("cycles_node_walk", "cycles_leaf_tests", "cycles_shading")}
    res[v] = {"simd_efficiency": eff, "per_sample": per_sample, "cycle_share": shares,
              "wave_cycles_per_sample": round(tot / st["samples"] * 64, 1),
              "lane_idle_after_pixel_done": round(st["cycles_lane_idle"] / (64.0 * tot), 3),
              "lane_utilisation": lane_utilisation(st)}
print(json.dumps({"scene": pathlib.Path(a.scene).name, "image": f"{a.width}x{a.height}", "spp": a.spp * a.chunks,
                  "variants": res}))
