"""How often the rising-t_max rebuild runs on a real workload (VERDICT r04 "do this" 1): one
instrumented launch of the default kernel (pt_render_instrumented; `repairs` = leaf rounds whose
sphere test raised t_max, Hittable.inl:152-158, and rebuilt the pending far children) against the
oracle's count of leaf visits that raise t_max over the same samples (the reference's hitBVH,
trace.cu:48-98, restated in oracle/pt_oracle.c).  Both walks visit the same leaves in the same order,
so the two counts must be equal.
    python tools/rise_count.py [--scene generated_scene] [--width 1920 --height 1080 --spp 8 --chunks 12]
"""
import argparse
import json
import pathlib
import sys
import time

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import pathtracercuda_amd as pa  # noqa: E402
from oracle import pyoracle as po  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--scene", default="generated_scene")
ap.add_argument("--width", type=int, default=1920)
ap.add_argument("--height", type=int, default=1080)
ap.add_argument("--spp", type=int, default=8)
ap.add_argument("--chunks", type=int, default=12)
ap.add_argument("--oracle", type=int, default=1)
a = ap.parse_args()
path = ROOT / "scenes" / f"{a.scene}.scene.json"
pt = pa.Pathtracer(a.width, a.height)
cam = pt.load_scene(str(path))
st = pt.render_instrumented(cam, a.spp, a.chunks, True)
out = {"scene": a.scene, "image": f"{a.width}x{a.height}", "spp": a.spp * a.chunks,
       "samples": st["samples"], "segments": st["segments"], "wave_leaf_rounds": st["leaf_rounds"],
       "repairs": st["repairs"], "repairs_per_Msample": round(st["repairs"] / st["samples"] * 1e6, 3)}
if a.oracle:
    osc = po.load_scene(path, a.width, a.height)
    ref = po.OracleRenderer(osc, a.width, a.height, fast=True)
    t0 = time.perf_counter()
    ref.render(osc.camera, a.spp, True, chunks=a.chunks, collect_stats=True)
    out.update({"oracle_rises": int(ref.stats[7]), "oracle_s": round(time.perf_counter() - t0, 1),
                "counts_equal": int(ref.stats[7]) == st["repairs"]})
    import numpy as np
    out["accum_bitexact"] = bool(np.array_equal(pt.accum().view(np.uint32), ref.accum.view(np.uint32)))
print(json.dumps(out))
