"""First-launch (cold) time of a one-shot render (GPU box): a fresh context renders the workload once
-- the built-in cost pre-pass, its sort and the launch in the pre-pass's order -- for several cold-start
settings (pt_set_cold_start: pre-pass spp, issue priority on the pre-pass order), then renders it
twice more (the order rebuilt from the cold launch), against a warm reference (cost order from a full
launch, graded priority).  Results are checked bit-identical across settings.
    python tools/cold_start.py [--width 1920 --height 1080 --spp 1024] [--settings 2:0,8:0,2:1,8:1]
"""
import argparse
import json
import pathlib
import sys

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import pathtracercuda_amd as pa  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--width", type=int, default=1920)
ap.add_argument("--height", type=int, default=1080)
ap.add_argument("--spp", type=int, default=1024)
ap.add_argument("--reps", type=int, default=2)
ap.add_argument("--settings", default="0:1,0:0,2:1,8:1,2:0")
ap.add_argument("--scene", default=str(ROOT / "scenes/generated_scene.scene.json"))
a = ap.parse_args()
samples = a.width * a.height * a.spp
res = {"image": f"{a.width}x{a.height}", "spp": a.spp, "runs": []}
ref = None
ok = True
for rep in range(a.reps):
    row = {}
    for tok in ["warm"] + a.settings.split(","):
        pt = pa.Pathtracer(a.width, a.height)
        cam = pt.load_scene(a.scene)
        st = pt.rng_state()
        if tok == "warm":
            for _ in range(2):                                # cold launch, then one that rebuilds the
                pt.render_raw(cam, 8, a.spp // 8, True)       # order without priority
                pt.set_rng_state(st)                          # (a state write keeps the order)
            ms = [pt.render_raw(cam, 8, a.spp // 8, True)]
        else:
            pre, prio = (int(x) for x in tok.split(":"))
            pt.set_cold_start(pre, bool(prio))            # 0:x = first call split off
            ms = [pt.render_raw(cam, 8, a.spp // 8, True)]   # gpu_ms includes the pre-pass
            acc = pt.accum().view(np.uint32).copy()
            if ref is None:
                ref = acc
            ok = ok and np.array_equal(acc, ref)
            for _ in range(3):
                pt.set_rng_state(st)
                ms.append(pt.render_raw(cam, 8, a.spp // 8, True))
        row[tok] = [round(m, 2) for m in ms]
        pt.close()
    res["runs"].append(row)
    print(json.dumps(row), flush=True)
res["bit_identical"] = bool(ok)
print(json.dumps(res))
