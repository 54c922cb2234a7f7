"""Per-call GPU times of the reference's call loop (render(cam, 8, i == 0) per call) under run-ahead
modes (pt_set_run_ahead: 1 off, 3 make-but-never-use, 0 automatic),
interleaved rounds in one process; results cross-checked bit-identical.
    python tools/ahead_probe.py [--calls 32] [--modes 1,3,0] [--rounds 3]
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
ap.add_argument("--scene", default=str(ROOT / "scenes/generated_scene.scene.json"))
ap.add_argument("--width", type=int, default=1920)
ap.add_argument("--height", type=int, default=1080)
ap.add_argument("--calls", type=int, default=32)
ap.add_argument("--call-spp", type=int, default=8)
ap.add_argument("--modes", default="1,3,0")
ap.add_argument("--rounds", type=int, default=3)
a = ap.parse_args()
pt = pa.Pathtracer(a.width, a.height)
cam = pt.load_scene(a.scene)
st = pt.rng_state()
pt.render(cam, a.call_spp, True)                      # cost order from an 8-spp call
modes = [int(m) for m in a.modes.split(",")]
res = {m: [] for m in modes}
ref = None
ok = True
for r in range(a.rounds):
    for m in modes:
        pt.set_run_ahead(m)
        pt.set_rng_state(st)
        t = []
        for i in range(a.calls):
            pt.render(cam, a.call_spp, i == 0)
            t.append(pt.get_timing())
        res[m].append(t)
        acc = pt.accum().view(np.uint32).copy()
        if ref is None:
            ref = acc
        ok = ok and np.array_equal(acc, ref)
out = {"image": f"{a.width}x{a.height}", "calls": a.calls, "call_spp": a.call_spp, "bit_identical": bool(ok), "modes": {}}
for m in modes:
    t = np.array(res[m])                               # rounds x calls
    out["modes"][m] = {"first_call_ms": round(float(np.median(t[:, 0])), 3),
                       "later_call_ms_median": round(float(np.median(t[:, 1:])), 3),
                       "total_ms_median": round(float(np.median(t.sum(1))), 2)}
print(json.dumps(out))
