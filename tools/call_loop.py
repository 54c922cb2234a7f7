"""The reference's headless loop unchanged (main.cpp:272-279: spp/8 separate render(cam, 8, i == 0)
calls, one synchronous launch each) against the same work as one chunked launch, for trace-kernel
variants, strip-unit settings (pt_set_strip_units) and run-ahead modes (pt_set_run_ahead), in one
process, interleaved rounds; results cross-checked bit-identical.
    python tools/call_loop.py [--variants 0] [--strips 1,2,4] [--aheads 0,1] [--spp 1024] [--rounds 3]
"""
import argparse
import json
import pathlib
import sys
import time

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import pathtracercuda_amd as pa  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--scene", default=str(ROOT / "scenes/generated_scene.scene.json"))
ap.add_argument("--width", type=int, default=1920)
ap.add_argument("--height", type=int, default=1080)
ap.add_argument("--spp", type=int, default=1024)
ap.add_argument("--rounds", type=int, default=3)
ap.add_argument("--variants", default="0")
ap.add_argument("--strips", default="1,2,4")
ap.add_argument("--aheads", default="1", help="run-ahead modes (0 automatic, 1 off, 2 always)")
ap.add_argument("--call-spp", type=int, default=8, help="spp per render() call")
ap.add_argument("--frames", type=int, default=0, help="also time this many 1-spp progressive frames per setting")
a = ap.parse_args()
pt = pa.Pathtracer(a.width, a.height)
cam = pt.load_scene(a.scene)
st = pt.rng_state()
settings = [(int(v), int(k), int(h)) for v in a.variants.split(",") for k in a.strips.split(",")
            for h in a.aheads.split(",")]
res = {f"{v}/k{k}/a{h}": {"loop_ms": [], "gpu_ms": [], "frame_ms": []} for v, k, h in settings}
ref = None
mismatches = []
for r in range(a.rounds):
    for v, k, h in settings:
        key = f"{v}/k{k}/a{h}"
        pt.set_kernel_variant(v)
        pt.set_strip_units(k)
        pt.set_run_ahead(h)
        pt.set_rng_state(st)
        t0 = time.perf_counter()
        g = 0.0
        for i in range(a.spp // a.call_spp):
            pt.render(cam, a.call_spp, i == 0)
            g += pt.get_timing()
        res[key]["loop_ms"].append((time.perf_counter() - t0) * 1e3)
        res[key]["gpu_ms"].append(g)
        acc = pt.accum().view(np.uint32)
        if ref is None:
            ref = acc.copy()
        if not np.array_equal(acc, ref):
            bad = np.argwhere((acc != ref).any(-1))
            mismatches.append({"setting": key, "round": r, "pixels": int(len(bad)),
                               "first": [int(x) for x in bad[0]], "got": [float(x) for x in acc[tuple(bad[0])].view(np.float32)],
                               "want": [float(x) for x in ref[tuple(bad[0])].view(np.float32)]})
        if a.frames:
            t0 = time.perf_counter()
            for f in range(a.frames):
                pt.render(cam, 1, f == 0)
            res[key]["frame_ms"].append((time.perf_counter() - t0) * 1e3 / a.frames)
pt.set_strip_units(0)
pt.set_run_ahead(1)
pt.set_kernel_variant(0)
pt.set_rng_state(st)
fused = []
for r in range(a.rounds):
    pt.set_rng_state(st)
    fused.append(pt.render_raw(cam, 8, a.spp // 8, True))
out = {"image": f"{a.width}x{a.height}", "spp": a.spp, "calls": a.spp // a.call_spp, "call_spp": a.call_spp, "fused_ms_median": float(np.median(fused)),
       "bit_identical": not mismatches, "mismatches": mismatches[:8], "settings": {}}
for key, d in res.items():
    m = float(np.median(d["loop_ms"]))
    out["settings"][key] = {"loop_ms_median": round(m, 2), "gpu_ms_median": round(float(np.median(d["gpu_ms"])), 2),
                            "loop_over_fused": round(m / out["fused_ms_median"], 4),
                            "Msamples_s": round(a.width * a.height * a.spp / m / 1e3, 1)}
    if d["frame_ms"]:
        out["settings"][key]["frame_ms_median"] = round(float(np.median(d["frame_ms"])), 4)
print(json.dumps(out))
if mismatches:
    sys.exit(3)
