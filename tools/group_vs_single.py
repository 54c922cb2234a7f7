"""Same-process timing of the in-process device group (pt_group_*, one device) against a plain
context on the same image (1 GPU): does the group path cost anything beyond the gather?  Optionally
with torch imported first (its bundled HIP runtime then serves the process, as in bench.py's
single-GPU path).  Usage on the GPU box:
    python tools/group_vs_single.py [--torch 1] [--spp 1024] [--rounds 3]
"""
import argparse
import json
import pathlib
import sys

ap = argparse.ArgumentParser()
ap.add_argument("--torch", type=int, default=0)
ap.add_argument("--spp", type=int, default=1024)
ap.add_argument("--rounds", type=int, default=3)
a = ap.parse_args()
if a.torch:
    import torch  # noqa: F401  (loads torch/lib/libamdhip64.so before libpt_hip.so)
ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import pathtracercuda_amd as pa  # noqa: E402

W, H = 1920, 1080
scene = str(ROOT / "scenes/generated_scene.scene.json")
g = pa.Pathtracer(W, H, devices=[0])
s = pa.Pathtracer(W, H)
cam = g.load_scene(scene)
s.load_scene(scene)
for pt in (g, s):
    pt.render_raw(cam, 8, 2, True)          # cold start: cost order
res = {"group": [], "single": []}
for _ in range(a.rounds):
    for name, pt in (("group", g), ("single", s)):
        res[name].append(round(pt.render_raw(cam, 8, a.spp // 8, True), 2))
print(json.dumps({"torch_first": a.torch, "spp": a.spp, "kernel_ms": res,
                  "Msamples_s": {k: round(W * H * a.spp / min(v) / 1e3, 1) for k, v in res.items()}}))
