"""Compare our render with the reference's published 8-bit render, pixel for pixel (GPU box).

The reference's cornell_box_4096spp.png was made by its windowed loop: render(cam, 1, false) once
per frame (main.cpp:387-399), tonemap by the frame count (tonemap.cu:16-26).  Per pixel the sample
sequence is the pixel's own XORWOW stream, so the same loop here draws the same random numbers; the
remaining differences are the reference's floating point (nvcc FMA contraction, libdevice
transcendentals, the texture unit), which can send an individual path elsewhere.
    python tools/pin_png.py [--scene cornell_box --spp 4096 --out gpurun_out/pin]
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
ap.add_argument("--scene", default="cornell_box", choices=["cornell_box"])
ap.add_argument("--spp", type=int, default=4096)
ap.add_argument("--per-call", type=int, default=1, help="spp per render() call (1 = the windowed loop)")
ap.add_argument("--out", default="gpurun_out/pin")
ap.add_argument("--corr", action="store_true", help="print the path-level pin of tests/pin.py as JSON and exit")
a = ap.parse_args()
if a.corr:
    sys.path.insert(0, str(ROOT / "tests"))
    import pin  # noqa: E402
    print(json.dumps(pin.reference_pin(ROOT, ROOT / "scenes")))
    sys.exit(0)
ref = np.load(ROOT / "tests" / "golden" / f"{a.scene}_4096spp_ref8.npz")["rgb"].astype(np.int16)
H, W, _ = ref.shape
pt = pa.Pathtracer(W, H)
cam = pt.load_scene(str(ROOT / "scenes" / f"{a.scene}.scene.json"))
pt.render(cam, a.per_call, False, chunks=a.spp // a.per_call)
ours = pt.tonemap(a.spp)[..., :3].astype(np.int16)
d = ours - ref
ad = np.abs(d).max(-1)
out = pathlib.Path(a.out)
out.mkdir(parents=True, exist_ok=True)
np.savez_compressed(out / f"{a.scene}_diff.npz", d=d.astype(np.int8), ours=ours.astype(np.uint8),
                    accum=pt.accum()[..., :3])
res = {"scene": a.scene, "image": f"{W}x{H}", "spp": a.spp, "per_call": a.per_call,
       "frac_equal": float((ad == 0).mean()), "frac_le1": float((ad <= 1).mean()),
       "frac_le2": float((ad <= 2).mean()), "frac_le8": float((ad <= 8).mean()),
       "mean_signed_rgb": [float(x) for x in d.reshape(-1, 3).mean(0)],
       "mean_abs_rgb": [float(x) for x in np.abs(d).reshape(-1, 3).mean(0)]}
print(json.dumps(res))
