"""Progressive (interactive) call pattern of the reference's windowed loop (main.cpp:298-437):
one render(camera, 1 spp, reset) per frame plus a tonemap into a device pixel buffer, optionally
with a camera move every K frames (which resets the accumulation, as the controls do).  Not the
headline bench (bench.py is); this reports what a viewer would see.  Usage on the GPU box:
    python tools/bench_progressive.py [--frames 200] [--move-every 0] [--width 1920 --height 1080]
"""
import argparse
import json
import pathlib
import sys
import time

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import torch  # noqa: E402,F401  (loads the HIP runtime first: one libamdhip64 for torch and the library)

import pathtracercuda_amd as pa  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default=str(ROOT / "scenes/generated_scene.scene.json"))
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--frames", type=int, default=200)
    ap.add_argument("--move-every", type=int, default=0, help="rotate the camera every K frames (0: never)")
    a = ap.parse_args()
    pt = pa.Pathtracer(a.width, a.height)
    cam = pt.load_scene(a.scene)
    pbo = torch.empty((a.height, a.width, 4), dtype=torch.uint8, device="cuda:0")
    for _ in range(3):                                   # warmup (also records the tile costs)
        pt.render(cam, 1, True)
        pt.tonemap_device(pbo.data_ptr(), pbo.numel())
    gpu_ms = 0.0
    reset = True
    t0 = time.perf_counter()
    for f in range(a.frames):
        if a.move_every and f % a.move_every == 0 and f > 0:
            pa.camera_rotate(cam, 0.0, 0.002, 0.0)
            reset = True
        pt.render(cam, 1, reset)
        gpu_ms += pt.get_timing()
        reset = False
        pt.tonemap_device(pbo.data_ptr(), pbo.numel())
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    samples = a.width * a.height * a.frames
    print(json.dumps({"mode": "progressive 1 spp/frame + device tonemap", "scene": pathlib.Path(a.scene).name,
                      "width": a.width, "height": a.height, "frames": a.frames, "move_every": a.move_every,
                      "ms_per_frame": round(wall * 1e3 / a.frames, 3), "fps": round(a.frames / wall, 1),
                      "kernel_ms_per_frame": round(gpu_ms / a.frames, 3),
                      "Msamples_s": round(samples / wall / 1e6, 1)}))


if __name__ == "__main__":
    main()
