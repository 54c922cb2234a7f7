"""Seeded generator of the deep-BVH stress scene (BASELINE.json config C5: "100k random quadrics").

Mirrors the layout of the reference's generateSceneFile (SceneLoader.cpp:94-114) on a larger grid:
a floor quad, then for every grid cell (a, b) one object at (a + 0.9 U, 0.2, b + 0.9 U) with a
uniformly chosen shape (0..6), LAMBERT_GGX, albedo U*U, roughness U, metalness U > 0.5, scale 0.2;
camera and sky as generated_scene.json.  The reference draws from std::default_random_engine
(implementation-defined), so this uses numpy's PCG64 with a fixed seed: the scene is deterministic
but not the reference's draw sequence.  grid=317 gives 100,489 objects (~40 MB of JSON), so the
file is generated on demand (tests, bench) instead of being committed.

    python tools/make_stress_scene.py [out.json] [--grid 317] [--seed 1984]
"""
import argparse
import json
import pathlib
import sys

import numpy as np

SHAPES = ["SPHERE", "CYLINDER", "DISK", "CONE", "PARABOLOID", "QUAD", "CUBE"]


def make_scene(grid: int = 317, seed: int = 1984, skybox: str = "skybox.hdr") -> dict:
    rng = np.random.default_rng(seed)
    half = grid // 2
    n = grid * grid
    u = rng.random((n, 11), dtype=np.float32)
    a, b = np.meshgrid(np.arange(-half, grid - half), np.arange(-half, grid - half), indexing="ij")
    a = a.ravel().astype(np.float32)
    b = b.ravel().astype(np.float32)
    cx = a + np.float32(0.9) * u[:, 0]
    cz = b + np.float32(0.9) * u[:, 1]
    albedo = u[:, 2:5] * u[:, 5:8]
    metal = np.where(u[:, 8] > 0.5, 1.0, 0.0)
    rough = u[:, 9]
    shape = np.minimum((u[:, 10] * 7).astype(int), 6)
    objs = [{"type": "QUAD", "position": [0.0, 0.0, 0.0], "rotation": [0.0, 0.0, 0.0],
             "scale": [float(half + 2)] * 3,
             "material": {"type": "LAMBERT", "baseColor": [1.0, 1.0, 1.0], "emissive": [0.0, 0.0, 0.0],
                          "roughness": 1.0, "metalness": 0.0, "texture": ""}}]
    for i in range(n):
        objs.append({"type": SHAPES[shape[i]], "position": [float(cx[i]), 0.2, float(cz[i])],
                     "rotation": [0.0, 0.0, 0.0], "scale": [0.2, 0.2, 0.2],
                     "material": {"type": "LAMBERT_GGX",
                                  "baseColor": [float(x) for x in albedo[i]],
                                  "emissive": [0.0, 0.0, 0.0], "roughness": float(rough[i]),
                                  "metalness": float(metal[i]), "texture": ""}})
    return {"camera": {"position": [13.0, 2.0, 3.0], "look_at": [0.0, 0.0, 0.0], "fovy": 60.0},
            "skybox": skybox, "objects": objs}


def write_scene(path: pathlib.Path, grid: int = 317, seed: int = 1984, skybox: str = "skybox.hdr") -> pathlib.Path:
    path = pathlib.Path(path)
    path.write_text(json.dumps(make_scene(grid, seed, skybox), separators=(",", ":")))
    return path


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("out", nargs="?", default="stress_100k.scene.json")
    ap.add_argument("--grid", type=int, default=317)
    ap.add_argument("--seed", type=int, default=1984)
    ap.add_argument("--skybox", default=str(pathlib.Path(__file__).resolve().parents[1] / "scenes" / "skybox.hdr"))
    a = ap.parse_args()
    p = write_scene(pathlib.Path(a.out), a.grid, a.seed, a.skybox)
    print(f"wrote {p} ({a.grid * a.grid + 1} objects)")
    return 0


if __name__ == "__main__":
    sys.exit(main())
