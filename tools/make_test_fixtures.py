"""Deterministic test fixtures (committed outputs):
  scenes/test_shapes.scene.json  every shape type x every material type, textured quad / disk /
                                 sphere / cylinder, an emissive light, metals, roughness extremes,
                                 a JSON-integer roughness (ignored by the loader, SceneLoader.cpp:165),
                                 an unknown material string, skybox lighting;
  scenes/checker.png             64x32 RGB texture standing in for the reference's missing earth.png;
  scenes/rise_repair.scene.json  the camera and every object inside one large emissive sphere, with
                                 overlapping spheres and boxes: nearly every ray starts inside a
                                 sphere, so the sphere test's far-root quirk (Hittable.inl:152-158,
                                 t1 accepted beyond t_max when t0 <= t_min) raises t_max in mid
                                 traversal and the reference then tests popped boxes at the larger
                                 value (trace.cu:48-98) -- the case repair_pending exists for;
  scenes/rise_pair.scene.json    three objects -- a dome sphere around the camera, a sphere A and a
                                 back wall B behind it -- for the caller BVH of tests/bvh_edit.py
                                 rise_pair_bvh(), in which every ray that hits A raises t_max at the
                                 dome's leaf with B's leaf dropped by the hit-now rule: the pixels of
                                 A then differ unless the pending set is rebuilt.
"""
import json
import pathlib
import struct
import sys
import zlib

ROOT = pathlib.Path(__file__).resolve().parents[1]
SHAPES = ["SPHERE", "CYLINDER", "DISK", "CONE", "PARABOLOID", "QUAD", "CUBE"]
MATS = ["LAMBERT", "GGX", "LAMBERT_GGX"]


def checker_png(path: pathlib.Path, w: int = 64, h: int = 32) -> None:
    rows = []
    for y in range(h):
        row = bytearray([0])
        for x in range(w):
            c = ((x // 8) + (y // 8)) % 2
            r = 40 + 200 * c
            g = (x * 255) // (w - 1)
            b = (y * 255) // (h - 1)
            row += bytes([r, g, b])
        rows.append(bytes(row))
    raw = b"".join(rows)

    def chunk(t, d):
        return struct.pack(">I", len(d)) + t + d + struct.pack(">I", zlib.crc32(t + d) & 0xFFFFFFFF)

    png = b"\x89PNG\r\n\x1a\n" + chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, 8, 2, 0, 0, 0))
    png += chunk(b"IDAT", zlib.compress(raw, 9)) + chunk(b"IEND", b"")
    path.write_bytes(png)


def obj(t, pos, rot, scale, mtype, base, emissive=(0.0, 0.0, 0.0), rough=0.5, metal=0.0, tex=""):
    return {"type": t, "position": list(pos), "rotation": list(rot), "scale": list(scale),
            "material": {"type": mtype, "baseColor": list(base), "emissive": list(emissive),
                         "roughness": rough, "metalness": metal, "texture": tex}}


def scene() -> dict:
    objs = [obj("QUAD", (0.0, 0.0, 0.0), (0.0, 0.0, 0.0), (12.0, 12.0, 12.0), "LAMBERT", (0.8, 0.8, 0.8))]
    for i, s in enumerate(SHAPES):
        for j, m in enumerate(MATS):
            x = -4.5 + 1.5 * i
            z = -2.0 + 1.6 * j
            rot = (15.0 * j, 30.0 * i + 10.0, -20.0 * (i % 3))
            sc = (0.45, 0.55 if s not in ("DISK", "QUAD") else 1.0, 0.45)
            base = (0.2 + 0.1 * i, 0.9 - 0.1 * i, 0.3 + 0.2 * j)
            rough = [0.02, 0.3, 0.75][(i + j) % 3]
            metal = 1.0 if (i + j) % 2 else 0.0
            objs.append(obj(s, (x, 0.6, z), rot, sc, m, base, rough=rough, metal=metal))
    objs.append(obj("SPHERE", (0.0, 1.6, -3.5), (0.0, 30.0, 0.0), (0.8, 0.8, 0.8), "LAMBERT_GGX", (1.0, 1.0, 1.0), rough=0.2, tex="checker.png"))
    objs.append(obj("CYLINDER", (2.5, 1.2, -3.5), (10.0, 0.0, 5.0), (0.4, 0.8, 0.4), "LAMBERT", (1.0, 1.0, 1.0), tex="checker.png"))
    objs.append(obj("QUAD", (-2.5, 1.2, -3.8), (80.0, 0.0, 0.0), (0.8, 1.0, 0.6), "LAMBERT", (1.0, 1.0, 1.0), tex="checker.png"))
    objs.append(obj("DISK", (-4.0, 0.02, 2.5), (0.0, 0.0, 0.0), (0.7, 1.0, 0.7), "GGX", (1.0, 1.0, 1.0), rough=0.4, metal=1.0, tex="checker.png"))
    objs.append(obj("SPHERE", (3.5, 2.5, 1.5), (0.0, 0.0, 0.0), (0.3, 0.3, 0.3), "LAMBERT", (1.0, 1.0, 1.0), emissive=(8.0, 6.0, 4.0)))
    o = obj("CUBE", (4.0, 0.5, 2.5), (0.0, 45.0, 0.0), (0.5, 0.5, 0.5), "LAMBERT_GGX", (0.9, 0.5, 0.1), metal=1.0)
    o["material"]["roughness"] = 1          # JSON integer: ignored (default 0.5 kept)
    objs.append(o)
    o = obj("SPHERE", (-4.0, 0.5, -3.0), (0.0, 0.0, 0.0), (0.5, 0.5, 0.5), "PLASTIC", (0.3, 0.6, 0.9))
    objs.append(o)                          # unknown material string: LAMBERT kept
    return {"camera": {"position": [0.5, 4.0, 9.0], "look_at": [0.0, 0.5, -0.5], "fovy": 45.0},
            "skybox": "skybox.hdr", "objects": objs}


def rise_scene() -> dict:
    objs = [obj("SPHERE", (0.0, 1.0, 0.0), (0.0, 0.0, 0.0), (6.0, 6.0, 6.0), "LAMBERT", (0.7, 0.7, 0.8),
                emissive=(0.6, 0.6, 0.7)),
            obj("QUAD", (0.0, 0.0, 0.0), (0.0, 0.0, 0.0), (3.0, 3.0, 3.0), "LAMBERT", (0.8, 0.8, 0.8))]
    for i in range(4):
        for j in range(3):
            x = -1.8 + 1.2 * i
            z = -1.5 + 1.2 * j
            r = 0.25 + 0.05 * ((i + j) % 3)
            m = MATS[(i + 2 * j) % 3]
            base = (0.3 + 0.15 * i, 0.8 - 0.2 * j, 0.4 + 0.1 * (i + j) % 0.5)
            shape = "SPHERE" if (i + j) % 2 == 0 else "CUBE"
            objs.append(obj(shape, (x, r + 0.05 * j, z), (0.0, 20.0 * i, 10.0 * j), (r, r, r), m, base,
                            rough=[0.1, 0.4, 0.8][j], metal=float((i + j) % 2)))
    # overlapping pairs: a sphere cut by a box and a sphere around a smaller one (rays start inside)
    objs.append(obj("SPHERE", (0.6, 0.9, 1.4), (0.0, 0.0, 0.0), (0.6, 0.6, 0.6), "GGX", (0.9, 0.9, 0.9), rough=0.3, metal=1.0))
    objs.append(obj("CUBE", (0.9, 0.7, 1.6), (0.0, 35.0, 0.0), (0.35, 0.35, 0.35), "LAMBERT", (0.9, 0.3, 0.2)))
    objs.append(obj("SPHERE", (-0.9, 1.2, 0.8), (0.0, 0.0, 0.0), (0.9, 0.9, 0.9), "LAMBERT_GGX", (0.4, 0.6, 0.9), rough=0.2))
    objs.append(obj("SPHERE", (-0.9, 1.2, 0.8), (0.0, 0.0, 0.0), (0.3, 0.3, 0.3), "LAMBERT", (1.0, 1.0, 1.0), emissive=(4.0, 3.0, 2.0)))
    objs.append(obj("CYLINDER", (1.8, 0.8, -0.4), (0.0, 0.0, 0.0), (0.3, 0.8, 0.3), "LAMBERT", (0.5, 0.9, 0.5)))
    return {"camera": {"position": [0.0, 1.3, 4.0], "look_at": [0.0, 0.6, 0.0], "fovy": 50.0}, "objects": objs}


def rise_pair_scene() -> dict:
    return {"camera": {"position": [0.0, 1.0, 4.0], "look_at": [0.0, 1.0, 0.0], "fovy": 45.0},
            "objects": [obj("SPHERE", (0.0, 1.0, 0.0), (0.0, 0.0, 0.0), (8.0, 8.0, 8.0), "LAMBERT", (0.6, 0.6, 0.7),
                            emissive=(0.5, 0.5, 0.6)),
                        obj("SPHERE", (0.0, 1.0, 0.0), (0.0, 0.0, 0.0), (0.6, 0.6, 0.6), "LAMBERT", (0.9, 0.2, 0.2)),
                        obj("QUAD", (0.0, 1.0, -2.0), (-90.0, 0.0, 0.0), (3.0, 3.0, 3.0), "LAMBERT", (0.2, 0.8, 0.3),
                            emissive=(0.2, 0.6, 0.2))]}


def main() -> int:
    checker_png(ROOT / "scenes" / "checker.png")
    (ROOT / "scenes" / "test_shapes.scene.json").write_text(json.dumps(scene(), indent=1) + "\n")
    (ROOT / "scenes" / "rise_repair.scene.json").write_text(json.dumps(rise_scene(), indent=1) + "\n")
    (ROOT / "scenes" / "rise_pair.scene.json").write_text(json.dumps(rise_pair_scene(), indent=1) + "\n")
    print("wrote scenes/checker.png, scenes/test_shapes.scene.json, scenes/rise_repair.scene.json, "
          "scenes/rise_pair.scene.json")
    return 0


if __name__ == "__main__":
    sys.exit(main())
