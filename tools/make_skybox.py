"""Deterministic synthetic HDR environment map (stand-in for the reference's missing skybox.hdr).

The reference's generated_scene.json is lit only by "skybox.hdr", which is absent from the
reference checkout (.MISSING_LARGE_BLOBS:2), so the scene renders black without a substitute
(SURVEY.md fact 6).  This writes a 512x256 equirectangular Radiance RGBE file laid out the way the
reference samples it (trace.cu:120-130): v = acos(dir.y)/pi (row 0 = zenith), u = atan2(z, x)/2pi
(wrapped).  Content: a blue-to-white sky gradient, a dim brown ground below the horizon and a
warm sun lobe (peak radiance ~40).  Pure numpy float32 arithmetic, so the file is byte-identical
on every run; the committed copy is scenes/skybox.hdr.
"""
import pathlib
import sys

import numpy as np

W, H = 512, 256


def sky(width: int = W, height: int = H) -> np.ndarray:
    j = (np.arange(height, dtype=np.float64) + 0.5) / height
    i = (np.arange(width, dtype=np.float64) + 0.5) / width
    theta = np.pi * j[:, None]                 # 0 = up
    phi = 2.0 * np.pi * (i[None, :] - 0.5)     # u = phi / 2pi wrapped to [0, 1)
    dy = np.cos(theta)
    dx = np.sin(theta) * np.cos(phi)
    dz = np.sin(theta) * np.sin(phi)
    up = np.clip(dy, 0.0, 1.0)
    zenith = np.array([0.25, 0.45, 0.95])
    horizon = np.array([1.10, 1.10, 1.05])
    t = up[..., None] ** 0.5
    rgb = horizon * (1.0 - t) + zenith * t
    ground = np.array([0.22, 0.18, 0.14]) * (1.0 - 0.5 * np.clip(-dy, 0.0, 1.0))[..., None]
    rgb = np.where((dy >= 0.0)[..., None], rgb, ground)
    # sun: elevation 40 deg, azimuth chosen so it lights generated_scene's camera side
    el, az = np.radians(40.0), np.radians(25.0)
    s = np.array([np.cos(el) * np.cos(az), np.sin(el), np.cos(el) * np.sin(az)])
    cosang = dx * s[0] + dy * s[1] + dz * s[2]
    lobe = np.exp((cosang - 1.0) / 0.0015)      # ~3 deg core
    glow = np.exp((cosang - 1.0) / 0.05)        # wide halo
    rgb = rgb + (40.0 * lobe + 1.5 * glow)[..., None] * np.array([1.0, 0.92, 0.80])
    return rgb.astype(np.float32)


def to_rgbe(rgb: np.ndarray) -> np.ndarray:
    rgb = rgb.astype(np.float64)
    v = rgb.max(axis=-1)
    m, e = np.frexp(v)
    scale = np.where(v > 1e-32, m * 256.0 / np.where(v > 1e-32, v, 1.0), 0.0)
    out = np.zeros(rgb.shape[:-1] + (4,), dtype=np.uint8)
    out[..., :3] = np.floor(rgb * scale[..., None]).clip(0, 255).astype(np.uint8)
    out[..., 3] = np.where(v > 1e-32, e + 128, 0).astype(np.uint8)
    return out


def write_hdr(path: pathlib.Path, rgb: np.ndarray) -> None:
    h, w, _ = rgb.shape
    header = f"#?RADIANCE\nFORMAT=32-bit_rle_rgbe\n\n-Y {h} +X {w}\n".encode()
    path.write_bytes(header + to_rgbe(rgb).tobytes())


def main() -> int:
    out = pathlib.Path(sys.argv[1]) if len(sys.argv) > 1 else pathlib.Path(__file__).resolve().parents[1] / "scenes" / "skybox.hdr"
    write_hdr(out, sky())
    print(f"wrote {out}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
