"""Analytic known-answer tests (KATs) for the features the reference's published render cannot pin.

Both the GPU kernel and the oracle are checked against these.  The expected values here come from
numerical integration in float64 of formulas restated from the reference's source.  They share
no code with the oracle (oracle/pt_oracle.c) or the kernel:
  * sky lookup: camera ray (Camera.inl:4-62, trace.cu:190-192), spherical mapping
    (trace.cu:120-130), CUDA bilinear filtering with wrap in u and clamp in v (Pathtracer.cpp:275-279);
    the per-pixel expectation over the jittered footprint is a 2-D midpoint quadrature;
  * white furnace: a flat GGX or Lambert+GGX quad under a uniform sky of radiance 1.  The pixel
    expectation is the directional albedo integral of the reference's BRDF (brdf.h:11-72,
    Material.inl:74-144) over the upper hemisphere.  VNDF sampling with the pdf of
    MonteCarlo.h:107-114 is an unbiased estimator of that integral, so this checks the sampler,
    the pdf and the weight (trace.cu:150) together.
The test scenes are written as JSON + Radiance RGBE files into a temporary directory.
"""
from __future__ import annotations

import json
import math
import pathlib

import numpy as np


# ---- Radiance RGBE (flat scanlines; decode as stb_image does: m * 2^(e - 136)) ---------------
def write_rgbe(path: pathlib.Path, rgb: np.ndarray) -> np.ndarray:
    """Write float RGB (h x w x 3) as flat RGBE; returns the texel values a decoder reads back."""
    h, w, _ = rgb.shape
    mx = rgb.max(-1)
    e = np.where(mx > 0, np.floor(np.log2(np.maximum(mx, 1e-30))) + 1, -128).astype(np.int64)
    scale = np.ldexp(1.0, (8 - e).astype(np.int64))
    m = np.clip(np.floor(rgb * scale[..., None]), 0, 255).astype(np.uint8)
    ebyte = np.where(mx > 0, e + 128, 0).astype(np.uint8)
    data = np.concatenate([m, ebyte[..., None]], -1)
    # a flat scanline must not start with the RLE marker (2, 2): keep the first red byte != 2
    assert not ((data[:, 0, 0] == 2) & (data[:, 0, 1] == 2)).any()
    with open(path, "wb") as f:
        f.write(b"#?RADIANCE\nFORMAT=32-bit_rle_rgbe\n\n" + f"-Y {h} +X {w}\n".encode())
        f.write(data.tobytes())
    return decode_rgbe(data)


def decode_rgbe(data: np.ndarray) -> np.ndarray:
    e = data[..., 3].astype(np.int64)
    f = np.where(e > 0, np.ldexp(1.0, e - 136), 0.0)
    return data[..., :3].astype(np.float64) * f[..., None]


# ---- scenes --------------------------------------------------------------------------------
def write_scene(path: pathlib.Path, objects, camera, skybox: str) -> pathlib.Path:
    path.write_text(json.dumps({"camera": camera, "skybox": skybox, "objects": objects}))
    return path


def material(mtype="LAMBERT", base=(1.0, 1.0, 1.0), rough=1.0, metal=0.0, emissive=(0.0, 0.0, 0.0)):
    return {"type": mtype, "baseColor": list(base), "emissive": list(emissive), "roughness": rough,
            "metalness": metal, "texture": ""}


def obj(kind, pos=(0.0, 0.0, 0.0), rot=(0.0, 0.0, 0.0), scale=(1.0, 1.0, 1.0), mat=None):
    return {"type": kind, "name": "", "position": list(pos), "rotation": list(rot), "scale": list(scale),
            "material": mat or material()}


# ---- camera (Camera.inl:4-62) in float64 ----------------------------------------------------
def camera_dirs(position, look_at, fovy_deg, W, H, sx, sy):
    """Unit ray directions for image-plane coordinates s = (x + sx)/W, t = (y + sy)/H, for every pixel
    (H x W) and every sub-pixel offset pair (sx, sy) (broadcast)."""
    p = np.asarray(position, float)
    back = p - np.asarray(look_at, float)
    back /= np.linalg.norm(back)
    right = np.cross([0.0, 1.0, 0.0], back)
    right /= np.linalg.norm(right)
    up = np.cross(back, right)
    hh = math.tan(math.radians(fovy_deg) * 0.5)
    hw = (W / H) * hh
    llc = -hw * right - hh * up - back
    s = (np.arange(W)[None, :, None] + np.asarray(sx)[None, None, :]) / W
    t = (np.arange(H)[:, None, None] + np.asarray(sy)[None, None, :]) / H
    d = llc + s[..., None] * (2 * hw * right) + t[..., None] * (2 * hh * up)
    return d / np.linalg.norm(d, axis=-1, keepdims=True)


# ---- sky lookup (trace.cu:120-130) + CUDA linear filter (wrap u, clamp v) ---------------------
def sky_lookup(tex: np.ndarray, d: np.ndarray) -> np.ndarray:
    h, w, _ = tex.shape
    theta = np.arccos(np.clip(d[..., 1], -1.0, 1.0))
    phi = np.arctan2(d[..., 2], d[..., 0])
    u = phi / (2 * np.pi)
    v = theta / np.pi
    x = u * w - 0.5
    y = v * h - 0.5
    x0 = np.floor(x)
    y0 = np.floor(y)
    a = (x - x0)[..., None]
    b = (y - y0)[..., None]
    i0 = np.mod(x0.astype(np.int64), w)
    i1 = np.mod(i0 + 1, w)
    j0 = np.clip(y0.astype(np.int64), 0, h - 1)
    j1 = np.clip(y0.astype(np.int64) + 1, 0, h - 1)
    return ((1 - a) * (1 - b) * tex[j0, i0] + a * (1 - b) * tex[j0, i1]
            + (1 - a) * b * tex[j1, i0] + a * b * tex[j1, i1])


def sky_pixel_expectation(tex, position, look_at, fovy_deg, W, H, q=24):
    """Mean and per-sample standard deviation of the sky seen through each pixel's footprint."""
    g = (np.arange(q) + 0.5) / q
    sx = np.repeat(g, q)
    sy = np.tile(g, q)
    d = camera_dirs(position, look_at, fovy_deg, W, H, sx, sy)
    c = sky_lookup(tex, d)                          # H x W x q^2 x 3
    return c.mean(axis=2), c.std(axis=2)


def sky_test_texture(w=64, h=32) -> np.ndarray:
    """Asymmetric in u and v, so a flipped or shifted mapping shows: red ramps with u, green with v,
    blue is a smooth bump at (u, v) = (0.3, 0.35)."""
    u = (np.arange(w) + 0.5) / w
    v = (np.arange(h) + 0.5) / h
    U, V = np.meshgrid(u, v)
    r = 0.2 + 1.5 * U
    gch = 0.1 + 2.0 * V
    b = 0.3 + 3.0 * np.exp(-((U - 0.3) ** 2 + (V - 0.35) ** 2) / 0.01)
    return np.stack([r, gch, b], -1)


# ---- GGX directional albedo (brdf.h, Material.inl) ------------------------------------------
def _d_ggx(nh, a2):
    d = (nh * a2 - nh) * nh + 1.0
    return a2 / (np.pi * d * d)


def _vis(nv, nl, a2):
    gv = nl * np.sqrt((-nv * a2 + nv) * nv + a2)
    gl = nv * np.sqrt((-nl * a2 + nl) * nl + a2)
    return 0.5 / (gv + gl + 1e-5)


def _pow5(x):
    return x ** 5


def directional_albedo(mu: float, roughness: float, mtype: str, base: float = 1.0, metal: float = 1.0,
                       n_theta: int = 3000, n_phi: int = 720) -> float:
    """E[weight] for one view direction: integral of f(V, L) * L.z over the upper hemisphere, with the
    reference's BRDF (including its 1e-5 terms); the integral runs over half vectors H (dL = 4 V.H dH)
    with a GGX-adapted theta grid, so the lobe is resolved at any roughness."""
    rough = max(roughness, 0.04)                        # Material.inl:13
    a = rough * rough
    a2 = a * a
    V = np.array([math.sqrt(max(0.0, 1 - mu * mu)), 0.0, mu])
    # theta_H = atan(a * tan(pi/2 * s)), s in (0, 1): midpoint rule in s
    s = (np.arange(n_theta) + 0.5) / n_theta
    ts = np.tan(0.5 * np.pi * s)
    th = np.arctan(a * ts)
    dth = a * (0.5 * np.pi) * (1 + ts * ts) / (1 + (a * ts) ** 2) / n_theta
    ph = (np.arange(n_phi) + 0.5) / n_phi * 2 * np.pi
    dph = 2 * np.pi / n_phi
    TH, PH = np.meshgrid(th, ph, indexing="ij")
    Hh = np.stack([np.sin(TH) * np.cos(PH), np.sin(TH) * np.sin(PH), np.cos(TH)], -1)
    vh = Hh @ V
    L = 2 * vh[..., None] * Hh - V
    ok = (vh > 0) & (L[..., 2] > 0)
    nl = np.clip(L[..., 2], 0, 1)
    nh = np.clip(Hh[..., 2], 0, 1)
    vhc = np.clip(vh, 0, 1)
    nv = abs(V[2]) + 1e-5
    F0 = 0.04 + (base - 0.04) * metal                    # lerp(0.04, base, metal)
    p5 = _pow5(1 - vhc)
    F = p5 + F0 * (1 - p5)
    spec = _d_ggx(nh, a2) * _vis(nv, nl, a2) * F
    f = spec if mtype == "GGX" else (base / np.pi) * (1 - metal) + spec
    jac = 4 * vhc                                        # dL = 4 (V.H) dH
    dH = np.sin(TH) * dth[:, None] * dph
    return float(np.sum(np.where(ok, f * nl * jac * dH, 0.0)))


# ---- the KAT cases, shared by the oracle (CPU) and GPU tests --------------------------------
SKY_CAM = {"position": [0.0, 0.0, 0.0], "look_at": [0.3, 0.2, 1.0], "fovy": 90.0}
FURNACE_CAM = {"position": [0.0, 1.0, 1.0], "look_at": [0.0, 0.0, 0.0], "fovy": 2.0}
FURNACE_CASES = [("GGX", 0.3, 1.0), ("GGX", 0.6, 1.0), ("GGX", 1.0, 1.0), ("LAMBERT_GGX", 0.5, 0.0),
                 ("LAMBERT", 1.0, 0.0)]


def sky_case(tmp: pathlib.Path):
    """Sky-only scene: one tiny sphere behind the camera (never seen, so every path is one sky
    lookup).  Returns (scene path, decoded texture)."""
    tex = write_rgbe(tmp / "kat_sky.hdr", sky_test_texture())
    p = write_scene(tmp / "kat_sky.json", [obj("SPHERE", pos=(0.0, 0.0, -50.0), scale=(0.01, 0.01, 0.01))],
                    SKY_CAM, str(tmp / "kat_sky.hdr"))
    return p, tex


def furnace_case(tmp: pathlib.Path, mtype: str, rough: float, metal: float):
    """A 200 x 200 quad of the given material under a uniform sky of radiance 1 (exact in RGBE)."""
    write_rgbe(tmp / "kat_white.hdr", np.ones((8, 16, 3)))
    m = material(mtype, base=(1.0, 1.0, 1.0), rough=rough, metal=metal)
    return write_scene(tmp / f"kat_furnace_{mtype}_{rough}.json", [obj("QUAD", scale=(100.0, 1.0, 100.0), mat=m)],
                       FURNACE_CAM, str(tmp / "kat_white.hdr"))


def furnace_expectation(W: int, H: int, mtype: str, rough: float, metal: float) -> float:
    """Mean over the pixels' centre rays of the directional albedo at each pixel's view angle."""
    if mtype == "LAMBERT":
        return 1.0
    d = camera_dirs(FURNACE_CAM["position"], FURNACE_CAM["look_at"], FURNACE_CAM["fovy"], W, H, [0.5], [0.5])
    mu = -d[..., 0, 1]
    grid = np.linspace(mu.min(), mu.max(), 5)
    vals = [directional_albedo(m, rough, mtype, metal=metal) for m in grid]
    return float(np.interp(mu.ravel(), grid, vals).mean())


def check_furnace(mean_img: np.ndarray, expected: float, what: str) -> None:
    """mean_img: per-pixel sample means (H x W x 3).  All three channels carry the same value."""
    v = mean_img[..., :3]
    finite = np.isfinite(v).all(-1)
    assert finite.mean() > 0.99, f"{what}: {(~finite).sum()} non-finite pixels"
    px = v[finite].mean(-1)
    m = float(px.mean())
    sigma = float(px.std() / math.sqrt(px.size))
    tol = 5 * sigma + 2e-4
    assert abs(m - expected) < tol, f"{what}: mean {m:.6f} vs analytic {expected:.6f} (tol {tol:.2e})"


def check_sky(mean_img: np.ndarray, tex: np.ndarray, W: int, H: int, spp: int, what: str) -> None:
    mu, sd = sky_pixel_expectation(tex, SKY_CAM["position"], SKY_CAM["look_at"], SKY_CAM["fovy"], W, H)
    got = mean_img[..., :3].astype(np.float64)
    # Monte Carlo error of the pixel mean + the 1/256 filter-weight quantisation (App. C)
    tol = 5 * sd / math.sqrt(spp) + 2.5e-3 * (1 + np.abs(mu))
    bad = np.abs(got - mu) > tol
    assert not bad.any(), (f"{what}: {bad.any(-1).sum()} pixels off; worst |diff| "
                           f"{np.abs(got - mu).max():.4g}, e.g. pixel {np.argwhere(bad)[0]}")
    # and the image as a whole: the mapping is not flipped or shifted
    assert np.abs(got.mean((0, 1)) - mu.mean((0, 1))).max() < 2e-3
