"""Path-level pin of the restatement against the reference's own published render.

The reference's `cornell_box_4096spp.png` was made by its windowed loop (main.cpp:387-399): one
render(cam, 1, false) call per frame, tonemapped by the frame count (tonemap.cu:16-26).  Every pixel
draws its own cuRAND XORWOW stream, seeded curand_init(1984 + idx, 0, 0) (initRandState.cu:16), two
uniforms for the jitter (trace.cu:190-191) and two per hit (Material.inl:40-41).  If our restatement
of those is right, our windowed render S draws, per pixel, the same random
numbers as the reference's, so most of its paths are the reference's paths: its Monte Carlo noise
is the reference's noise.  A render D of the same pixels from samples 4096..8191 of the same streams
(disjoint from S's) has noise independent of the reference's.

Statistic (VERDICT r02 "do this" 1): estimate each pixel's expectation E from a third disjoint run of
samples (8192 .. 8192 + e_spp), tonemapped into 8-bit units without quantisation, and correlate the
residuals (S - E) and (D - E) with (ref - E) over the unmasked pixels and all three channels.  Shared
biases (E's own noise, the tonemap's Jensen bias, the reference's missing earth texture) enter both
correlations alike; only path-level agreement separates them.  Under "the streams differ" rho_S and
rho_D have the same distribution, with sigma ~ 1/sqrt(n).

Used by tests/test_gpu_kat.py (the asserted pin) and tools/pin_png.py --corr (the record).
"""
from __future__ import annotations

import math

import numpy as np

import pathtracercuda_amd as pa


def pin_mask() -> np.ndarray:
    """Blocks (32 x 32 pixels, row 0 = bottom) around the textured earth sphere and its reflection in
    the GGX cube: the reference rendered them with earth.png, which its checkout does not contain."""
    mb = np.ones((32, 32), bool)
    mb[2:11, 11:20] = False
    mb[4:12, 8:13] = False
    return np.kron(mb, np.ones((32, 32), bool))


def mask_distance() -> np.ndarray:
    """Per 32 x 32 block: Chebyshev distance in blocks to the nearest masked block (0 = masked)."""
    mb = pin_mask()[::32, ::32]
    iy, ix = np.nonzero(~mb)
    yy, xx = np.mgrid[0:mb.shape[0], 0:mb.shape[1]]
    d = np.maximum(np.abs(yy[..., None] - iy), np.abs(xx[..., None] - ix)).min(-1)
    return d


def bias_by_ring(x: np.ndarray, ref: np.ndarray, m: np.ndarray) -> list:
    """Mean (x - ref) per channel over the unmasked pixels of the blocks at each distance from the
    masked earth sphere (its light is missing from our render: the reference's earth.png is absent,
    so our sphere is untextured white, cornell_box.json:136-141, Material.inl:26-34)."""
    dist = np.kron(mask_distance(), np.ones((32, 32), int))
    d = (x - ref).astype(np.float64)
    out = []
    for r in range(1, int(dist.max()) + 1):
        sel = m & (dist == r)
        if sel.any():
            out.append({"ring": r, "pixels": int(sel.sum()), "bias": [round(float(v), 4) for v in d[sel].mean(0)]})
    return out


def tonemap_f(hdr: np.ndarray) -> np.ndarray:
    """tonemap.cu:16-26 without the final truncation (float64, 8-bit units)."""
    c = np.maximum(hdr.astype(np.float64), 0.0)
    return 255.0 * (c / (c + 1.0)) ** (1.0 / 2.2)


def _corr(a: np.ndarray, b: np.ndarray) -> float:
    a = a - a.mean()
    b = b - b.mean()
    return float((a * b).sum() / math.sqrt((a * a).sum() * (b * b).sum()))


def _agree(x: np.ndarray, ref: np.ndarray, m: np.ndarray) -> dict:
    d = (x - ref)
    ad = np.abs(d).max(-1)[m]
    return {"eq": float((ad == 0).mean()), "le1": float((ad <= 1).mean()), "le2": float((ad <= 2).mean()),
            "le4": float((ad <= 4).mean()), "bias": [float(v) for v in d[m].mean(0)]}


def reference_pin(root, scenes, e_spp: int = 16384, spp: int = 4096) -> dict:
    ref = np.load(root / "tests" / "golden" / "cornell_box_4096spp_ref8.npz")["rgb"].astype(np.int16)
    H, W, _ = ref.shape
    pt = pa.Pathtracer(W, H)
    cam = pt.load_scene(str(scenes / "cornell_box.scene.json"))
    # S: samples 0 .. spp-1 of every pixel's stream, one sample per render() call as the reference
    pt.render(cam, 1, True, chunks=spp)
    s8 = pt.tonemap(spp)[..., :3].astype(np.int16)
    finite = np.isfinite(pt.accum()[..., :3]).all(-1)
    # D: samples spp .. 2 spp - 1 (the streams continue where S ended)
    pt.render(cam, 1, True, chunks=spp)
    d8 = pt.tonemap(spp)[..., :3].astype(np.int16)
    finite &= np.isfinite(pt.accum()[..., :3]).all(-1)
    # E: samples 2 spp .. 2 spp + e_spp - 1, the expectation estimate
    pt.render(cam, 8, True, chunks=e_spp // 8)
    acc = pt.accum()[..., :3]
    finite &= np.isfinite(acc).all(-1)
    e = tonemap_f(np.where(np.isfinite(acc), acc, 0.0) / float(e_spp))
    pt.close()
    # pixels a NaN sample poisoned (the reference's 0/0 VNDF pdf, MonteCarlo.h:110-113, reproduced)
    # carry no residual; they are left out of the correlation (a handful per render)
    m = pin_mask()
    mc = m & finite
    rr = (ref - e)[mc].ravel()
    rho_s = _corr((s8 - e)[mc].ravel(), rr)
    rho_d = _corr((d8 - e)[mc].ravel(), rr)
    n = rr.size
    sigma = 1.0 / math.sqrt(n)
    out = {"image": f"{W}x{H}", "spp": spp, "e_spp": e_spp, "values": n, "rho_same": rho_s, "rho_disjoint": rho_d,
           "sigma": sigma, "excess_sigmas": (rho_s - rho_d) / sigma, "nan_pixels_excluded": int((m & ~finite).sum()),
           "same_stream": _agree(s8, ref, m), "disjoint": _agree(d8, ref, m)}
    out["eq_excess"] = out["same_stream"]["eq"] - out["disjoint"]["eq"]
    out["bias_by_ring_same"] = bias_by_ring(s8, ref, m)
    # E - ref: the same table for the noise-free expectation (8-bit units, no truncation)
    out["bias_by_ring_expectation"] = bias_by_ring(e, ref, mc)
    return out
