"""GPU kernel against the analytic KATs (tests/kat.py) and against the reference's own published
render, pixel for pixel (tests/golden/cornell_box_4096spp_ref8.npz, from the reference's
cornell_box_4096spp.png by tools/make_png_fixture.py)."""
import numpy as np
import pytest

import kat
import pathtracercuda_amd as pa

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gpu_available():
    if pa.device_count() < 1:
        pytest.skip("no GPU")


def render_mean(scene, W, H, spp):
    pt = pa.Pathtracer(W, H)
    cam = pt.load_scene(str(scene))
    pt.render(cam, 8, True, chunks=spp // 8)
    acc = pt.accum()
    pt.close()
    return acc / spp


def test_gpu_sky_only_kat(gpu_available, tmp_path):
    p, tex = kat.sky_case(tmp_path)
    W, H, spp = 48, 32, 4096
    kat.check_sky(render_mean(p, W, H, spp), tex, W, H, spp, "gpu sky")


@pytest.mark.parametrize("mtype,rough,metal", kat.FURNACE_CASES)
def test_gpu_white_furnace(gpu_available, tmp_path, mtype, rough, metal):
    W, H, spp = 32, 32, 2048
    p = kat.furnace_case(tmp_path, mtype, rough, metal)
    kat.check_furnace(render_mean(p, W, H, spp), kat.furnace_expectation(W, H, mtype, rough, metal),
                      f"gpu {mtype} r={rough}")


# Blocks (32 x 32 pixels, row 0 = bottom) around the textured earth sphere and its reflection in the
# GGX cube: the reference rendered them with earth.png, which its checkout does not contain.
def _pin_mask():
    mb = np.ones((32, 32), bool)
    mb[2:11, 11:20] = False
    mb[4:12, 8:13] = False
    return np.kron(mb, np.ones((32, 32), bool))


def _windowed_render(scenes, decorrelate):
    """The reference's windowed loop (main.cpp:387-399): render(cam, 1, false) per frame, tonemap by
    the frame count; decorrelate = consume 8 samples per pixel first, so every path differs."""
    pt = pa.Pathtracer(1024, 1024)
    cam = pt.load_scene(str(scenes / "cornell_box.scene.json"))
    if decorrelate:
        pt.render(cam, 8, True)
    pt.render(cam, 1, decorrelate, chunks=4096)
    img = pt.tonemap(4096)[..., :3].astype(np.int16)
    pt.close()
    return img


def test_pixel_pin_vs_reference_png(gpu_available, scenes, root):
    """Per pixel, the reference's 4096-spp cornell render and ours draw the same random numbers in
    the same order; the reference's float arithmetic (nvcc FMA contraction, libdevice, texture unit)
    rounds differently, and in a closed box those differences grow over five bounces, so most
    paths end up elsewhere: the pixels agree at the level of their 8-bit Monte Carlo noise, with a
    small path-level excess.  Measured on MI355X (unmasked 90 % of the image): same stream 57.8 %
    of the pixels equal, 81.9 % within 1 LSB, 93.4 % within 2; decorrelated (8 samples consumed
    first) 52.6 / 80.8 / 92.9 %; mean difference +0.45/+0.38/+0.32 LSB (R/G/B) in both -- the
    expectation gap, which the missing earth texture's indirect light explains.  A wrong jitter,
    lobe, BRDF, pdf or normalisation moves the expectation by many LSB and fails the thresholds
    (the 2 %-level block test in test_gpu_parity is the coarse version of this one)."""
    ref = np.load(root / "tests" / "golden" / "cornell_box_4096spp_ref8.npz")["rgb"].astype(np.int16)
    m = _pin_mask()
    stats = {}
    for tag, dec in (("same_stream", False), ("decorrelated", True)):
        d = _windowed_render(scenes, dec) - ref
        ad = np.abs(d).max(-1)[m]
        stats[tag] = {"eq": float((ad == 0).mean()), "le1": float((ad <= 1).mean()), "le2": float((ad <= 2).mean()),
                      "le4": float((ad <= 4).mean()), "bias": [float(x) for x in d[m].mean(0)]}
    s, u = stats["same_stream"], stats["decorrelated"]
    print(stats)
    assert s["eq"] >= 0.5 and s["le1"] >= 0.75 and s["le2"] >= 0.9 and s["le4"] >= 0.97, stats
    assert max(abs(b) for b in s["bias"]) < 1.0, stats           # < 1 LSB mean difference
    assert s["eq"] >= u["eq"] - 0.01, stats                      # the same stream is never further away
