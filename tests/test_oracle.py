"""Oracle (CPU restatement) checks: pinned against the reference's published render, plus
known-answer tests of the restated third-party pieces (XORWOW, transcendentals, sampler)."""
import ctypes as C
import json
import math

import numpy as np
import pytest

from oracle import pyoracle as po


def test_struct_sizes():
    # Material.h:22-27 (40 B), Hittable.h:23-27 (96 B), BVH.h:6-11 (32 B), Camera.h:14-22 (92 B)
    L = po.lib()
    assert [L.or_sizeof(i) for i in (0, 1, 3, 4, 5)] == [40, 96, 32, 92, 24]
    assert C.sizeof(po.Hittable) == 96 and C.sizeof(po.BVHNode) == 32 and C.sizeof(po.Camera) == 92


def xorwow_ref(seed):
    """Independent numpy restatement of cuRAND's curand_init(seed, 0, 0)."""
    u = np.uint32
    s0 = u(seed & 0xFFFFFFFF) ^ u(0xAAD26B49)
    s1 = u(seed >> 32) ^ u(0xF7DCEFDD)
    with np.errstate(over="ignore"):
        t0 = u(1099087573) * s0
        t1 = u(2591861531) * s1
        d = u(6615241) + t1 + t0
        v = [u(123456789) + t0, u(362436069) ^ t0, u(521288629) + t1, u(88675123) ^ t1, u(5783321) + t0]
    return d, v


def test_xorwow_stream():
    L = po.lib()
    for seed in (1984, 1984 + 1919 + 1079 * 1920, 12345678901):
        st = po.Xorwow()
        L.or_xorwow_init(seed, C.byref(st))
        d, v = xorwow_ref(seed)
        assert st.d == d and list(st.v) == [int(x) for x in v]
        with np.errstate(over="ignore"):
            for _ in range(50):
                t = v[0] ^ (v[0] >> np.uint32(2))
                v = v[1:] + [(v[4] ^ (v[4] << np.uint32(4))) ^ (t ^ (t << np.uint32(1)))]
                d = d + np.uint32(362437)
                assert L.or_xorwow_next(C.byref(st)) == int(v[4] + d)


def test_uniform_range():
    L = po.lib()
    st = po.Xorwow()
    L.or_xorwow_init(1984, C.byref(st))
    us = np.array([L.or_xorwow_uniform(C.byref(st)) for _ in range(20000)], dtype=np.float32)
    assert us.min() > 0.0 and us.max() <= 1.0            # curand_uniform: (0, 1]
    assert abs(us.mean() - 0.5) < 0.01


def ulp_err(got, want):
    got = np.float64(np.float32(got))
    return abs(got - want) / np.spacing(np.float32(want if want != 0 else 1e-38))


def test_transcendentals_accuracy():
    L = po.lib()
    rng = np.random.default_rng(1)
    xs = np.concatenate([rng.uniform(0, 2 * np.pi, 3000), np.linspace(0, 6.2831855, 500)]).astype(np.float32)
    for x in xs:
        x = float(x)
        assert ulp_err(L.pm_sinf(x), math.sin(x)) < 4 or abs(L.pm_sinf(x) - math.sin(x)) < 2e-7
        assert ulp_err(L.pm_cosf(x), math.cos(x)) < 4 or abs(L.pm_cosf(x) - math.cos(x)) < 2e-7
    for y in np.linspace(-1, 1, 4001).astype(np.float32):
        y = float(y)
        assert abs(L.pm_acosf(y) - math.acos(y)) < 4e-7 * max(1.0, math.acos(y))
    for _ in range(3000):
        y, x = rng.normal(size=2).astype(np.float32)
        want = math.atan2(float(y), float(x))
        assert abs(L.pm_atan2f(float(y), float(x)) - want) < 3e-7 * max(1.0, abs(want))
    for b in rng.uniform(0, 1, 3000).astype(np.float32):
        for e in (2.2, 1.0 / 2.2):
            want = float(b) ** float(np.float32(e))
            assert abs(L.pm_powf(float(b), float(np.float32(e))) - want) <= 3e-6 * max(want, 1e-30)
    assert L.pm_powf(0.0, 2.2) == 0.0 and L.pm_powf(1.0, 0.4545) == 1.0
    assert L.pm_atan2f(0.0, -1.0) == np.float32(np.pi) and L.pm_atan2f(-0.0, -1.0) == -np.float32(np.pi)


def test_bilinear_sampler_rule():
    # wrap u, clamp v, weights on a 1/256 grid
    tex = np.zeros((2, 4, 4), dtype=np.float32)
    tex[..., 0] = np.arange(8, dtype=np.float32).reshape(2, 4)
    t = po.Texture(4, 2, po.fptr(tex))
    L = po.lib()
    out = (C.c_float * 4)()
    L.or_tex2d(C.byref(t), 0.125, 0.25, out)        # texel centre (0, 0)
    assert out[0] == 0.0
    L.or_tex2d(C.byref(t), 0.0, 0.25, out)          # halfway between texel 3 (wrapped) and 0
    assert out[0] == 1.5
    L.or_tex2d(C.byref(t), 0.125, -3.0, out)        # clamped to row 0
    assert out[0] == 0.0
    L.or_tex2d(C.byref(t), 0.125 + 0.25 * 0.3, 0.25, out)
    assert out[0] == np.float32(77.0 / 256.0)        # 0.3 -> 77/256


def test_camera_corner_rays():
    L = po.lib()
    cam = po.Camera()
    L.or_camera_make(po.f3([0, 0, 0]), po.f3([0, 0, -1]), po.f3([0, 1, 0]), L.or_radians(90.0), 2.0, C.byref(cam))
    assert np.allclose(list(cam.lowerLeftCorner), [-2.0, -1.0, -1.0], atol=1e-6)
    assert np.allclose(list(cam.horizontal), [4.0, 0.0, 0.0], atol=1e-6)
    assert np.allclose(list(cam.vertical), [0.0, 2.0, 0.0], atol=1e-6)


def test_transform_roundtrip():
    # worldTransform (Hittable.cpp:6-103): the inverse rows map the world AABB corners into [-1,1]^3
    L = po.lib()
    rng = np.random.default_rng(3)
    for _ in range(50):
        pos, rot = rng.uniform(-5, 5, 3), rng.uniform(-180, 180, 3)
        scale = rng.uniform(0.2, 3, 3)
        m = po.Material()
        L.or_material_make(0, po.f3([1, 1, 1]), po.f3([0, 0, 0]), 0.5, 0.0, 0, C.byref(m))
        h = po.CpuHittable()
        L.or_cpu_hittable_make(6, po.f3(pos), po.f3([L.or_radians(float(r)) for r in rot]), po.f3(scale), C.byref(m), C.byref(h))
        R = np.array([list(r) for r in h.rows], dtype=np.float64)
        # object-space centre of the world position is the origin
        assert np.allclose(R[:, :3] @ pos.astype(np.float32) + R[:, 3], 0.0, atol=1e-4)
        # AABB contains the transformed unit cube: its centre maps near the origin
        c = (np.array(list(h.aabbMin)) + np.array(list(h.aabbMax))) / 2
        assert np.allclose(c, pos, atol=1e-4)


def test_oracle_pinned_to_reference_render(root, scenes):
    """The reference's own published output, cornell_box_4096spp.png (1024x1024, windowed mode,
    earth.png present), reduced to linear block means in tests/golden/: the oracle at 16 spp must
    agree away from the textured sphere (whose texture is missing here)."""
    ref = np.array(json.loads((root / "tests/golden/cornell_ref_blocks.json").read_text())["blocks"])
    sc = po.load_scene(scenes / "cornell_box.scene.json", 1024, 1024)
    r = po.OracleRenderer(sc, 1024, 1024)
    r.render(sc.camera, 8, True, chunks=2)
    ours = (r.accum[..., :3] / 16.0).reshape(32, 32, 32, 32, 3).mean(axis=(1, 3))
    mask = np.ones((32, 32), bool)
    mask[3:10, 12:19] = False
    mask[5:11, 9:12] = False
    ratio = ours[mask].mean(0) / ref[mask].mean(0)
    assert np.all(np.abs(ratio - 1.0) < 0.02), ratio
    rel = np.abs(ours[mask] - ref[mask]) / (ref[mask] + 0.02)
    assert np.median(rel) < 0.04, np.median(rel)
    assert np.percentile(rel, 95) < 0.25


def test_white_furnace_bounded(scenes, tmp_path):
    # A Lambert sphere of albedo a inside a constant-1 environment: radiance <= sum_k a^k (k < 5)
    import struct
    W = H = 8
    hdr = tmp_path / "white.hdr"
    hdr.write_bytes(b"#?RADIANCE\nFORMAT=32-bit_rle_rgbe\n\n-Y %d +X %d\n" % (H, W) + bytes([128, 128, 128, 129]) * (W * H))
    a = 0.6
    scene = {"camera": {"position": [0.0, 0.0, 3.0], "look_at": [0.0, 0.0, 0.0], "fovy": 30.0},
             "skybox": str(hdr),
             "objects": [{"type": "SPHERE", "position": [0.0, 0.0, 0.0], "rotation": [0.0, 0.0, 0.0],
                          "scale": [1.0, 1.0, 1.0], "material": {"type": "LAMBERT", "baseColor": [a, a, a]}}]}
    p = tmp_path / "furnace.json"
    p.write_text(json.dumps(scene))
    sc = po.load_scene(p, 16, 16)
    r = po.OracleRenderer(sc, 16, 16)
    r.render(sc.camera, 16, True, chunks=4)
    lin = r.accum[..., :3] / 64.0
    bound = sum(a ** k for k in range(5))
    centre = lin[6:10, 6:10].mean()
    assert abs(centre - a) < 0.03          # one bounce into a convex sphere, then the sky (=1)
    assert lin.max() <= bound + 1e-3


def test_fast_timing_build_is_bit_identical(scenes):
    # bench.py's CPU baseline times liboracle_fast.so (-O3 -march=x86-64-v3, contraction off): it
    # must compute the checker's bits, with any thread count (rows are handed out dynamically)
    sc = po.load_scene(scenes / "test_shapes.scene.json", 40, 24)
    a = po.OracleRenderer(sc, 40, 24, threads=1)
    a.render(sc.camera, 4, True, chunks=2)
    b = po.OracleRenderer(sc, 40, 24, threads=5, fast=True)
    b.render(sc.camera, 4, True, chunks=2)
    assert np.array_equal(a.accum.view(np.uint32), b.accum.view(np.uint32))
    assert np.array_equal(a.rng_array(), b.rng_array())


def test_rise_scene_exercises_the_far_root_quirk(scenes):
    # scenes/rise_repair.scene.json puts the camera and every object inside one large sphere, so the
    # reference's hitBVH (trace.cu:48-98) meets leaves whose sphere test returns the far root beyond
    # t_max (Hittable.inl:152-158) and raises t_max mid-traversal.  The oracle counts such leaf visits
    # ("rises"); the GPU parity test asserts its repairs counter equals this count.  The shipped
    # scenes meet the case rarely (generated_scene) or never at this size.
    W, H = 48, 32
    osc = po.load_scene(scenes / "rise_repair.scene.json", W, H)
    r = po.OracleRenderer(osc, W, H)
    r.render(osc.camera, 4, True, collect_stats=True)
    rises = int(r.stats[7])
    assert rises > 0.05 * int(r.stats[5]), f"rise scene: only {rises} rises in {int(r.stats[5])} samples"
    osc = po.load_scene(scenes / "cornell_box.scene.json", W, H)
    r = po.OracleRenderer(osc, W, H)
    r.render(osc.camera, 4, True, collect_stats=True)
    assert int(r.stats[7]) < rises
