"""Speculative sample groups: a pixel's sample chain cut into groups started at
guessed draw offsets and stitched where the parses meet.  The bar is the same as for every other
schedule: bit-identical accumulation sums and XORWOW states (trace.cu:183-198: one serial stream
per pixel, the chunk fold color + accum)."""
import numpy as np
import pytest

import pathtracercuda_amd as pa
from oracle import pyoracle as po

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gpu_available():
    if pa.device_count() < 1:
        pytest.skip("no GPU")


def bits(a):
    return np.ascontiguousarray(a).view(np.uint32)


def same(a, b, what):
    if not np.array_equal(bits(a), bits(b)):
        bad = np.argwhere(bits(a) != bits(b))
        raise AssertionError(f"{what}: {len(bad)} words differ, first at {bad[0]}: {a[tuple(bad[0][:2])]} vs "
                             f"{b[tuple(bad[0][:2])]}")


@pytest.mark.parametrize("name,W,H,spp,chunks,groups", [
    ("cornell_box", 64, 64, 8, 8, 2),
    ("cornell_box", 37, 21, 3, 11, 5),        # ragged tiles, odd spp: the groups cut render() calls
    ("generated_scene", 96, 54, 8, 16, 8),
    ("test_shapes", 80, 50, 8, 8, 3),
])
@pytest.mark.parametrize("variant", [39, 40, 60, 61])  # grouped walk without / with deferred shading, 6 waves
def test_groups_bitexact_vs_oracle(gpu_available, scenes, name, W, H, spp, chunks, groups, variant):
    p = scenes / f"{name}.scene.json"
    pt = pa.Pathtracer(W, H)
    cam = pt.load_scene(str(p))
    pt.set_kernel_variant(variant)
    pt.set_sample_groups(groups)
    pt.render(cam, spp, True, chunks=chunks)
    assert pt.last_sample_groups == groups
    osc = po.load_scene(p, W, H)
    ref = po.OracleRenderer(osc, W, H)
    ref.render(osc.camera, spp, True, chunks=chunks)
    same(pt.accum(), ref.accum, f"{name} G={groups}")
    assert np.array_equal(pt.rng_state(), ref.rng_array())
    # a second launch continues the history (ignoreHistory = false) from the stitched state
    pt.render(cam, spp, False, chunks=chunks)
    ref.render(osc.camera, spp, False, chunks=chunks)
    same(pt.accum(), ref.accum, f"{name} G={groups}, second launch")
    assert np.array_equal(pt.rng_state(), ref.rng_array())


@pytest.mark.parametrize("rounds", [6, 0])
def test_groups_equal_plain_launch_patch_and_resume(gpu_available, scenes, rounds):
    """One rank's share of the 1080p image at N = 8 (8-row bands): the automatic choice groups it, and
    the result equals the plain launch bit for bit.  Many groups over short chains make guesses miss,
    so patch rounds run (rounds = 6) or the plain resume launch takes the dead ends (rounds = 0)."""
    W, H = 1920, 1080
    p = str(scenes / "generated_scene.scene.json")
    out = {}
    for mode in (1, 0, 16):
        pt = pa.Pathtracer(W, H, row_offset=3, row_stride=8, band_rows=8)
        cam = pt.load_scene(p)
        pt.set_sample_groups(mode)
        pt.set_patch_rounds(rounds)
        pt.render(cam, 8, True, chunks=32)
        out[mode] = (pt.accum(), pt.rng_state(), pt.last_sample_groups, pt.group_stats())
        pt.close()
    assert out[1][2] == 0 and out[0][2] >= 2 and out[16][2] == 16
    for mode in (0, 16):
        same(out[mode][0], out[1][0], f"mode {mode}")
        assert np.array_equal(out[mode][1], out[1][1])
    st = out[16][3]
    assert st["dead_ends"][0] > 0, st                    # guesses missed somewhere: the later passes ran
    if rounds:
        assert st["patch_rounds"] >= 1, st


@pytest.mark.parametrize("groups", [2, 4])
def test_group_lookback_bitexact(gpu_available, scenes, groups):
    """The second phases' lag tolerance (pt_set_group_lookback) is scheduling only: every setting
    gives the plain launch's bits, on a rank share (ground pixels: many second phases) and on a
    ragged image."""
    for W, H, kw, name in ((1920, 1080, dict(row_offset=5, row_stride=8, band_rows=8), "generated_scene"),
                           (37, 21, {}, "cornell_box")):
        p = str(scenes / f"{name}.scene.json")
        out = {}
        for cfg in ("plain", (0, 0), (1, 0), (8, 0), (32, 8), (256, 3)):
            pt = pa.Pathtracer(W, H, **kw)
            cam = pt.load_scene(p)
            pt.set_sample_groups(1 if cfg == "plain" else groups)
            if cfg != "plain":
                pt.set_group_lookback(*cfg)
            pt.render(cam, 8, True, chunks=16)
            assert pt.last_sample_groups == (0 if cfg == "plain" else groups)
            out[cfg] = (pt.accum(), pt.rng_state())
            pt.close()
        for cfg, (acc, st) in out.items():
            same(acc, out["plain"][0], f"{name} G={groups} lookback {cfg}")
            assert np.array_equal(st, out["plain"][1]), cfg


def test_groups_refused_beyond_the_fold_word(gpu_available, scenes):
    # the fold state packs (sample in call, call) as sIdx | c << 16, so a launch of more
    # than 65,535 render() calls (or spp) must not run grouped; forced groups then run plain and the
    # result equals the launch without groups, bit for bit
    W, H, chunks = 16, 16, 70000
    a = pa.Pathtracer(W, H)
    cam = a.load_scene(str(scenes / "cornell_box.scene.json"))
    b = pa.Pathtracer(W, H)
    b.load_scene(str(scenes / "cornell_box.scene.json"))
    a.set_sample_groups(2)
    b.set_sample_groups(1)
    a.render(cam, 1, True, chunks=chunks)
    assert a.last_sample_groups == 0
    b.render(cam, 1, True, chunks=chunks)
    assert np.array_equal(a.accum().view(np.uint32), b.accum().view(np.uint32))
    assert np.array_equal(a.rng_state(), b.rng_state())


def test_groups_after_plain_launch_reallocate(gpu_available, scenes):
    # a plain launch releases the group logs (pt_kernels.hip ssg_release); a later grouped launch
    # allocates them again and still reproduces the plain sequence bit for bit
    W, H = 96, 54
    a = pa.Pathtracer(W, H)
    cam = a.load_scene(str(scenes / "generated_scene.scene.json"))
    b = pa.Pathtracer(W, H)
    b.load_scene(str(scenes / "generated_scene.scene.json"))
    b.set_sample_groups(1)
    for mode, ignore in ((4, True), (1, False), (4, False)):
        a.set_sample_groups(mode)
        a.render(cam, 8, ignore, chunks=16)
        assert a.last_sample_groups == (4 if mode == 4 else 0)
        b.render(cam, 8, ignore, chunks=16)
        same(a.accum(), b.accum(), f"groups {mode}")
        assert np.array_equal(a.rng_state(), b.rng_state())
