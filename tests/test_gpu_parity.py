"""GPU parity: the HIP megakernel against the CPU restatement (oracle/), through the C ABI.

Bar: bit-exact accumulation sums and XORWOW states (integer and float work share one fixed
operation order; SURVEY.md §8c "GPU vs build's CPU restatement: expect bit-exact").  Sizes are
chosen so the oracle finishes in seconds; full BASELINE sizes are covered by exact parity on a
row subset of the full 1080p image and by size-independent properties (determinism, tiling,
chunking).
"""
import numpy as np
import pytest

import pathtracercuda_amd as pa
from oracle import pyoracle as po
from pathtracercuda_amd import _native as N

pytestmark = pytest.mark.gpu


def bits(a):
    return np.ascontiguousarray(a).view(np.uint32)


def assert_bitexact(gpu, ref, what):
    if np.array_equal(bits(gpu), bits(ref)):
        return
    diff = np.argwhere(bits(gpu) != bits(ref))
    y, x = diff[0][:2]
    e = np.linalg.norm(gpu[..., :3] - ref[..., :3], axis=-1)
    raise AssertionError(f"{what}: {len(diff)} words differ; first pixel (row {y}, x {x}) gpu={gpu[y, x]} "
                         f"ref={ref[y, x]}; max L2 {e.max():.3g}, pixels > 1e-4: {(e > 1e-4).mean():.2%}")


SHIPPED_VARIANTS = (1, 4, 6, 20, 39, 40, 41, 46, 47, 48, 60, 61)


def pair(scene_path, W, H, row_offset=0, row_stride=1, band_rows=1):
    pt = pa.Pathtracer(W, H, device=0, row_offset=row_offset, row_stride=row_stride, band_rows=band_rows)
    cam = pt.load_scene(str(scene_path))
    osc = po.load_scene(scene_path, W, H)
    ref = po.OracleRenderer(osc, W, H, row_offset, row_stride, band_rows=band_rows)
    assert bytes(cam) == bytes(osc.camera)
    return pt, cam, ref, osc


@pytest.fixture(scope="module")
def gpu_available():
    if pa.device_count() < 1:
        pytest.skip("no GPU")


def test_rng_seeding(gpu_available, scenes):
    # initRandState.cu:16 curand_init(1984 + idx, 0, 0): fresh contexts carry the same state
    for (W, H, off, stride) in [(37, 29, 0, 1), (64, 64, 3, 4)]:
        pt = pa.Pathtracer(W, H, row_offset=off, row_stride=stride)
        ref = po.OracleRenderer(po.OracleScene(), W, H, off, stride)
        assert np.array_equal(pt.rng_state(), ref.rng_array())


@pytest.mark.parametrize("name,W,H,spp,chunks", [
    ("cornell_box", 64, 64, 8, 2),
    ("cornell_box", 37, 21, 3, 3),          # ragged tiles, odd spp
    ("generated_scene", 96, 54, 8, 2),      # 484 quadrics + HDR sky
    ("test_shapes", 80, 50, 8, 2),          # every shape x material, textures, emission
])
def test_render_bitexact(gpu_available, scenes, name, W, H, spp, chunks):
    pt, cam, ref, osc = pair(scenes / f"{name}.scene.json", W, H)
    pt.render(cam, spp, True, chunks=chunks)
    ref.render(osc.camera, spp, True, chunks=chunks)
    assert_bitexact(pt.accum(), ref.accum, f"{name} accum")
    assert np.array_equal(pt.rng_state(), ref.rng_array()), "RNG streams diverged"
    assert pt.frames == ref.frames == chunks


@pytest.mark.parametrize("variant", SHIPPED_VARIANTS)
def test_every_kernel_variant_bitexact(gpu_available, scenes, variant):
    # all trace-kernel variants (schedules, LDS staging, occupancy) produce the reference's bits
    pt, cam, ref, osc = pair(scenes / "test_shapes.scene.json", 72, 40)
    pt.set_kernel_variant(variant)
    pt.render(cam, 4, True, chunks=2)
    ref.render(osc.camera, 4, True, chunks=2)
    assert_bitexact(pt.accum(), ref.accum, f"variant {variant}")
    assert np.array_equal(pt.rng_state(), ref.rng_array())


def test_persistent_variants_large_grid(gpu_available, scenes):
    # the persistent variants fall back to the plain kernel when the grid fits on the chip in one
    # pass, so run them on a frame with more tiles than resident waves, several launches in a row
    # (the last wave of each launch rewinds the tile cursor for the next), against variant 1
    pt = pa.Pathtracer(1280, 720)
    cam = pt.load_scene(scenes / "generated_scene.scene.json")
    st = pt.rng_state()
    pt.set_kernel_variant(1)
    pt.render(cam, 3, True, chunks=3)
    want = pt.accum().view(np.uint32).copy()       # bits: the reference's NaN pixels stay NaN
    for variant in (39, 40, 41, 46, 47, 48, 60, 61):
        pt.set_kernel_variant(variant)
        pt.set_rng_state(st)
        pt.render(cam, 3, True, chunks=3)
        assert np.array_equal(pt.accum().view(np.uint32), want), f"variant {variant}"


@pytest.mark.parametrize("nprims", [484, 200])
def test_single_leaf_bvh_every_traversal(gpu_available, scenes, nprims):
    # a caller-supplied BVH through pt_set_scene: the root is one leaf of nprims primitives.  484 is
    # beyond the child-box encoding (leaf counts < 256), so those variants fall back; 200 runs the
    # child-box traversal with a leaf root.  Results must still be the reference's.
    import ctypes as C
    from pathtracercuda_amd import _native as N
    W, H = 48, 32
    pt, cam, ref, osc = pair(scenes / "generated_scene.scene.json", W, H)
    root = po.BVHNode.from_buffer_copy(bytes(osc.nodes[0]))
    root.offset = 0
    root.primitiveCountAxis = nprims << 16
    osc.nodes = (po.BVHNode * 1)(root)
    osc.node_count = 1
    osc.prim_count = nprims
    nodes = (pa.PtBvhNode * 1).from_buffer_copy(bytes(osc.nodes))
    prims = (pa.PtHittable * nprims).from_buffer_copy(bytes(osc.prims)[:nprims * C.sizeof(pa.PtHittable)])
    N.check_ctx(N.hip().pt_set_scene(pt._ctx, nodes, 1, prims, nprims), pt._ctx)
    ref.render(osc.camera, 2, True, chunks=1)
    for variant in (0,) + SHIPPED_VARIANTS:
        st = pt.rng_state()
        pt.set_kernel_variant(variant)
        pt.render_raw(cam, 2, 1, True)
        assert_bitexact(pt.accum(), ref.accum, f"single leaf {nprims}, variant {variant}")
        pt.set_rng_state(st)


def test_tile_schedule_does_not_change_results(gpu_available, scenes):
    # cost-sorted tile dispatch (default) vs row-major: same bits, ragged tile grid, row tiles
    for (W, H, off, stride) in [(75, 43, 0, 1), (64, 90, 1, 3)]:
        pt, cam, ref, osc = pair(scenes / "generated_scene.scene.json", W, H, off, stride)
        st = pt.rng_state()
        pt.render(cam, 2, True)                      # records the tile costs
        pt.set_rng_state(st)
        pt.render_raw(cam, 2, 1, True)               # runs in cost order
        sorted_acc = pt.accum()
        sorted_rng = pt.rng_state()
        for mode in (1, 2):                           # row-major tiles, scattered pixels
            pt.set_schedule(mode)
            pt.set_rng_state(st)
            pt.render_raw(cam, 2, 1, True)
            assert np.array_equal(bits(sorted_acc), bits(pt.accum())), f"schedule {mode}"
            assert np.array_equal(pt.rng_state(), sorted_rng), f"schedule {mode}: RNG state"
        ref.render(osc.camera, 2, True)
        assert_bitexact(sorted_acc, ref.accum, f"sorted schedule {W}x{H}")
        assert np.array_equal(sorted_rng, ref.rng_array())


def test_schedule_knobs_do_not_change_results(gpu_available, scenes):
    # issue priority by cost-order position, occupancy caps: only which wave renders a tile and when
    # changes
    W, H = 1280, 720
    pt = pa.Pathtracer(W, H)
    cam = pt.load_scene(scenes / "generated_scene.scene.json")
    st = pt.rng_state()
    pt.render(cam, 8, True, chunks=2)                 # cost order
    pt.set_rng_state(st)
    pt.render(cam, 4, True, chunks=3)
    want = pt.accum().view(np.uint32).copy()
    want_rng = pt.rng_state()
    for prio, occ in [((2, 64, 64, 64), 0), ((1, 0, 0, 0), 0), ((2, 100, 2000, 6000), 0), ((0, 0, 0, 0), 2),
                      ((0, 0, 0, 0), 1)]:
        pt.set_issue_priority(*prio)
        pt.set_occupancy(occ)
        pt.set_rng_state(st)
        pt.render(cam, 4, True, chunks=3)
        assert np.array_equal(pt.accum().view(np.uint32), want), (prio, occ)
        assert np.array_equal(pt.rng_state(), want_rng), (prio, occ)


def test_priority_bounds_and_trace_do_not_change_results(gpu_available, scenes):
    # issue-priority bounds, automatic (the dealt positions raised into the first band) and explicit,
    # on the five-wave build (automatic at 2.3 tiles per six-wave slot) and the forced six- and
    # four-wave builds, plain and instrumented with the schedule trace: only which wave issues first
    # changes.  The trace holds one start and one hardware id per tile.
    W, H = 1280, 720
    pt = pa.Pathtracer(W, H)
    cam = pt.load_scene(scenes / "generated_scene.scene.json")
    st = pt.rng_state()
    pt.render(cam, 8, True, chunks=2)                 # cost order
    pt.set_rng_state(st)
    pt.render(cam, 4, True, chunks=3)
    want = pt.accum().view(np.uint32).copy()
    want_rng = pt.rng_state()
    pt.set_tile_trace(True)
    for variant, bounds in [(0, None), (0, (5120, 5120, 12000)), (60, None), (46, (100, 7000, 7000))]:
        pt.set_kernel_variant(variant)
        if bounds:
            pt.set_issue_priority(2, *bounds)
        else:
            pt.set_issue_priority(0)
        for instrumented in (False, True):
            pt.set_rng_state(st)
            if instrumented:
                pt.render_instrumented(cam, 4, 3, True)
                tr = pt.tile_trace().reshape(-1, 2)
                cu = (tr[:, 1] >> 16) << 8 | ((tr[:, 1] & 0xffff) >> 8)
                assert len(np.unique(cu)) > 200, "tiles ran on every CU"
            else:
                pt.render_raw(cam, 4, 3, True)
            assert np.array_equal(pt.accum().view(np.uint32), want), (variant, bounds, instrumented)
            assert np.array_equal(pt.rng_state(), want_rng), (variant, bounds, instrumented)
    pt.set_tile_trace(False)
    pt.set_issue_priority(0)
    pt.set_kernel_variant(0)


def test_fast_reciprocal_and_sqrt_exhaustive(gpu_available, root):
    # pt::rcp_rn / pt::sqrt_rn (pt_math.h) against hipcc's correctly rounded 1.0f/x and sqrtf(x)
    # for every one of the 2^32 float inputs
    import json
    import subprocess
    exe = root / "pathtracercuda_amd" / "lib" / "fp_exhaustive"
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300, check=True).stdout
    res = json.loads(out)
    assert res["inputs"] == 2 ** 32
    assert res["rcp_rn"]["mismatches"] == 0, res["rcp_rn"]
    assert res["sqrt_rn"]["mismatches"] == 0, res["sqrt_rn"]
    assert res["rcp_rn_u"]["mismatches"] == 0, res["rcp_rn_u"]
    assert res["sqrt_rn_u"]["mismatches"] == 0, res["sqrt_rn_u"]
    for k in ("acos_sel", "atan_pos_sel", "atan2_sel_y", "atan2_sel_x",   # select forms = branchy forms
              "sqrt_dom", "nan_through_rcp_sqrt"):                         # guard-free forms on their domains
        assert res[k]["mismatches"] == 0, (k, res[k])
    # the guards matter: the raw sequences are not correctly rounded everywhere
    assert res["diag_rcp_newton_unguarded"]["mismatches"] > 0
    assert res["diag_sqrt_rsq_newton_unguarded"]["mismatches"] > 0


def test_progressive_frames_with_camera_moves(gpu_available, scenes):
    # the windowed loop's call pattern (main.cpp:298-437): render(cam, 1, reset) per frame, a
    # tonemap into a device pixel buffer every frame (Pathtracer.cpp:207-221), camera rotate /
    # translate resetting the accumulation
    import ctypes as C
    import torch
    W, H = 48, 32
    pt, cam, ref, osc = pair(scenes / "generated_scene.scene.json", W, H)
    L = po.lib()
    ocam = po.Camera.from_buffer_copy(bytes(osc.camera))
    dev = torch.empty((H, W, 4), dtype=torch.uint8, device="cuda:0")
    reset = True
    for frame in range(9):
        if frame == 3:
            pa.camera_rotate(cam, 0.05, -0.1, 0.0)
            L.or_camera_rotate(C.byref(ocam), 0.05, -0.1, 0.0)
            reset = True
        if frame == 6:
            pa.camera_translate(cam, 0.5, 0.0, -1.5)
            L.or_camera_translate(C.byref(ocam), 0.5, 0.0, -1.5)
            reset = True
        assert bytes(cam) == bytes(ocam)
        pt.render(cam, 1, reset)
        ref.render(ocam, 1, reset)
        reset = False
        pt.tonemap_device(dev.data_ptr(), dev.numel())
        assert pt.frames == ref.frames
        assert np.array_equal(dev.cpu().numpy(), ref.tonemap()), f"frame {frame}"
        assert_bitexact(pt.accum(), ref.accum, f"frame {frame}")


def test_history_semantics(gpu_available, scenes):
    # render(cam, spp, ignoreHistory) sequence: trace.cu:196 and Pathtracer.cpp:164-167,226
    pt, cam, ref, osc = pair(scenes / "test_shapes.scene.json", 48, 40)
    for spp, ignore, chunks in [(2, True, 1), (3, False, 2), (1, False, 1), (4, True, 1), (2, False, 3)]:
        pt.render(cam, spp, ignore, chunks=chunks)
        ref.render(osc.camera, spp, ignore, chunks=chunks)
        assert_bitexact(pt.accum(), ref.accum, f"after render({spp}, {ignore}, x{chunks})")
        assert pt.frames == ref.frames
    assert np.array_equal(pt.get_image_data(), ref.tonemap())
    hdr = pt.get_hdr_image_data()
    assert_bitexact(hdr, ref.hdr(), "getHDRImageData")


def test_chunked_launch_equals_separate_launches(gpu_available, scenes):
    # one launch of k chunks == k render() calls (the headless loop, main.cpp:275-279)
    a, cam, _, _ = pair(scenes / "generated_scene.scene.json", 64, 40)
    b = pa.Pathtracer(64, 40)
    b.load_scene(str(scenes / "generated_scene.scene.json"))
    a.render(cam, 8, True, chunks=4)
    for i in range(4):
        b.render(cam, 8, i == 0)
    assert np.array_equal(bits(a.accum()), bits(b.accum()))
    assert np.array_equal(a.rng_state(), b.rng_state())


def test_row_tiles_compose_full_image(gpu_available, scenes):
    W, H, N = 40, 30, 4
    full, cam, _, _ = pair(scenes / "cornell_box.scene.json", W, H)
    full.render(cam, 4, True, chunks=2)
    img = full.accum()
    for r in range(N):
        t = pa.Pathtracer(W, H, row_offset=r, row_stride=N)
        tc = t.load_scene(str(scenes / "cornell_box.scene.json"))
        t.render(tc, 4, True, chunks=2)
        assert np.array_equal(bits(t.accum()), bits(img[r::N]))


@pytest.mark.parametrize("band,N", [(8, 3), (8, 8), (2, 4)])
def test_band_tiles_compose_full_image(gpu_available, scenes, band, N):
    # the multi-GPU partition (band b of `band` rows -> tile b mod N), ragged last band, one tile
    # per context on one GPU: the union is the single-context image, and each tile is the oracle's
    W, H = 40, 45
    full, cam, _, _ = pair(scenes / "generated_scene.scene.json", W, H)
    full.render(cam, 4, True, chunks=2)
    img = full.accum()
    from pathtracercuda_amd.distributed import global_rows
    for r in range(N):
        t, tc, ref, osc = pair(scenes / "generated_scene.scene.json", W, H, r, N, band_rows=band)
        t.render(tc, 4, True, chunks=2)
        rows = global_rows(H, r, N, band)
        assert t.rows == len(rows)
        if not rows:
            continue
        assert np.array_equal(bits(t.accum()), bits(img[rows])), f"tile {r}/{N}"
        ref.render(osc.camera, 4, True, chunks=2)
        assert_bitexact(t.accum(), ref.accum, f"band tile {r}/{N}")


def test_c4_rank_tiles_union(gpu_available, scenes):
    # BASELINE config C4 geometry (generated_scene at 3840x2160, image tiled over 8 GPUs in 8-row
    # bands): the 8 rank tiles, rendered one after another on this GPU, are bit-identical to the
    # full single-context render, and one rank's whole tile is bit-identical to the oracle
    from pathtracercuda_amd.distributed import global_rows
    W, H, N = 3840, 2160, 8
    scene = scenes / "generated_scene.scene.json"
    full = pa.Pathtracer(W, H)
    cam = full.load_scene(str(scene))
    full.render(cam, 4, True, chunks=2)
    img = full.accum()
    del full
    for r in range(N):
        t = pa.Pathtracer(W, H, row_offset=r, row_stride=N, band_rows=8)
        tc = t.load_scene(str(scene))
        t.render(tc, 4, True, chunks=2)
        acc = t.accum()
        assert np.array_equal(bits(acc), bits(img[global_rows(H, r, N, 8)])), f"rank {r}"
        if r == 5:
            osc = po.load_scene(scene, W, H)
            ref = po.OracleRenderer(osc, W, H, r, N, band_rows=8)
            ref.render(osc.camera, 4, True, chunks=2)
            assert_bitexact(acc, ref.accum, "C4 rank 5 tile")
            assert np.array_equal(t.rng_state(), ref.rng_array())
        del t


def test_group_rccl_gather_single_device(gpu_available, scenes):
    # the in-process multi-device Pathtracer (pt_group_*: ncclCommInitAll, grouped ncclSend/ncclRecv
    # to device 0, unpermute kernel) with a 1-device communicator: the full RCCL path, bit-exact
    # against the plain single-context render and the oracle, through the Pathtracer interface
    W, H = 72, 53
    scene = scenes / "test_shapes.scene.json"
    g = pa.Pathtracer(W, H, devices=[0])
    cam = g.load_scene(str(scene))
    single, scam, ref, osc = pair(scene, W, H)
    for spp, ignore, chunks in [(4, True, 2), (3, False, 1)]:
        g.render(cam, spp, ignore, chunks=chunks)
        single.render(scam, spp, ignore, chunks=chunks)
        ref.render(osc.camera, spp, ignore, chunks=chunks)
        assert g.gather() >= 0.0
        acc = g.accum()
        assert np.array_equal(bits(acc), bits(single.accum()))
        assert_bitexact(acc, ref.accum, f"group render({spp}, {ignore}, x{chunks})")
    assert g.frames == ref.frames
    assert np.array_equal(g.get_image_data(), ref.tonemap())
    assert_bitexact(g.get_hdr_image_data(), ref.hdr(), "group getHDRImageData")


def test_group_python_api_routes_through_the_group(gpu_available, scenes):
    # a device group's Python methods act on the whole group -- knobs on every context,
    # render_raw through pt_group_render, tonemap / rng_state over the full image -- and the
    # per-context diagnostics refuse instead of returning one device's share
    W, H = 72, 53
    scene = scenes / "test_shapes.scene.json"
    g = pa.Pathtracer(W, H, devices=[0])
    assert g.band_rows == 8                      # the C++ constructor's and the CLI's default
    cam = g.load_scene(str(scene))
    single = pa.Pathtracer(W, H)
    single.load_scene(str(scene))
    assert np.array_equal(g.rng_state(), single.rng_state())
    g.set_kernel_variant(20)
    g.set_schedule(1)
    g.set_sample_groups(1)
    ms = g.render_raw(cam, 4, 2, True)
    assert ms > 0.0
    single.render_raw(cam, 4, 2, True)
    assert np.array_equal(bits(g.accum()), bits(single.accum()))
    assert np.array_equal(g.rng_state(), single.rng_state())
    assert np.array_equal(g.tonemap(8), single.tonemap(8))
    # a direct launch after a gather must not leave the gathered image stale
    g.gather()
    g.render_raw(cam, 4, 1, False)
    single.render_raw(cam, 4, 1, False)
    assert np.array_equal(bits(g.accum()), bits(single.accum()))
    st = single.rng_state()
    st[3, 5, 0] ^= 1
    g.set_rng_state(st)
    assert np.array_equal(g.rng_state(), st)
    for call in (g.tile_costs, g.group_stats, lambda: g.render_instrumented(cam, 1, 1, True)):
        with pytest.raises(pa.PathtracerError):
            call()


def test_group_two_devices(gpu_available, scenes):
    # the multi-device group (RCCL send/recv across devices, one host thread per device)
    # against the single-context render, bit for bit; needs two visible GPUs
    if pa.device_count() < 2:
        pytest.skip("one GPU visible")
    W, H = 200, 120
    scene = scenes / "generated_scene.scene.json"
    g = pa.Pathtracer(W, H, devices=[0, 1])
    cam = g.load_scene(str(scene))
    single = pa.Pathtracer(W, H)
    single.load_scene(str(scene))
    g.render(cam, 8, True, chunks=3)
    single.render(cam, 8, True, chunks=3)
    assert np.array_equal(bits(g.accum()), bits(single.accum()))
    assert np.array_equal(g.rng_state(), single.rng_state())
    assert np.array_equal(g.get_image_data(), single.get_image_data())


def test_c2_exact_size(gpu_available, scenes):
    # BASELINE config C2 exactly: cornell_box 512x512, 64 spp as the headless loop runs it (8
    # render() calls of 8), bit-exact against the oracle; a cold launch (cost pre-pass first)
    pt, cam, ref, osc = pair(scenes / "cornell_box.scene.json", 512, 512)
    pt.render(cam, 8, True, chunks=8)
    ref.render(osc.camera, 8, True, chunks=8)
    assert_bitexact(pt.accum(), ref.accum, "C2 512x512x64")
    assert np.array_equal(pt.rng_state(), ref.rng_array())
    assert np.array_equal(pt.get_image_data(), ref.tonemap())


def test_cold_start_prepass_keeps_results(gpu_available, scenes):
    # a cold launch runs the cost pre-pass (nothing written back) and then the launch in cost order:
    # bits and RNG state equal a row-major launch, and the pre-pass left no trace in the state
    W, H = 320, 180
    a = pa.Pathtracer(W, H)
    cam = a.load_scene(str(scenes / "generated_scene.scene.json"))
    b = pa.Pathtracer(W, H)
    b.load_scene(str(scenes / "generated_scene.scene.json"))
    b.set_schedule(1)
    a.render(cam, 8, True, chunks=4)          # cold: pre-pass + sorted order
    b.render(cam, 8, True, chunks=4)          # row-major, no pre-pass
    assert np.array_equal(bits(a.accum()), bits(b.accum()))
    assert np.array_equal(a.rng_state(), b.rng_state())
    pa.camera_rotate(cam, 0.02, 0.03, 0.0)    # camera change: cold again
    a.render(cam, 8, False, chunks=2)
    b.render(cam, 8, False, chunks=2)
    assert np.array_equal(bits(a.accum()), bits(b.accum()))
    # cold launches beyond the run-ahead range: the first render() call split off as a launch of its
    # own (ignoreHistory on it only), then a one-call launch (discarded pre-pass), each after a camera
    # change, then warm launches (the order rebuilt once more without priority)
    for spp, chunks, ignore, move in ((8, 9, True, True), (8, 9, False, False), (32, 3, False, True),
                                      (72, 1, False, True), (8, 12, False, False), (8, 12, True, False)):
        if move:
            pa.camera_rotate(cam, -0.01, 0.02, 0.0)
        a.render(cam, spp, ignore, chunks=chunks)
        b.render(cam, spp, ignore, chunks=chunks)
        assert np.array_equal(bits(a.accum()), bits(b.accum())), (spp, chunks, ignore)
        assert np.array_equal(a.rng_state(), b.rng_state()), (spp, chunks, ignore)
        assert a.frames == b.frames


def test_tonemap_bitexact(gpu_available, scenes):
    pt, cam, ref, osc = pair(scenes / "generated_scene.scene.json", 64, 36)
    pt.render(cam, 8, True, chunks=1)
    ref.render(osc.camera, 8, True, chunks=1)
    for frames in (1, 3, 8):
        assert np.array_equal(pt.tonemap(frames), ref.tonemap(frames))


def test_edge_cases(gpu_available, scenes):
    # 1x1 image, spp 0 (no launch, frame still counted: Pathtracer.cpp:174,226)
    pt, cam, ref, osc = pair(scenes / "cornell_box.scene.json", 1, 1)
    pt.render(cam, 1, True)
    ref.render(osc.camera, 1, True)
    assert_bitexact(pt.accum(), ref.accum, "1x1")
    before = pt.accum()
    pt.render(cam, 0, False)
    assert np.array_equal(bits(pt.accum()), bits(before))
    assert pt.frames == 2
    # no scene: no launch, black image
    empty = pa.Pathtracer(16, 16)
    c = pa.make_camera((0, 0, 0), (0, 0, -1), aspect=1.0)
    empty.render(c, 4, True)
    assert not empty.accum().any()


def test_context_size_limits(gpu_available):
    # tiles are addressed by packed 16-bit coordinates and pixels by 32-bit indices: contexts beyond
    # that are refused with an error, never created with wrapped indices
    with pytest.raises(pa.PathtracerError):
        pa.Pathtracer(32768, 32768)                  # 2^30 pixels
    with pytest.raises(pa.PathtracerError):
        pa.Pathtracer(8 * 65536, 8)                  # 65,536 tiles across
    pt = pa.Pathtracer(8 * 65535, 8)                 # the widest accepted image
    assert pt.rows == 8
    pt.close()


def test_full_resolution_row_subset(gpu_available, scenes):
    # BASELINE config C3 geometry (1920x1080, generated_scene + sky): exact parity on every 45th row
    W, H, stride = 1920, 1080, 45
    pt, cam, ref, osc = pair(scenes / "generated_scene.scene.json", W, H, row_offset=7, row_stride=stride)
    pt.render(cam, 8, True, chunks=1)
    ref.render(osc.camera, 8, True, chunks=1)
    assert_bitexact(pt.accum(), ref.accum, "1080p row subset")


def test_full_frame_bitexact_and_nan_pixels(gpu_available, scenes):
    # BASELINE config C3 geometry, the whole 1920x1080 frame at 32 spp (4 render() calls of 8)
    # against the oracle: every word, and the pixels poisoned by the reference's 0/0 VNDF pdf
    # (MonteCarlo.h:110-113; LAMBERT_GGX with VdotH clamped to 0) counted on both sides -- the one
    # full-frame statistic a change in the pdf path would move
    # 96 spp (12 calls): rays whose t_max rises mid-traversal (the sphere's far-root quirk) are rare;
    # round 4 found a walk that dropped pending boxes on them at the 11th call of this frame
    W, H = 1920, 1080
    pt, cam, ref, osc = pair(scenes / "generated_scene.scene.json", W, H)
    pt.render(cam, 8, True, chunks=12)
    ref.render(osc.camera, 8, True, chunks=12)
    acc = pt.accum()
    nan_gpu = int((~np.isfinite(acc)).any(-1).sum())
    nan_ref = int((~np.isfinite(ref.accum)).any(-1).sum())
    print(f"NaN pixels at 1080p x 96 spp: gpu {nan_gpu}, oracle {nan_ref}")
    assert nan_gpu == nan_ref
    assert_bitexact(acc, ref.accum, "1080p full frame x 96 spp")
    assert np.array_equal(pt.rng_state(), ref.rng_array())


def test_full_size_determinism(gpu_available, scenes):
    # size-independent properties at 1080p: two contexts give identical bits; chunk split invariance
    W, H = 1920, 1080
    a = pa.Pathtracer(W, H)
    cam = a.load_scene(str(scenes / "generated_scene.scene.json"))
    b = pa.Pathtracer(W, H)
    b.load_scene(str(scenes / "generated_scene.scene.json"))
    a.render(cam, 8, True, chunks=4)
    b.render(cam, 8, True, chunks=2)
    b.render(cam, 8, False, chunks=2)
    assert np.array_equal(bits(a.accum()), bits(b.accum()))
    acc = a.accum()
    assert (acc[..., 3] == 1.0).all()
    # LAMBERT_GGX can return pdf = 0/0 = NaN (VNDF pdf with VdotH clamped to 0, MonteCarlo.h:110-113);
    # the reference poisons those pixels too (the oracle reproduces them), but they must stay rare.
    finite = np.isfinite(acc).all(-1)
    assert finite.mean() > 1 - 1e-4
    assert (acc[finite][:, :3] >= 0).all()


def test_statistical_pin_vs_reference_render(gpu_available, scenes, root):
    # The reference's own published cornell_box_4096spp.png (linear block means, tests/golden/):
    # GPU render at 1024x1024 normalised by the sample count must match away from the textured
    # sphere (earth.png is absent here).
    import json
    ref = np.array(json.loads((root / "tests/golden/cornell_ref_blocks.json").read_text())["blocks"])
    pt = pa.Pathtracer(1024, 1024)
    cam = pt.load_scene(str(scenes / "cornell_box.scene.json"))
    pt.render(cam, 8, True, chunks=16)
    lin = pt.accum()[..., :3] / 128.0
    ours = lin.reshape(32, 32, 32, 32, 3).mean(axis=(1, 3))
    mask = np.ones((32, 32), bool)
    mask[3:10, 12:19] = False
    mask[5:11, 9:12] = False
    ratio = ours[mask].mean(0) / ref[mask].mean(0)
    assert np.all(np.abs(ratio - 1.0) < 0.02), ratio
    rel = np.abs(ours[mask] - ref[mask]) / (ref[mask] + 0.02)
    assert np.median(rel) < 0.03, np.median(rel)


def _stress_scene(tmp_path, root):
    import importlib.util
    spec = importlib.util.spec_from_file_location("make_stress_scene", root / "tools" / "make_stress_scene.py")
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod.write_scene(tmp_path / "stress_100k.json", grid=317, skybox=str(root / "scenes" / "skybox.hdr"))


def test_stress_100k_row_subset(gpu_available, tmp_path, root):
    # BASELINE config C5 scene (100,490 objects, 66,737-node BVH in global memory): exact parity on
    # a row subset of the 1080p image with the kernel variant chosen for large scenes
    p = _stress_scene(tmp_path, root)
    W, H, stride = 1920, 1080, 72
    pt, cam, ref, osc = pair(p, W, H, row_offset=5, row_stride=stride)
    pt.render(cam, 4, True, chunks=1)
    ref.render(osc.camera, 4, True, chunks=1)
    assert_bitexact(pt.accum(), ref.accum, "stress 100k row subset")
    assert np.array_equal(pt.rng_state(), ref.rng_array())


def test_stress_100k_rises_exact_and_counted(gpu_available, tmp_path, root):
    # the C5 check above (115 k samples) meets no rising t_max at C5's 0.66 repairs per
    # million samples, so the repair on the deep cache-read walk (variant 46, the build C5 runs) had
    # never met the oracle.  Every 8th row of the 1080p image at 160 spp (41 M samples; 40 spp hold
    # none, 160 hold 5): the oracle's rise count is positive, the default launch and variant 46 are
    # bit-exact, and the instrumented variant-46 launch repairs exactly as often as the oracle's walk
    # raises t_max.
    p = _stress_scene(tmp_path, root)
    W, H, stride, spp, chunks = 1920, 1080, 8, 8, 20
    pt, cam, ref, osc = pair(p, W, H, row_offset=3, row_stride=stride)
    st = pt.rng_state()
    ref.render(osc.camera, spp, True, chunks=chunks, collect_stats=True)
    rises = int(ref.stats[7])
    assert rises > 0, "the sample reaches no rising t_max"
    for variant in (0, 46):
        pt.set_kernel_variant(variant)
        pt.set_rng_state(st)
        pt.render_raw(cam, spp, chunks, True)
        assert_bitexact(pt.accum(), ref.accum, f"stress 100k rises, variant {variant}")
        assert np.array_equal(pt.rng_state(), ref.rng_array()), f"stress 100k rises, variant {variant}: RNG"
    pt.set_kernel_variant(46)
    pt.set_rng_state(st)
    stats = pt.render_instrumented(cam, spp, chunks, True)
    assert stats["repairs"] == rises, (stats["repairs"], rises)
    assert_bitexact(pt.accum(), ref.accum, "stress 100k rises, instrumented variant 46")


def test_cli_headless_outputs(gpu_available, tmp_path, scenes):
    # the `pathtracer` CLI (main.cpp headless path): PNG = tonemapped image flipped vertically,
    # -ohdr = accumulation / frames; the default (one launch) and -call_loop give the same files
    import subprocess
    from pathtracercuda_amd import _native as N
    from PIL import Image
    scene = scenes / "test_shapes.scene.json"
    W, H, SPP = 64, 40, 20                       # 20 spp = render() calls of 8, 8, 4
    outs = {}
    for tag, extra in [("loop", ["-call_loop"]), ("single", [])]:
        png = tmp_path / f"{tag}.png"
        r = subprocess.run([str(N.CLI), "-w", str(W), "-h", str(H), "-spp", str(SPP), *extra, "-o", str(png), str(scene)],
                           capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, r.stdout + r.stderr
        assert "Finished accumulating 20 samples" in r.stdout
        outs[tag] = np.asarray(Image.open(png).convert("RGBA"))
    assert np.array_equal(outs["loop"], outs["single"])
    osc = po.load_scene(scene, W, H)
    ref = po.OracleRenderer(osc, W, H)
    ref.render(osc.camera, 8, True, chunks=2)
    ref.render(osc.camera, 4, False, chunks=1)
    assert np.array_equal(outs["loop"], ref.tonemap()[::-1])
    hdr = tmp_path / "out.hdr"
    r = subprocess.run([str(N.CLI), "-w", str(W), "-h", str(H), "-spp", str(SPP), "-ohdr", "-o", str(hdr), str(scene)],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0
    back = po.read_rgbe(hdr)[::-1]
    want = ref.hdr()
    tol = np.nan_to_num(want[..., :3]).max(-1, keepdims=True) / 128.0 + 1e-30
    finite = np.isfinite(want).all(-1)
    assert (np.abs(back[..., :3] - want[..., :3])[finite] <= tol[finite]).all()


def test_torchrun_unpermute_matches_row_map(gpu_available, root):
    # the one-process-per-GPU gather scatters with the native unpermute kernel (pt_unpermute_bands,
    # the kernel pt_group_gather runs); it must place every band as global_rows() says
    # (own process: a torch.cuda context next to the suite's native contexts)
    import subprocess
    import sys
    code = (
        "from pathtracercuda_amd import _native as N\n"
        "N.hip()\n"
        "import torch\n"
        "from pathtracercuda_amd.distributed import global_rows, max_rows\n"
        "W = 72\n"
        "for H, world, band in ((64, 3, 8), (61, 2, 8), (37, 4, 1)):\n"
        "    g = torch.Generator().manual_seed(H)\n"
        "    full = torch.full((H, W, 4), -1.0, device='cuda')\n"
        "    want = torch.full((H, W, 4), -1.0)\n"
        "    for r in range(world):\n"
        "        part = torch.rand((max_rows(H, world, band), W, 4), generator=g)\n"
        "        idx = torch.tensor(global_rows(H, r, world, band), dtype=torch.long)\n"
        "        want.index_copy_(0, idx, part[: idx.numel()])\n"
        "        pd = part.cuda()\n"
        "        assert N.hip().pt_unpermute_bands(0, full.data_ptr(), pd.data_ptr(), W, H, band, r, world) == 0\n"
        "    assert torch.equal(full.cpu().view(torch.int32), want.view(torch.int32)), (H, world, band)\n"
        "print('ok')\n")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, cwd=str(root), timeout=120)
    assert r.returncode == 0 and r.stdout.strip().endswith("ok"), (r.stdout, r.stderr)


@pytest.mark.parametrize("W,H,band", [(1280, 720, 0), (1004, 604, 0), (1920, 1080, 3)])
def test_strip_units_bitexact(gpu_available, scenes, W, H, band):
    # strip units (a lane whose pixel is done moves on to the next tile of its row strip) change
    # which lane renders a pixel, never how: every K gives the unit-less launch's bits, for 8-spp
    # calls with and without history and for 1-spp frames, on odd image sizes (partial tiles, strips
    # cut by the right edge) and on a band tile (row offset 3 of 8, as a rank's share)
    pt = (pa.Pathtracer(W, H, row_offset=band, row_stride=8, band_rows=8) if band
          else pa.Pathtracer(W, H))
    cam = pt.load_scene(scenes / "generated_scene.scene.json")
    st = pt.rng_state()
    want = None
    for K in (1, 2, 3, 4):
        pt.set_strip_units(K)
        pt.set_rng_state(st)
        pt.render(cam, 8, True)
        pt.render(cam, 8, False)
        pt.render(cam, 1, False, chunks=2)
        pt.render(cam, 4, False, chunks=5)     # >= 16 samples: the cold-start cost pre-pass runs first
        got = (pt.accum().view(np.uint32).copy(), pt.rng_state())
        if want is None:
            want = got
        assert np.array_equal(got[0], want[0]) and np.array_equal(got[1], want[1]), f"strip K={K}"


def test_walk_variants_full_frame_match(gpu_available, scenes):
    # the walk variants (deferred / undeferred, records in LDS / through the caches, 4 / 5 waves per
    # SIMD) on the whole 1080p frame over 16 render() calls with history: rare traversal paths (a
    # leaf that raises t_max and the rebuilt pending set) show up only at this many rays
    W, H = 1920, 1080
    pt = pa.Pathtracer(W, H)
    cam = pt.load_scene(scenes / "generated_scene.scene.json")
    pt.set_strip_units(1)
    st = pt.rng_state()
    want = None
    for variant in (40, 39, 41, 46, 20, 60, 61):
        pt.set_kernel_variant(variant)
        pt.set_rng_state(st)
        for i in range(16):
            pt.render(cam, 8, i == 0)
        got = pt.accum().view(np.uint32).copy()
        if want is None:
            want = got
        diff = int((got != want).any(-1).sum())
        assert diff == 0, f"variant {variant}: {diff} pixels differ from variant 40"


@pytest.mark.parametrize("scene,W,H,calls", [("generated_scene", 1920, 1080, 16), ("test_shapes", 640, 400, 16),
                                              ("cornell_box", 512, 512, 16)])
def test_rise_repair_matches_reference_rule(gpu_available, scenes, scene, W, H, calls):
    # t_max rises only on rays that meet a sphere with t0 <= t_min (the far-root quirk); the child-box
    # walks keep a far child only if it is hit now and rebuild the reference's pending set when a
    # leaf raises t_max (repair_pending).  Variant 1 is the reference's control flow (every far child
    # pushed, tested when popped): the bits must be the same over many calls of whole frames
    pt = pa.Pathtracer(W, H)
    cam = pt.load_scene(scenes / f"{scene}.scene.json")
    pt.set_strip_units(1)
    st = pt.rng_state()
    out = []
    for variant in (0, 1):
        pt.set_kernel_variant(variant)
        pt.set_rng_state(st)
        for i in range(calls):
            pt.render(cam, 8, i == 0)
        out.append(pt.accum().view(np.uint32).copy())
    diff = int((out[0] != out[1]).any(-1).sum())
    assert diff == 0, f"{scene}: {diff} pixels differ from the reference's control flow"


def test_rise_repair_runs_and_is_exact_vs_oracle(gpu_available, scenes):
    # VERDICT r04 "do this" 1.  scenes/rise_repair.scene.json (tools/make_test_fixtures.py) puts the
    # camera and every object inside one large sphere: leaves whose sphere test takes the far root
    # (Hittable.inl:152-158) raise t_max in mid traversal on about a third of the samples, and the
    # reference then tests the boxes it pops at the larger t_max (trace.cu:48-98).
    #  1. the default launch is bit-exact against the ORACLE (not only against variant 1);
    #  2. the instrumented launch's repairs counter (leaf rounds that rebuilt the pending set) is
    #     positive and equals the oracle's count of leaf visits that raised t_max -- the two walks
    #     visit the same leaves in the same order;
    # The negative control (the rebuild switched off changes the result) is test_rise_pair_needs_the_repair:
    # here the BVH puts the dome's leaf where no box was dropped before a rise (0 pixels differ).
    W, H, spp, chunks = 96, 64, 4, 2
    pt, cam, ref, osc = pair(scenes / "rise_repair.scene.json", W, H)
    st = pt.rng_state()
    ref.render(osc.camera, spp, True, chunks=chunks, collect_stats=True)
    rises = int(ref.stats[7])
    assert rises > 0
    for variant in (0, 40, 20, 60, 46):
        pt.set_kernel_variant(variant)
        pt.set_rng_state(st)
        pt.render_raw(cam, spp, chunks, True)
        assert_bitexact(pt.accum(), ref.accum, f"rise scene, variant {variant}")
        assert np.array_equal(pt.rng_state(), ref.rng_array()), f"rise scene, variant {variant}: RNG"
    for variant in (40, 20, 60, 61, 46):
        pt.set_kernel_variant(variant)
        pt.set_rng_state(st)
        stats = pt.render_instrumented(cam, spp, chunks, True)
        assert stats["repairs"] == rises, (variant, stats["repairs"], rises)
        assert_bitexact(pt.accum(), ref.accum, f"rise scene, instrumented variant {variant}")


def test_rise_pair_needs_the_repair(gpu_available, scenes):
    # scenes/rise_pair.scene.json with the caller BVH of tests/bvh_edit.py rise_pair_bvh(): every ray
    # that hits sphere A raises t_max at the dome's leaf after the wall B's leaf was dropped by the
    # hit-now rule; the reference pops B's leaf at the raised t_max and B wins (trace.cu:48-98).
    #  1. default launch (and the child-box variants) bit-exact vs the oracle on that BVH;
    #  2. repairs counter == the oracle's rise count, and positive;
    #  3. negative control: variant 40 built without the rebuild (pt_set_rise_repair(0)) is NOT the
    #     oracle's -- on most pixels of A -- so the scene exercises the repair.
    import ctypes as C
    import bvh_edit as be
    W, H, spp, chunks = 96, 64, 4, 2
    path = scenes / "rise_pair.scene.json"
    pt, cam, ref, osc = pair(path, W, H)
    objs, aabbs = pa.Scene(str(path), W, H).objects()
    nodes, order = be.rise_pair_bvh(aabbs)
    sz = C.sizeof(pa.PtHittable)
    raw = b"".join(bytes(objs)[o * sz:(o + 1) * sz] for o in order)
    ref_nodes = (po.BVHNode * len(nodes))()
    for i, (lo, hi, off, pca) in enumerate(nodes):
        ref_nodes[i].bmin[:] = list(lo)
        ref_nodes[i].bmax[:] = list(hi)
        ref_nodes[i].offset = off
        ref_nodes[i].primitiveCountAxis = pca
    osc.nodes, osc.node_count = ref_nodes, len(nodes)
    osc.prims, osc.prim_count = (po.Hittable * len(order)).from_buffer_copy(raw), len(order)
    ref.render(osc.camera, spp, True, chunks=chunks, collect_stats=True)
    rises = int(ref.stats[7])
    assert rises > 0
    N.check_ctx(N.hip().pt_set_scene(pt._ctx, _bvh_array(nodes), len(nodes),
                                     (pa.PtHittable * len(order)).from_buffer_copy(raw), len(order)), pt._ctx)
    st = pt.rng_state()
    for variant in (0, 40, 41, 39, 20, 1, 60, 61, 46):
        pt.set_kernel_variant(variant)
        pt.set_rng_state(st)
        pt.render_raw(cam, spp, chunks, True)
        assert_bitexact(pt.accum(), ref.accum, f"rise pair, variant {variant}")
        assert np.array_equal(pt.rng_state(), ref.rng_array()), f"rise pair, variant {variant}: RNG"
    for variant in (40, 20, 60, 61, 46):
        pt.set_kernel_variant(variant)
        pt.set_rng_state(st)
        assert pt.render_instrumented(cam, spp, chunks, True)["repairs"] == rises, variant
    pt.set_kernel_variant(40)
    pt.set_rise_repair(False)
    pt.set_rng_state(st)
    pt.render_raw(cam, spp, chunks, True)
    got = pt.accum()
    pt.set_rise_repair(True)
    differ = int((bits(got) != bits(ref.accum)).any(-1).sum())
    assert differ > 0.05 * W * H, f"negative control: only {differ} pixels differ without the repair"


def _bvh_array(nodes):
    arr = (pa.PtBvhNode * len(nodes))()
    for i, (lo, hi, off, pca) in enumerate(nodes):
        arr[i].aabb_min[:] = list(lo)
        arr[i].aabb_max[:] = list(hi)
        arr[i].offset = off
        arr[i].primitive_count_axis = pca
    return arr


def _set_caller_bvh(pt, osc, nodes):
    """Hand a caller BVH (tests/bvh_edit.py node tuples) to pt_set_scene with the scene's primitives."""
    import ctypes as C
    arr = _bvh_array(nodes)
    prims = (pa.PtHittable * osc.prim_count).from_buffer_copy(bytes(osc.prims)[:osc.prim_count * C.sizeof(pa.PtHittable)])
    N.check_ctx(N.hip().pt_set_scene(pt._ctx, arr, len(nodes), prims, osc.prim_count), pt._ctx)


def test_orphan_node_bvh_renders_exactly(gpu_available, scenes):
    # a caller BVH with an unreachable interior node that names a deep reachable node as
    # its child.  The stack-row bound is now taken over the tree reachable from the root (the
    # array-order form gave 16 rows instead of 29 here, tests/test_bvh_validation.py), so the walks
    # stay inside their LDS rows; the render equals the oracle's on the same tree without the orphan.
    from test_bvh_validation import orphan_caterpillar
    W, H = 96, 64
    pt, cam, ref, osc = pair(scenes / "generated_scene.scene.json", W, H)
    cat, bad = orphan_caterpillar(osc)
    ref_nodes = (po.BVHNode * len(cat))()
    for i, (lo, hi, off, pca) in enumerate(cat):
        ref_nodes[i].bmin[:] = list(lo)
        ref_nodes[i].bmax[:] = list(hi)
        ref_nodes[i].offset = off
        ref_nodes[i].primitiveCountAxis = pca
    osc.nodes = ref_nodes
    osc.node_count = len(cat)
    ref.render(osc.camera, 4, True, chunks=2)
    _set_caller_bvh(pt, osc, bad)
    st = pt.rng_state()
    for variant in (0, 40, 41, 39, 20, 60, 61):
        pt.set_kernel_variant(variant)
        pt.set_rng_state(st)
        pt.render_raw(cam, 4, 2, True)
        assert_bitexact(pt.accum(), ref.accum, f"orphan BVH, variant {variant}")
    # unreachable nodes whose offsets point outside the arrays (and one at the last
    # index) are never read by the upload either; the render is unchanged
    from bvh_edit import append_malformed_orphans
    _set_caller_bvh(pt, osc, append_malformed_orphans(bad))
    for variant in (0, 60, 20):
        pt.set_kernel_variant(variant)
        pt.set_rng_state(st)
        pt.render_raw(cam, 4, 2, True)
        assert_bitexact(pt.accum(), ref.accum, f"malformed orphans, variant {variant}")


def test_forced_strip_variant_without_child_box_layout(gpu_available, scenes):
    # a forced child-box variant with strip units on a scene outside the child-box
    # encoding (one leaf of 484 > 255 primitives) runs the node-at-a-time walk, unit-less: every tile
    # rendered, the oracle's bits (before round 5 only the first tile of each strip was rendered)
    import ctypes as C
    from pathtracercuda_amd import _native as N
    W, H = 256, 96
    pt, cam, ref, osc = pair(scenes / "generated_scene.scene.json", W, H)
    root = po.BVHNode.from_buffer_copy(bytes(osc.nodes[0]))
    root.offset = 0
    root.primitiveCountAxis = osc.prim_count << 16
    osc.nodes = (po.BVHNode * 1)(root)
    osc.node_count = 1
    nodes = (pa.PtBvhNode * 1).from_buffer_copy(bytes(osc.nodes))
    prims = (pa.PtHittable * osc.prim_count).from_buffer_copy(bytes(osc.prims)[:osc.prim_count * C.sizeof(pa.PtHittable)])
    N.check_ctx(N.hip().pt_set_scene(pt._ctx, nodes, 1, prims, osc.prim_count), pt._ctx)
    ref.render(osc.camera, 1, True, chunks=2)
    st = pt.rng_state()
    for variant in (40, 41, 46, 60, 61):
        pt.set_kernel_variant(variant)
        pt.set_strip_units(4)
        pt.set_rng_state(st)
        pt.render_raw(cam, 1, 2, True)
        assert_bitexact(pt.accum(), ref.accum, f"no child-box layout, forced variant {variant}, strip 4")


CALL_PLAN = [  # (spp, ignore_history, camera move before the call): the reference's loop with changes
    (8, True, False), (8, False, False), (8, False, False), (8, False, False), (8, False, True),
    (8, False, False), (8, False, False), (4, False, False), (4, False, False), (16, False, False),
    (8, True, False), (8, False, False), (1, False, False), (8, False, False), (8, False, False), (8, False, False)]


@pytest.mark.parametrize("W,H", [(200, 120), (1280, 720)])
def test_run_ahead_call_loop_bitexact_vs_oracle(gpu_available, scenes, W, H):
    # VERDICT r04 "do this" 3: run-ahead across render() calls (MODE 4).  16 separate render() calls
    # as main.cpp:272-279 makes them, with a camera move, spp changes (8 -> 4: stashes longer than the
    # call are dropped; 4 -> 16; a 1-spp call), an ignoreHistory reset and an RNG overwrite in between;
    # after every call the accumulation and RNG state are the oracle's.  1280x720 runs the persistent
    # grid, 200x120 the one-pass grid.  Mode 2 makes a stash at every launch.
    pt, cam, ref, osc = pair(scenes / "generated_scene.scene.json", W, H)
    pt.set_run_ahead(2)
    cam_g, cam_o = cam, osc.camera
    for i, (spp, ignore, move) in enumerate(CALL_PLAN):
        if move:
            cam_g = pa.camera_rotate(pa.PtCamera.from_buffer_copy(bytes(cam_g)), 0.02, -0.03)
            cam_o = po.Camera.from_buffer_copy(bytes(cam_g))
        if i == 14:                                  # pt_write_rng voids a stash (stateEpoch)
            s = pt.rng_state()
            pt.set_rng_state(s)
        pt.render(cam_g, spp, ignore)
        ref.render(cam_o, spp, ignore)
        if i in (0, 3, 4, 7, 9, 10, 12, 15):
            assert_bitexact(pt.accum(), ref.accum, f"call {i} ({spp} spp)")
            assert np.array_equal(pt.rng_state(), ref.rng_array()), f"call {i}: RNG"
    assert pt.frames == ref.frames


def test_run_ahead_modes_same_bits_full_frame(gpu_available, scenes):
    # the whole 1080p frame, 24 calls of 8 spp: run-ahead automatic, off, always, made but never used
    # -- identical accumulation and RNG state; the fused launch agrees
    W, H = 1920, 1080
    pt = pa.Pathtracer(W, H)
    cam = pt.load_scene(scenes / "generated_scene.scene.json")
    st = pt.rng_state()
    want = None
    for mode in (0, 1, 2, 3):
        pt.set_run_ahead(mode)
        pt.set_rng_state(st)
        for i in range(24):
            pt.render(cam, 8, i == 0)
        got = (pt.accum().view(np.uint32).copy(), pt.rng_state())
        if want is None:
            want = got
        assert np.array_equal(got[0], want[0]) and np.array_equal(got[1], want[1]), f"run-ahead mode {mode}"
    pt.set_run_ahead(1)
    pt.set_rng_state(st)
    pt.render(cam, 8, True, chunks=24)
    assert np.array_equal(pt.accum().view(np.uint32), want[0]) and np.array_equal(pt.rng_state(), want[1])


def test_six_wave_policy(gpu_available, scenes):
    # the default runs the six-wave build (variant 60) on a
    # launch of many tiles per slot and the five-wave build on a chain-bound share of few tiles per
    # slot; the bits are the same either way
    pt = pa.Pathtracer(1920, 1080)
    cam = pt.load_scene(scenes / "generated_scene.scene.json")
    st = pt.rng_state()
    pt.render_raw(cam, 8, 16, True)
    assert pt.last_variant == 60
    want = pt.accum().view(np.uint32).copy()
    pt.set_kernel_variant(40)
    pt.set_rng_state(st)
    pt.render_raw(cam, 8, 16, True)
    assert pt.last_variant == 40 and np.array_equal(pt.accum().view(np.uint32), want)
    share = pa.Pathtracer(1920, 1080, row_offset=0, row_stride=2, band_rows=8)
    cam = share.load_scene(scenes / "generated_scene.scene.json")
    share.set_sample_groups(1)
    share.render_raw(cam, 8, 16, True)
    assert share.last_variant == 40
