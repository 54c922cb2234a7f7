"""MI355X-native path tracer with the capabilities of DoerriesT/PathtracerCUDA's hot path.

Python mirror of the reference's host interface (PathtracerCUDA/src/pathtracer/Pathtracer.h:12-68,
SceneLoader.h, Camera.h) over the native libraries:

    pt = Pathtracer(width, height)            # Pathtracer(w, h)            Pathtracer.cpp:30
    cam = pt.load_scene("scene.json")         # loadScene(pt, params)        SceneLoader.cpp:124
    pt.render(cam, 8, ignore_history=True)    # render(camera, spp, ignore)  Pathtracer.cpp:162
    ms = pt.get_timing()                      # getTiming()                  Pathtracer.cpp:229
    hdr = pt.get_hdr_image_data()             # getHDRImageData()            Pathtracer.cpp:299
    rgba8 = pt.get_image_data()               # getImageData()               Pathtracer.cpp:317

All rendering runs in hand-written HIP kernels for gfx950 (libpt_hip.so); scene loading, the SAH
BVH and frame accounting run in host C++ (libpt_host.so).  There is no CPU fallback.
"""
from __future__ import annotations

import ctypes as C
import os
from typing import Dict, Optional, Sequence

import numpy as np

from . import _native as N
from ._native import PathtracerError, PtBvhNode, PtCamera, PtHittable, PtRenderStats, device_count

__all__ = ["Pathtracer", "Scene", "make_camera", "camera_rotate", "camera_translate", "radians", "device_count", "PathtracerError", "PtCamera",
           "PtBvhNode", "PtHittable", "write_png", "write_hdr", "HITTABLE_TYPES", "MATERIAL_TYPES"]

HITTABLE_TYPES = ["SPHERE", "CYLINDER", "DISK", "CONE", "PARABOLOID", "QUAD", "CUBE"]   # Hittable.h:9-12
MATERIAL_TYPES = ["LAMBERT", "GGX", "LAMBERT_GGX"]                                     # Material.h:9-12


def _f3(v: Sequence[float]):
    return (C.c_float * 3)(*[float(np.float32(x)) for x in v])


def radians(degrees: float) -> float:
    """SceneLoader.cpp:193-196 (float arithmetic)."""
    return float(N.host().pth_radians(float(degrees)))


def make_camera(position, look_at, up=(0.0, 1.0, 0.0), fovy_radians: float = 1.0471976, aspect: float = 1.0) -> PtCamera:
    """Camera ctor (Camera.inl:4-23)."""
    cam = PtCamera()
    N.check_host(N.host().pth_camera_make(_f3(position), _f3(look_at), _f3(up), float(fovy_radians), float(aspect),
                                          C.byref(cam)))
    return cam


def camera_rotate(camera: PtCamera, pitch: float, yaw: float, roll: float = 0.0) -> PtCamera:
    """Camera::rotate (Camera.inl:30-45), in place; returns the camera."""
    N.check_host(N.host().pth_camera_rotate(C.byref(camera), float(pitch), float(yaw), float(roll)))
    return camera


def camera_translate(camera: PtCamera, x: float, y: float, z: float) -> PtCamera:
    """Camera::translate (Camera.inl:47-51), in place; returns the camera."""
    N.check_host(N.host().pth_camera_translate(C.byref(camera), float(x), float(y), float(z)))
    return camera


def write_png(path: str, rgba: np.ndarray, flip: bool = True) -> None:
    a = np.ascontiguousarray(rgba, dtype=np.uint8)
    h, w = a.shape[:2]
    N.check_host(N.host().pth_write_png(os.fsencode(path), w, h, a.ctypes.data_as(C.POINTER(C.c_uint8)), int(flip)))


def write_hdr(path: str, rgba: np.ndarray, flip: bool = True) -> None:
    a = np.ascontiguousarray(rgba, dtype=np.float32)
    h, w = a.shape[:2]
    N.check_host(N.host().pth_write_hdr(os.fsencode(path), w, h, a.ctypes.data_as(C.POINTER(C.c_float)), int(flip)))


class Scene:
    """A parsed scene file (no GPU): objects in file order, the SAH BVH, camera, textures."""

    def __init__(self, path: str, width: int, height: int) -> None:
        self._h = C.c_void_p()
        N.check_host(N.host().pth_scene_load(os.fsencode(str(path)), int(width), int(height), C.byref(self._h)))
        self.path = str(path)

    def __del__(self) -> None:
        h = getattr(self, "_h", None)
        if h:
            N.host().pth_scene_free(h)
            self._h = None

    def timing(self) -> Dict[str, float]:
        """Host wall time of the load: {"parse_ms": JSON + transforms, "bvh_ms": SAH build}."""
        a, b = C.c_double(), C.c_double()
        N.check_host(N.host().pth_scene_timing(self._h, C.byref(a), C.byref(b)))
        return {"parse_ms": a.value, "bvh_ms": b.value}

    @property
    def object_count(self) -> int:
        return int(N.host().pth_scene_object_count(self._h))

    @property
    def node_count(self) -> int:
        return int(N.host().pth_scene_node_count(self._h))

    @property
    def bvh_depth(self) -> int:
        return int(N.host().pth_scene_bvh_depth(self._h))

    def objects(self):
        n = self.object_count
        objs = (PtHittable * max(1, n))()
        aabbs = np.zeros((n, 6), dtype=np.float32)
        N.check_host(N.host().pth_scene_objects(self._h, objs, aabbs.ctypes.data_as(C.POINTER(C.c_float))))
        return objs, aabbs

    def bvh(self):
        nodes = (PtBvhNode * max(1, self.node_count))()
        prims = (PtHittable * max(1, self.object_count))()
        N.check_host(N.host().pth_scene_bvh(self._h, nodes, prims))
        return nodes, prims

    def camera(self) -> PtCamera:
        cam = PtCamera()
        N.check_host(N.host().pth_scene_camera(self._h, C.byref(cam)))
        return cam

    @property
    def skybox(self) -> int:
        return int(N.host().pth_scene_skybox(self._h))

    def textures(self):
        out = []
        for handle in range(1, int(N.host().pth_scene_texture_count(self._h)) + 1):
            w, h = C.c_uint32(), C.c_uint32()
            N.check_host(N.host().pth_scene_texture_info(self._h, handle, C.byref(w), C.byref(h)))
            t = np.zeros((h.value, w.value, 4), dtype=np.float32)
            N.check_host(N.host().pth_scene_texture_data(self._h, handle, t.ctypes.data_as(C.POINTER(C.c_float))))
            out.append(t)
        return out


class Pathtracer:
    """The reference's Pathtracer on one MI355X, on a row-band tile of the image, or on several GPUs.

    Tiles: the image is cut into bands of `band_rows` rows and this object renders the bands
    b = row_offset + k * row_stride (band_rows = 1: rows y = row_offset + k * row_stride).
    `devices=[...]` spans several GPUs of this process (pt_group_*, RCCL gather; 8-row bands unless
    `band_rows` says otherwise, as the C++ constructor and the CLI): the image calls (accum,
    get_hdr_image_data, get_image_data, tonemap, rng_state) then cover the full image, the tuning
    knobs apply to every device, and the per-context diagnostics raise PathtracerError.
    """

    def __init__(self, width: int, height: int, device: int = 0, row_offset: int = 0, row_stride: int = 1,
                 band_rows: Optional[int] = None, devices: Optional[Sequence[int]] = None) -> None:
        self._r = C.c_void_p()
        if band_rows is None:
            band_rows = 8 if devices is not None else 1
        if devices is not None:
            devs = (C.c_int * len(devices))(*[int(d) for d in devices])
            N.check_host(N.host().pth_renderer_create_group(int(width), int(height), len(devices), devs, int(band_rows),
                                                            C.byref(self._r)))
        else:
            N.check_host(N.host().pth_renderer_create_banded(int(width), int(height), int(device), int(band_rows),
                                                             int(row_offset), int(row_stride), C.byref(self._r)))
        self.width, self.height = int(width), int(height)
        self.device = int(device)
        self.row_offset, self.row_stride, self.band_rows = int(row_offset), int(row_stride), int(band_rows)
        self.devices = list(devices) if devices is not None else None
        self.rows = int(N.host().pth_renderer_local_rows(self._r))
        self._ctx = N.host().pth_renderer_context(self._r)
        self._group = N.host().pth_renderer_group(self._r)

    # --- device groups ------------------------------------------------------------------------
    def _contexts(self):
        """Every device context: the group's, or this object's one."""
        if not self._group:
            return [self._ctx]
        return [N.hip().pt_group_context(self._group, i) for i in range(int(N.hip().pt_group_size(self._group)))]

    def _single(self, what: str) -> None:
        if self._group:
            raise PathtracerError(N.PT_ERR_STATE, f"{what}: per-context call, not available on a device group "
                                                  f"(use pt_group_context(i) through the C ABI)")

    def _group_rows(self):
        """Per device of a group: (context, its local rows' global row indices)."""
        out = []
        n = len(self.devices)
        shift = self.band_rows.bit_length() - 1
        for i, c in enumerate(self._contexts()):
            rows = int(N.hip().pt_local_rows(c))
            ly = np.arange(rows, dtype=np.int64)
            out.append((c, ((i + (ly >> shift) * n) << shift) + (ly & (self.band_rows - 1))))
        return out

    def close(self) -> None:
        if getattr(self, "_r", None):
            N.host().pth_renderer_destroy(self._r)
            self._r = None

    def __del__(self) -> None:
        self.close()

    def __enter__(self) -> "Pathtracer":
        return self

    def __exit__(self, *exc) -> None:
        self.close()

    # --- reference API --------------------------------------------------------------------------
    def load_scene(self, path: str) -> PtCamera:
        cam = PtCamera()
        N.check_host(N.host().pth_renderer_load_scene(self._r, os.fsencode(str(path)), C.byref(cam)))
        return cam

    def render(self, camera: PtCamera, spp: int, ignore_history: bool, chunks: int = 1) -> None:
        """`chunks` x render(camera, spp, ignore_history and first) in one kernel launch."""
        N.check_host(N.host().pth_renderer_render(self._r, C.byref(camera), int(spp), int(chunks), int(bool(ignore_history))))

    def get_timing(self) -> float:
        return float(N.host().pth_renderer_timing(self._r))

    @property
    def frames(self) -> int:
        return int(N.host().pth_renderer_frames(self._r))

    def get_hdr_image_data(self) -> np.ndarray:
        p = N.host().pth_renderer_hdr(self._r)
        if not p:
            N.check_host(N.PT_ERR_HIP)
        return np.ctypeslib.as_array(p, shape=(self.rows, self.width, 4)).copy()

    def get_image_data(self) -> np.ndarray:
        p = N.host().pth_renderer_image(self._r)
        if not p:
            N.check_host(N.PT_ERR_HIP)
        return np.ctypeslib.as_array(p, shape=(self.rows, self.width, 4)).copy()

    # --- device-layer access (C ABI of pt_hip.h) ------------------------------------------------
    def accum(self) -> np.ndarray:
        """Raw accumulation sums (rows x width x 4 float32); the gathered full image for a group."""
        out = np.zeros((self.rows, self.width, 4), dtype=np.float32)
        if self._group:
            N.check_group(N.hip().pt_group_read_accum(self._group, out.ctypes.data_as(C.POINTER(C.c_float))), self._group)
        else:
            N.check_ctx(N.hip().pt_read_accum(self._ctx, out.ctypes.data_as(C.POINTER(C.c_float))), self._ctx)
        return out

    def gather(self) -> float:
        """Group only: RCCL gather of every device's rows to devices[0]; returns its wall time in ms."""
        ms = C.c_float(0.0)
        N.check_group(N.hip().pt_group_gather(self._group, C.byref(ms)), self._group)
        return float(ms.value)

    def rng_state(self) -> np.ndarray:
        out = np.zeros((self.rows, self.width, 6), dtype=np.uint32)
        if self._group:
            for c, gy in self._group_rows():
                part = np.zeros((gy.size, self.width, 6), dtype=np.uint32)
                N.check_ctx(N.hip().pt_read_rng(c, part.ctypes.data_as(C.POINTER(C.c_uint32))), c)
                out[gy] = part
            return out
        N.check_ctx(N.hip().pt_read_rng(self._ctx, out.ctypes.data_as(C.POINTER(C.c_uint32))), self._ctx)
        return out

    def set_rng_state(self, state: np.ndarray) -> None:
        s = np.ascontiguousarray(state, dtype=np.uint32)
        if s.shape != (self.rows, self.width, 6):
            raise PathtracerError(N.PT_ERR_ARG, f"set_rng_state: shape {s.shape}, expected {(self.rows, self.width, 6)}")
        if self._group:
            for c, gy in self._group_rows():
                part = np.ascontiguousarray(s[gy])
                N.check_ctx(N.hip().pt_write_rng(c, part.ctypes.data_as(C.POINTER(C.c_uint32))), c)
            return
        N.check_ctx(N.hip().pt_write_rng(self._ctx, s.ctypes.data_as(C.POINTER(C.c_uint32))), self._ctx)

    def render_raw(self, camera: PtCamera, spp: int, chunks: int, ignore_history: bool) -> float:
        """Device-layer launch without frame accounting; returns the kernel time in ms (a group: every
        device concurrently, the slowest device's time; the next image read gathers again)."""
        ms = C.c_float(0.0)
        if self._group:
            N.check_group(N.hip().pt_group_render(self._group, C.byref(camera), int(spp), int(chunks),
                                                  int(bool(ignore_history)), C.byref(ms)), self._group)
            return float(ms.value)
        N.check_ctx(N.hip().pt_render(self._ctx, C.byref(camera), int(spp), int(chunks), int(bool(ignore_history)),
                                      C.byref(ms)), self._ctx)
        return float(ms.value)

    def render_instrumented(self, camera: PtCamera, spp: int, chunks: int, ignore_history: bool) -> Dict[str, int]:
        self._single("render_instrumented")
        ms = C.c_float(0.0)
        st = PtRenderStats()
        N.check_ctx(N.hip().pt_render_instrumented(self._ctx, C.byref(camera), int(spp), int(chunks),
                                                   int(bool(ignore_history)), C.byref(ms), C.byref(st)), self._ctx)
        d = {name: int(getattr(st, name)) for name, _ in PtRenderStats._fields_}
        d["ms"] = float(ms.value)
        return d

    def set_kernel_variant(self, variant: int) -> None:
        """pt_set_kernel_variant on every device context."""
        for c in self._contexts():
            N.check_ctx(N.hip().pt_set_kernel_variant(c, int(variant)), c)

    def set_occupancy(self, workgroups_per_cu: int) -> None:
        """Persistent grids hold at most this many 4-wave workgroups per CU (waves per SIMD); 0 = all
        that fit (pt_set_occupancy).  A measurement knob: results are identical."""
        for c in self._contexts():
            N.check_ctx(N.hip().pt_set_occupancy(c, int(workgroups_per_cu)), c)

    def set_issue_priority(self, mode: int, level3: int = 0, level2: int = 0, level1: int = 0) -> None:
        """Issue priority by cost-order position (pt_set_issue_priority): mode 0 automatic, 1 off,
        2 explicit (positions < level3 at priority 3, < level2 at 2, < level1 at 1).  Results are
        identical."""
        for c in self._contexts():
            N.check_ctx(N.hip().pt_set_issue_priority(c, int(mode), int(level3), int(level2), int(level1)), c)

    def set_schedule(self, mode: int) -> None:
        """0 = cost-sorted tile dispatch (default), 1 = row-major (pt_set_schedule), every device."""
        for c in self._contexts():
            N.check_ctx(N.hip().pt_set_schedule(c, int(mode)), c)

    def set_strip_units(self, mode: int) -> None:
        """pt_set_strip_units on every device context (0 automatic, 1 off, K >= 2 always K tiles per unit)."""
        for c in self._contexts():
            N.check_ctx(N.hip().pt_set_strip_units(c, int(mode)), c)

    def set_run_ahead(self, mode: int) -> None:
        """Run-ahead across render() calls (pt_set_run_ahead): 0 automatic, 1 off, 2 always make a
        stash, 3 make stashes but never use them (diagnostic).  Results are the reference's for every
        setting."""
        for c in self._contexts():
            N.check_ctx(N.hip().pt_set_run_ahead(c, int(mode)), c)

    def set_cold_start(self, prepass_spp: int = 0, priority: bool = True) -> None:
        """Cold-start scheduling (pt_set_cold_start): cost pre-pass spp (0 = default) and issue
        priority on the pre-pass's order.  Results are identical for every setting."""
        for c in self._contexts():
            N.check_ctx(N.hip().pt_set_cold_start(c, int(prepass_spp), int(bool(priority))), c)

    def set_rise_repair(self, enabled: bool) -> None:
        """Test knob (pt_set_rise_repair): False skips the rebuild of the pending far children after a
        leaf raised t_max, so results are NOT the reference's on such rays (negative control)."""
        for c in self._contexts():
            N.check_ctx(N.hip().pt_set_rise_repair(c, int(bool(enabled))), c)

    def set_sample_groups(self, mode: int) -> None:
        """Speculative sample groups (pt_set_sample_groups): 0 = automatic, 1 = off, G >= 2 = always G."""
        for c in self._contexts():
            N.check_ctx(N.hip().pt_set_sample_groups(c, int(mode)), c)

    @property
    def last_sample_groups(self) -> int:
        """Groups of the last launch (a device group: the largest over its devices)."""
        return max(int(N.hip().pt_last_sample_groups(c)) for c in self._contexts())

    @property
    def last_variant(self) -> int:
        """Trace-kernel variant of the last launch's main pass (a device group: device 0's)."""
        return int(N.hip().pt_last_variant(self._contexts()[0]))

    def set_patch_rounds(self, rounds: int) -> None:
        for c in self._contexts():
            N.check_ctx(N.hip().pt_set_patch_rounds(c, int(rounds)), c)

    def set_group_lookback(self, far: int = 64, near: int = 16) -> None:
        """Sample groups: a second phase also stops on a junction with its first phase `far` or
        `near` samples back (0 = off).  Scheduling only (pt_set_group_lookback)."""
        for c in self._contexts():
            N.check_ctx(N.hip().pt_set_group_lookback(c, int(far), int(near)), c)

    def group_fold_word(self, word: int) -> np.ndarray:
        """Diagnostics: a plane of the grouped launch's fold state (pt_read_group_fold); words 19 /
        20 / 21 = the guess statistics (float32): draw pairs per sample, odd-length fraction, variance."""
        self._single("group_fold_word")
        out = np.zeros((self.rows, self.width), dtype=np.uint32)
        N.check_ctx(N.hip().pt_read_group_fold(self._ctx, int(word), out.ctypes.data_as(C.POINTER(C.c_uint32))), self._ctx)
        return out.view(np.float32) if word >= 19 else out

    def group_stats(self) -> Dict[str, object]:
        """How the last grouped launch went: groups, patch rounds, dead-end pixels after each fold."""
        self._single("group_stats")
        out = (C.c_uint32 * 10)()
        N.check_ctx(N.hip().pt_read_group_stats(self._ctx, out), self._ctx)
        v = list(out)
        return {"groups": v[0], "patch_rounds": v[1], "dead_ends": v[2:2 + v[1] + 1] if v[0] else []}

    def group_log_counts(self) -> np.ndarray:
        """Samples each (tile, item) of the last grouped launch logged: (tiles, 2 * groups - 1, 64), tiles
        in dispatch (cost) order; item 0 = group 0, items 2g - 1 and 2g = group g at its guess and one
        draw pair later."""
        self._single("group_log_counts")
        g = 2 * self.last_sample_groups - 1
        tiles = ((self.width + 7) // 8) * ((self.rows + 7) // 8)
        out = np.zeros((tiles, g, 64), dtype=np.uint32)
        N.check_ctx(N.hip().pt_read_group_log_counts(self._ctx, out.ctypes.data_as(C.POINTER(C.c_uint32)), out.size),
                    self._ctx)
        return out

    def tile_costs(self) -> np.ndarray:
        """Shader-clock cycles of each 8x8 tile in the last launch (tiles_y x tiles_x)."""
        self._single("tile_costs")
        tx, ty = (self.width + 7) // 8, (self.rows + 7) // 8
        out = np.zeros(tx * ty, dtype=np.uint32)
        N.check_ctx(N.hip().pt_read_tile_costs(self._ctx, out.ctypes.data_as(C.POINTER(C.c_uint32)), tx * ty), self._ctx)
        return out.reshape(ty, tx)

    def tile_idle(self) -> np.ndarray:
        """Per tile of the last instrumented launch: mean lane cycles spent done while the tile ran
        (tiles_y x tiles_x; divide by tile_costs() for the idle-lane fraction)."""
        self._single("tile_idle")
        tx, ty = (self.width + 7) // 8, (self.rows + 7) // 8
        out = np.zeros(tx * ty, dtype=np.uint32)
        N.check_ctx(N.hip().pt_read_tile_idle(self._ctx, out.ctypes.data_as(C.POINTER(C.c_uint32)), tx * ty), self._ctx)
        return out.reshape(ty, tx)

    def set_tile_trace(self, enabled: bool) -> None:
        """Instrumented launches also record per tile the start cycle and hardware ids of the wave
        that ran it (diagnostics)."""
        for c in self._contexts():
            N.check_ctx(N.hip().pt_set_tile_trace(c, int(bool(enabled))), c)

    def tile_trace(self) -> np.ndarray:
        """Last traced launch: (tiles_y x tiles_x x 2) u32 -- start cycle (low 32 bits) and
        XCC_ID << 16 | HW_ID (bits 0-15) of the wave that ran each tile."""
        self._single("tile_trace")
        tx, ty = (self.width + 7) // 8, (self.rows + 7) // 8
        out = np.zeros(2 * tx * ty, dtype=np.uint32)
        N.check_ctx(N.hip().pt_read_tile_trace(self._ctx, out.ctypes.data_as(C.POINTER(C.c_uint32)), 2 * tx * ty),
                    self._ctx)
        return out.reshape(ty, tx, 2)

    def copy_accum_to_device(self, dst_ptr: int, nbytes: int) -> None:
        self._single("copy_accum_to_device")
        N.check_ctx(N.hip().pt_copy_accum_device(self._ctx, C.c_void_p(int(dst_ptr)), int(nbytes)), self._ctx)

    def tonemap_device(self, dst_ptr: int, nbytes: int, frames: Optional[int] = None) -> None:
        """Tonemap into a device buffer (RGBA8, rows x width) -- the pixel-buffer path of render()."""
        self._single("tonemap_device")
        f = self.frames if frames is None else int(frames)
        N.check_ctx(N.hip().pt_tonemap_device(self._ctx, f, C.c_void_p(int(dst_ptr)), int(nbytes)), self._ctx)

    def tonemap(self, frames: Optional[int] = None) -> np.ndarray:
        out = np.zeros((self.rows, self.width, 4), dtype=np.uint8)
        f = self.frames if frames is None else int(frames)
        if self._group:
            N.check_group(N.hip().pt_group_tonemap(self._group, f, out.ctypes.data_as(C.POINTER(C.c_uint8))), self._group)
            return out
        N.check_ctx(N.hip().pt_tonemap(self._ctx, f, out.ctypes.data_as(C.POINTER(C.c_uint8))), self._ctx)
        return out
