"""ctypes bindings of the native libraries (include/pt_hip.h, include/pt_host.h).

The libraries are built in-tree by `make` (or __graft_entry__.build()) into
pathtracercuda_amd/lib/.  There is no fallback: if they are missing the import fails loudly.
"""
from __future__ import annotations

import ctypes as C
import importlib.util
import os
import pathlib
import sys

LIB_DIR = pathlib.Path(__file__).resolve().parent / "lib"
HIP_LIB = LIB_DIR / "libpt_hip.so"
HOST_LIB = LIB_DIR / "libpt_host.so"
CLI = LIB_DIR / "pathtracer"

PT_OK, PT_ERR_HIP, PT_ERR_ARG, PT_ERR_STATE, PT_ERR_DEPTH, PT_ERR_NO_DEVICE = range(6)
PT_MAX_TEXTURES = 64


class PtCamera(C.Structure):
    """pt_camera (reference Camera.h:14-22)."""
    _fields_ = [("tan_half_fovy", C.c_float), ("aspect_ratio", C.c_float), ("origin", C.c_float * 3),
                ("lower_left_corner", C.c_float * 3), ("horizontal", C.c_float * 3), ("vertical", C.c_float * 3),
                ("right", C.c_float * 3), ("up", C.c_float * 3), ("backward", C.c_float * 3)]


class PtBvhNode(C.Structure):
    """pt_bvh_node (reference BVH.h:6-11)."""
    _fields_ = [("aabb_min", C.c_float * 3), ("aabb_max", C.c_float * 3), ("offset", C.c_uint32),
                ("primitive_count_axis", C.c_uint32)]


class PtHittable(C.Structure):
    """pt_hittable (reference Hittable.h:23-27 + Material.h:22-27)."""
    _fields_ = [("inv_transform_rows", (C.c_float * 4) * 3), ("base_color", C.c_float * 3), ("roughness", C.c_float),
                ("emissive", C.c_float * 3), ("metalness", C.c_float), ("texture_index", C.c_uint32),
                ("material_type", C.c_uint32), ("type", C.c_uint32), ("pad", C.c_uint32)]


class PtRenderStats(C.Structure):
    _fields_ = [("node_tests", C.c_uint64), ("prim_tests", C.c_uint64), ("hits", C.c_uint64),
                ("sky_lookups", C.c_uint64), ("segments", C.c_uint64), ("samples", C.c_uint64),
                ("wave_node_iters", C.c_uint64), ("wave_prim_iters", C.c_uint64), ("wave_hits", C.c_uint64),
                ("wave_sky", C.c_uint64), ("wave_segments", C.c_uint64), ("cycles_node_walk", C.c_uint64),
                ("cycles_leaf_tests", C.c_uint64), ("cycles_shading", C.c_uint64), ("cycles_total", C.c_uint64),
                ("cycles_lane_idle", C.c_uint64), ("leaf_rounds", C.c_uint64), ("family_execs", C.c_uint64),
                ("family_execs_compacted", C.c_uint64), ("leaf_round_lanes", C.c_uint64), ("leaf_pairs", C.c_uint64),
                ("family_execs_compacted_in_round", C.c_uint64), ("repairs", C.c_uint64)]


# symbol -> (restype, argtypes); the CPU test suite checks that every declaration in include/*.h
# is exported and bound here.
P = C.POINTER
_HIP_SYMBOLS = {
    "pt_device_count": (C.c_int, [P(C.c_int)]),
    "pt_create": (C.c_int, [C.c_int, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, P(C.c_void_p)]),
    "pt_create_banded": (C.c_int, [C.c_int, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, P(C.c_void_p)]),
    "pt_band_rows": (C.c_uint32, [C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32]),
    "pt_destroy": (None, [C.c_void_p]),
    "pt_set_scene": (C.c_int, [C.c_void_p, P(PtBvhNode), C.c_uint32, P(PtHittable), C.c_uint32]),
    "pt_set_texture": (C.c_int, [C.c_void_p, C.c_uint32, P(C.c_float), C.c_uint32, C.c_uint32]),
    "pt_set_skybox": (C.c_int, [C.c_void_p, C.c_uint32]),
    "pt_render": (C.c_int, [C.c_void_p, P(PtCamera), C.c_uint32, C.c_uint32, C.c_int, P(C.c_float)]),
    "pt_render_instrumented": (C.c_int, [C.c_void_p, P(PtCamera), C.c_uint32, C.c_uint32, C.c_int, P(C.c_float),
                                         P(PtRenderStats)]),
    "pt_read_accum": (C.c_int, [C.c_void_p, P(C.c_float)]),
    "pt_copy_accum_device": (C.c_int, [C.c_void_p, C.c_void_p, C.c_size_t]),
    "pt_tonemap": (C.c_int, [C.c_void_p, C.c_uint32, P(C.c_uint8)]),
    "pt_tonemap_device": (C.c_int, [C.c_void_p, C.c_uint32, C.c_void_p, C.c_size_t]),
    "pt_read_rng": (C.c_int, [C.c_void_p, P(C.c_uint32)]),
    "pt_write_rng": (C.c_int, [C.c_void_p, P(C.c_uint32)]),
    "pt_local_rows": (C.c_uint32, [C.c_void_p]),
    "pt_read_tile_costs": (C.c_int, [C.c_void_p, P(C.c_uint32), C.c_uint32]),
    "pt_read_tile_idle": (C.c_int, [C.c_void_p, P(C.c_uint32), C.c_uint32]),
    "pt_set_strip_units": (C.c_int, [C.c_void_p, C.c_int]),
    "pt_set_rise_repair": (C.c_int, [C.c_void_p, C.c_int]),
    "pt_set_run_ahead": (C.c_int, [C.c_void_p, C.c_int]),
    "pt_set_cold_start": (C.c_int, [C.c_void_p, C.c_uint32, C.c_int]),
    "pt_unpermute_bands": (C.c_int, [C.c_int, C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32,
                                     C.c_uint32]),
    "pt_set_kernel_variant": (C.c_int, [C.c_void_p, C.c_int]),
    "pt_set_occupancy": (C.c_int, [C.c_void_p, C.c_uint32]),
    "pt_set_tile_trace": (C.c_int, [C.c_void_p, C.c_int]),
    "pt_read_tile_trace": (C.c_int, [C.c_void_p, P(C.c_uint32), C.c_uint32]),
    "pt_set_issue_priority": (C.c_int, [C.c_void_p, C.c_int, C.c_uint32, C.c_uint32, C.c_uint32]),
    "pt_set_schedule": (C.c_int, [C.c_void_p, C.c_int]),
    "pt_set_sample_groups": (C.c_int, [C.c_void_p, C.c_int]),
    "pt_last_sample_groups": (C.c_int, [C.c_void_p]),
    "pt_last_variant": (C.c_int, [C.c_void_p]),
    "pt_read_group_stats": (C.c_int, [C.c_void_p, P(C.c_uint32)]),
    "pt_set_patch_rounds": (C.c_int, [C.c_void_p, C.c_uint32]),
    "pt_set_group_lookback": (C.c_int, [C.c_void_p, C.c_uint32, C.c_uint32]),
    "pt_read_group_fold": (C.c_int, [C.c_void_p, C.c_uint32, P(C.c_uint32)]),
    "pt_read_group_log_counts": (C.c_int, [C.c_void_p, P(C.c_uint32), C.c_size_t]),
    "pt_last_error": (C.c_char_p, [C.c_void_p]),
    "pt_group_create": (C.c_int, [C.c_int, P(C.c_int), C.c_uint32, C.c_uint32, C.c_uint32, P(C.c_void_p)]),
    "pt_group_destroy": (None, [C.c_void_p]),
    "pt_group_size": (C.c_int, [C.c_void_p]),
    "pt_group_context": (C.c_void_p, [C.c_void_p, C.c_int]),
    "pt_group_set_scene": (C.c_int, [C.c_void_p, P(PtBvhNode), C.c_uint32, P(PtHittable), C.c_uint32]),
    "pt_group_set_texture": (C.c_int, [C.c_void_p, C.c_uint32, P(C.c_float), C.c_uint32, C.c_uint32]),
    "pt_group_set_skybox": (C.c_int, [C.c_void_p, C.c_uint32]),
    "pt_group_render": (C.c_int, [C.c_void_p, P(PtCamera), C.c_uint32, C.c_uint32, C.c_int, P(C.c_float)]),
    "pt_group_gather": (C.c_int, [C.c_void_p, P(C.c_float)]),
    "pt_group_read_accum": (C.c_int, [C.c_void_p, P(C.c_float)]),
    "pt_group_tonemap": (C.c_int, [C.c_void_p, C.c_uint32, P(C.c_uint8)]),
    "pt_group_last_error": (C.c_char_p, [C.c_void_p]),
}

_HOST_SYMBOLS = {
    "pth_last_error": (C.c_char_p, []),
    "pth_scene_load": (C.c_int, [C.c_char_p, C.c_uint32, C.c_uint32, P(C.c_void_p)]),
    "pth_scene_free": (None, [C.c_void_p]),
    "pth_scene_timing": (C.c_int, [C.c_void_p, P(C.c_double), P(C.c_double)]),
    "pth_scene_object_count": (C.c_uint32, [C.c_void_p]),
    "pth_scene_node_count": (C.c_uint32, [C.c_void_p]),
    "pth_scene_bvh_depth": (C.c_uint32, [C.c_void_p]),
    "pth_scene_objects": (C.c_int, [C.c_void_p, P(PtHittable), P(C.c_float)]),
    "pth_scene_bvh": (C.c_int, [C.c_void_p, P(PtBvhNode), P(PtHittable)]),
    "pth_scene_camera": (C.c_int, [C.c_void_p, P(PtCamera)]),
    "pth_scene_skybox": (C.c_uint32, [C.c_void_p]),
    "pth_scene_texture_count": (C.c_uint32, [C.c_void_p]),
    "pth_scene_texture_info": (C.c_int, [C.c_void_p, C.c_uint32, P(C.c_uint32), P(C.c_uint32)]),
    "pth_scene_texture_data": (C.c_int, [C.c_void_p, C.c_uint32, P(C.c_float)]),
    "pth_camera_make": (C.c_int, [P(C.c_float), P(C.c_float), P(C.c_float), C.c_float, C.c_float, P(PtCamera)]),
    "pth_camera_rotate": (C.c_int, [P(PtCamera), C.c_float, C.c_float, C.c_float]),
    "pth_camera_translate": (C.c_int, [P(PtCamera), C.c_float, C.c_float, C.c_float]),
    "pth_radians": (C.c_float, [C.c_float]),
    "pth_renderer_create": (C.c_int, [C.c_uint32, C.c_uint32, C.c_int, C.c_uint32, C.c_uint32, P(C.c_void_p)]),
    "pth_renderer_create_banded": (C.c_int, [C.c_uint32, C.c_uint32, C.c_int, C.c_uint32, C.c_uint32, C.c_uint32,
                                             P(C.c_void_p)]),
    "pth_renderer_create_group": (C.c_int, [C.c_uint32, C.c_uint32, C.c_int, P(C.c_int), C.c_uint32, P(C.c_void_p)]),
    "pth_renderer_gather_ms": (C.c_float, [C.c_void_p]),
    "pth_renderer_destroy": (None, [C.c_void_p]),
    "pth_renderer_load_scene": (C.c_int, [C.c_void_p, C.c_char_p, P(PtCamera)]),
    "pth_renderer_render": (C.c_int, [C.c_void_p, P(PtCamera), C.c_uint32, C.c_uint32, C.c_int]),
    "pth_renderer_timing": (C.c_float, [C.c_void_p]),
    "pth_renderer_frames": (C.c_uint32, [C.c_void_p]),
    "pth_renderer_local_rows": (C.c_uint32, [C.c_void_p]),
    "pth_renderer_hdr": (P(C.c_float), [C.c_void_p]),
    "pth_renderer_image": (P(C.c_uint8), [C.c_void_p]),
    "pth_renderer_context": (C.c_void_p, [C.c_void_p]),
    "pth_renderer_group": (C.c_void_p, [C.c_void_p]),
    "pth_write_png": (C.c_int, [C.c_char_p, C.c_uint32, C.c_uint32, P(C.c_uint8), C.c_int]),
    "pth_write_hdr": (C.c_int, [C.c_char_p, C.c_uint32, C.c_uint32, P(C.c_float), C.c_int]),
}

_hip = None
_host = None


def _bind(lib: C.CDLL, table: dict) -> C.CDLL:
    for name, (res, args) in table.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


def mapped_hip_runtimes() -> list:
    """Distinct HIP runtime files (libamdhip64*) mapped into this process, from /proc/self/maps."""
    seen = []
    try:
        with open("/proc/self/maps") as f:
            for line in f:
                parts = line.split(None, 5)
                if len(parts) == 6 and "/libamdhip64" in parts[5]:
                    path = os.path.realpath(parts[5].strip())
                    if path not in seen:
                        seen.append(path)
    except OSError:
        pass
    return seen


def check_single_runtime() -> None:
    """Raise PathtracerError when two HIP runtimes are mapped: two copies of the runtime in one process
    corrupt the heap at exit ("double free or corruption", rc 134)."""
    paths = mapped_hip_runtimes()
    if len(paths) > 1:
        raise PathtracerError(PT_ERR_STATE, "two HIP runtimes are mapped into this process ("
                              + ", ".join(paths) + "); load libpt_hip.so through pathtracercuda_amd._native.hip() "
                              "before any other HIP user, or import torch first")


def _unify_runtime() -> None:
    """Load the HIP runtime stack the process will use before libpt_hip.so binds one.

    The torch wheel ships its own libamdhip64 / librccl / libhsa-runtime64 and resolves them by file
    name through RPATH $ORIGIN, so a torch imported after libpt_hip.so maps a second runtime next to
    /opt/rocm's.  Preloading the wheel's files is not enough: with the wheel's own librccl.so mapped
    before libtorch_hip.so, the process aborts at exit ("double free or corruption", measured in this
    container with nothing else loaded).  So when torch is importable it is imported first, which is
    the configuration every test runs; libpt_hip.so then binds the wheel's runtime by soname
    (libamdhip64.so.7, librccl.so.1).  Without torch the system runtime (/opt/rocm) is used.
    """
    if "torch" in sys.modules:
        return
    try:
        spec = importlib.util.find_spec("torch")
    except (ImportError, ValueError):
        spec = None
    if spec is not None:
        import torch  # noqa: F401


def hip() -> C.CDLL:
    global _hip
    if _hip is None:
        if not HIP_LIB.exists():
            raise RuntimeError(f"{HIP_LIB} is missing: build it with `make` (or __graft_entry__.build())")
        _unify_runtime()
        lib = C.CDLL(str(HIP_LIB), mode=C.RTLD_GLOBAL)
        check_single_runtime()
        _hip = _bind(lib, _HIP_SYMBOLS)
    return _hip


def host() -> C.CDLL:
    global _host
    if _host is None:
        hip()
        if not HOST_LIB.exists():
            raise RuntimeError(f"{HOST_LIB} is missing: build it with `make` (or __graft_entry__.build())")
        _host = _bind(C.CDLL(str(HOST_LIB)), _HOST_SYMBOLS)
    return _host


class PathtracerError(RuntimeError):
    def __init__(self, code: int, message: str):
        super().__init__(f"[{code}] {message}")
        self.code = code


def check_host(rc: int) -> None:
    if rc != PT_OK:
        raise PathtracerError(rc, (host().pth_last_error() or b"").decode(errors="replace"))


def check_ctx(rc: int, ctx) -> None:
    if rc != PT_OK:
        raise PathtracerError(rc, (hip().pt_last_error(ctx) or b"").decode(errors="replace"))


def check_group(rc: int, group) -> None:
    if rc != PT_OK:
        raise PathtracerError(rc, (hip().pt_group_last_error(group) or b"").decode(errors="replace"))


def device_count() -> int:
    n = C.c_int(0)
    hip().pt_device_count(C.byref(n))
    return int(n.value)
