"""ctypes driver for the CPU restatement (liboracle.so).  TEST INFRASTRUCTURE ONLY.

Imported by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg -- never by the
product package.  Mirrors the reference's host flow so tests read like the reference's own code:
  SceneLoader.cpp:124-348 (loadScene)  -> load_scene()
  Pathtracer.cpp:111-160 (setScene)    -> OracleScene.bvh (BVH::build, leaf size 4)
  Pathtracer.cpp:162-227 (render)      -> OracleRenderer.render()
  tonemap.cu / Pathtracer.cpp:299-339  -> OracleRenderer.tonemap()/hdr()
JSON is parsed with Python's json (numbers -> double, like nlohmann 3.9.0) and narrowed to float32
exactly as `get<float>()` does.  Parity status: see the header of pt_oracle.c (unpinned vs the CUDA
binary; pinned statistically to the reference's published render).
"""
from __future__ import annotations

import ctypes as C
import json
import os
import pathlib
import struct
from typing import List, Optional, Sequence

import numpy as np

HERE = pathlib.Path(__file__).resolve().parent
LIB_PATH = HERE / "liboracle.so"
FAST_LIB_PATH = HERE / "liboracle_fast.so"      # -O3 build of the same source (bench.py cpu_baseline)

SHAPES = ["SPHERE", "CYLINDER", "DISK", "CONE", "PARABOLOID", "QUAD", "CUBE"]
MATERIALS = ["LAMBERT", "GGX", "LAMBERT_GGX"]


class Material(C.Structure):
    _fields_ = [("baseColor", C.c_float * 3), ("roughness", C.c_float), ("emissive", C.c_float * 3),
                ("metalness", C.c_float), ("textureIndex", C.c_uint32), ("materialType", C.c_uint32)]


class Hittable(C.Structure):
    _fields_ = [("rows", (C.c_float * 4) * 3), ("mat", Material), ("type", C.c_uint32), ("pad", C.c_uint32)]


class CpuHittable(C.Structure):
    _fields_ = [("rows", (C.c_float * 4) * 3), ("mat", Material), ("aabbMin", C.c_float * 3),
                ("aabbMax", C.c_float * 3), ("type", C.c_uint32)]


class BVHNode(C.Structure):
    _fields_ = [("bmin", C.c_float * 3), ("bmax", C.c_float * 3), ("offset", C.c_uint32),
                ("primitiveCountAxis", C.c_uint32)]


class Camera(C.Structure):
    _fields_ = [("tanHalfFovy", C.c_float), ("aspectRatio", C.c_float), ("origin", C.c_float * 3),
                ("lowerLeftCorner", C.c_float * 3), ("horizontal", C.c_float * 3), ("vertical", C.c_float * 3),
                ("right", C.c_float * 3), ("up", C.c_float * 3), ("backward", C.c_float * 3)]


class Texture(C.Structure):
    _fields_ = [("width", C.c_uint32), ("height", C.c_uint32), ("texels", C.POINTER(C.c_float))]


class Xorwow(C.Structure):
    _fields_ = [("d", C.c_uint32), ("v", C.c_uint32 * 5)]


_lib = None
_fast = None


def lib(fast: bool = False) -> C.CDLL:
    global _lib, _fast
    if fast:
        if _fast is None:
            if not FAST_LIB_PATH.exists():
                raise RuntimeError(f"{FAST_LIB_PATH} missing: run `make -C oracle`")
            _fast = _bind(C.CDLL(str(FAST_LIB_PATH)))
        return _fast
    if _lib is None:
        if not LIB_PATH.exists():
            raise RuntimeError(f"{LIB_PATH} missing: run `make -C oracle` (or __graft_entry__.build())")
        _lib = _bind(C.CDLL(str(LIB_PATH)))
    return _lib


def _bind(L: C.CDLL) -> C.CDLL:
    if True:   # (indentation kept from the single-library loader)
        f = C.c_float
        P = C.POINTER
        L.or_radians.restype = f
        L.or_radians.argtypes = [f]
        L.or_material_make.argtypes = [C.c_uint32, P(f), P(f), f, f, C.c_uint32, P(Material)]
        L.or_cpu_hittable_make.argtypes = [C.c_uint32, P(f), P(f), P(f), P(Material), P(CpuHittable)]
        L.or_gpu_hittable.argtypes = [P(CpuHittable), P(Hittable)]
        L.or_camera_make.argtypes = [P(f), P(f), P(f), f, f, P(Camera)]
        L.or_camera_rotate.argtypes = [P(Camera), f, f, f]
        L.or_camera_translate.argtypes = [P(Camera), f, f, f]
        L.or_bvh_build.restype = C.c_uint32
        L.or_bvh_build.argtypes = [C.c_size_t, P(CpuHittable), C.c_uint32, P(BVHNode)]
        L.or_init_rand_state.argtypes = [C.c_uint32] * 5 + [P(Xorwow)]
        L.or_view_rows.restype = C.c_uint32
        L.or_view_rows.argtypes = [C.c_uint32] * 4
        L.or_render.restype = C.c_int
        L.or_render.argtypes = [P(Hittable), C.c_uint32, P(BVHNode), C.c_uint32, P(Camera), C.c_uint32, P(Texture),
                                C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, P(f), P(Xorwow),
                                C.c_uint32, C.c_uint32, C.c_int, C.c_int, P(C.c_uint64)]
        L.or_tonemap.argtypes = [P(f), C.c_size_t, C.c_uint32, P(C.c_uint8)]
        L.or_hdr_normalize.argtypes = [P(f), C.c_size_t, C.c_uint32, P(f)]
        L.or_xorwow_init.argtypes = [C.c_uint64, P(Xorwow)]
        L.or_xorwow_next.restype = C.c_uint32
        L.or_xorwow_next.argtypes = [P(Xorwow)]
        L.or_xorwow_uniform.restype = f
        L.or_xorwow_uniform.argtypes = [P(Xorwow)]
        for name in ("pm_sinf", "pm_cosf", "pm_acosf"):
            getattr(L, name).restype = f
            getattr(L, name).argtypes = [f]
        for name in ("pm_atan2f", "pm_powf"):
            getattr(L, name).restype = f
            getattr(L, name).argtypes = [f, f]
        L.or_tex2d.argtypes = [P(Texture), f, f, P(f)]
        L.or_xorwow_skip.argtypes = [P(Xorwow), C.c_uint64]
        L.or_sample_log.restype = C.c_int
        L.or_sample_log.argtypes = [P(Hittable), C.c_uint32, P(BVHNode), C.c_uint32, P(Camera), C.c_uint32, P(Texture),
                                    C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, P(Xorwow), C.c_uint32,
                                    P(f), P(C.c_uint8)]
        L.or_sizeof.restype = C.c_uint32
        L.or_sizeof.argtypes = [C.c_int]
    return L


def fptr(a: np.ndarray):
    return a.ctypes.data_as(C.POINTER(C.c_float))


def f3(v: Sequence[float]):
    return (C.c_float * 3)(*[float(np.float32(x)) for x in v])


# ------------------------------------------------------------------------------------------------
# image decoding for textures (stb_image semantics for the formats the scenes use)
# ------------------------------------------------------------------------------------------------
def read_rgbe(path: os.PathLike) -> np.ndarray:
    """Radiance .hdr -> float32 RGBA (H, W, 4); stbi__hdr_convert (stb_image.h:7036-7061):
    f = ldexp(1, e - 136); rgb = byte * f; A = 1; e == 0 -> (0, 0, 0, 1)."""
    data = pathlib.Path(path).read_bytes()
    pos = 0

    def line() -> bytes:
        nonlocal pos
        end = data.index(b"\n", pos)
        s = data[pos:end]
        pos = end + 1
        return s

    first = line()
    if first not in (b"#?RADIANCE", b"#?RGBE"):
        raise ValueError("not a Radiance file")
    while True:
        s = line()
        if s == b"":
            break
    dims = line().split()
    if len(dims) != 4 or dims[0] != b"-Y" or dims[2] != b"+X":
        raise ValueError("unsupported HDR orientation")
    h, w = int(dims[1]), int(dims[3])
    rgbe = np.zeros((h, w, 4), dtype=np.uint8)
    buf = memoryview(data)
    for j in range(h):
        if 8 <= w < 32768 and pos + 4 <= len(data) and data[pos] == 2 and data[pos + 1] == 2 and not (data[pos + 2] & 0x80):
            pos += 4
            for k in range(4):
                i = 0
                while i < w:
                    count = data[pos]
                    pos += 1
                    if count > 128:
                        count -= 128
                        rgbe[j, i:i + count, k] = data[pos]
                        pos += 1
                    else:
                        rgbe[j, i:i + count, k] = np.frombuffer(buf[pos:pos + count], dtype=np.uint8)
                        pos += count
                    i += count
        else:
            rgbe[j] = np.frombuffer(buf[pos:pos + 4 * w], dtype=np.uint8).reshape(w, 4)
            pos += 4 * w
    e = rgbe[..., 3].astype(np.int32)
    f = np.where(e != 0, np.ldexp(np.float32(1.0), e - 136), 0.0).astype(np.float32)
    out = np.empty((h, w, 4), dtype=np.float32)
    out[..., :3] = rgbe[..., :3].astype(np.float32) * f[..., None]
    out[..., 3] = 1.0
    return out


def read_ldr(path: os.PathLike) -> np.ndarray:
    """8-bit texture -> float32 RGBA normalised c/255 (cudaReadModeNormalizedFloat, Pathtracer.cpp:276-283)."""
    from PIL import Image  # test infrastructure only
    img = np.asarray(Image.open(path).convert("RGBA"), dtype=np.uint8)
    return (img.astype(np.float32) / np.float32(255.0)).astype(np.float32)


def is_hdr(path: os.PathLike) -> bool:
    try:
        with open(path, "rb") as fh:
            head = fh.read(11)
        return head.startswith(b"#?RADIANCE") or head.startswith(b"#?RGBE")
    except OSError:
        return False


# ------------------------------------------------------------------------------------------------
# scene loading (SceneLoader.cpp:124-348)
# ------------------------------------------------------------------------------------------------
class OracleScene:
    def __init__(self) -> None:
        self.cpu: List[CpuHittable] = []
        self.textures: List[np.ndarray] = []
        self.skybox = 0
        self.camera = Camera()
        self.nodes = None
        self.prims = None
        self.node_count = 0
        self.prim_count = 0
        self._tex_structs = None

    def load_texture(self, path: str) -> int:
        """Pathtracer::loadTexture (Pathtracer.cpp:234-292): 0 on failure or when 64 are loaded."""
        if len(self.textures) >= 64:
            return 0
        p = pathlib.Path(path)
        try:
            tex = read_rgbe(p) if is_hdr(p) else read_ldr(p)
        except Exception:
            return 0
        self.textures.append(np.ascontiguousarray(tex, dtype=np.float32))
        return len(self.textures)

    def texture_table(self):
        arr = (Texture * max(1, len(self.textures)))()
        for i, t in enumerate(self.textures):
            arr[i].width = t.shape[1]
            arr[i].height = t.shape[0]
            arr[i].texels = fptr(t)
        self._tex_structs = arr
        return arr

    def set_scene(self, cpu: Sequence[CpuHittable]) -> None:
        """Pathtracer::setScene (Pathtracer.cpp:111-160): BVH build (leaf <= 4) + getGpuHittable."""
        L = lib()
        n = len(cpu)
        if n == 0:
            return
        elems = (CpuHittable * n)(*cpu)
        nodes = (BVHNode * (2 * n))()
        count = L.or_bvh_build(n, elems, 4, nodes)
        prims = (Hittable * n)()
        for i in range(n):
            L.or_gpu_hittable(C.byref(elems[i]), C.byref(prims[i]))
        self.bvh_elements = elems
        self.nodes = nodes
        self.node_count = int(count)
        self.prims = prims
        self.prim_count = n


def _resolve(path: str, scene_dir: pathlib.Path) -> str:
    # The reference resolves texture paths against the CWD (SceneLoader.cpp:145); fall back to the
    # scene file's directory so the fixtures under scenes/ work from any CWD.
    if os.path.exists(path):
        return path
    alt = scene_dir / path
    return str(alt) if alt.exists() else path


def load_scene(path: os.PathLike, width: int, height: int) -> OracleScene:
    L = lib()
    scene_path = pathlib.Path(path)
    j = json.loads(scene_path.read_text())
    sc = OracleScene()
    handles = {}

    def tex_handle(p: str) -> int:
        if p == "":
            return 0
        if p in handles:
            return handles[p]
        h = sc.load_texture(_resolve(p, scene_path.parent))
        handles[p] = h
        return h

    def get_vec3(o, key, default):
        v = o.get(key) if isinstance(o, dict) else None
        if isinstance(v, list) and len(v) == 3:
            return [np.float32(x) for x in v]
        return default

    def get_float(o, key, default):
        v = o.get(key)
        if isinstance(v, float):          # is_number_float(): JSON integers are ignored
            return np.float32(v)
        return default

    objs = j.get("objects")
    if isinstance(objs, list):
        cpu = []
        for o in objs:
            htype, pos, rot, scale = 0, [0.0] * 3, [0.0] * 3, [1.0] * 3
            mtype, base, emis, rough, metal, texh = 0, [1.0] * 3, [0.0] * 3, np.float32(0.5), np.float32(0.0), 0
            t = o.get("type")
            if isinstance(t, str):
                if t in SHAPES:
                    htype = SHAPES.index(t)
                else:
                    print(f"Failed to parse object type: {t}")
            pos = get_vec3(o, "position", pos)
            rot = get_vec3(o, "rotation", rot)
            scale = get_vec3(o, "scale", scale)
            m = o.get("material")
            if isinstance(m, dict):
                mt = m.get("type")
                if isinstance(mt, str):
                    if mt in MATERIALS:
                        mtype = MATERIALS.index(mt)
                    else:
                        print(f"Failed to parse material type: {mt}")
                base = get_vec3(m, "baseColor", base)
                emis = get_vec3(m, "emissive", emis)
                rough = get_float(m, "roughness", rough)
                metal = get_float(m, "metalness", metal)
                tp = m.get("texture")
                if isinstance(tp, str):
                    texh = tex_handle(tp)
            mat = Material()
            L.or_material_make(mtype, f3(base), f3(emis), float(rough), float(metal), texh, C.byref(mat))
            rrad = [L.or_radians(float(x)) for x in rot]
            h = CpuHittable()
            L.or_cpu_hittable_make(htype, f3(pos), f3(rrad), f3(scale), C.byref(mat), C.byref(h))
            cpu.append(h)
        sc.cpu = cpu
        sc.set_scene(cpu)
    sky = j.get("skybox")
    if isinstance(sky, str):
        sc.skybox = tex_handle(sky)
    cpos, look, fovy = [0.0] * 3, [0.0, 0.0, -1.0], np.float32(60.0)
    c = j.get("camera")
    if isinstance(c, dict):
        cpos = get_vec3(c, "position", cpos)
        look = get_vec3(c, "look_at", look)
        fovy = get_float(c, "fovy", fovy)
    aspect = float(np.float32(np.float32(width) / np.float32(height)))
    L.or_camera_make(f3(cpos), f3(look), f3([0.0, 1.0, 0.0]), L.or_radians(float(fovy)), aspect, C.byref(sc.camera))
    return sc


def rows_of(height: int, row_offset: int, row_stride: int, band_rows: int = 1) -> int:
    return int(lib().or_view_rows(height, band_rows, row_offset, row_stride))


def default_threads() -> int:
    """Every CPU this process may use: the affinity mask, capped by the cgroup's CPU quota (the GPU
    boxes show 256 logical CPUs but grant 16; more threads only time-slice them)."""
    n = max(1, len(os.sched_getaffinity(0)))
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            n = min(n, max(1, int(-(-float(q) // float(per)))))
    except (OSError, ValueError):
        pass
    return n


class OracleRenderer:
    """Per-pixel state of the reference Pathtracer (accum buffer, curandState, frame counter)
    restricted to the row bands b = row_offset + k * row_stride of band_rows rows (band_rows = 1:
    rows y = row_offset + k * row_stride)."""

    def __init__(self, scene: OracleScene, width: int, height: int, row_offset: int = 0, row_stride: int = 1,
                 threads: Optional[int] = None, band_rows: int = 1, fast: bool = False) -> None:
        self.scene = scene
        self.width, self.height = width, height
        self.row_offset, self.row_stride, self.band_rows = row_offset, row_stride, band_rows
        self.rows = rows_of(height, row_offset, row_stride, band_rows)
        self.accum = np.zeros((self.rows, width, 4), dtype=np.float32)
        self.rng = (Xorwow * max(1, self.rows * width))()
        lib().or_init_rand_state(width, height, band_rows, row_offset, row_stride, self.rng)
        self.frames = 0
        self.threads = threads or default_threads()
        self.stats = np.zeros(8, dtype=np.uint64)   # node, prim tests, hits, sky, segments, samples, max stack, rises
        self.fast = fast

    def render(self, camera: Camera, spp: int, ignore_history: bool, chunks: int = 1, collect_stats: bool = False) -> None:
        """`chunks` successive reference render(camera, spp, ignore_history and c == 0) calls."""
        sc = self.scene
        tex = sc.texture_table()
        st = (C.c_uint64 * 8)() if collect_stats else None
        rc = lib(self.fast).or_render(sc.prims, sc.prim_count, sc.nodes, sc.node_count, C.byref(camera), sc.skybox, tex,
                             len(sc.textures), self.width, self.height, self.band_rows, self.row_offset, self.row_stride,
                             fptr(self.accum), self.rng, spp, chunks, int(bool(ignore_history)), self.threads, st)
        if rc != 0:
            raise RuntimeError("oracle: BVH traversal stack overflow (reference UB)")
        if collect_stats:
            self.stats = np.frombuffer(bytes(st), dtype=np.uint64).copy()
        for c in range(chunks):
            if ignore_history and c == 0:
                self.frames = 0
            self.frames += 1

    def rng_array(self) -> np.ndarray:
        return np.frombuffer(bytes(self.rng), dtype=np.uint32)[:self.rows * self.width * 6].reshape(self.rows, self.width, 6)

    def tonemap(self, frames: Optional[int] = None) -> np.ndarray:
        out = np.zeros((self.rows, self.width, 4), dtype=np.uint8)
        lib().or_tonemap(fptr(self.accum), self.rows * self.width, self.frames if frames is None else frames,
                         out.ctypes.data_as(C.POINTER(C.c_uint8)))
        return out

    def hdr(self) -> np.ndarray:
        out = np.zeros_like(self.accum)
        lib().or_hdr_normalize(fptr(self.accum), self.rows * self.width, self.frames, fptr(out))
        return out


def struct_bytes(arr) -> bytes:
    return bytes(arr)


def pixel_state(width: int, x: int, y: int, draws: int = 0) -> Xorwow:
    """The pixel's XORWOW state (initRandState.cu:16) after `draws` draws."""
    st = Xorwow()
    lib().or_xorwow_init(1984 + x + y * width, C.byref(st))
    if draws:
        lib().or_xorwow_skip(C.byref(st), draws)
    return st


def sample_log(scene: OracleScene, width: int, height: int, x: int, y: int, state: Xorwow, n: int):
    """n samples of pixel (x, y) from `state` (advanced in place): per-sample colours (n x 3 float32,
    what getColor returns) and draw pairs consumed (n uint8)."""
    cols = np.zeros((n, 3), dtype=np.float32)
    pairs = np.zeros(n, dtype=np.uint8)
    tex = scene.texture_table()
    rc = lib().or_sample_log(scene.prims, scene.prim_count, scene.nodes, scene.node_count, C.byref(scene.camera),
                             scene.skybox, tex, len(scene.textures), width, height, x, y, C.byref(state), n,
                             fptr(cols), pairs.ctypes.data_as(C.POINTER(C.c_uint8)))
    if rc != 0:
        raise RuntimeError("oracle: BVH traversal stack overflow (reference UB)")
    return cols, pairs

