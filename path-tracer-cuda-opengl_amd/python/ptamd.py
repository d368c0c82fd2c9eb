"""ptamd — ctypes binding of libpt.so (include/pt.h) for tests, smoke() and bench.py.

This module only marshals arguments: every computation happens in libpt.so (host C++ for
scene assembly / PNG, HIP kernels for the LBVH build, traversal and render).  There is no
CPU fallback: if libpt.so is missing, importing this module raises; if no GPU is visible,
device calls fail with PT_ERR_NODEVICE.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.dirname(HERE)
REPO = os.path.dirname(PKG)
LIB_PATH = os.environ.get("PT_LIB") or os.path.join(PKG, "libpt.so")   # PT_LIB: A/B builds
MODELS_DIR = os.path.join(REPO, "models")

PT_OK = 0
PT_SPHERE, PT_TRIANGLE = 1, 3
PT_LAMBERTIAN, PT_METAL, PT_DIELECTRIC = 1, 2, 4
PT_BVH_ORIGIN_BOUNDS, PT_BVH_HOST_KEYS, PT_BVH_WIDE_DEVICE = 1, 2, 4

# numpy mirrors of the C structs (all 4-byte fields, no padding)
OBJECT_DTYPE = np.dtype([("type", "<i4"), ("mat", "<i4"), ("v", "<f4", (9,))])
MATERIAL_DTYPE = np.dtype([("type", "<i4"), ("albedo", "<f4", (3,)), ("fuzz", "<f4"), ("ir", "<f4")])
RAY_DTYPE = np.dtype([("o", "<f4", (3,)), ("d", "<f4", (3,))])
HIT_DTYPE = np.dtype([("hit", "<i4"), ("obj", "<i4"), ("mat", "<i4"), ("front_face", "<i4"),
                      ("t", "<f4"), ("p", "<f4", (3,)), ("n", "<f4", (3,))])
NODE_DTYPE = np.dtype([("left", "<i4"), ("right", "<i4"), ("parent", "<i4"), ("objid", "<i4"),
                       ("bmin", "<f4", (3,)), ("bmax", "<f4", (3,))])
assert OBJECT_DTYPE.itemsize == 44 and MATERIAL_DTYPE.itemsize == 24 and HIT_DTYPE.itemsize == 44


class Camera(C.Structure):
    _fields_ = [("origin", C.c_float * 3), ("lower_left", C.c_float * 3), ("horizontal", C.c_float * 3),
                ("vertical", C.c_float * 3), ("right", C.c_float * 3), ("up", C.c_float * 3),
                ("front", C.c_float * 3), ("focus_dist", C.c_float), ("lens_radius", C.c_float),
                ("time0", C.c_float), ("time1", C.c_float)]


class Stats(C.Structure):
    _fields_ = [("rays", C.c_uint64), ("node_visits", C.c_uint64), ("box_tests", C.c_uint64),
                ("tri_tests", C.c_uint64), ("sphere_tests", C.c_uint64), ("paths", C.c_uint64),
                ("kernel_ms", C.c_double), ("algo_bytes", C.c_uint64)]

    def as_dict(self) -> dict:
        return {k: getattr(self, k) for k, _ in self._fields_}


class RenderOpts(C.Structure):
    _fields_ = [("kernel", C.c_int32), ("leaf_batch", C.c_int32), ("shade_batch", C.c_int32), ("flags", C.c_int32),
                ("rng", C.c_int32), ("chunk", C.c_int32), ("out_format", C.c_int32), ("reserved1", C.c_int32)]


RNG_COMPAT, RNG_SAMPLE = 0, 1
IDENTITY_ORDER, ACCUMULATE = 1, 2
OUT_RGB32F, OUT_RGBA8, OUT_RGBA8_SURFACE = 0, 1, 2


KERNEL_DEFAULT, KERNEL_SIMPLE, KERNEL_WAVEFRONT, KERNEL_WIDE = 0, 1, 2, 3


class SceneDesc(C.Structure):
    _fields_ = [("objects", C.c_void_p), ("n_objects", C.c_int64), ("materials", C.c_void_p),
                ("n_materials", C.c_int64), ("camera", Camera), ("width", C.c_int32), ("height", C.c_int32),
                ("spp", C.c_int32), ("max_depth", C.c_int32), ("name", C.c_char * 64)]


INSTANCE_DTYPE = np.dtype([("m", np.float32, 12), ("mesh", np.int32), ("reserved", np.int32)])


class InstancedDesc(C.Structure):
    _fields_ = [("objects", C.c_void_p), ("n_objects", C.c_int64), ("mesh_first", C.c_void_p),
                ("mesh_count", C.c_void_p), ("n_meshes", C.c_int32), ("instances", C.c_void_p),
                ("n_instances", C.c_int64), ("materials", C.c_void_p), ("n_materials", C.c_int64),
                ("camera", Camera), ("width", C.c_int32), ("height", C.c_int32), ("spp", C.c_int32),
                ("max_depth", C.c_int32), ("name", C.c_char * 64)]


# Every symbol include/pt.h declares (checked by the CPU tests).
EXPORTS = [
    "pt_last_error", "pt_abi_version", "pt_device_count", "pt_camera_make", "pt_camera_move",
    "pt_preset_scene", "pt_scene_desc_free", "pt_load_obj", "pt_free", "pt_morton_keys", "pt_write_png",
    "pt_quantize_rgba8", "pt_scene_create", "pt_scene_build_bvh", "pt_scene_bvh_info", "pt_scene_download_bvh",
    "pt_trace_closest", "pt_film_create", "pt_film_info", "pt_film_rows", "pt_film_get_rng", "pt_film_set_rng",
    "pt_render", "pt_render_ex", "pt_film_reset", "pt_film_destroy", "pt_scene_destroy",
    "pt_film_clear", "pt_film_accumulated", "pt_write_png_rgba8", "pt_scene_build_time",
    "pt_scene_update_objects", "pt_trace_closest_ex", "pt_scene_wide_info", "pt_trace_closest_device",
    "pt_scene_build_bvh_ex", "pt_film_stats", "pt_preset_instanced", "pt_instanced_desc_free",
    "pt_scene_create_instanced",
]

if not os.path.exists(LIB_PATH):
    raise ImportError(f"{LIB_PATH} not built (run `make -C path-tracer-cuda-opengl_amd` or __graft_entry__.build())")
# torch first when it is installed: libpt.so then binds the HIP runtime torch already loaded (one
# runtime per process -- a second one, loaded after libpt.so's, sees no GPU: torch.cuda reports
# "No HIP GPUs are available" although libpt.so works).  Torch stays optional for the C ABI.
try:
    import torch  # noqa: F401
except ImportError:
    pass
lib = C.CDLL(LIB_PATH)

_P = C.c_void_p
_sig = {
    "pt_last_error": (C.c_char_p, []),
    "pt_abi_version": (C.c_int, []),
    "pt_device_count": (C.c_int, [C.POINTER(C.c_int)]),
    "pt_camera_make": (C.c_int, [_P, _P, C.c_float, C.c_float, C.c_float, C.c_float, C.c_float, C.c_float,
                                 C.POINTER(Camera)]),
    "pt_camera_move": (C.c_int, [C.POINTER(Camera), C.c_int, C.c_float]),
    "pt_preset_scene": (C.c_int, [C.c_char_p, C.c_char_p, C.c_int, C.c_int, C.POINTER(SceneDesc)]),
    "pt_scene_desc_free": (None, [C.POINTER(SceneDesc)]),
    "pt_load_obj": (C.c_int, [C.c_char_p, C.c_float, _P, C.c_int32, C.POINTER(C.c_void_p), C.POINTER(C.c_int64)]),
    "pt_free": (None, [_P]),
    "pt_morton_keys": (C.c_int, [_P, C.c_int64, C.c_int, _P]),
    "pt_write_png": (C.c_int, [C.c_char_p, _P, C.c_int, C.c_int]),
    "pt_quantize_rgba8": (C.c_int, [_P, C.c_int, C.c_int, _P]),
    "pt_scene_create": (C.c_int, [C.c_int, _P, C.c_int64, _P, C.c_int64, C.POINTER(C.c_void_p)]),
    "pt_scene_build_bvh": (C.c_int, [_P, C.c_int]),
    "pt_preset_instanced": (C.c_int, [C.c_char_p, C.c_char_p, C.c_int, C.c_int, C.POINTER(InstancedDesc)]),
    "pt_instanced_desc_free": (None, [C.POINTER(InstancedDesc)]),
    "pt_scene_create_instanced": (C.c_int, [C.c_int, _P, C.c_int64, _P, _P, C.c_int, _P, C.c_int64, _P, C.c_int64,
                                            C.POINTER(C.c_void_p)]),
    "pt_scene_build_bvh_ex": (C.c_int, [_P, C.c_int, _P]),
    "pt_film_stats": (C.c_int, [_P, C.POINTER(Stats)]),
    "pt_scene_build_time": (C.c_int, [_P, C.POINTER(C.c_double)]),
    "pt_scene_update_objects": (C.c_int, [_P, _P, C.c_int64, C.c_int64]),
    "pt_scene_bvh_info": (C.c_int, [_P, C.POINTER(C.c_int), C.POINTER(C.c_int64), C.POINTER(C.c_int64)]),
    "pt_scene_download_bvh": (C.c_int, [_P, _P]),
    "pt_scene_wide_info": (C.c_int, [_P, C.POINTER(C.c_int), C.POINTER(C.c_int64), C.POINTER(C.c_double),
                                     C.POINTER(C.c_int)]),
    "pt_trace_closest": (C.c_int, [_P, _P, C.c_int64, C.c_float, C.c_float, _P, C.POINTER(Stats)]),
    "pt_trace_closest_ex": (C.c_int, [_P, _P, C.c_int64, C.c_float, C.c_float, C.c_int, _P, C.POINTER(Stats)]),
    "pt_trace_closest_device": (C.c_int, [_P, _P, C.c_int64, C.c_float, C.c_float, C.c_int, _P, _P,
                                          C.POINTER(Stats)]),
    "pt_film_create": (C.c_int, [C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_uint64,
                                 C.POINTER(C.c_void_p)]),
    "pt_film_info": (C.c_int, [_P, C.POINTER(C.c_int), C.POINTER(C.c_int64)]),
    "pt_film_rows": (C.c_int, [_P, _P]),
    "pt_film_get_rng": (C.c_int, [_P, _P]),
    "pt_film_set_rng": (C.c_int, [_P, _P]),
    "pt_render": (C.c_int, [_P, _P, C.POINTER(Camera), C.c_int, C.c_int, _P, C.c_int, _P, C.POINTER(Stats)]),
    "pt_render_ex": (C.c_int, [_P, _P, C.POINTER(Camera), C.c_int, C.c_int, _P, C.c_int, _P, C.POINTER(RenderOpts),
                               C.POINTER(Stats)]),
    "pt_film_reset": (C.c_int, [_P, _P]),
    "pt_film_clear": (C.c_int, [_P, _P]),
    "pt_film_accumulated": (C.c_int, [_P, C.POINTER(C.c_int64)]),
    "pt_write_png_rgba8": (C.c_int, [C.c_char_p, _P, C.c_int, C.c_int]),
    "pt_film_destroy": (None, [_P]),
    "pt_scene_destroy": (None, [_P]),
}
for _name, (_res, _args) in _sig.items():
    _f = getattr(lib, _name)
    _f.restype = _res
    _f.argtypes = _args


class PtError(RuntimeError):
    def __init__(self, code: int, where: str):
        msg = lib.pt_last_error().decode(errors="replace")
        super().__init__(f"{where} failed with status {code}: {msg}")
        self.code = code


def _check(rc: int, where: str) -> None:
    if rc != PT_OK:
        raise PtError(rc, where)


def _ptr(a: np.ndarray) -> int:
    assert a.flags["C_CONTIGUOUS"]
    return a.ctypes.data


def device_count() -> int:
    n = C.c_int(0)
    _check(lib.pt_device_count(C.byref(n)), "pt_device_count")
    return n.value


def camera_make(frm, at, vfov, aspect, aperture=0.0, focus=10.0, t0=0.0, t1=1.0) -> Camera:
    cam = Camera()
    f = np.asarray(frm, np.float32)
    a = np.asarray(at, np.float32)
    _check(lib.pt_camera_make(_ptr(f), _ptr(a), vfov, aspect, aperture, focus, t0, t1, C.byref(cam)), "pt_camera_make")
    return cam


def camera_move(cam: Camera, direction: int, delta_time: float) -> None:
    """camera::processKeyboard (camera.h:41-56): 0 FORWARD 1 BACKWARD 2 LEFT 3 RIGHT 4 UP 5 DOWN."""
    _check(lib.pt_camera_move(C.byref(cam), direction, delta_time), "pt_camera_move")


def camera_to_array(cam: Camera) -> np.ndarray:
    return np.frombuffer(bytes(cam), dtype=np.float32).copy()


class Preset:
    """Host-side scene description produced by pt_preset_scene."""

    def __init__(self, name: str, width: int = 0, height: int = 0, models_dir: str = MODELS_DIR):
        d = SceneDesc()
        _check(lib.pt_preset_scene(name.encode(), models_dir.encode(), width, height, C.byref(d)), "pt_preset_scene")
        try:
            ob = (C.c_char * (d.n_objects * OBJECT_DTYPE.itemsize)).from_address(d.objects) if d.n_objects else b""
            mb = (C.c_char * (d.n_materials * MATERIAL_DTYPE.itemsize)).from_address(d.materials) if d.n_materials else b""
            self.objects = np.frombuffer(bytes(ob), dtype=OBJECT_DTYPE).copy()
            self.materials = np.frombuffer(bytes(mb), dtype=MATERIAL_DTYPE).copy()
            self.camera = Camera.from_buffer_copy(bytes(d.camera))
            self.width, self.height, self.spp, self.max_depth = d.width, d.height, d.spp, d.max_depth
            self.name = d.name.decode()
        finally:
            lib.pt_scene_desc_free(C.byref(d))


def _copy_array(ptr, n, dtype):
    if not n:
        return np.zeros(0, dtype)
    return np.frombuffer(bytes((C.c_char * (n * np.dtype(dtype).itemsize)).from_address(ptr)), dtype=dtype).copy()


class InstancedPreset:
    """pt_preset_instanced: meshes (object ranges, object space) placed by instance transforms."""

    def __init__(self, name: str, width: int = 0, height: int = 0, models_dir: str = MODELS_DIR):
        d = InstancedDesc()
        _check(lib.pt_preset_instanced(name.encode(), models_dir.encode(), width, height, C.byref(d)),
               "pt_preset_instanced")
        try:
            self.objects = _copy_array(d.objects, d.n_objects, OBJECT_DTYPE)
            self.mesh_first = _copy_array(d.mesh_first, d.n_meshes, np.int64)
            self.mesh_count = _copy_array(d.mesh_count, d.n_meshes, np.int64)
            self.instances = _copy_array(d.instances, d.n_instances, INSTANCE_DTYPE)
            self.materials = _copy_array(d.materials, d.n_materials, MATERIAL_DTYPE)
            self.camera = Camera.from_buffer_copy(bytes(d.camera))
            self.width, self.height, self.spp, self.max_depth = d.width, d.height, d.spp, d.max_depth
            self.name = d.name.decode()
        finally:
            lib.pt_instanced_desc_free(C.byref(d))

    def flattened_count(self) -> int:
        return int(sum(self.mesh_count[i["mesh"]] for i in self.instances))


def load_obj(path: str, scale: float = 1.0, translate=(0.0, 0.0, 0.0), mat: int = 0) -> np.ndarray:
    out = C.c_void_p()
    n = C.c_int64()
    t = np.asarray(translate, np.float32)
    _check(lib.pt_load_obj(path.encode(), scale, _ptr(t), mat, C.byref(out), C.byref(n)), "pt_load_obj")
    try:
        buf = (C.c_char * (n.value * OBJECT_DTYPE.itemsize)).from_address(out.value)
        return np.frombuffer(bytes(buf), dtype=OBJECT_DTYPE).copy()
    finally:
        lib.pt_free(out)


def morton_keys(objects: np.ndarray, include_origin: bool = True) -> np.ndarray:
    objects = np.ascontiguousarray(objects, OBJECT_DTYPE)
    keys = np.zeros(len(objects), np.uint64)
    _check(lib.pt_morton_keys(_ptr(objects) if len(objects) else None, len(objects), int(include_origin),
                              _ptr(keys) if len(keys) else None), "pt_morton_keys")
    return keys


def quantize_rgba8(rgb: np.ndarray, width: int, height: int) -> np.ndarray:
    rgb = np.ascontiguousarray(rgb, np.float32)
    out = np.zeros((height, width, 4), np.uint8)
    _check(lib.pt_quantize_rgba8(_ptr(rgb), width, height, _ptr(out)), "pt_quantize_rgba8")
    return out


def write_png_rgba8(path: str, rgba: np.ndarray, width: int, height: int) -> None:
    """PNG of a device-quantised frame (OUT_RGBA8 rows, row 0 = bottom; flipped on output)."""
    rgba = np.ascontiguousarray(rgba, np.uint8)
    assert rgba.size == width * height * 4
    _check(lib.pt_write_png_rgba8(path.encode(), _ptr(rgba), width, height), "pt_write_png_rgba8")


def write_png(path: str, rgb: np.ndarray, width: int, height: int) -> None:
    rgb = np.ascontiguousarray(rgb, np.float32)
    _check(lib.pt_write_png(path.encode(), _ptr(rgb), width, height), "pt_write_png")


class Scene:
    """Device-resident scene (objects, materials, LBVH) on one GPU."""

    def __init__(self, objects: np.ndarray, materials: np.ndarray, device: int = 0, build: bool = True,
                 flags: int = PT_BVH_ORIGIN_BOUNDS):
        self.objects = np.ascontiguousarray(objects, OBJECT_DTYPE)
        self.materials = np.ascontiguousarray(materials, MATERIAL_DTYPE)
        self.device = device
        h = C.c_void_p()
        _check(lib.pt_scene_create(device, _ptr(self.objects) if len(self.objects) else None, len(self.objects),
                                   _ptr(self.materials) if len(self.materials) else None, len(self.materials),
                                   C.byref(h)), "pt_scene_create")
        self.h = h
        if build:
            self.build_bvh(flags)

    @classmethod
    def instanced(cls, objects: np.ndarray, mesh_first, mesh_count, instances: np.ndarray, materials: np.ndarray,
                  device: int = 0, build: bool = True) -> "Scene":
        """pt_scene_create_instanced: each mesh stored once (object space), placed by `instances`
        (INSTANCE_DTYPE); rendered and traced by the wide kernel over a two-level tree."""
        self = cls.__new__(cls)
        self.objects = np.ascontiguousarray(objects, OBJECT_DTYPE)
        self.materials = np.ascontiguousarray(materials, MATERIAL_DTYPE)
        self.mesh_first = np.ascontiguousarray(mesh_first, np.int64)
        self.mesh_count = np.ascontiguousarray(mesh_count, np.int64)
        self.instances = np.ascontiguousarray(instances, INSTANCE_DTYPE)
        self.device = device
        self.h = None
        h = C.c_void_p()
        _check(lib.pt_scene_create_instanced(
            device, _ptr(self.objects) if len(self.objects) else None, len(self.objects),
            _ptr(self.mesh_first) if len(self.mesh_first) else None,
            _ptr(self.mesh_count) if len(self.mesh_count) else None, len(self.mesh_first),
            _ptr(self.instances) if len(self.instances) else None, len(self.instances),
            _ptr(self.materials) if len(self.materials) else None, len(self.materials), C.byref(h)),
            "pt_scene_create_instanced")
        self.h = h
        if build:
            self.build_bvh()
        return self

    def build_bvh(self, flags: int = PT_BVH_ORIGIN_BOUNDS, stream=None) -> None:
        """pt_scene_build_bvh_ex: the build's device work on `stream` (a hipStream_t handle or None)."""
        _check(lib.pt_scene_build_bvh_ex(self.h, flags, C.c_void_p(int(stream) if stream else 0)),
               "pt_scene_build_bvh_ex")

    def update_objects(self, objects: np.ndarray, first: int = 0) -> None:
        """Overwrite objects [first, first + len(objects)); the BVH must be rebuilt (build_bvh)
        before the next render or trace (dynamic scenes, one rebuild per frame)."""
        objs = np.ascontiguousarray(objects, OBJECT_DTYPE)
        _check(lib.pt_scene_update_objects(self.h, _ptr(objs) if len(objs) else None, first, len(objs)),
               "pt_scene_update_objects")
        self.objects = self.objects.copy()
        self.objects[first:first + len(objs)] = objs

    @property
    def build_ms(self) -> float:
        """Device time of the last LBVH build (HIP events)."""
        ms = C.c_double()
        _check(lib.pt_scene_build_time(self.h, C.byref(ms)), "pt_scene_build_time")
        return ms.value

    def bvh_info(self) -> dict:
        d, n, b = C.c_int(), C.c_int64(), C.c_int64()
        _check(lib.pt_scene_bvh_info(self.h, C.byref(d), C.byref(n), C.byref(b)), "pt_scene_bvh_info")
        return {"depth": d.value, "nodes": n.value, "device_bytes": b.value}

    def wide_info(self) -> dict:
        """The wide kernel's tree: depth, node slots, build ms, source (0 none yet, 1 host SAH, 2 device)."""
        d, n, ms, src = C.c_int(), C.c_int64(), C.c_double(), C.c_int()
        _check(lib.pt_scene_wide_info(self.h, C.byref(d), C.byref(n), C.byref(ms), C.byref(src)), "pt_scene_wide_info")
        return {"depth": d.value, "slots": n.value, "build_ms": ms.value, "source": src.value}

    def download_bvh(self) -> np.ndarray:
        n = len(self.objects)
        out = np.zeros(max(0, 2 * n - 1), NODE_DTYPE)
        _check(lib.pt_scene_download_bvh(self.h, _ptr(out) if len(out) else None), "pt_scene_download_bvh")
        return out

    def trace(self, rays: np.ndarray, tmin: float = 0.001, tmax: float = float("inf"), kernel: int = KERNEL_DEFAULT):
        """Closest hits (pt_trace_closest_ex): kernel=KERNEL_WIDE traverses the 8-wide tree."""
        rays = np.ascontiguousarray(rays, RAY_DTYPE)
        hits = np.zeros(len(rays), HIT_DTYPE)
        st = Stats()
        _check(lib.pt_trace_closest_ex(self.h, _ptr(rays) if len(rays) else None, len(rays), tmin, tmax, kernel,
                                       _ptr(hits) if len(hits) else None, C.byref(st)), "pt_trace_closest_ex")
        return hits, st

    def trace_device(self, rays_ptr: int, n: int, hits_ptr: int, tmin: float = 0.001, tmax: float = float("inf"),
                     kernel: int = KERNEL_DEFAULT, stream=None):
        """pt_trace_closest_device: rays_ptr / hits_ptr are device pointers to n RAY_DTYPE / HIT_DTYPE
        records (e.g. torch uint8 tensors' data_ptr()); returns the stats."""
        st = Stats()
        _check(lib.pt_trace_closest_device(self.h, rays_ptr or None, n, tmin, tmax, kernel, hits_ptr or None,
                                           stream, C.byref(st)), "pt_trace_closest_device")
        return st

    def close(self) -> None:
        if self.h:
            lib.pt_scene_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Film:
    """Per-pixel XORWOW streams for the rows of one stripe partition of a frame."""

    def __init__(self, width: int, height: int, seed: int, device: int = 0, stripe_height: int = 8,
                 n_parts: int = 1, part: int = 0):
        h = C.c_void_p()
        _check(lib.pt_film_create(device, width, height, stripe_height, n_parts, part, seed, C.byref(h)),
               "pt_film_create")
        self.h = h
        self.width, self.height = width, height
        nr, npix = C.c_int(), C.c_int64()
        _check(lib.pt_film_info(self.h, C.byref(nr), C.byref(npix)), "pt_film_info")
        self.n_rows, self.n_pixels = nr.value, npix.value
        self.rows = np.zeros(self.n_rows, np.int32)
        if self.n_rows:
            _check(lib.pt_film_rows(self.h, _ptr(self.rows)), "pt_film_rows")

    def get_rng(self) -> np.ndarray:
        out = np.zeros((self.n_pixels, 6), np.uint32)
        if self.n_pixels:
            _check(lib.pt_film_get_rng(self.h, _ptr(out)), "pt_film_get_rng")
        return out

    def set_rng(self, states: np.ndarray) -> None:
        states = np.ascontiguousarray(states, np.uint32)
        assert states.shape == (self.n_pixels, 6)
        _check(lib.pt_film_set_rng(self.h, _ptr(states)), "pt_film_set_rng")

    def reset(self, stream=None) -> None:
        """Back to the initRandom state: curand_init(seed, pixel, 0) for every pixel."""
        _check(lib.pt_film_reset(self.h, C.c_void_p(int(stream) if stream else 0)), "pt_film_reset")

    def clear(self, stream=None) -> None:
        """Progressive rendering: restart the accumulation (e.g. after the camera moved)."""
        _check(lib.pt_film_clear(self.h, C.c_void_p(int(stream) if stream else 0)), "pt_film_clear")

    def stats(self) -> "Stats":
        """pt_film_stats: counters and kernel time of the last render (waits for it)."""
        st = Stats()
        _check(lib.pt_film_stats(self.h, C.byref(st)), "pt_film_stats")
        return st

    @property
    def accumulated(self) -> int:
        n = C.c_int64()
        _check(lib.pt_film_accumulated(self.h, C.byref(n)), "pt_film_accumulated")
        return n.value

    def close(self) -> None:
        if self.h:
            lib.pt_film_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def render(scene: Scene, film: Film, camera: Camera, spp: int, max_depth: int, out=None, stream=None,
           kernel: int = KERNEL_DEFAULT, leaf_batch: int = 0, shade_batch: int = 0, rng: int = RNG_COMPAT,
           chunk: int = 0, flags: int = 0, accumulate: bool = False, out_format: int = OUT_RGB32F,
           wait: bool = True):
    """Render spp samples per pixel of the film's rows.  `out` may be a numpy array (host) or
    an integer device pointer (then `stream` is a hipStream_t handle or None).  Returns
    (rgb or None, Stats); rgb is float32 (n_pixels, 3), or uint8 (n_pixels, 4) for the 8-bit
    output formats.  accumulate=True adds the frame to the film's running sums (progressive).
    wait=False (device output only): the frame is enqueued and the call returns at once with
    Stats None -- film.stats() waits for it and returns its counters."""
    st = Stats()
    if accumulate:
        flags |= ACCUMULATE
    opts = RenderOpts(kernel, leaf_batch, shade_batch, flags, rng, chunk, out_format, 0)
    if out is None or isinstance(out, np.ndarray):
        if out is None:
            rgb = (np.zeros((film.n_pixels, 3), np.float32) if out_format == OUT_RGB32F
                   else np.zeros((film.n_pixels, 4), np.uint8))
        else:
            rgb = out
            want = (np.float32, 3) if out_format == OUT_RGB32F else (np.uint8, 4)
            assert rgb.dtype == want[0] and rgb.flags["C_CONTIGUOUS"] and rgb.size >= film.n_pixels * want[1]
        _check(lib.pt_render_ex(scene.h, film.h, C.byref(camera), spp, max_depth, _ptr(rgb), 0, None, C.byref(opts),
                                C.byref(st)), "pt_render_ex")
        return rgb, st
    _check(lib.pt_render_ex(scene.h, film.h, C.byref(camera), spp, max_depth, C.c_void_p(int(out)), 1,
                            C.c_void_p(int(stream) if stream else 0), C.byref(opts), C.byref(st) if wait else None),
           "pt_render_ex")
    return None, (st if wait else None)
