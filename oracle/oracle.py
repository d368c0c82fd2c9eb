"""ctypes wrapper of oracle/liboracle.so — the CPU restatement (TEST INFRASTRUCTURE ONLY).

Imported only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg, as the
checker; the product (libpt.so) never uses it.  Parity status: see pt_oracle.h.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")

OBJECT_DTYPE = np.dtype([("type", "<i4"), ("mat", "<i4"), ("v", "<f4", (9,))])
MATERIAL_DTYPE = np.dtype([("type", "<i4"), ("albedo", "<f4", (3,)), ("fuzz", "<f4"), ("ir", "<f4")])
HIT_DTYPE = np.dtype([("hit", "<i4"), ("obj", "<i4"), ("mat", "<i4"), ("front_face", "<i4"),
                      ("t", "<f4"), ("p", "<f4", (3,)), ("n", "<f4", (3,))])
NODE_DTYPE = np.dtype([("left", "<i4"), ("right", "<i4"), ("parent", "<i4"), ("objid", "<i4"),
                       ("bmin", "<f4", (3,)), ("bmax", "<f4", (3,))])
CAMERA_FLOATS = 25


def build() -> str:
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB_PATH


if not os.path.exists(LIB_PATH):
    build()
lib = C.CDLL(LIB_PATH)


class Stats(C.Structure):
    _fields_ = [(k, C.c_uint64) for k in ("rays", "node_visits", "box_tests", "tri_tests", "sphere_tests", "paths")]

    def as_dict(self) -> dict:
        return {k: getattr(self, k) for k, _ in self._fields_}


_P = C.c_void_p
for name, res, args in [
    ("orc_camera_make", None, [_P, _P, C.c_float, C.c_float, C.c_float, C.c_float, C.c_float, C.c_float, _P]),
    ("orc_xorwow_init", None, [C.c_uint64, C.c_uint64, _P]),
    ("orc_xorwow_init_range", None, [C.c_uint64, C.c_uint64, C.c_int64, _P]),
    ("orc_xorwow_skip_subsequences", None, [_P, C.c_uint64]),
    ("orc_xorwow_next", C.c_uint32, [_P]),
    ("orc_curand_uniform", C.c_float, [_P]),
    ("orc_set_draw_order", None, [C.c_int]),
    ("orc_morton_keys", C.c_int, [_P, C.c_int64, C.c_int, _P]),
    ("orc_build_lbvh", C.c_int, [_P, C.c_int64, _P, C.c_int, _P]),
    ("orc_bvh_depth", C.c_int, [_P, C.c_int64]),
    ("orc_trace", C.c_int, [_P, C.c_int64, _P, _P, C.c_int64, C.c_float, C.c_float, C.c_int, _P, C.POINTER(Stats)]),
    ("orc_scatter_tape", C.c_int, [_P, _P, _P, _P, C.c_int, C.POINTER(C.c_int), _P, _P]),
    ("orc_render2", C.c_int, [_P, C.c_int64, _P, C.c_int64, _P, _P, C.c_int, C.c_int, _P, C.c_int, C.c_int,
                              C.c_int, _P, _P, C.POINTER(Stats), C.c_int, _P]),
    ("orc_render_sample", C.c_int, [_P, C.c_int64, _P, C.c_int64, _P, _P, C.c_int, C.c_int, _P, C.c_int, C.c_int,
                                    C.c_int, C.c_uint64, C.c_int, _P, C.POINTER(Stats), C.c_int]),
    ("orc_render3", C.c_int, [_P, C.c_int64, _P, C.c_int64, _P, _P, C.c_int, C.c_int, _P, C.c_int, C.c_int,
                              C.c_int, _P, _P, C.POINTER(Stats), C.c_int, _P, _P]),
    ("orc_render_sample2", C.c_int, [_P, C.c_int64, _P, C.c_int64, _P, _P, C.c_int, C.c_int, _P, C.c_int, C.c_int,
                                     C.c_int, C.c_uint64, C.c_int, _P, C.POINTER(Stats), C.c_int, C.c_uint32, _P]),
    ("orc_philox_word", C.c_uint32, [C.c_uint64, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, C.c_int]),
    ("orc_sample_stream", None, [C.c_uint64, C.c_uint32, C.c_uint64, C.c_void_p]),
    ("orc_render", C.c_int, [_P, C.c_int64, _P, C.c_int64, _P, _P, C.c_int, C.c_int, _P, C.c_int, C.c_int,
                             C.c_int, _P, _P, C.POINTER(Stats), C.c_int]),
]:
    f = getattr(lib, name)
    f.restype = res
    f.argtypes = args


def _ptr(a):
    if a is None:
        return None
    assert a.flags["C_CONTIGUOUS"]
    return a.ctypes.data if a.size else None


def camera_make(frm, at, vfov, aspect, aperture=0.0, focus=10.0, t0=0.0, t1=1.0) -> np.ndarray:
    out = np.zeros(CAMERA_FLOATS, np.float32)
    f = np.asarray(frm, np.float32)
    a = np.asarray(at, np.float32)
    lib.orc_camera_make(_ptr(f), _ptr(a), vfov, aspect, aperture, focus, t0, t1, _ptr(out))
    return out


def xorwow_init(seed: int, subsequence: int) -> np.ndarray:
    s = np.zeros(6, np.uint32)
    lib.orc_xorwow_init(seed, subsequence, _ptr(s))
    return s


def xorwow_init_range(seed: int, first: int, count: int) -> np.ndarray:
    s = np.zeros((count, 6), np.uint32)
    lib.orc_xorwow_init_range(seed, first, count, _ptr(s))
    return s


def xorwow_skip(state: np.ndarray, n: int) -> np.ndarray:
    s = np.ascontiguousarray(state, np.uint32).copy()
    lib.orc_xorwow_skip_subsequences(_ptr(s), n)
    return s


def curand_uniform(state: np.ndarray, count: int) -> np.ndarray:
    """Draw `count` uniforms; `state` (uint32[6]) is advanced in place."""
    assert state.dtype == np.uint32 and state.flags["C_CONTIGUOUS"]
    return np.array([lib.orc_curand_uniform(state.ctypes.data) for _ in range(count)], np.float32)


def set_draw_order(zyx: bool) -> None:
    """Test-only: draw vec3(u - 0.5f, u - 0.5f, u - 0.5f)'s three coordinates z, y, x instead of x, y, z.
    utility.h:55-58 / 76-79 leave the order to the compiler (C++ argument evaluation order is
    unspecified); the oracle's default x, y, z is an assumption (pt_oracle.cpp draw3)."""
    lib.orc_set_draw_order(1 if zyx else 0)


def morton_keys(objects: np.ndarray, include_origin: bool = True) -> np.ndarray:
    objects = np.ascontiguousarray(objects, OBJECT_DTYPE)
    keys = np.zeros(len(objects), np.uint64)
    lib.orc_morton_keys(_ptr(objects), len(objects), int(include_origin), _ptr(keys))
    return keys


def build_lbvh(objects: np.ndarray, keys: np.ndarray | None = None, tight: bool = True) -> np.ndarray:
    objects = np.ascontiguousarray(objects, OBJECT_DTYPE)
    if keys is None:
        keys = morton_keys(objects)
    keys = np.ascontiguousarray(keys, np.uint64)
    nodes = np.zeros(max(0, 2 * len(objects) - 1), NODE_DTYPE)
    lib.orc_build_lbvh(_ptr(objects), len(objects), _ptr(keys), int(tight), _ptr(nodes))
    return nodes


def bvh_depth(nodes: np.ndarray, n: int) -> int:
    return lib.orc_bvh_depth(_ptr(nodes), n)


def trace(objects, nodes, rays: np.ndarray, tmin=0.001, tmax=float("inf"), brute=False):
    """rays: float32 (n, 6) = origin, direction."""
    objects = np.ascontiguousarray(objects, OBJECT_DTYPE)
    rays = np.ascontiguousarray(rays, np.float32).reshape(-1, 6)
    hits = np.zeros(len(rays), HIT_DTYPE)
    st = Stats()
    lib.orc_trace(_ptr(objects), len(objects), _ptr(nodes), _ptr(rays), len(rays), tmin, tmax, int(brute),
                  _ptr(hits), C.byref(st))
    return hits, st


def scatter_tape(material: np.ndarray, ray, hit: np.ndarray, tape):
    m = np.ascontiguousarray(material, MATERIAL_DTYPE).reshape(1)
    r = np.ascontiguousarray(ray, np.float32).reshape(6)
    h = np.ascontiguousarray(hit, HIT_DTYPE).reshape(1)
    t = np.ascontiguousarray(tape, np.float32)
    used = C.c_int(0)
    out = np.zeros(6, np.float32)
    att = np.zeros(3, np.float32)
    ok = lib.orc_scatter_tape(_ptr(m), _ptr(r), _ptr(h), _ptr(t), len(t), C.byref(used), _ptr(out), _ptr(att))
    return bool(ok), out, att, used.value


def render(objects, materials, nodes, camera: np.ndarray, width: int, height: int, rows, spp: int,
           max_depth: int, states: np.ndarray, nthreads: int = 1):
    """Returns (rgb float32 (len(rows)*width, 3), Stats); `states` ((npix, 6) uint32) is advanced."""
    objects = np.ascontiguousarray(objects, OBJECT_DTYPE)
    materials = np.ascontiguousarray(materials, MATERIAL_DTYPE)
    rows = np.ascontiguousarray(rows, np.int32)
    camera = np.ascontiguousarray(camera, np.float32)
    assert states.dtype == np.uint32 and states.flags["C_CONTIGUOUS"] and states.shape == (len(rows) * width, 6)
    out = np.zeros((len(rows) * width, 3), np.float32)
    st = Stats()
    lib.orc_render(_ptr(objects), len(objects), _ptr(materials), len(materials), _ptr(nodes), _ptr(camera), width,
                   height, _ptr(rows), len(rows), spp, max_depth, _ptr(states), _ptr(out), C.byref(st), nthreads)
    return out, st


def render_sample(objects, materials, nodes, camera, width, height, rows, spp, max_depth, seed, chunk=64,
                  nthreads=1):
    """Sample mode (Philox per pixel-sample, chunked sums): (rgb float32 (npix, 3), Stats)."""
    objects = np.ascontiguousarray(objects, OBJECT_DTYPE)
    materials = np.ascontiguousarray(materials, MATERIAL_DTYPE)
    rows = np.ascontiguousarray(rows, np.int32)
    camera = np.ascontiguousarray(camera, np.float32)
    out = np.zeros((len(rows) * width, 3), np.float32)
    st = Stats()
    lib.orc_render_sample(_ptr(objects), len(objects), _ptr(materials), len(materials), _ptr(nodes), _ptr(camera),
                          width, height, _ptr(rows), len(rows), spp, max_depth, seed, chunk, _ptr(out), C.byref(st),
                          nthreads)
    return out, st


def render_sums(objects, materials, nodes, camera, width, height, rows, spp, max_depth, states, nthreads=1):
    """orc_render + the raw per-pixel sample sums: (rgb, sums float32 (npix, 3), Stats)."""
    objects = np.ascontiguousarray(objects, OBJECT_DTYPE)
    materials = np.ascontiguousarray(materials, MATERIAL_DTYPE)
    rows = np.ascontiguousarray(rows, np.int32)
    camera = np.ascontiguousarray(camera, np.float32)
    assert states.dtype == np.uint32 and states.flags["C_CONTIGUOUS"] and states.shape == (len(rows) * width, 6)
    out = np.zeros((len(rows) * width, 3), np.float32)
    sums = np.zeros((len(rows) * width, 3), np.float32)
    st = Stats()
    lib.orc_render3(_ptr(objects), len(objects), _ptr(materials), len(materials), _ptr(nodes), _ptr(camera), width,
                    height, _ptr(rows), len(rows), spp, max_depth, _ptr(states), _ptr(out), C.byref(st), nthreads,
                    None, _ptr(sums))
    return out, sums, st


def render_sample_sums(objects, materials, nodes, camera, width, height, rows, spp, max_depth, seed, chunk,
                       sample_base=0, nthreads=1):
    """Sample mode with samples numbered from sample_base: (rgb, sums float32 (npix, 3), Stats)."""
    objects = np.ascontiguousarray(objects, OBJECT_DTYPE)
    materials = np.ascontiguousarray(materials, MATERIAL_DTYPE)
    rows = np.ascontiguousarray(rows, np.int32)
    camera = np.ascontiguousarray(camera, np.float32)
    out = np.zeros((len(rows) * width, 3), np.float32)
    sums = np.zeros((len(rows) * width, 3), np.float32)
    st = Stats()
    lib.orc_render_sample2(_ptr(objects), len(objects), _ptr(materials), len(materials), _ptr(nodes), _ptr(camera),
                           width, height, _ptr(rows), len(rows), spp, max_depth, seed, chunk, _ptr(out), C.byref(st),
                           nthreads, sample_base, _ptr(sums))
    return out, sums, st


def accumulate(frame_sums, frame_spps):
    """Progressive resolve (pt_render_ex with PT_RENDER_ACCUMULATE after each frame): the running
    fp32 sum A_k = A_{k-1} + S_k (A_0 = 0) and the image sqrt(A_k * (1 / samples so far)), in
    float32 arithmetic.  Returns the list of images, one per frame."""
    a = np.zeros_like(np.asarray(frame_sums[0], np.float32))
    n, out = 0, []
    for s, spp in zip(frame_sums, frame_spps):
        a = (a + np.asarray(s, np.float32)).astype(np.float32)
        n += spp
        out.append(np.sqrt((a * (np.float32(1.0) / np.float32(n))).astype(np.float32)).astype(np.float32))
    return out


def quantize_png(rgb):
    """PngImage::saveColor (png_image.h:24-30): (uint8)(clamp(c, 0, 0.999f) * 256), alpha 255;
    rows kept in film order.  (npix, 3) float32 -> (npix, 4) uint8."""
    c = np.asarray(rgb, np.float32)
    c = np.where(c < 0, np.float32(0), np.where(c > np.float32(0.999), np.float32(0.999), c)).astype(np.float32)
    q = np.full((c.shape[0], 4), 255, np.uint8)
    q[:, :3] = (c * np.float32(256.0)).astype(np.float32).astype(np.uint8)
    return q


def quantize_surface(rgb):
    """renderBySurface (main.cu:327-331): (unsigned)(c * 255) stored in an 8-bit field, alpha 255.
    (A negative value -- never produced by the path -- converts to 0, as v_cvt_u32_f32 does.)"""
    c = np.asarray(rgb, np.float32)
    q = np.full((c.shape[0], 4), 255, np.uint8)
    x = np.maximum((c * np.float32(255.0)).astype(np.float32), np.float32(0))
    q[:, :3] = (x.astype(np.uint32) & 0xFF).astype(np.uint8)
    return q


def render_pixel_rays(objects, materials, nodes, camera, width, height, rows, spp, max_depth, states, nthreads=1):
    """orc_render + per-pixel ray counts: (rgb, rays uint32 (npix,), Stats)."""
    objects = np.ascontiguousarray(objects, OBJECT_DTYPE)
    materials = np.ascontiguousarray(materials, MATERIAL_DTYPE)
    rows = np.ascontiguousarray(rows, np.int32)
    camera = np.ascontiguousarray(camera, np.float32)
    out = np.zeros((len(rows) * width, 3), np.float32)
    cnt = np.zeros(len(rows) * width, np.uint32)
    st = Stats()
    lib.orc_render2(_ptr(objects), len(objects), _ptr(materials), len(materials), _ptr(nodes), _ptr(camera), width,
                    height, _ptr(rows), len(rows), spp, max_depth, _ptr(states), _ptr(out), C.byref(st), nthreads,
                    _ptr(cnt))
    return out, cnt, st


def film_states(seed: int, width: int, rows) -> np.ndarray:
    """XORWOW states for every pixel of `rows` (global row indices), curand_init(seed, pixel, 0)."""
    rows = np.asarray(rows, np.int64)
    out = np.zeros((len(rows) * width, 6), np.uint32)
    # consecutive rows share one jump chain: init each contiguous run in one call
    i = 0
    while i < len(rows):
        j = i
        while j + 1 < len(rows) and rows[j + 1] == rows[j] + 1:
            j += 1
        out[i * width:(j + 1) * width] = xorwow_init_range(seed, int(rows[i]) * width, (j - i + 1) * width)
        i = j + 1
    return out


def philox_word(key: int, counter, word: int) -> int:
    """Philox4x32-10 output word `word` of block (counter[0..3], key)."""
    return int(lib.orc_philox_word(key, *[int(c) for c in counter], word))


def sample_stream(seed: int, sample: int, pixel: int) -> np.ndarray:
    """Sample-mode XORWOW state {d, v0..v4} of pixel-sample (pixel, sample)."""
    st = np.zeros(6, np.uint32)
    lib.orc_sample_stream(seed, sample, pixel, _ptr(st))
    return st
