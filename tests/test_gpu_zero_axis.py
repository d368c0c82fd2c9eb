"""Rays parallel to an axis plane (a direction component of exactly +-0, |1/d| = inf).

The reference's slab test (aabb.h:21-34) handles them exactly: (plane - o) * inf is -inf / +inf by
the side of the plane the origin lies on, so the axis bounds nothing when o lies between a box's
planes and rejects the box otherwise.  The wide tree's decomposed plane distances
q * (s * inv) + (p - o) * inv are NaN for every plane of such an axis, which the NaN-ignoring min /
max drop: conservative, but the ray then enters every box it overlaps in the other two axes (round
4: 1,000-1,500 node visits per query for C5 rays at the origin's height).  Two fixes, both guarded
here by a bound on the node visits as well as by the hit records:
  * flattened scenes: such a ray takes the reference-order query (mixUnsafe) -- hits bit-exact;
  * instanced scenes (no reference-order query): the children a lane's exact slab test rejects on
    that axis are culled before the node test (zeroAxisKeep / wideHitsInst) -- hits within the
    instancing tolerance of the flattened scene (test_gpu_instancing.py).
The bound compares a batch with exact zeros against the same rays with the zeros nudged to +-2^-30
(finite reciprocals, the wide path's ordinary arithmetic): a regression to the NaN planes multiplies
the zero batch's visits many times over while every hit record stays the same.
"""
import os

import numpy as np
import pytest
import torch  # before libpt.so loads (the two must share torch's HIP runtime)

from helpers import rays_to_struct
from test_gpu_instancing import compare, instanced_scene

pytestmark = pytest.mark.gpu

NUDGE = np.float32(2.0 ** -30)


def zero_rays(objs, n, seed, height_frac=(0.02, 0.2)):
    """Rays at the height of the scene's lower geometry (the bunnies on the floor), from in front of
    the box and from inside it: d.y = 0 exactly (and for a quarter also d.x or d.z = 0); returns
    (rays with exact zeros, the same rays with every zero nudged to +-2^-30)."""
    rng = np.random.default_rng(seed)
    lo, hi = objs["v"][:, :3].min(0), objs["v"][:, :3].max(0)
    ext = hi - lo
    o = np.empty((n, 3), np.float32)
    o[:, 0] = lo[0] + ext[0] * rng.uniform(0.05, 0.95, n)
    o[:, 1] = lo[1] + ext[1] * rng.uniform(height_frac[0], height_frac[1], n)
    inside = rng.random(n) < 0.5
    o[:, 2] = np.where(inside, lo[2] + ext[2] * rng.uniform(0.05, 0.95, n), lo[2] - 0.5 * ext[2])
    ang = rng.uniform(-0.6, 0.6, n) + np.where(rng.random(n) < 0.3, np.pi, 0.0) * inside
    d = np.stack([np.sin(ang), np.zeros(n), np.cos(ang)], 1).astype(np.float32)
    q = rng.random(n)
    d[q < 0.125, 0] = 0.0          # along z
    d[(q >= 0.125) & (q < 0.25), 2] = 0.0   # along x
    d[(q >= 0.25) & (q < 0.3), 1] = -0.0    # a negative zero
    d[(d[:, 0] == 0) & (d[:, 2] == 0), 2] = 1.0
    zero = np.concatenate([o, d], 1).astype(np.float32)
    nud = zero.copy()
    dd = nud[:, 3:]
    z = dd == 0
    dd[z] = np.where(np.signbit(dd[z]), -NUDGE, NUDGE)
    assert (zero[:, 3:] == 0).sum() >= n
    return zero, nud


@pytest.mark.parametrize("stride", ["0", "1"])
@pytest.mark.parametrize("name", ["bunny_cornell", "bunny_field"])
def test_zero_direction_flattened_trace(pt, orc, gpu, name, stride, monkeypatch):
    """C3 and C5 (flattened): hit records bit-exact against the oracle; the zero batch's wide node
    visits at most those of the nudged batch plus one per ray (its rays take the reference-order
    query, which the wide counter does not count); queued and grid-stride kernels."""
    monkeypatch.setenv("PT_TRACE_STRIDE", stride)
    p = pt.Preset(name, 32, 32)
    objs = p.objects
    n = 4096 if name == "bunny_field" else 8192
    zero, nud = zero_rays(objs, n, seed=11)
    s = pt.Scene(objs, p.materials, device=gpu)
    hz, stz = s.trace(rays_to_struct(zero, pt.RAY_DTYPE), kernel=pt.KERNEL_WIDE)
    hn, stn = s.trace(rays_to_struct(nud, pt.RAY_DTYPE), kernel=pt.KERNEL_WIDE)
    ref, _ = orc.trace(objs, orc.build_lbvh(objs, orc.morton_keys(objs), tight=True), zero, 0.001, np.inf)
    for f in ("hit", "obj", "mat", "front_face"):
        np.testing.assert_array_equal(hz[f], ref[f], err_msg=f)
    h = hz["hit"] == 1
    for f in ("t", "p", "n"):
        np.testing.assert_array_equal(hz[f][h].view(np.uint32), ref[f][h].view(np.uint32), err_msg=f)
    assert h.sum() > n // 4
    assert stn.node_visits > n   # the nudged rays do traverse the wide tree
    assert stz.node_visits <= stn.node_visits + n, (stz.node_visits / n, stn.node_visits / n)


@pytest.mark.parametrize("stride", ["0", "1"])
def test_zero_direction_instanced_trace(pt, gpu, stride, monkeypatch):
    """C5 instanced (two-level tree, no reference-order query): the zero batch's node visits stay
    within 1.25x of the nudged batch's (+ 2 per ray) -- not the 100x of the NaN planes -- and its hit
    records match the flattened scene's (whose zero rays take the reference-order query) within the
    instancing tolerance; queued and grid-stride kernels."""
    monkeypatch.setenv("PT_TRACE_STRIDE", stride)
    ip = pt.InstancedPreset("bunny_field")
    fp = pt.Preset("bunny_field")
    n = 8192
    zero, nud = zero_rays(fp.objects, n, seed=12)
    si = instanced_scene(pt, ip, gpu)
    sf = pt.Scene(fp.objects, fp.materials, device=gpu)
    gz, stz = si.trace(rays_to_struct(zero, pt.RAY_DTYPE), kernel=pt.KERNEL_WIDE)
    _, stn = si.trace(rays_to_struct(nud, pt.RAY_DTYPE), kernel=pt.KERNEL_WIDE)
    gf, _ = sf.trace(rays_to_struct(zero, pt.RAY_DTYPE), kernel=pt.KERNEL_WIDE)
    compare(gz, gf, 1e-4, 0.999, 0.9995, normals_exact=False)
    assert stz.rays == n and stn.node_visits > n
    assert stz.node_visits <= 1.25 * stn.node_visits + 2 * n, (stz.node_visits / n, stn.node_visits / n)


def slit_camera(pt, cam, tilt):
    """The preset camera with its vertical viewport extent replaced by (0, tilt, 0): tilt 0 gives
    every camera ray d.y = lower_left.y - origin.y = 0 exactly (a level camera's rows collapsed onto
    the horizon row)."""
    c = pt.Camera.from_buffer_copy(bytes(cam))
    c.vertical[0], c.vertical[1], c.vertical[2] = 0.0, tilt, 0.0
    c.lower_left[1] = c.origin[1] - tilt / 2
    return c


def test_zero_direction_instanced_render(pt, gpu):
    """The render kernel's instanced NODE step (wideHitsInst) on camera rays that are all parallel to
    the floor (d.y = 0 exactly) at the bunnies' height: the frame's node visits stay within 1.25x of
    the same camera tilted by a hair (finite reciprocals), and the frame matches the flattened
    scene's within the instancing render tolerance (per-channel mean 1 %, mean |difference| 0.02)."""
    w, h, spp = 96, 32, 8
    ip = pt.InstancedPreset("bunny_field", w, h)
    fp = pt.Preset("bunny_field", w, h)
    base = pt.Camera.from_buffer_copy(bytes(fp.camera))
    base.origin[1] = 20.0     # at the bunnies' height, level
    base.lower_left[1] = 20.0
    cz, ct = slit_camera(pt, base, 0.0), slit_camera(pt, base, 1e-3)
    c = pt.camera_to_array(cz)
    assert c[10] == 0.0 and c[4] == c[1]   # vertical.y = 0, lower_left.y = origin.y
    si = instanced_scene(pt, ip, gpu)
    sf = pt.Scene(fp.objects, fp.materials, device=gpu)
    depth = 1   # camera rays only: the rows with d.y = 0
    rz, stz = pt.render(si, pt.Film(w, h, 5, device=gpu), cz, spp, depth, kernel=pt.KERNEL_WIDE, rng=pt.RNG_SAMPLE)
    _, stt = pt.render(si, pt.Film(w, h, 5, device=gpu), ct, spp, depth, kernel=pt.KERNEL_WIDE, rng=pt.RNG_SAMPLE)
    rf, _ = pt.render(sf, pt.Film(w, h, 5, device=gpu), cz, spp, depth, kernel=pt.KERNEL_WIDE, rng=pt.RNG_SAMPLE)
    assert stz.rays == stt.rays == w * h * spp
    assert stz.node_visits <= 1.25 * stt.node_visits + 2 * stz.rays, (stz.node_visits / stz.rays,
                                                                       stt.node_visits / stt.rays)
    m_i, m_f = rz.mean(0), rf.mean(0)
    assert (np.abs(m_i - m_f) <= 0.01 * np.abs(m_f) + 1e-6).all(), (m_i, m_f)
    assert np.abs(rz - rf).mean() <= 0.02
    # full paths too: the bounces leave the floor plane, the first segment does not
    rd, std = pt.render(si, pt.Film(w, h, 5, device=gpu), cz, spp, ip.max_depth, kernel=pt.KERNEL_WIDE,
                        rng=pt.RNG_SAMPLE)
    assert np.isfinite(rd).all() and std.paths == w * h * spp
