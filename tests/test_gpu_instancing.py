"""Instanced scenes: meshes stored once in object space, placed by
instance transforms, traced through a two-level tree (top-level tree over instance boxes, one
8-wide tree per mesh) by the wide kernel.

The flattened scene (every instance's objects written out in world space, pt_preset_scene) stays
the bit-exact mode.  An instance transforms the RAY into object space instead of the geometry
into world space, so the two differ by float rounding; the bars below are stated per test:
  * identity instances: every hit record bit-exact against the flattened scene (the ray is not
    transformed; only exact ties may pick a different, equal-t object);
  * translation instances (the C5 bunny field): hit/miss agreement >= 99.95 %, same object for
    >= 99.9 % of common hits and on those |dt| <= 1e-4 * t + 1e-4, normal cosine >= 0.9999 on the same object
    (a triangle's normal comes from its object-space edges, the flattened one's from world-space
    edges: different roundings);
  * rotated + scaled instances: against the oracle on geometry transformed in float64,
    agreement >= 99.5 %, same object >= 99.5 % and on those |dt| <= 2e-4 * t + 1e-4, normal
    cosine >= 0.9999 for triangles; for spheres >= 0.995 (median >= 0.99999): the reference's
    sphere test solves its quadratic in float (cuda_object.h:44-68) and for far origins the
    cancellation places the hit point slightly off the surface, in world and object space
    differently (random soups also hold intersecting triangles: near an intersection line the
    closest object may differ);
  * renders: the frame's mean per channel within 1 % and the mean |difference| per channel
    within 0.02 (paths that diverge after a slightly different hit point re-sample).
"""
import numpy as np
import pytest
import torch  # before libpt.so loads (the two must share torch's HIP runtime)

from helpers import OBJECT_DTYPE, random_rays, random_soup, rays_to_struct

pytestmark = pytest.mark.gpu


def flatten(pt, ip):
    """World-space objects of an instanced description (float64 transform, rounded once)."""
    parts = []
    for inst in ip.instances:
        m = inst["m"].astype(np.float64).reshape(3, 4)
        f, c = int(ip.mesh_first[inst["mesh"]]), int(ip.mesh_count[inst["mesh"]])
        o = ip.objects[f:f + c].copy()
        v = o["v"].astype(np.float64)
        tri = o["type"] != 1
        pts = v.reshape(-1, 3, 3)
        w = pts @ m[:, :3].T + m[:, 3]
        out = w.reshape(-1, 9)
        sph = ~tri
        if sph.any():
            out[sph, :3] = v[sph, :3] @ m[:, :3].T + m[:, 3]
            out[sph, 3] = v[sph, 3] * np.cbrt(abs(np.linalg.det(m[:, :3])))
            out[sph, 4:] = 0
        o["v"] = out.astype(np.float32)
        parts.append(o)
    return np.concatenate(parts)


def camera_rays(pt, cam, w, h, seed=0):
    rng = np.random.default_rng(seed)
    c = pt.camera_to_array(cam)
    org, ll, hor, ver = c[0:3], c[3:6], c[6:9], c[9:12]
    ys, xs = np.mgrid[0:h, 0:w]
    u = ((xs + rng.random(xs.shape)) / w).reshape(-1, 1)
    v = ((ys + rng.random(ys.shape)) / h).reshape(-1, 1)
    rays = np.zeros((w * h, 6), np.float32)
    rays[:, :3] = org
    rays[:, 3:] = ll + u * hor + v * ver - org
    return rays


def compare(gi, gf, rel, same_obj_frac, hit_frac, normals_exact, types=None):
    agree = gi["hit"] == gf["hit"]
    assert agree.mean() >= hit_frac, agree.mean()
    both = (gi["hit"] == 1) & (gf["hit"] == 1)
    assert both.sum() > 100
    same = both & (gi["obj"] == gf["obj"])
    assert same.sum() >= same_obj_frac * both.sum(), same.sum() / both.sum()
    dt = np.abs(gi["t"][same] - gf["t"][same])
    assert (dt <= rel * gf["t"][same] + 1e-4).all(), (dt.max(), gf["t"][same][dt.argmax()])
    np.testing.assert_array_equal(gi["mat"][same], gf["mat"][same])
    np.testing.assert_array_equal(gi["front_face"][same], gf["front_face"][same])
    if normals_exact:
        np.testing.assert_array_equal(gi["n"][same].view(np.uint32), gf["n"][same].view(np.uint32))
    else:
        # directions: a sphere's normal (p - c) / r is unit only as far as the hit point lies on
        # the sphere (cuda_object.h:44-68 solves the quadratic in float; far rays cancel), and the
        # instanced normal is normalised after the inverse transpose
        ni = gi["n"][same] / np.linalg.norm(gi["n"][same], axis=1, keepdims=True)
        nf = gf["n"][same] / np.linalg.norm(gf["n"][same], axis=1, keepdims=True)
        cos = (ni * nf).sum(1)
        sph = np.zeros(len(cos), bool) if types is None else types[gf["obj"][same]] == 1
        assert (~sph).any() and cos[~sph].min() >= 0.9999, cos[~sph].min()
        if sph.any():   # the quadratic's cancellation moves the hit point along the sphere
            assert cos[sph].min() >= 0.995 and np.median(cos[sph]) >= 0.99999, (cos[sph].min(), np.median(cos[sph]))


def instanced_scene(pt, ip, gpu):
    return pt.Scene.instanced(ip.objects, ip.mesh_first, ip.mesh_count, ip.instances, ip.materials, device=gpu)


@pytest.mark.parametrize("name", ["cornell", "bunny_cornell", "bunny_field"])
def test_instanced_preset_trace_matches_flattened(pt, gpu, name):
    ip = pt.InstancedPreset(name)
    fp = pt.Preset(name)
    assert ip.flattened_count() == len(fp.objects)
    si = instanced_scene(pt, ip, gpu)
    sf = pt.Scene(fp.objects, fp.materials, device=gpu)
    lo, hi = fp.objects["v"][:, :3].min(0), fp.objects["v"][:, :3].max(0)
    rays = np.concatenate([camera_rays(pt, fp.camera, 320, 180, seed=1),
                           random_rays(16384, seed=3, center=(lo + hi) / 2,
                                       radius=float(np.linalg.norm(hi - lo)) * 0.6, objects=fp.objects)])
    r = rays_to_struct(rays, pt.RAY_DTYPE)
    gi, sti = si.trace(r, kernel=pt.KERNEL_WIDE)
    gf, _ = sf.trace(r, kernel=pt.KERNEL_WIDE)
    assert sti.rays == len(rays)
    assert si.wide_info()["source"] == 3
    if name == "cornell":   # identity instance: bit-exact but for exact ties between coplanar halves
        for f in ("hit", "mat", "front_face"):
            np.testing.assert_array_equal(gi[f], gf[f])
        h = gi["hit"] == 1
        for f in ("t", "p", "n"):
            np.testing.assert_array_equal(gi[f][h].view(np.uint32), gf[f][h].view(np.uint32))
    else:
        compare(gi, gf, 1e-4, 0.999, 0.9995, normals_exact=False)


def test_identity_instances_bit_exact(pt, gpu):
    """Two meshes, each placed once by the identity: the flattened scene's hit records bit for bit
    (no duplicated geometry, so no exact ties)."""
    a, mats = random_soup(1500, 200, seed=11)
    b, _ = random_soup(800, 100, seed=12)
    b["v"][:, :3] += 3.0
    objs = np.concatenate([a, b])
    inst = np.zeros(2, pt.INSTANCE_DTYPE)
    inst["m"][:] = [1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0]
    inst["mesh"] = [0, 1]
    si = pt.Scene.instanced(objs, [0, len(a)], [len(a), len(b)], inst, mats, device=gpu)
    sf = pt.Scene(objs, mats, device=gpu)
    rays = rays_to_struct(random_rays(16384, seed=13, objects=objs), pt.RAY_DTYPE)
    gi, _ = si.trace(rays, kernel=pt.KERNEL_WIDE)
    gf, _ = sf.trace(rays, kernel=pt.KERNEL_WIDE)
    for f in ("hit", "obj", "mat", "front_face"):
        np.testing.assert_array_equal(gi[f], gf[f], err_msg=f)
    h = gi["hit"] == 1
    assert h.sum() > 1000
    for f in ("t", "p", "n"):
        np.testing.assert_array_equal(gi[f][h].view(np.uint32), gf[f][h].view(np.uint32), err_msg=f)


def random_transforms(n, seed):
    rng = np.random.default_rng(seed)
    out = np.zeros((n, 12), np.float32)
    for i in range(n):
        q, _ = np.linalg.qr(rng.normal(size=(3, 3)))
        s = rng.uniform(0.5, 2.0)
        out[i] = np.concatenate([q * s, rng.uniform(-30, 30, (3, 1))], 1).reshape(-1)
    return out


def test_rotated_scaled_instances_match_oracle(pt, orc, gpu):
    """Rotations with uniform scales (spheres stay spheres), many instances of two meshes, against
    the oracle's trace of the flattened world geometry (float64 transform)."""
    a, mats = random_soup(600, 60, seed=21, spread=4.0)
    b, _ = random_soup(300, 30, seed=22, spread=3.0)
    objs = np.concatenate([a, b])
    inst = np.zeros(40, pt.INSTANCE_DTYPE)
    inst["m"] = random_transforms(40, seed=23)
    inst["mesh"] = np.arange(40) % 2
    si = pt.Scene.instanced(objs, [0, len(a)], [len(a), len(b)], inst, mats, device=gpu)

    class Desc:
        pass
    d = Desc()
    d.objects, d.mesh_first, d.mesh_count, d.instances = objs, np.array([0, len(a)]), np.array([len(a), len(b)]), inst
    flat = flatten(pt, d)
    rays = random_rays(16384, seed=24, radius=60.0, objects=flat)
    gi, _ = si.trace(rays_to_struct(rays, pt.RAY_DTYPE), kernel=pt.KERNEL_WIDE)
    ref, _ = orc.trace(flat, orc.build_lbvh(flat, orc.morton_keys(flat), tight=True), rays, 0.001, np.inf)
    compare(gi, ref, 2e-4, 0.995, 0.995, normals_exact=False, types=flat["type"])
    # the reported object index is the flattened order's
    assert gi["obj"][gi["hit"] == 1].max() < len(flat)


@pytest.mark.parametrize("name,w,h,spp", [("cornell", 96, 96, 8), ("bunny_cornell", 128, 128, 8),
                                          ("bunny_field", 192, 108, 4)])
def test_instanced_render_close_to_flattened(pt, gpu, name, w, h, spp):
    ip = pt.InstancedPreset(name, w, h)
    fp = pt.Preset(name, w, h)
    si = instanced_scene(pt, ip, gpu)
    sf = pt.Scene(fp.objects, fp.materials, device=gpu)
    ri, sti = pt.render(si, pt.Film(w, h, 7, device=gpu), ip.camera, spp, ip.max_depth, kernel=pt.KERNEL_WIDE,
                        rng=pt.RNG_SAMPLE)
    rf, stf = pt.render(sf, pt.Film(w, h, 7, device=gpu), fp.camera, spp, fp.max_depth, kernel=pt.KERNEL_WIDE,
                        rng=pt.RNG_SAMPLE)
    assert np.isfinite(ri).all()
    mi, mf = ri.mean(0), rf.mean(0)
    assert (np.abs(mi - mf) <= 0.01 * mf + 1e-4).all(), (mi, mf)
    assert (np.abs(ri - rf).mean(0) <= 0.02).all(), np.abs(ri - rf).mean(0)
    assert abs(sti.rays - stf.rays) <= 0.01 * stf.rays
    if name == "cornell":   # identity instance: the same frame
        np.testing.assert_array_equal(ri, rf)


def test_instanced_memory_and_build(pt, gpu):
    ip = pt.InstancedPreset("bunny_field")
    fp = pt.Preset("bunny_field")
    si = instanced_scene(pt, ip, gpu)
    sf = pt.Scene(fp.objects, fp.materials, device=gpu)
    sf.trace(rays_to_struct(np.zeros((1, 6), np.float32) + 1, pt.RAY_DTYPE), kernel=pt.KERNEL_WIDE)  # wide tree
    bi, bf = si.bvh_info()["device_bytes"], sf.bvh_info()["device_bytes"]
    assert bi * 20 < bf, (bi, bf)
    wi = si.wide_info()
    assert wi["source"] == 3 and wi["depth"] > 0 and wi["build_ms"] < 1000.0


def test_instanced_scene_rules(pt, gpu):
    ip = pt.InstancedPreset("bunny_cornell", 32, 32)
    si = instanced_scene(pt, ip, gpu)
    rays = rays_to_struct(camera_rays(pt, ip.camera, 8, 8), pt.RAY_DTYPE)
    for k in (pt.KERNEL_SIMPLE, pt.KERNEL_WAVEFRONT):
        with pytest.raises(pt.PtError):
            si.trace(rays, kernel=k)
        with pytest.raises(pt.PtError):
            pt.render(si, pt.Film(32, 32, 1, device=gpu), ip.camera, 1, 4, kernel=k)
    hits, _ = si.trace(rays)   # the default kernel is the wide one
    assert hits["hit"].sum() > 0
    with pytest.raises(pt.PtError):
        si.update_objects(ip.objects[:1])
    with pytest.raises(pt.PtError):
        si.download_bvh()
    # compat-mode RNG works too (per-pixel XORWOW streams)
    rgb, st = pt.render(si, pt.Film(32, 32, 1, device=gpu), ip.camera, 2, 8, kernel=pt.KERNEL_WIDE)
    assert np.isfinite(rgb).all() and st.rays > 0


@pytest.mark.parametrize("size,dist,same_frac", [(20.0, 300.0, 0.995), (20.0, 1200.0, 0.995), (20.0, 60000.0, 0.97)])
def test_far_origins_into_small_instances(pt, gpu, size, dist, same_frac):
    """A small mesh (the bunny, 5,000 triangles, scaled to `size` units) placed by translations
    about 1,000 units apart, traced from origins `dist` units away -- up to 3,000 mesh sizes, far
    beyond the range a tree quantised against the mesh's own size covers (its box
    tests could then drop true hits).  The mesh trees are now quantised against the world's reach into object
    space, and origins beyond 8 world extents (dist 60,000) start at their entry into the world
    (instEntry).  Against the flattened scene (whose far origins take the reference-order query),
    at the float resolution of the distance (rays that graze a silhouette or an edge may go
    either way, in both directions alike): hit / miss agreement >= 99.8 %, the hits lost not
    more than twice the hits gained (+ 10) -- a traversal that drops boxes loses hits one way --,
    the same triangle on >= same_frac of common hits (at 60,000 units a float step is 0.004-0.008,
    a fair share of a small triangle), |dt| within the translation bar."""
    ip = pt.InstancedPreset("bunny_field", 32, 32)
    f, c = int(ip.mesh_first[1]), int(ip.mesh_count[1])
    a = ip.objects[f:f + c].copy()
    v = a["v"][:, :9].reshape(-1, 3, 3)
    cen = v.reshape(-1, 3).mean(0)
    span = float((v.reshape(-1, 3).max(0) - v.reshape(-1, 3).min(0)).max())
    a["v"][:, :9] = ((v - cen) * (size / span)).reshape(-1, 9)
    mats = ip.materials
    inst = np.zeros(5, pt.INSTANCE_DTYPE)
    offs = np.array([[0, 0, 0], [1000, 0, 0], [0, 1000, 0], [-800, 300, 200], [300, -900, 600]], np.float32)
    inst["m"][:] = [1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0]
    inst["m"][:, 3], inst["m"][:, 7], inst["m"][:, 11] = offs[:, 0], offs[:, 1], offs[:, 2]
    inst["mesh"] = 0
    si = pt.Scene.instanced(a, [0], [len(a)], inst, mats, device=gpu)
    flat = np.concatenate([a.copy() for _ in range(5)])
    for k in range(5):
        for j in range(3):
            flat["v"][k * len(a):(k + 1) * len(a), 3 * j:3 * j + 3] += offs[k]
    sf = pt.Scene(flat, mats, device=gpu)
    rng = np.random.default_rng(32)
    n = 20000
    k = rng.integers(0, 5, n)
    tri = rng.integers(0, len(a), n)
    tgt = (a["v"][tri, 0:3] + a["v"][tri, 3:6] + a["v"][tri, 6:9]) / 3 + offs[k] + rng.normal(0, 0.025 * size, (n, 3))
    dirs = rng.normal(size=(n, 3))
    dirs /= np.linalg.norm(dirs, axis=1, keepdims=True)
    org = tgt - dirs * dist
    rays = np.zeros((n, 6), np.float32)
    rays[:, :3] = org
    rays[:, 3:] = (tgt - org) / dist
    r = rays_to_struct(rays, pt.RAY_DTYPE)
    gi, _ = si.trace(r, kernel=pt.KERNEL_WIDE)
    gf, _ = sf.trace(r, kernel=pt.KERNEL_WIDE)
    assert (gf["hit"] == 1).mean() > 0.3
    lost = ((gf["hit"] == 1) & (gi["hit"] == 0)).sum()
    gained = ((gf["hit"] == 0) & (gi["hit"] == 1)).sum()
    assert lost <= 2 * gained + 10, (lost, gained)
    compare(gi, gf, 1e-4, same_frac, 0.998, normals_exact=False)


def test_far_camera_instanced_render(pt, gpu):
    """The render kernel's far-camera path for instanced scenes: a camera beyond 8 world extents
    (the bunny field seen from 40 extents away through a narrow field of view) starts its rays at
    their entry into the world (instEntry).  Camera rays only (depth 1): the flattened scene's
    frame (whose far camera rays take the reference-order query) pixel for pixel within 1e-5 but
    for grazing silhouettes at 26,000 units (<= 0.2 % of the pixels).  Deeper bounces are not compared: from a hit point
    computed off a 26,000-unit origin the reference's bounce rays re-hit their own surface
    depending on its rounding (self-intersection noise about the 0.001 ray offset), which the
    instanced path's better-conditioned hit points do not reproduce."""
    w, h, spp = 96, 64, 4
    ip = pt.InstancedPreset("bunny_field", w, h)
    fp = pt.Preset("bunny_field", w, h)
    lo, hi = fp.objects["v"][:, :3].min(0), fp.objects["v"][:, :3].max(0)
    c = (lo + hi) / 2
    ext = float((hi - lo).max())
    cam = pt.camera_make(c + np.array([0.3, 0.5, -1.0], np.float32) * 40 * ext, c, 1.2, w / h)
    si = instanced_scene(pt, ip, gpu)
    sf = pt.Scene(fp.objects, fp.materials, device=gpu)
    ri, sti = pt.render(si, pt.Film(w, h, 3, device=gpu), cam, spp, 1, kernel=pt.KERNEL_WIDE, rng=pt.RNG_SAMPLE)
    rf, stf = pt.render(sf, pt.Film(w, h, 3, device=gpu), cam, spp, 1, kernel=pt.KERNEL_WIDE, rng=pt.RNG_SAMPLE)
    assert sti.rays == stf.rays == w * h * spp
    assert (np.abs(ri - rf).max(1) > 1e-5).mean() <= 0.002
    # and the full path count stays finite and close
    rd, std = pt.render(si, pt.Film(w, h, 3, device=gpu), cam, spp, ip.max_depth, kernel=pt.KERNEL_WIDE,
                        rng=pt.RNG_SAMPLE)
    assert np.isfinite(rd).all() and std.paths == w * h * spp


@pytest.mark.parametrize("rng", ["sample", "compat"])
def test_instanced_frame_independent_of_scheduling(pt, gpu, rng):
    """The instanced kernels' frame is a function of scene, camera, seed and spp only, as the
    flattened kernels' is (pt.h: neither the scheduling nor the stripe partition changes the image):
    other LEAF / SHADE thresholds (the instanced defaults are 16 / 20), the identity launch order and
    a 2-way partition of 8-row stripes give the same bits and rays."""
    w, h, spp = 96, 54, 4
    ip = pt.InstancedPreset("bunny_field", w, h)
    s = instanced_scene(pt, ip, gpu)
    r = pt.RNG_SAMPLE if rng == "sample" else pt.RNG_COMPAT

    def frame(film_kw=None, **kw):
        f = pt.Film(w, h, 7, device=gpu, **(film_kw or {}))
        img, st = pt.render(s, f, ip.camera, spp, ip.max_depth, kernel=pt.KERNEL_WIDE, rng=r, **kw)
        return img, st, f

    a, sa, _ = frame()
    for kw in ({"leaf_batch": 5, "shade_batch": 40}, {"leaf_batch": 40, "shade_batch": 6},
               {"flags": pt.IDENTITY_ORDER}):
        b, sb, _ = frame(**kw)
        np.testing.assert_array_equal(b.view(np.uint32), a.view(np.uint32), err_msg=str(kw))
        assert sb.rays == sa.rays, kw
    full = a.reshape(h, w, 3)
    rays = 0
    for part in (0, 1):
        img, st, f = frame({"stripe_height": 8, "n_parts": 2, "part": part})
        np.testing.assert_array_equal(img.reshape(-1, w, 3).view(np.uint32), full[f.rows].view(np.uint32))
        rays += st.rays
    assert rays == sa.rays
