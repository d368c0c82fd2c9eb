"""Generate the oracle golden fixtures of SURVEY.md §8(c) (F1-F5) -> tests/golden/oracle_fixtures.npz.

The fixtures freeze the CPU restatement's outputs (oracle/, itself pinned to the reference's
committed render exp2.png and its probe counters) on fixed inputs, so that both the
oracle and the HIP path are checked against committed data: tests/test_fixtures.py (CPU: the
oracle and the host builders reproduce every array bit for bit) and tests/test_gpu_fixtures.py
(GPU: the device LBVH, closest hits and frames equal them).  Inputs are stored next to outputs.

  F1  sorted 64-bit Morton keys ((code << 32) | objID)        C2, C3
  F2  LBVH left/right/parent/objID + boxes (tight; origin-inflated for C2 and TRIANGLEWORLD)
  F3  2,048 seeded rays per scene -> closest-hit records (the BVH traversal; brute force agrees)
  F4  Material::scatter for each material type driven by scripted uniform tapes
  F5  compat-mode frames: C1 (RTIOW 400x225 @8 spp, depth 50, seed 1) fp32 RGB + its PNG bytes
      (saveColor), a 64x64 C2 @16 spp depth 8; and a sample-mode 96x54 C3 @4 spp (chunk 2)

usage: python tools/make_fixtures.py        (CPU; a few seconds on 8 threads)
"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "path-tracer-cuda-opengl_amd", "python"))
sys.path.insert(0, os.path.join(REPO, "oracle"))
sys.path.insert(0, os.path.join(REPO, "tests"))
import oracle  # noqa: E402
import ptamd  # noqa: E402
from helpers import random_rays  # noqa: E402

OUT = os.path.join(REPO, "tests", "golden", "oracle_fixtures.npz")
NTHREADS = 8

# (fixture prefix, preset, width, height): scene inputs stored for every prefix
SCENES = [("c1", "rtiow", 400, 225), ("tw", "triangle_world", 0, 0), ("c2", "cornell", 64, 64),
          ("c3", "bunny_cornell", 96, 54)]


def scene_rays(objects, seed):
    lo = objects["v"][:, :3].min(0)
    hi = objects["v"][:, :3].max(0)
    center = np.clip((lo + hi) / 2, -1e3, 1e3)
    radius = float(min(np.linalg.norm(hi - lo), 3000.0)) * 0.75 + 1.0
    return random_rays(2048, seed=seed, center=center, radius=radius, objects=objects)


def scatter_cases(objects, hits, rays, rng):
    """F4: for each material type, 16 (ray, hit, tape) cases from real hits of F3."""
    mats = np.zeros(3, oracle.MATERIAL_DTYPE)
    mats["type"] = [1, 2, 4]                          # LAMBERTIAN, METAL, DIELECTRIC
    mats["albedo"] = [(0.7, 0.3, 0.2), (0.8, 0.8, 0.9), (1.0, 1.0, 1.0)]
    mats["fuzz"] = [0.0, 0.3, 0.0]
    mats["ir"] = [0.0, 0.0, 1.5]
    idx = np.flatnonzero(hits["hit"] == 1)[:16]
    rows = []
    for m in range(3):
        for i in idx:
            # a tape long enough for any rejection loop; values in (0, 1] like curand_uniform
            tape = rng.uniform(0.0, 1.0, 64).astype(np.float32)
            tape[tape == 0] = np.float32(0.5)
            ok, out, att, used = oracle.scatter_tape(mats[m], rays[i], hits[i], tape)
            rows.append((m, i, tape, int(ok), out, att, used))
    return {
        "f4_materials": mats,
        "f4_mat": np.array([r[0] for r in rows], np.int32),
        "f4_case": np.array([r[1] for r in rows], np.int32),
        "f4_tape": np.stack([r[2] for r in rows]),
        "f4_ok": np.array([r[3] for r in rows], np.int32),
        "f4_out": np.stack([r[4] for r in rows]).astype(np.float32),
        "f4_att": np.stack([r[5] for r in rows]).astype(np.float32),
        "f4_used": np.array([r[6] for r in rows], np.int32),
    }


def main():
    fx = {}
    for key, name, w, h in SCENES:
        p = ptamd.Preset(name, w, h)
        fx[f"{key}_objects"] = p.objects
        fx[f"{key}_materials"] = p.materials
        fx[f"{key}_camera"] = ptamd.camera_to_array(p.camera)
        fx[f"{key}_size"] = np.array([p.width, p.height], np.int32)
    # F1 / F2
    for key in ("c2", "c3", "tw"):
        objs = fx[f"{key}_objects"]
        keys = oracle.morton_keys(objs)
        if key in ("c2", "c3"):
            fx[f"f1_{key}_keys"] = keys
        fx[f"f2_{key}_tight"] = oracle.build_lbvh(objs, keys, tight=True)
        if key in ("c2", "tw"):
            fx[f"f2_{key}_ref"] = oracle.build_lbvh(objs, keys, tight=False)
    # F3 (+ F4 from the C3 hits)
    for n, key in enumerate(("c2", "c3", "tw")):
        objs = fx[f"{key}_objects"]
        rays = scene_rays(objs, seed=100 + n)
        hits, st = oracle.trace(objs, fx[f"f2_{key}_tight"], rays)
        brute, _ = oracle.trace(objs, None, rays, brute=True)
        assert (hits["obj"] == brute["obj"]).all(), key
        assert hits["hit"].sum() > 100, key
        fx[f"f3_{key}_rays"] = rays
        fx[f"f3_{key}_hits"] = hits
        fx[f"f3_{key}_counts"] = np.array([st.node_visits, st.tri_tests, st.sphere_tests], np.int64)
    fx.update(scatter_cases(fx["c3_objects"], fx["f3_c3_hits"], fx["f3_c3_rays"], np.random.default_rng(5)))
    # F5
    for key, spp, depth in (("c1", 8, 50), ("c2", 16, 8)):
        objs, mats, cam = fx[f"{key}_objects"], fx[f"{key}_materials"], fx[f"{key}_camera"]
        w, h = (int(v) for v in fx[f"{key}_size"])
        rows = np.arange(h, dtype=np.int32)
        nodes = oracle.build_lbvh(objs, oracle.morton_keys(objs), tight=True)
        states = oracle.film_states(1, w, rows)
        rgb, st = oracle.render(objs, mats, nodes, cam, w, h, rows, spp, depth, states, nthreads=NTHREADS)
        fx[f"f5_{key}_rgb"] = rgb
        if key == "c2":   # (C1's 2.2 MB of advanced states would not compress: C2's pin the streams)
            fx[f"f5_{key}_rng_after"] = states
        fx[f"f5_{key}_params"] = np.array([spp, depth, 1], np.int64)
        fx[f"f5_{key}_counts"] = np.array([st.rays, st.paths], np.int64)
        if key == "c1":
            fx["f5_c1_rgba8"] = oracle.quantize_png(rgb)
    objs, mats, cam = fx["c3_objects"], fx["c3_materials"], fx["c3_camera"]
    w, h = (int(v) for v in fx["c3_size"])
    nodes = oracle.build_lbvh(objs, oracle.morton_keys(objs), tight=True)
    rgb, st = oracle.render_sample(objs, mats, nodes, cam, w, h, np.arange(h, dtype=np.int32), 4, 50, 1, 2,
                                   nthreads=NTHREADS)
    fx["f5_c3_sample_rgb"] = rgb
    fx["f5_c3_sample_params"] = np.array([4, 50, 1, 2], np.int64)   # spp, depth, seed, chunk
    fx["f5_c3_sample_counts"] = np.array([st.rays, st.paths], np.int64)
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    np.savez_compressed(OUT, **fx)
    print(f"{OUT}: {len(fx)} arrays, {os.path.getsize(OUT) / 1e6:.2f} MB")


if __name__ == "__main__":
    main()
