"""CPU tests of the wide tree (host/pt_wide8.cpp) and of the wide kernels' traversal rule.

tests/cpp/wide8_check.cpp (test infrastructure, built here with g++) builds the 8-wide tree
exactly as libpt.so does, checks its structure (every primitive once, outward-quantised child
planes strictly containing every primitive box below them) and traces rays through a scalar
restatement of renderKernelWF<.., WIDE>'s steps.  Every ray whose result the wide rule decides
(no `redo`) must give the oracle's reference-order closest hit, bit for bit; `redo` rays are
re-traced by the kernels in the reference order (tests/test_gpu_wide.py covers that path).
"""
import os
import subprocess

import numpy as np
import pytest

from helpers import deep_stack_scene, random_rays, random_soup

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def harness(tmp_path_factory):
    d = tmp_path_factory.mktemp("w8")
    exe = str(d / "wide8_check")
    subprocess.run(["g++", "-std=c++17", "-O2", "-ffp-contract=off", "-pthread",
                    "-I", os.path.join(ROOT, "include"), "-I", os.path.join(ROOT, "path-tracer-cuda-opengl_amd", "host"),
                    os.path.join(ROOT, "tests", "cpp", "wide8_check.cpp"),
                    os.path.join(ROOT, "path-tracer-cuda-opengl_amd", "host", "pt_wide8.cpp"),
                    "-L", os.path.join(ROOT, "oracle"), "-loracle", "-Wl,-rpath," + os.path.join(ROOT, "oracle"),
                    "-o", exe], check=True)
    return exe, d


def run(harness, objs, rays):
    exe, d = harness
    objs = np.ascontiguousarray(objs)
    ob, rb, out = str(d / "o.bin"), str(d / "r.bin"), str(d / "out.bin")
    objs.tofile(ob)
    np.ascontiguousarray(rays, np.float32).tofile(rb)
    r = subprocess.run([exe, ob, rb, out], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    res = np.fromfile(out, np.float32).reshape(-1, 3)
    return res[:, 0].astype(np.int64), res[:, 1], res[:, 2] != 0, r.stdout


def compare(orc, harness, objs, rays, max_redo=0.01):
    leaf, t, redo, info = run(harness, objs, rays)
    keys = orc.morton_keys(objs)
    obj = np.where(leaf >= 0, (keys[np.maximum(leaf, 0)] & 0xffffffff).astype(np.int64), -1)
    ref, _ = orc.trace(objs, orc.build_lbvh(objs, keys, tight=True), rays)
    ok = ~redo
    np.testing.assert_array_equal(obj[ok], np.where(ref["hit"] == 1, ref["obj"], -1)[ok])
    h = ok & (ref["hit"] == 1)
    np.testing.assert_array_equal(t[h].view(np.uint32), ref["t"][h].view(np.uint32))
    assert redo.mean() <= max_redo, (redo.mean(), info)
    return redo.mean()


@pytest.mark.parametrize("name", ["triangle_world", "random_world", "test_world", "rtiow", "cornell", "bunny_cornell"])
def test_wide_rule_matches_reference_order(pt, orc, harness, name):
    p = pt.Preset(name)
    lo, hi = p.objects["v"][:, :3].min(0), p.objects["v"][:, :3].max(0)
    center = np.clip((lo + hi) / 2, -1e3, 1e3)
    radius = float(min(np.linalg.norm(hi - lo), 3000.0)) * 0.75 + 1.0
    rays = random_rays(4096, seed=2, center=center, radius=radius, objects=p.objects)
    # rtiow, random_world: origins inside the r = 1000 ground sphere lose digits in the quadratic (grazing
    # hits whose box entry rounds past the hit): those rays are order-dependent and redone
    compare(orc, harness, p.objects, rays, max_redo=0.02 if name in ("rtiow", "random_world") else 0.001)


@pytest.mark.parametrize("seed", [0, 1])
def test_wide_rule_random_soup_and_ties(orc, harness, seed):
    objs, mats = random_soup(1500, 300, seed=seed)
    compare(orc, harness, objs, random_rays(4096, seed=seed + 20, objects=objs))
    dup = np.concatenate([objs, objs, objs])   # exact ties: identical copies
    dup = dup[np.random.default_rng(seed).permutation(len(dup))]
    compare(orc, harness, dup, random_rays(4096, seed=seed + 30, objects=dup))


def test_wide_rule_identical_spheres(orc, harness):
    objs, _ = deep_stack_scene(n_group=256)
    compare(orc, harness, objs, random_rays(2048, seed=8, center=(1024.0, 1024.0, 1024.0), radius=3000.0,
                                            objects=objs))


@pytest.mark.parametrize("n", [1, 2, 3, 4, 9, 25])
def test_wide_rule_tiny_scenes(orc, harness, n):
    objs, _ = random_soup(n - n // 2, n // 2, seed=n)
    compare(orc, harness, objs, random_rays(1024, seed=n, objects=objs))


def test_wide_tree_c5_structure(pt, orc, harness):
    """The 1,043,312-triangle field: structure checks and 2,048 rays."""
    p = pt.Preset("bunny_field", 64, 36)
    rays = random_rays(2048, seed=9, center=(278, 150, 280), radius=700, objects=p.objects)
    compare(orc, harness, p.objects, rays)
