"""The queued closest-hit kernels (traceKernelQ / traceKernelWideQ: persistent waves whose lanes
take the next ray of the batch by a ballot + mbcnt prefix count as soon as their own ray is done)
against the grid-stride kernels (PT_TRACE_STRIDE=1) and the oracle: the same hit records bit for
bit and the same work counters, on every tree (binary LBVH in the reference order, 8-wide,
instanced), for ragged batch sizes around the wave and pool sizes (64, 256 rays).
"""
import numpy as np
import pytest

from helpers import random_rays, random_soup, rays_to_struct
from test_gpu_parity import assert_hits_equal

pytestmark = pytest.mark.gpu


def both(s, r, kernel, monkeypatch):
    monkeypatch.setenv("PT_TRACE_STRIDE", "1")
    ref, rst = s.trace(r, kernel=kernel)
    monkeypatch.delenv("PT_TRACE_STRIDE")
    q, qst = s.trace(r, kernel=kernel)
    return q, qst, ref, rst


def same_work(a, b):
    assert (a.rays, a.node_visits, a.tri_tests, a.sphere_tests) == (b.rays, b.node_visits, b.tri_tests, b.sphere_tests)


@pytest.mark.parametrize("n", [1, 63, 64, 65, 255, 257, 4097, 100_003])
def test_queued_trace_equals_grid_stride(pt, orc, gpu, n, monkeypatch):
    objs, mats = random_soup(3000, 500, seed=5)
    s = pt.Scene(objs, mats, device=gpu)
    rays = random_rays(n, seed=n, objects=objs)
    r = rays_to_struct(rays, pt.RAY_DTYPE)
    for kernel in (pt.KERNEL_WAVEFRONT, pt.KERNEL_WIDE):
        q, qst, ref, rst = both(s, r, kernel, monkeypatch)
        assert_hits_equal(q, ref)
        same_work(qst, rst)
        assert qst.rays == n
    if n <= 4097:   # and the oracle (the reference's order) for the binary tree's records
        o, ost = orc.trace(objs, orc.build_lbvh(objs, orc.morton_keys(objs), tight=True), rays)
        q, qst = s.trace(r, kernel=pt.KERNEL_WAVEFRONT)
        assert_hits_equal(q, o)
        assert qst.node_visits == ost.node_visits and qst.tri_tests == ost.tri_tests


def test_queued_trace_c3_and_empty_batch(pt, gpu, monkeypatch):
    p = pt.Preset("bunny_cornell")
    s = pt.Scene(p.objects, p.materials, device=gpu)
    rng = np.random.default_rng(2)
    n = 200_000
    inco = np.zeros(n, pt.RAY_DTYPE)   # incoherent rays inside the box: long and short queries mixed
    inco["o"] = rng.uniform((10, 10, 10), (545, 540, 550), (n, 3)).astype(np.float32)
    d = rng.normal(size=(n, 3)).astype(np.float32)
    inco["d"] = d / np.linalg.norm(d, axis=1, keepdims=True)
    for kernel in (pt.KERNEL_WAVEFRONT, pt.KERNEL_WIDE):
        q, qst, ref, rst = both(s, inco, kernel, monkeypatch)
        assert_hits_equal(q, ref)
        same_work(qst, rst)
        assert q["hit"].mean() > 0.5
        h, st = s.trace(inco[:0], kernel=kernel)
        assert len(h) == 0 and st.rays == 0


def test_queued_trace_instanced(pt, gpu, monkeypatch):
    ip = pt.InstancedPreset("bunny_field")
    si = pt.Scene.instanced(ip.objects, ip.mesh_first, ip.mesh_count, ip.instances, ip.materials, device=gpu)
    fp = pt.Preset("bunny_field")
    lo, hi = fp.objects["v"][:, :3].min(0), fp.objects["v"][:, :3].max(0)
    rays = random_rays(50_001, seed=9, center=(lo + hi) / 2, radius=float(np.linalg.norm(hi - lo)) * 0.6,
                       objects=fp.objects)
    r = rays_to_struct(rays, pt.RAY_DTYPE)
    q, qst, ref, rst = both(si, r, pt.KERNEL_WIDE, monkeypatch)
    assert_hits_equal(q, ref)
    same_work(qst, rst)
    assert q["hit"].sum() > 1000
