"""CPU restatements of the two rules the device-built wide tree (csrc/pt_wide_build.hip) relies
on, checked without a GPU:

* rankKernel: leaf k's reference rank (its position in RenderManager::hitBvh's leaf order,
  render_manager.h:105-133) computed by climbing from the leaf and summing its offset in each
  ancestor's visit -- must equal the order of the reference's DFS itself;
* plocNearestKernel: nearest neighbours under the order (area, |i - j|, min odd, min) -- the
  globally first pair is mutual (every pass merges), and equal boxes pair off so a pass halves
  them (no quadratic pass count on duplicated geometry).

The GPU tests (tests/test_gpu_wide.py on both trees, tests/test_gpu_dynamic.py) check the kernels
themselves against the oracle's hits.
"""
import numpy as np
import pytest

from helpers import deep_stack_scene, random_soup


def dfs_ranks(nodes, n):
    """The reference's visiting order of leaves: at a node its leaf children (left, right), then
    the right subtree, then the left one (the left child is pushed first)."""
    rank = np.zeros(n, np.int64)
    nxt = 0
    stack = [0]
    leaf0 = n - 1
    while stack:
        i = stack.pop()
        l, r = int(nodes["left"][i]), int(nodes["right"][i])
        for c in (l, r):
            if c >= leaf0:
                rank[c - leaf0] = nxt
                nxt += 1
        for c in (l, r):
            if c < leaf0:
                stack.append(c)
    return rank


def climb_ranks(nodes, n):
    """rankKernel's rule: per ancestor, the child's offset in the ancestor's visit."""
    leaf0 = n - 1
    size = np.zeros(2 * n - 1, np.int64)
    size[leaf0:] = 1
    # sizes bottom-up (post order by an explicit stack)
    order, stack = [], [0]
    while stack:
        i = stack.pop()
        order.append(i)
        for c in (int(nodes["left"][i]), int(nodes["right"][i])):
            if c < leaf0:
                stack.append(c)
    for i in reversed(order):
        size[i] = size[nodes["left"][i]] + size[nodes["right"][i]]
    rank = np.zeros(n, np.int64)
    for k in range(n):
        r, child, p = 0, leaf0 + k, int(nodes["parent"][leaf0 + k])
        while p >= 0:
            l, rr = int(nodes["left"][p]), int(nodes["right"][p])
            l_leaf, r_leaf = l >= leaf0, rr >= leaf0
            nl = int(l_leaf) + int(r_leaf)
            is_left = child == l
            if child >= leaf0:
                r += 1 if (not is_left and l_leaf) else 0
            elif not is_left:
                r += nl
            else:
                r += nl + (0 if r_leaf else int(size[rr]))
            child, p = p, int(nodes["parent"][p])
        rank[k] = r
    return rank


@pytest.mark.parametrize("case", ["soup0", "soup1", "dups", "deep", "tiny2", "tiny3"])
def test_climb_ranks_equal_reference_dfs(orc, case):
    if case.startswith("soup"):
        objs, _ = random_soup(700, 300, seed=int(case[-1]))
    elif case == "dups":
        objs, _ = random_soup(200, 100, seed=7)
        objs = np.concatenate([objs, objs, objs])
    elif case == "deep":
        objs, _ = deep_stack_scene(n_group=64)
    else:
        objs, _ = random_soup(int(case[-1]) - 1, 1, seed=3)
    n = len(objs)
    nodes = orc.build_lbvh(objs, orc.morton_keys(objs), tight=True)
    want = dfs_ranks(nodes, n)
    assert sorted(want.tolist()) == list(range(n))
    np.testing.assert_array_equal(climb_ranks(nodes, n), want)


def area(lo, hi):
    d = (hi - lo).astype(np.float32)
    return d[..., 0] * d[..., 1] + d[..., 1] * d[..., 2] + d[..., 2] * d[..., 0]


def nearest(lo, hi, radius):
    m = len(lo)
    nn = np.full(m, -1, np.int64)
    for i in range(m):
        best, best_key = -1, None
        for o in range(-radius, radius + 1):
            j = i + o
            if o == 0 or j < 0 or j >= m:
                continue
            a = area(np.minimum(lo[i], lo[j]), np.maximum(hi[i], hi[j]))
            mn = min(i, j)
            key = (float(a), abs(o), mn & 1, mn)
            if best_key is None or key < best_key:
                best, best_key = j, key
        nn[i] = best
    return nn


def ploc_pass(lo, hi, radius):
    nn = nearest(lo, hi, radius)
    keep_lo, keep_hi, merged = [], [], 0
    for i in range(len(lo)):
        j = nn[i]
        mutual = j >= 0 and nn[j] == i
        if mutual and i > j:
            continue
        if mutual:
            keep_lo.append(np.minimum(lo[i], lo[j]))
            keep_hi.append(np.maximum(hi[i], hi[j]))
            merged += 1
        else:
            keep_lo.append(lo[i])
            keep_hi.append(hi[i])
    return np.array(keep_lo), np.array(keep_hi), merged


@pytest.mark.parametrize("seed", [0, 1])
def test_ploc_every_pass_merges(seed):
    rng = np.random.default_rng(seed)
    c = rng.uniform(-10, 10, (300, 3)).astype(np.float32)
    c = c[np.argsort(c[:, 0])]   # roughly spatial order, like Morton order
    e = rng.uniform(0.01, 1.0, (300, 3)).astype(np.float32)
    lo, hi = c - e, c + e
    passes = 0
    while len(lo) > 1:
        lo, hi, merged = ploc_pass(lo, hi, 8)
        assert merged >= 1
        passes += 1
    assert passes < 40


def test_ploc_equal_boxes_halve_per_pass():
    m = 500
    lo = np.zeros((m, 3), np.float32)
    hi = np.ones((m, 3), np.float32)
    passes = 0
    while len(lo) > 1:
        before = len(lo)
        lo, hi, merged = ploc_pass(lo, hi, 8)
        assert merged == before // 2
        passes += 1
    assert passes == int(np.ceil(np.log2(m)))


def test_device_build_child_bases_fit_24_bits(tmp_path):
    """the device build caps its node slots at 2^24 (pt_wide_dev.hpp wideDevSlotCap),
    so a child base the kernels truncate to 24 bits is reported as an error, never written."""
    import os
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    exe = str(tmp_path / "wide_dev_limits")
    subprocess.run(["g++", "-std=c++17", "-O1", "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include",
                    "-I" + os.path.join(root, "path-tracer-cuda-opengl_amd", "host"),
                    os.path.join(root, "tests", "cpp", "wide_dev_limits.cpp"), "-o", exe], check=True)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0 and r.stdout.strip() == "ok", r.stdout + r.stderr
