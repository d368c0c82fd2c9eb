"""Scene / ray generators shared by the CPU and GPU test modules (seeded, deterministic)."""
import struct
import zlib

import numpy as np

OBJECT_DTYPE = np.dtype([("type", "<i4"), ("mat", "<i4"), ("v", "<f4", (9,))])
MATERIAL_DTYPE = np.dtype([("type", "<i4"), ("albedo", "<f4", (3,)), ("fuzz", "<f4"), ("ir", "<f4")])


def random_soup(n_tri: int, n_sph: int, seed: int, spread: float = 10.0, n_mat: int = 4):
    """Random triangles and spheres with a mix of all three material types."""
    rng = np.random.default_rng(seed)
    objs = np.zeros(n_tri + n_sph, OBJECT_DTYPE)
    c = rng.uniform(-spread, spread, (n_tri, 3)).astype(np.float32)
    objs["type"][:n_tri] = 3
    for k in range(3):
        objs["v"][:n_tri, 3 * k:3 * k + 3] = c + rng.uniform(-1, 1, (n_tri, 3)).astype(np.float32)
    objs["type"][n_tri:] = 1
    objs["v"][n_tri:, :3] = rng.uniform(-spread, spread, (n_sph, 3)).astype(np.float32)
    objs["v"][n_tri:, 3] = rng.uniform(0.2, 1.5, n_sph).astype(np.float32)
    objs["mat"] = rng.integers(0, n_mat, len(objs))
    perm = rng.permutation(len(objs))
    objs = objs[perm]
    mats = np.zeros(n_mat, MATERIAL_DTYPE)
    for m in range(n_mat):
        t = [1, 2, 4, 1][m % 4]
        mats[m]["type"] = t
        mats[m]["albedo"] = rng.uniform(0.2, 0.9, 3)
        mats[m]["fuzz"] = 0.3 if t == 2 else 0.0
        mats[m]["ir"] = 1.5 if t == 4 else 0.0
    return objs, mats


def duplicate_centroids(n: int):
    """n identical tiny triangles (all Morton codes equal: exercises objID tie-breaking)."""
    objs = np.zeros(n, OBJECT_DTYPE)
    objs["type"] = 3
    objs["v"][:] = [0, 0, 0, 1, 0, 0, 0, 1, 0]
    objs["mat"] = 0
    mats = np.zeros(1, MATERIAL_DTYPE)
    mats["type"] = 1
    mats["albedo"] = 0.5
    return objs, mats


def random_rays(n: int, seed: int, center=(0, 0, 0), radius: float = 15.0, objects=None):
    """Rays from a sphere of origins toward the scene, plus rays aimed at object centres."""
    rng = np.random.default_rng(seed)
    o = rng.normal(size=(n, 3))
    o = o / np.linalg.norm(o, axis=1, keepdims=True) * radius + np.asarray(center)
    tgt = rng.uniform(-radius / 2, radius / 2, (n, 3)) + np.asarray(center)
    if objects is not None and len(objects):
        k = rng.integers(0, len(objects), n // 2)
        v = objects["v"][k]
        cen = np.where((objects["type"][k] == 1)[:, None], v[:, :3], (v[:, 0:3] + v[:, 3:6] + v[:, 6:9]) / 3)
        tgt[: n // 2] = cen
    d = tgt - o
    rays = np.zeros((n, 6), np.float32)
    rays[:, :3] = o
    rays[:, 3:] = d * rng.uniform(0.3, 3.0, (n, 1))   # unnormalised, as the reference's rays
    # a few axis-aligned directions (zero components -> infinite slab reciprocals)
    m = min(64, n)
    rays[:m, 3:] = 0
    rays[:m, 3 + (np.arange(m) % 3)] = np.where(np.arange(m) % 2, 1.0, -1.0)
    return rays


def rays_to_struct(rays: np.ndarray, ray_dtype) -> np.ndarray:
    out = np.zeros(len(rays), ray_dtype)
    out["o"] = rays[:, :3]
    out["d"] = rays[:, 3:]
    return out


def read_png(path):
    """Minimal reader for the 8-bit RGBA, filter-0 PNGs PngImage::write produces: (h, w, 4) uint8."""
    data = open(path, "rb").read()
    assert data[:8] == b"\x89PNG\r\n\x1a\n"
    pos, idat, w, h = 8, b"", 0, 0
    while pos < len(data):
        n, typ = struct.unpack(">I4s", data[pos:pos + 8])
        body = data[pos + 8:pos + 8 + n]
        assert zlib.crc32(typ + body) == struct.unpack(">I", data[pos + 8 + n:pos + 12 + n])[0]
        if typ == b"IHDR":
            w, h = struct.unpack(">II", body[:8])
        elif typ == b"IDAT":
            idat += body
        pos += 12 + n
    raw = np.frombuffer(zlib.decompress(idat), np.uint8).reshape(h, 1 + 4 * w)
    assert (raw[:, 0] == 0).all()
    return raw[:, 1:].reshape(h, w, 4)


def deep_stack_scene(n_group: int = 2048, L: float = 2048.0):
    """Spheres whose LBVH makes a traversal stack deeper than 32 entries (the sample-mode kernel
    keeps 32 per lane in LDS and the rest in global memory).  Every sphere's box contains the
    point (L/2, L/2, L/2), so a ray starting there hits every box and visits the whole tree.
    Morton cells are placed exactly: with radius r = L/2 and anchors at 0 and L the scene box is
    [-r, L + r] and cell = (c + r) / 4 for L = 2048.  A group of n_group spheres in cell
    (511, 511, 511) (27 one-bits in its code), plus a pair per low cell bit with that bit cleared:
    each pair is an internal left sibling on the path to the group (one push per pair), and the
    group's object-id bits add ~log2(n_group) more."""
    r = L / 2

    def centre(cell):
        return 4.0 * cell - r + 2.0

    g = 511
    cells = []
    for axis in range(3):
        for b in range(8):
            c = [g, g, g]
            c[axis] = g & ~(1 << b)
            cells += [c, c]
    cells += [[g, g, g]] * n_group
    objs = np.zeros(len(cells) + 2, OBJECT_DTYPE)
    objs["type"] = 1
    objs["mat"] = 0
    objs["v"][:len(cells), :3] = [[centre(x) for x in c] for c in cells]
    objs["v"][len(cells), :3] = 0.0
    objs["v"][len(cells) + 1, :3] = L
    objs["v"][:, 3] = r
    mats = np.zeros(1, MATERIAL_DTYPE)
    mats["type"] = 1
    mats["albedo"] = (0.5, 0.6, 0.7)
    return objs, mats


def max_stack(nodes: np.ndarray, n: int) -> int:
    """Deepest traversal stack (push left, descend right) when every box is hit."""
    best, todo = 0, [(0, 0)]
    while todo:
        i, d = todo.pop()
        best = max(best, d)
        left, right = nodes["left"][i], nodes["right"][i]
        li, ri = left < n - 1, right < n - 1
        if ri:
            todo.append((right, d + (1 if li else 0)))
        if li:
            todo.append((left, d))
    return best



def run_logged(cmd, timeout, cwd=None, env=None, log_path=None):
    """subprocess.run for the multi-process tests: stdout and stderr go to one log file (every
    rank's lines, each tagged by bench.py / ptdist with its rank and phase), the child runs in its
    own session, and on a timeout the whole process group is killed and the AssertionError carries
    the log's tail -- so a hang names its rank and phase.  Keep `timeout` below the test's pytest
    timeout so this report, not pytest-timeout's stack of the parent, is what a hang produces.
    Returns (returncode, stdout+stderr text, wall seconds)."""
    import os
    import signal
    import subprocess
    import tempfile
    import time
    if log_path is None:
        log_path = tempfile.mktemp(suffix=".log")
    t0 = time.perf_counter()
    # Every multi-process log is kept as evidence, written there WHILE the children run (a hang
    # leaves its ranks' last phases and the watchdog's stack dumps behind even if the whole call is
    # killed): PT_TEST_LOG_DIR, default gpurun_out/test_logs/ (the directory a GPU box's results
    # come back in); the test's own log_path then names the file.
    keep = os.environ.get("PT_TEST_LOG_DIR") or os.path.join(
        os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpurun_out", "test_logs")
    if keep:
        os.makedirs(keep, exist_ok=True)
        log_path = os.path.join(keep, os.path.basename(os.path.dirname(str(log_path))) + "_" +
                                os.path.basename(str(log_path)))

    def kept(text, rc):
        with open(log_path, "a") as f:
            f.write(f"\n[run_logged] rc={rc} wall={time.perf_counter() - t0:.1f} s\n")
        return text

    with open(log_path, "w+") as log:
        # the parent's situation when the child starts: its own GPU state and the box's load
        log.write(f"[run_logged] parent pid {os.getpid()}: loadavg {os.getloadavg()}, "
                  f"parent GPU context {'yes' if _parent_gpu_state() else 'no'}{_device_memory()}\n")
        log.flush()
        p = subprocess.Popen(cmd, cwd=cwd, env=env, stdout=log, stderr=subprocess.STDOUT, start_new_session=True)
        try:
            rc = p.wait(timeout=timeout)
        except subprocess.TimeoutExpired:
            try:
                os.killpg(p.pid, signal.SIGKILL)
            except ProcessLookupError:
                pass
            p.wait()
            log.seek(0)
            raise AssertionError(f"{' '.join(map(str, cmd[:8]))} ... still running after {timeout} s; log tail:\n"
                                 + kept(log.read(), "timeout")[-4000:])
        log.seek(0)
        return rc, kept(log.read(), rc), time.perf_counter() - t0


def _device_memory():
    """', device memory free / total GiB' when this process's torch has a GPU context, else ''."""
    import sys
    t = sys.modules.get("torch")
    try:
        if t is not None and t.cuda.is_initialized():
            free, total = t.cuda.mem_get_info()
            return f", device memory free {free / 2**30:.1f} of {total / 2**30:.1f} GiB"
    except Exception:   # noqa: BLE001  (diagnostic only)
        pass
    return ""


def _parent_gpu_state():
    """Whether this (pytest) process has created GPU state: torch initialised CUDA/HIP, or libpt
    (ptamd) was imported (its films and scenes hold device memory and streams)."""
    import sys
    t = sys.modules.get("torch")
    return bool((t is not None and t.cuda.is_initialized()) or "ptamd" in sys.modules)


def failure_digest(text, tail=2500):
    """The lines of a multi-rank log that name a failure (a rank's FAILED line, timeouts, errors,
    the watchdog's stack dumps and every rank's last traced phase) and then its tail."""
    keys = ("FAILED", "Timeout", "Timed out", "Error", "error", "Traceback", "Thread 0x", "File \"")
    picked = [ln for ln in text.splitlines() if any(k in ln for k in keys)]
    phases = {}
    for ln in text.splitlines():
        if "] phase: " in ln:
            phases[ln.split("]")[0] + "]"] = ln
    return ("last phase per rank:\n" + "\n".join(phases.values()) + "\n--- failure lines:\n" +
            "\n".join(picked[:80]) + "\n--- tail:\n" + text[-tail:])


def last_json(text):
    import json
    return json.loads([x for x in text.splitlines() if x.startswith("{")][-1])
