"""Independent pin of the XORWOW skip-ahead of `curand_init(seed, pixel, 0)` (main.cu:262-269,
utility.h:46-62) against rocRAND's host-callable XORWOW engine.

cuRAND itself is absent from this image, so the oracle restates its semantics: the seed scramble
of curand_kernel.h, then the state after 2^67 * subsequence draws, by GF(2) jump matrices of its
own (oracle/pt_oracle.cpp).  rocRAND (/opt/rocm/include/rocrand/rocrand_xorwow.h) implements the
same generator -- the same xorshift recurrence and Weyl increment, the same 2^67-draw subsequences
-- with jump tables of its own, so it checks the oracle's skip-ahead and recurrence bit for bit.
rocRAND's seed scramble uses different constants from cuRAND's, so the probe starts from the
oracle's subsequence-0 state: the scramble stays pinned only by cuRAND's documented constants,
and the float mapping (curand_uniform != rocrand_uniform) is not compared here.

tests/cpp/rocrand_xorwow_probe.cpp is compiled with hipcc (host code only; no GPU is used).
"""
import os
import shutil
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROBE_SRC = os.path.join(ROOT, "tests", "cpp", "rocrand_xorwow_probe.cpp")
HIPCC = "/opt/rocm/bin/hipcc"
DRAWS = 16


@pytest.fixture(scope="module")
def probe(tmp_path_factory):
    if not (os.path.exists(HIPCC) and os.path.exists("/opt/rocm/include/rocrand/rocrand_xorwow.h")):
        pytest.skip("hipcc / rocRAND headers not present")
    exe = str(tmp_path_factory.mktemp("rocrand") / "rocrand_xorwow_probe")
    subprocess.run([HIPCC, "-std=c++17", "-O2", "--offload-arch=gfx950", PROBE_SRC, "-o", exe], check=True,
                   capture_output=True)
    return exe


def _rocrand(exe, state0, subsequence, k=DRAWS):
    r = subprocess.run([exe, str(k), str(subsequence), *[str(int(x)) for x in state0]], capture_output=True,
                       text=True, check=True, timeout=60)
    lines = r.stdout.split("\n")
    state = np.array([int(x) for x in lines[0].split()], np.uint32)
    draws = np.array([int(x) for x in lines[1:1 + k]], np.uint32)
    return state, draws


def _oracle_draws(orc, state, k=DRAWS):
    s = np.ascontiguousarray(state, np.uint32).copy()
    return np.array([orc.lib.orc_xorwow_next(s.ctypes.data) for _ in range(k)], np.uint32)


PIXELS = [0, 1, 2, 3, 7, 64, 1 << 10, 1 << 16, (1 << 20) + 12345, 1920 * 1080 - 1, 1920 * 1080 * 8 - 1, (1 << 31) + 5]


@pytest.mark.parametrize("seed", [1, 7, 0x1234567890ABCDEF])
def test_skip_ahead_matches_rocrand(orc, probe, seed):
    """State after curand_init(seed, pixel, 0) == rocRAND's discard_subsequence(pixel) applied to
    the oracle's pixel-0 state, for pixels spanning one bit to 2^31; and the next 16 integer draws
    agree (rocrand() vs the oracle's curand() recurrence)."""
    s0 = orc.xorwow_init(seed, 0)
    for pixel in PIXELS:
        mine = orc.xorwow_init(seed, pixel)
        theirs, tdraws = _rocrand(probe, s0, pixel)
        np.testing.assert_array_equal(mine, theirs, err_msg=f"seed {seed} pixel {pixel}: state")
        np.testing.assert_array_equal(_oracle_draws(orc, mine), tdraws, err_msg=f"seed {seed} pixel {pixel}: draws")


def test_film_states_match_rocrand(orc, probe):
    """The film's per-pixel states (the device rngInitKernel's reference, oracle.film_states over a
    1080p frame's rows) at scattered pixels, each re-derived by rocRAND from pixel 0."""
    w = 1920
    rows = np.array([0, 1, 539, 1079], np.int32)
    states = orc.film_states(1, w, rows)
    s0 = orc.xorwow_init(1, 0)
    rng = np.random.default_rng(5)
    for i, row in enumerate(rows):
        for col in [0, w - 1, int(rng.integers(1, w - 1))]:
            pixel = int(row) * w + col
            theirs, _ = _rocrand(probe, s0, pixel, 0)
            np.testing.assert_array_equal(states[i * w + col], theirs, err_msg=f"pixel {pixel}")


def test_probe_detects_a_wrong_jump(orc, probe):
    """Negative control: one subsequence off, or the recurrence without the jump, disagrees."""
    s0 = orc.xorwow_init(1, 0)
    theirs, _ = _rocrand(probe, s0, 5)
    assert not np.array_equal(orc.xorwow_init(1, 4), theirs)
    assert not np.array_equal(orc.xorwow_init(1, 6), theirs)
    assert shutil.which(HIPCC) or os.path.exists(HIPCC)
