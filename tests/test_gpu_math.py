"""The render kernels' reciprocal (csrc/pt_math.hpp: v_rcp_f32 + one fused Newton step, the IEEE
division outside the checked exponent range) equals the IEEE division 1.0f / x for all 2^32 fp32
inputs, on the GPU (tools/micro/rcp_check.hip, built by the package Makefile with the kernels'
flags).  Tolerance: 0 ulp -- every triangle test, ray setup and normalisation of the reference
(triangle determinant, aabb.h:24, vec3.h:89-91) goes through it, and the frames stay bit-exact
against the oracle (test_gpu_parity.py).  The same run checks the XORWOW draw mappings
(curand_uniform and the unit-sphere coordinates 2 * (u - 0.5f), each one FMA) against their
separately rounded forms for all 2^32 draws."""
import json
import os
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHECK = os.path.join(REPO, "tools", "micro", "rcp_check")


@pytest.mark.gpu
def test_fast_reciprocal_equals_ieee_division_for_every_input():
    assert os.path.exists(CHECK), "tools/micro/rcp_check not built (make -C path-tracer-cuda-opengl_amd)"
    out = subprocess.run([CHECK], capture_output=True, text=True, timeout=120)
    assert out.returncode in (0, 1), out.stderr
    res = json.loads(out.stdout.strip().splitlines()[-1])
    assert res["inputs"] == 2 ** 32
    assert res["rcpRN_mismatches"] == 0
    assert res["newton_mismatches_in_fast_range"] == 0
    # the bare Newton step differs only for zeros / denormals and |x| >= 2^126 (denormal results)
    lo, hi = res["fast_range"]
    assert all(not (lo <= int(e) <= hi) for e in res["newton_mismatches_by_exponent"])
    # the draw mappings: uniformOf (one FMA) == x * 2^-32 + 2^-33, centered2Of == (u - 0.5f) * 2
    assert res["uniform_fma_mismatches"] == 0
    # sample mode's fast fixed-point conversion of non-negative block sums below 2^24 (blockFixedSmall)
    assert res["block_fixed_small_checked"] == 0x4B800000 + 1 and res["block_fixed_small_mismatches"] == 0
    assert res["centered2_fma_mismatches"] == 0
    assert out.returncode == 0


@pytest.mark.gpu
def test_fp16_denormal_plane_arithmetic_is_exact():
    """The wide NODE step's plane distances (pt_math.hpp planePairLo/Hi + fmaMixLo/Hi: v_perm_b32
    into fp16 denormals q * 2^-24, v_fma_mix_f32 with the scale times 2^24) equal
    fma((float)q, a, c) bit for bit: every plane byte, 2^32 random (byte, scale, offset) cases and
    the denormal / overflow edges (tools/micro/fmamix_check.hip).  Tolerance: 0 ulp."""
    check = os.path.join(REPO, "tools", "micro", "fmamix_check")
    assert os.path.exists(check), "tools/micro/fmamix_check not built (make -C path-tracer-cuda-opengl_amd)"
    out = subprocess.run([check], capture_output=True, text=True, timeout=120)
    assert out.returncode in (0, 1), out.stderr
    res = json.loads(out.stdout.strip().splitlines()[-1])
    assert res["random_tests"] == 2 ** 32
    assert res["random_mismatches"] == 0 and res["edge_mismatches"] == 0
    assert out.returncode == 0


@pytest.mark.gpu
def test_hand_written_radix_sort_and_scans():
    """The build path's device primitives (csrc/pt_sort.hip, replacing rocPRIM): the stable LSD
    radix sort equals std::stable_sort by key (values carried, inputs untouched) at sizes around its
    1024-pair tile up to 2^22 pairs, with heavy duplicates and all-equal keys, for 30 / 32 / 8 bits;
    the decoupled look-back scans (uint32 and the wide build's {x, y, z} uint4 sums) equal the
    sequential exclusive sums up to 2^23 items (tools/micro/sort_check.hip).  Exact."""
    check = os.path.join(REPO, "tools", "micro", "sort_check")
    assert os.path.exists(check), "tools/micro/sort_check not built (make -C path-tracer-cuda-opengl_amd)"
    out = subprocess.run([check], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-2000:]
    assert out.stdout.strip().splitlines()[-1] == "ok"
