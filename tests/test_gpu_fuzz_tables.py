"""GPU parity of runtime scene tables under seeded random uniforms: the tables of
test_gpu_scene.py (random entries of every type, with and without extra planes,
and reference-shaped floor-last tables) seen from the random cameras and lights
of test_gpu_fuzz_uniforms.py.

Each case: the generic table kernel's counting build against the oracle's table
mode (test_gpu_parity's bar) and its production build equal to the counting
build; for the first few cases, the hiprtc-specialised kernels (rm_jit.hip)
equal to the generic kernel bit for bit, counters and sdf counts included.
"""
import os

import numpy as np
import pytest

from test_gpu_fuzz_uniforms import CASES as UCASES, H, W, _uniforms
from test_gpu_parity import _compare
from test_gpu_scene import _render, _render_spec, _same, floor_last_scene, random_scene

pytestmark = pytest.mark.gpu

# RM_FUZZ_TABLES widens the run
NTABLES = int(os.environ.get("RM_FUZZ_TABLES", "96"))
NSPEC = 6  # specialised cases: each compiles its table with hiprtc


def _case(rm, i):
    kind = i % 3
    if kind == 0:
        scene = random_scene(rm, 5000 + i)
    elif kind == 1:
        scene = random_scene(rm, 5000 + i, nplanes=1 + i % 4)
    else:
        scene = floor_last_scene(rm, 5000 + i)
    return scene, _uniforms(rm, UCASES[(7 * i) % len(UCASES)])


@pytest.mark.parametrize("i", range(NTABLES))
def test_random_tables_random_uniforms(rm, oracle, gpu, i):
    scene, u = _case(rm, i)
    ref = oracle.render(u, W, H, scene=scene)
    got = _render(rm, u, W, H, scene=scene)
    _compare(ref, got, f"table case {i}")
    prod = _render(rm, u, W, H, scene=scene, counters=False)
    np.testing.assert_array_equal(prod["rgba32f"], got["rgba32f"], err_msg=f"table case {i}")
    np.testing.assert_array_equal(prod["rgba8"], got["rgba8"], err_msg=f"table case {i}")


@pytest.mark.parametrize("i", range(NSPEC))
def test_specialised_random_uniforms_equal_generic(rm, gpu, i):
    scene, u = _case(rm, i)
    for counters in (True, False):
        _same(_render_spec(rm, u, W, H, scene, counters=counters),
              _render(rm, u, W, H, scene=scene, counters=counters))
