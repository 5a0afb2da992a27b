"""The squared bounding-ball cull test (rm_scene.hpp ball_needs) culls only
where the square-root form's margin proves the primitive above the minimum.

ball_needs(x, U, R) evaluates primitive k iff RN(x (1 - 2^-11)) <= RN(a^2),
a = RN(U + CULL_ABS + R), x = |p - c_k|^2 (all float32, round to nearest).  It
replaced v_sqrt(x) (1 - 2^-12) - CULL_ABS - R <= U for the torus and capsule
(scene_cull, normal_samples) and all five primitives in the soft-shadow march
(DESIGN.md §4.4 item 13 e, f).  Soundness: a cull must imply, in real
arithmetic, sqrt(x) (1 - 2^-12) - CULL_ABS - R - U > -1.5 ulp (U + CULL_ABS + R):
the root form's 2^-12 relative margin less at most what the v_sqrt form it
replaced could lose (v_sqrt is within 1.5 ulp), far inside the margin, which
covers the ~2^-21 float error of the sdfs.  (Measured worst case of the squared
form: -0.46 ulp.)  Checked here on float32 samples packed around the
boundary, for every radius the kernels use, U both signs.  CPU only.
"""
import numpy as np
import pytest

CULL_ABS = np.float32(2.0 ** -18)
SQ_LO = np.float32(1.0 - 2.0 ** -11)
RADII = [3.0, 4.63682, 3.45115]  # spheres and torus (3), blend circumradius, capsule


def ball_needs(x, U, R):
    a = (U + np.float32(CULL_ABS + np.float32(R))).astype(np.float32)
    return (x * SQ_LO).astype(np.float32) <= (a * a).astype(np.float32)


@pytest.mark.parametrize("R", RADII)
def test_squared_cull_is_sound(R):
    rng = np.random.default_rng(12345)
    n = 400_000
    U = np.concatenate([rng.uniform(-8.0, 8.0, n // 2), rng.uniform(-8.0, 400.0, n // 2)]).astype(np.float32)
    c = float(np.float32(CULL_ABS + np.float32(R)))  # the float32 constant both forms use
    # x around the boundary sqrt(x) (1 - 2^-12) = U + c, relative offsets down to 2^-24
    rb = np.maximum((U.astype(np.float64) + c) / (1.0 - 2.0 ** -12), 0.0)
    delta = rng.choice([-1.0, 1.0], n) * np.exp2(rng.uniform(-24.0, -6.0, n))
    x = (rb * rb * (1.0 + delta)).astype(np.float32)
    x = np.where(rng.random(n) < 0.05, rng.uniform(0.0, 100.0, n).astype(np.float32), x)
    culled = ~ball_needs(x, U, R)
    U64 = U.astype(np.float64)
    slack = np.sqrt(x.astype(np.float64)) * (1.0 - 2.0 ** -12) - c - U64
    bad = culled & ~(slack > -1.5 * 2.0 ** -24 * np.maximum(U64 + c, 0.0))
    assert not bad.any(), f"{int(bad.sum())} unsound culls, e.g. x={x[bad][:3]} U={U[bad][:3]}"
    # the test is not vacuous: both outcomes occur near the boundary
    assert 0.2 < culled.mean() < 0.8


def test_squared_cull_nan_culls():
    assert not ball_needs(np.float32([4.0]), np.float32([np.nan]), 3.0)[0]
