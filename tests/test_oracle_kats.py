"""Known-answer tests of the CPU oracle, derived analytically from
shaders/computeShader.glsl (the reference ships no tests or fixtures).
Each test cites the GLSL lines it pins."""
import numpy as np
import pytest

f32 = np.float32


@pytest.fixture(scope="module")
def U(rm):
    return rm.sweep_uniforms(-1, 120, 0, False, 0)   # frame D, iTime 0


def test_sphere_centre_is_minus_radius(oracle, U):          # glsl:83,111-112
    h = oracle.sdf(U, (15.0, 0.0, -10.0))
    assert h.hitpoint == -3.0 and h.id == 0 and h.material == 1.0
    h = oracle.sdf(U, (-25.0, 0.0, -10.0))
    assert h.hitpoint == -3.0 and h.id == 1


def test_plane_far_from_objects(oracle, U):                  # glsl:85,121
    for p in [(200.0, 3.0, 200.0), (-300.0, -1.0, 150.0), (120.0, 0.25, -400.0)]:
        h = oracle.sdf(U, p)
        assert h.id == 7 and h.material == 0.0
        assert h.hitpoint == f32(p[1]) + f32(5.5)


def test_checkers_colour(oracle, U):                         # glsl:77-80
    # int(1000+x)%2 != int(1000+z)%2 ? 1.0 : 0.2
    assert oracle.sdf(U, (200.5, 0.0, 200.5)).color[0] == pytest.approx(0.2)
    assert oracle.sdf(U, (201.5, 0.0, 200.5)).color[0] == 1.0
    assert oracle.sdf(U, (200.5, 0.0, 201.5)).color[0] == 1.0
    assert oracle.sdf(U, (201.5, 0.0, 201.5)).color[0] == pytest.approx(0.2)


def test_checkers_int_saturates(oracle, U):                  # glsl:79, DESIGN.md §2
    # int() of a value beyond the int range: GLSL leaves it undefined; the
    # contract takes gfx950's v_cvt_i32_f32 (saturating, NaN -> 0): int(1000 +
    # 3e9) = INT_MAX (odd), int(1000 - 3e9) = INT_MIN (even)
    assert oracle.sdf(U, (3.0e9, 0.0, 200.5)).color[0] == 1.0
    assert oracle.sdf(U, (3.0e9, 0.0, 201.5)).color[0] == pytest.approx(0.2)
    assert oracle.sdf(U, (-3.0e9, 0.0, 200.5)).color[0] == pytest.approx(0.2)
    assert oracle.sdf(U, (-3.0e9, 0.0, 201.5)).color[0] == 1.0
    assert oracle.sdf(U, (3.0e9, 0.0, 3.0e9)).color[0] == pytest.approx(0.2)


def test_blend_follows_itime(rm, oracle):                    # glsl:115-117
    # at the box/sphere centre both sdfs are negative: box -2.5, sphere -3
    for it in (0.0, 1.0, 2.5):
        u = rm.sweep_uniforms(-1, 120, 0, False, 0)
        u.iTime = it
        a = f32(np.sin(f32(it))) / f32(2) + f32(0.5)
        want = f32(-2.5) * (f32(1) - a) + f32(-3.0) * a
        h = oracle.sdf(u, (-5.0, 0.0, -10.0))
        assert h.id == 4 and h.hitpoint == pytest.approx(want, abs=1e-6)


def test_sky_colour_on_miss(oracle, U):                      # glsl:220,247 + escape rule :136
    ro, rd = (0.0, 50.0, 0.0), (0.0, 1.0, 0.0)
    h, steps = oracle.raymarch(U, ro, rd)
    assert h.hitpoint == -1.0 and h.id == -1 and steps < 20
    c = oracle.render_ray(U, ro, rd)
    sky = np.array([0.30, 0.36, 0.60], f32) - f32(1.0) * f32(0.2)
    np.testing.assert_allclose(c, sky ** f32(0.4545), rtol=2e-7)


def test_floor_hit_distance(oracle, U):                      # glsl:125-142 hit test d < 1e-6 t
    s = f32(1) / np.sqrt(f32(2))
    ro, rd = (60.0, 0.0, 60.0), (0.0, -float(s), float(s))
    h, steps = oracle.raymarch(U, ro, rd)
    assert h.id == 7
    assert h.hitpoint == pytest.approx(5.5 * np.sqrt(2), rel=2e-5)
    assert steps < 512


def test_step_cap_counts_as_miss(oracle, U):                 # glsl:131-141 (Q3)
    rd = np.array([1.0, -1e-4, 0.0], f32)
    rd = rd / np.linalg.norm(rd)
    h, steps = oracle.raymarch(U, (0.0, 0.0, 100.0), tuple(rd.tolist()))
    assert steps == 512 and h.hitpoint == -1.0           # grazing ray: capped, not escaped
    h, steps = oracle.raymarch(U, (0.0, 0.0, 100.0), tuple(rd.tolist()), reflected=True)
    assert steps == 256 and h.hitpoint == -1.0           # reflectedRay: MAX_STEPS/2


def test_escape_is_on_step_size_not_distance(oracle, U):     # glsl:136 (Q3)
    # reflected march escapes once a single step exceeds 200
    h, steps = oracle.raymarch(U, (0.0, 300.0, 0.0), (0.0, 1.0, 0.0), reflected=True)
    assert h.hitpoint == -1.0 and steps == 1


def test_normal_on_floor(oracle, U):                         # glsl:278-288
    n = oracle.get_normal(U, (80.0, -5.5, 80.0))
    np.testing.assert_allclose(n, [0.0, 1.0, 0.0], atol=1e-6)


def test_normal_on_sphere(oracle, U):
    n = oracle.get_normal(U, (15.0, 3.0, -10.0))             # top of sphere 0
    np.testing.assert_allclose(n, [0.0, 1.0, 0.0], atol=2e-3)


def test_unoccluded_softshadow_is_one(oracle, U):            # glsl:201-216 (Q4: t=0 -> inf)
    r, steps = oracle.softshadow(U, (0.0, 100.0, 0.0), (0.0, 1.0, 0.0), 2.0)
    assert r == 1.0 and steps == 16


def test_occluded_softshadow(oracle, U):                     # glsl:208-209
    # start inside sphere 0: first step has h < 0.001
    r, steps = oracle.softshadow(U, (15.0, 0.0, -10.0), (0.0, 1.0, 0.0), 2.0)
    assert r == pytest.approx(0.05) and steps == 1


def test_hard_shadow_is_binary(rm, oracle):                  # extension k = +inf
    u = rm.sweep_uniforms(-1, 120, 0, False, 1)
    rng = np.random.default_rng(1)
    lp = np.array(u.light.position, f32)
    vals = set()
    pts = [np.array([rng.uniform(-40, 40), -5.48, rng.uniform(-40, 20)], f32) for _ in range(100)]
    pts += [np.array([rng.uniform(-8, -2), -5.48, rng.uniform(-13, -7)], f32) for _ in range(50)]
    for p in pts:  # random floor points, plus floor points under the box (occluded)
        r, _ = oracle.softshadow(u, tuple(p.tolist()), tuple((lp - p).tolist()), float("inf"))
        vals.add(round(float(r), 6))
    assert vals <= {0.05, 1.0} and len(vals) == 2


def test_point_light_formula(oracle, U):                     # glsl:253-276
    col, n, pos = (1.0, 1.0, 1.0), (0.0, 1.0, 0.0), (-5.0, -5.5, -10.0)
    got = oracle.point_light(U, col, n, pos)
    lp = np.array([-5, 5, -10], np.float64)
    d = np.linalg.norm(lp - np.array(pos))                   # 10.5 straight below the light
    att = 1 / (1 + 0.009 * d + 0.00032 * d * d)
    ld = (lp - pos) / d
    view = np.array(pos) / np.linalg.norm(pos)
    refl = ld - 2 * np.dot(n, ld) * np.array(n)
    spec = max(np.dot(view, refl), 0) ** 32
    want = (0.8 * max(np.dot(n, ld), 0) + np.array([0.03, 0.04, 0.1]) + 0.5 * spec) * att
    np.testing.assert_allclose(got, want, rtol=1e-5)


def test_cast_ray_centre_pixel_is_forward(oracle, U):        # glsl:68-74
    ro, rd = oracle.cast_ray(U, 0.0, 0.0)
    np.testing.assert_array_equal(ro, [0, 0, 0])
    np.testing.assert_allclose(rd, [0, 0, -1], atol=1e-7)


def test_supersample_offsets_are_cumulative(rm, oracle):     # glsl:309-335 (Q1)
    u = rm.sweep_uniforms(60, 120, 1, True, 0)
    W, H, px, py = 40, 30, 17, 9
    x = f32(px * 2 - W) / f32(W)
    y = f32(py * 2 - H) / f32(H)
    acc = np.zeros(3, f32)
    for ox, oy in ((0.25, 0.25), (0.75, 0.25), (0.25, 0.75), (0.75, 0.75)):
        x = f32(x + f32(ox) / f32(W))
        y = f32(y + f32(oy) / f32(H))
        ro, rd = oracle.cast_ray(u, float(x), float(y))
        acc = (acc + oracle.render_ray(u, ro, rd)).astype(f32)
    np.testing.assert_array_equal(oracle.pixel(u, W, H, px, py)[:3], acc / f32(4))
    # in pixel units the sample positions are 0.125, 0.5, 0.625, 1.0
    assert (0.25 + 0.75 + 0.25 + 0.75) / 2 == 1.0


def test_no_aspect_correction(rm, oracle):                   # glsl:302-303 (Q2)
    u = rm.sweep_uniforms(-1, 120, 0, False, 0)
    # the right edge of any image maps to uv.x -> 1 regardless of W/H
    for W, H in ((64, 64), (128, 32)):
        x = f32((W - 1) * 2 - W) / f32(W)
        assert x == pytest.approx(1 - 2 / W)


def test_primary_floor_hit_ignores_bounces(rm, oracle):      # glsl:232-240 (Q8)
    W, H = 32, 24
    a = oracle.render(rm.sweep_uniforms(10, 120, 0, False, 0), W, H)
    b = oracle.render(rm.sweep_uniforms(10, 120, 5, False, 0), W, H)
    floor = a["counters"]["normals"]  # rows near the bottom see only the floor
    np.testing.assert_array_equal(a["rgba32f"][:4], b["rgba32f"][:4])
    assert floor > 0


def test_live_counters_exclude_dead_bounce_tail(rm, oracle):  # glsl:189-190 (Q6)
    r = oracle.render(rm.sweep_uniforms(30, 120, 5, False, 0), 64, 48)
    live, full = r["counters"], r["full_counters"]
    for k in ("rays", "march_steps"):
        assert live[k] == full[k]
    assert live["reflect_steps"] < full["reflect_steps"]
    assert r["sdf_counts"].sum() == live["sdf_evals"]


@pytest.mark.parametrize("c,q", [(0.0, 0), (1.0, 255), (0.5, 128), (2.0, 255), (-1.0, 0),
                                 (float("nan"), 0), (1 / 255, 1), (0.998, 254)])
def test_quantize(oracle, c, q):
    assert oracle.quantize(c) == q


def test_oracle_is_deterministic_across_threads(rm, oracle):
    u = rm.sweep_uniforms(77, 120, 3, True, 0)
    a = oracle.render(u, 48, 32, nthreads=1)
    b = oracle.render(u, 48, 32, nthreads=4)
    np.testing.assert_array_equal(a["rgba32f"], b["rgba32f"])
    assert a["counters"] == b["counters"]


def test_rows_subset_matches_full(rm, oracle):
    u = rm.sweep_uniforms(5, 120, 1, False, 0)
    full = oracle.render(u, 40, 30)
    sub = oracle.render(u, 40, 30, rows=[29, 3, 3, 17])
    np.testing.assert_array_equal(sub["rgba32f"], full["rgba32f"][[29, 3, 3, 17]])
